"""HIP runtime settings a serving process applies before the runtime starts.

``GPU_MAX_HW_QUEUES`` (hardware queues per process; HIP's default is 4): a
server replays a HIP graph per lane on its own stream -- 4 lanes plus the
copy engines' streams.  With 4 queues, streams beyond the fourth share a
queue and their work serialises behind each other; with 8, four concurrent
ResNet-50 b32 replays ran 0.529 vs 0.595 ms per batch (0.604 vs 0.637 ms with
the H2D / D2H copies) in ``scripts/probe_concurrency.py``, and the headline
bench averaged 45.6k vs 40.8k RPC/s over four interleaved pairs on one box
(``profiles/round3/hw_queues/``).

With two models co-resident (8 lanes) the extra queues let more replays run
at once than the caches hold: config 5 measured 31.0k vs 35.3k ResNet RPC/s
and 25.3 vs 10.7 ms p99 during reloads (``profiles/round3/hw_queues/``), so
callers serving several models pass ``default="4"``.

``TFSERVE_HW_QUEUES`` overrides the count (0 leaves the environment alone);
a ``GPU_MAX_HW_QUEUES`` the operator exported is kept unless
``TFSERVE_HW_QUEUES`` asks otherwise.  Must run before anything initialises
HIP (importing torch does not; ``torch.cuda`` calls do).
"""
import os
import re
from typing import Optional, Sequence


def apply(default: str = "8", force: bool = False) -> None:
    """``force``: the caller's count replaces an inherited GPU_MAX_HW_QUEUES
    (bench.py, whose measured configuration must not depend on the box's
    environment); TFSERVE_HW_QUEUES still overrides both."""
    want = os.environ.get("TFSERVE_HW_QUEUES")
    if want is None:
        if os.environ.get("GPU_MAX_HW_QUEUES") and not force:
            return                      # the operator's explicit setting wins over our default
        want = default
    if want and want != "0":
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, max(1, int(want))))


def models_in_config(argv: Sequence[str]) -> int:
    """Models a server command line will load: the ``config { ... }`` entries
    of its ``--model_config_file`` (text-format ModelServerConfig), else 1."""
    path: Optional[str] = None
    for i, a in enumerate(argv):
        if a.startswith("--model_config_file="):
            path = a.split("=", 1)[1]
        elif a == "--model_config_file" and i + 1 < len(argv):
            path = argv[i + 1]
    if not path:
        return 1
    try:
        with open(path) as f:
            text = f.read()
    except OSError:
        return 1
    return max(1, len(re.findall(r"(?m)^\s*config\s*[:{]", text)))


def server_default(argv: Sequence[str]) -> str:
    """Queues for a server process: 8 for one model, 4 when the config names
    several (their lanes together would oversubscribe the caches, see above)."""
    return "4" if models_in_config(argv) > 1 else "8"
