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

``TFSERVE_HW_QUEUES`` overrides the count (0 leaves the environment alone).
Must run before anything initialises HIP (importing torch does not;
``torch.cuda`` calls do).
"""
import os


def apply(default: str = "8") -> None:
    want = os.environ.get("TFSERVE_HW_QUEUES", default)
    if want and want != "0":
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, max(1, int(want))))
