"""gfx950 HIP kernel bindings (``_hip``) + tile-config autotuning.

The extension is built in-tree by ``_build.build_hip`` (hipcc
--offload-arch=gfx950).  On a machine with a GPU the fused graph ops *require*
it: :func:`hip` raises if the ``.so`` is missing instead of silently falling
back to PyTorch, so a GPU test that passes has run the native kernels.
"""
from __future__ import annotations

import os
import threading
from typing import Callable, Dict, Tuple

import torch

_HIP = None
_LOCK = threading.Lock()


class KernelsUnavailable(RuntimeError):
    pass


def hip():
    """The loaded ``_hip`` extension (raises loudly when missing)."""
    global _HIP
    if _HIP is None:
        with _LOCK:
            if _HIP is None:
                try:
                    from .. import _hip as mod  # type: ignore
                except ImportError as e:
                    raise KernelsUnavailable(
                        "rust_tensorflow_serving2_amd._hip is not built (run "
                        "`python -m rust_tensorflow_serving2_amd._build`): " + str(e)) from e
                _HIP = mod
    return _HIP


def available() -> bool:
    try:
        hip()
        return torch.cuda.is_available()
    except KernelsUnavailable:
        return False


ACT = {"none": 0, "relu": 1, "gelu_tanh": 2, "gelu_erf": 3, "tanh": 4}

# ------------------------------------------------------------------ autotune
_TUNED: Dict[Tuple, int] = {}
_TUNE_LOCK = threading.Lock()
AUTOTUNE = os.environ.get("TFSERVE_AUTOTUNE", "1") != "0"


def heuristic_config(M: int, N: int) -> int:
    """0=128x128, 1=128x64, 2=64x128, 3=64x64 — fill 256 CUs first."""
    def tiles(bm, bn):
        return -(-M // bm) * -(-N // bn)
    if N <= 64:
        return 1 if tiles(128, 64) >= 256 else 3
    if tiles(128, 128) >= 512:
        return 0
    if tiles(128, 64) >= 256:
        return 1
    return 3


def tuned_config(key: Tuple, M: int, N: int, launch: Callable[[int], None]) -> int:
    """Pick the fastest tile config for ``key`` by timing each once (eager only —
    never during HIP-graph capture; falls back to the heuristic there)."""
    cfg = _TUNED.get(key)
    if cfg is not None:
        return cfg
    if not AUTOTUNE or torch.cuda.is_current_stream_capturing():
        return heuristic_config(M, N)
    with _TUNE_LOCK:
        cfg = _TUNED.get(key)
        if cfg is not None:
            return cfg
        n = hip().num_configs()
        best, best_t = heuristic_config(M, N), float("inf")
        for c in range(n):
            launch(c)   # warm (also sets the kernel's LDS attribute)
            start = torch.cuda.Event(enable_timing=True)
            end = torch.cuda.Event(enable_timing=True)
            start.record()
            for _ in range(3):
                launch(c)
            end.record()
            end.synchronize()
            t = start.elapsed_time(end)
            if t < best_t:
                best, best_t = c, t
        _TUNED[key] = best
        return best


def tuned_table() -> Dict[Tuple, int]:
    return dict(_TUNED)
