"""gfx950 HIP kernel bindings (``_hip``) + tile-config autotuning.

The extension is built in-tree by ``_build.build_hip`` (hipcc
--offload-arch=gfx950).  On a machine with a GPU the fused graph ops *require*
it: :func:`hip` raises if the ``.so`` is missing instead of silently falling
back to PyTorch, so a GPU test that passes has run the native kernels.
"""
from __future__ import annotations

import contextlib
import gc
import itertools
import os
import threading
import weakref
from typing import Callable, Dict, List, Optional, Sequence, Tuple

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
# per key: [(median cold launch ms, (config, splits))] ascending, from tuned_config
_TUNE_TIMES: Dict[Tuple, List[Tuple[float, Tuple[int, int]]]] = {}
_GRAPH_TUNED: set = set()
_REC = threading.local()
# tile picks another replica made (parallel/weights.py: the leader tunes, the
# followers install its table) keyed by repr(key): used instead of tuning
_REMOTE: Dict[str, Tuple[int, int]] = {}


def _table_schema() -> str:
    """Identity of the tile-config tables a cached pick refers to."""
    import hashlib
    return hashlib.sha1(repr(sorted(TILES.items())).encode()).hexdigest()[:12]


TUNED_CACHE = os.environ.get("TFSERVE_TUNED_CACHE",
                             os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned_mi355x.json"))


def load_tuned_cache(path: Optional[str] = None) -> int:
    """Install tile picks measured earlier on this GPU model (a committed
    table, like a library's performance database): keys found there are
    neither autotuned nor graph-tuned at capture.  The table is keyed by the
    exact launch shape and only used when its config-table schema and device
    (gfx arch, CU count) match this process.  Returns the entries installed."""
    import json
    path = path or TUNED_CACHE
    if not path or path == "0" or not os.path.exists(path):
        return 0
    try:
        with open(path) as f:
            doc = json.load(f)
    except (OSError, ValueError):
        return 0
    if doc.get("schema") != _table_schema():
        return 0
    if torch.cuda.is_available():
        p = torch.cuda.get_device_properties(torch.cuda.current_device())
        if doc.get("arch") != getattr(p, "gcnArchName", "").split(":")[0] or \
                int(doc.get("cus", -1)) != p.multi_processor_count:
            return 0
    install_remote_tuned(doc.get("picks", {}))
    return len(doc.get("picks", {}))


def save_tuned_cache(path: str, keys=None) -> int:
    """Write the current picks (all, or ``keys``) in load_tuned_cache's format."""
    import json
    p = torch.cuda.get_device_properties(torch.cuda.current_device())
    with _TUNE_LOCK:
        picks = {repr(k): list(v) for k, v in _TUNED.items() if keys is None or k in keys}
    doc = {"schema": _table_schema(), "arch": getattr(p, "gcnArchName", "").split(":")[0],
           "cus": p.multi_processor_count, "picks": picks}
    with open(path + ".tmp", "w") as f:
        json.dump(doc, f, indent=0, sort_keys=True)
    os.replace(path + ".tmp", path)
    return len(picks)


def install_remote_tuned(table: Dict[str, list]) -> None:
    with _TUNE_LOCK:
        for k, v in table.items():
            _REMOTE[k] = (int(v[0]), int(v[1]))


def tuned_table_for(keys) -> Dict[str, list]:
    """{repr(key): [cfg, splits]} of the picks made for ``keys`` (to publish)."""
    return {repr(k): list(_TUNED[k]) for k in keys if k in _TUNED}


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


# (BM, BN) per igemm config; configs 4.. add deeper direct-to-LDS DMA rings
# (kernels/igemm.hip kCfgST) and only apply to dense / im2col operands.
TILES = {0: (128, 128), 1: (128, 64), 2: (64, 128), 3: (64, 64),
         4: (128, 128), 5: (64, 64), 6: (128, 64), 7: (64, 128),
         8: (64, 256), 9: (256, 64), 10: (128, 256), 11: (256, 128),
         12: (64, 64), 13: (64, 64), 14: (64, 128), 15: (128, 64), 16: (128, 128)}
DMA_ONLY = {4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16}
TILE_BK = {12: 128, 13: 256, 14: 128, 15: 128, 16: 128}     # k-tile depth (default 64)
# pipelined cgemm kernel (kernels/cgemm.hip; 64-aligned operands only): config id -> (BM, BN)
CGEMM = {32: (128, 128), 33: (128, 128), 34: (64, 128), 35: (128, 64), 36: (64, 64),
         37: (256, 128), 38: (128, 256), 39: (128, 128), 40: (64, 256), 41: (256, 64),
         42: (64, 64), 43: (64, 128), 44: (128, 64), 45: (128, 96), 46: (128, 96), 47: (64, 96),
         64: (64, 64), 65: (64, 64), 66: (64, 64), 67: (128, 64), 68: (64, 128), 69: (128, 64), 70: (64, 128),
         71: (64, 64), 72: (256, 192), 73: (256, 144), 74: (128, 96), 75: (128, 96)}
# fragment-prefetch (PF) builds of 11 of those tiles (kernels/cgemm.hip kPfOf)
CGEMM_PF_OF = [32, 34, 35, 36, 39, 41, 42, 43, 44, 45, 71]
CGEMM.update({96 + k: CGEMM[base] for k, base in enumerate(CGEMM_PF_OF)})
# v_mfma_f32_32x32x16_bf16 builds (kernels/cgemm32.hip, ids 112..123: wave tiles in 32x32 blocks)
CGEMM32 = {112: (64, 64), 113: (64, 64), 114: (128, 128), 115: (128, 64), 116: (64, 128), 117: (128, 256),
           118: (256, 128), 119: (256, 64), 120: (128, 128), 121: (64, 128), 122: (128, 64), 123: (256, 192)}
CGEMM.update(CGEMM32)
# (ids 124..137, the 32-deep k-tile and persistent multi-tile builds, were removed in round 6:
# 0 of 192 picks in the round-5 table)
# big-tile ping-pong builds (kernels/bgemm.hip, ids 140..142): 8 waves of 128 x 64 / 128 x 32 / 128 x 48,
# dense operands only (other operand modes are rejected at launch and skipped by the tuner)
BGEMM = {140: (256, 256), 141: (256, 128), 142: (256, 192)}
CGEMM.update(BGEMM)
TILES.update(CGEMM)
# halo-tiled 3x3 stride-1 conv (kernels/halo.hip): config id -> (output pixels per tile, BN)
HALO = {48: (256, 64), 49: (128, 128), 50: (128, 64), 51: (64, 64), 52: (256, 128), 53: (64, 128), 54: (64, 64),
        55: (128, 64), 56: (256, 64), 57: (128, 64), 58: (128, 64)}
# the same tiles with the fragment-prefetch step pipeline (halo.hip PF)
HALO.update({cfg + 32: tile for cfg, tile in list(HALO.items()) if cfg != 52})
# (ids 144/145, the ping-pong halo kernel, were removed in round 6: 0 picks)
# the persistent halo kernel (halo.hip halo_persist_kernel): C == 64 and N == 64, the whole
# filter resident in LDS, plain bf16 output; other operand modes are rejected at launch
HALO_PERSIST = 146
HALO[HALO_PERSIST] = (128, 64)
# TFSERVE_PINGPONG=0: leave the ping-pong builds (bgemm 140-142) out of the
# tuner's candidates (A/B of the tile tables with and without them)
PINGPONG = os.environ.get("TFSERVE_PINGPONG", "1") != "0"
TILES.update(HALO)


def heuristic_splits(M: int, N: int, K: int, cfg: int) -> int:
    bm, bn = TILES[cfg]
    tiles = -(-M // bm) * -(-N // bn)
    nk = -(-K // 64)
    s = 1
    while tiles * s < 256 and nk // (s * 2) >= 4 and s < 16:
        s *= 2
    return s


def candidates(M: int, N: int, K: int, dma: bool = True, aligned64: bool = False, cgemm_only: bool = False,
               halo: bool = False, no_split: bool = False, stem: bool = False, ln: bool = False):
    """(tile config, split-K) pairs worth timing for an M x N x K problem
    (``dma``: the operand mode uses the direct-to-LDS path, so the deeper
    DMA-ring configs apply; ``aligned64``: K and the conv channels are
    multiples of 64, so the pipelined cgemm configs apply; ``halo``: a 3x3
    stride-1 conv with C % 64 == 0, so the halo-tiled configs apply too —
    their split-K granule is a 64-channel chunk of 9 taps; ``stem``: the
    padded RGBA stem operand, which the 32-deep and persistent builds do not
    take)."""
    nk = -(-K // 64)
    out = []
    if halo and aligned64 and K % 576 == 0 and N % 8 == 0:
        nch = K // 576
        for cfg, (bm, bn) in HALO.items():
            if bn > 64 and N <= bn // 2:
                continue
            if cfg == HALO_PERSIST:
                if K == 576 and N == 64:
                    out.append((cfg, 1))     # one chunk, no split-K
                continue
            tiles = -(-M // bm) * -(-N // bn)
            for s in (1, 2, 4, 8):
                if s > 1 and (nch // s < 1 or tiles >= 512 or tiles * s > 2048):
                    continue
                out.append((cfg, s))
    for cfg, (bm, bn) in TILES.items():
        if cfg in HALO:
            continue
        if cfg in DMA_ONLY and (not dma or (cfg in (4, 5, 6, 7) and nk < 3)):
            continue
        if cfg in CGEMM and not (aligned64 and K % 64 == 0 and N % 8 == 0):
            continue
        if cgemm_only and cfg not in CGEMM:
            continue
        if cfg in BGEMM and (stem or ln or not PINGPONG):
            continue   # dense operands, plain epilogues only
        if ln and (cfg not in CGEMM or bn % 32):
            continue   # deferred LayerNorm: cgemm tiles (4-aligned chunk lanes per row)
        if K < 2 * TILE_BK.get(cfg, 64) and cfg in TILE_BK:
            continue   # deep k-tiles only pay off with several of them
        if bn > 64 and N <= bn // 2 or bm > 64 and M <= bm // 2:
            continue   # mostly-empty tiles
        if bn % 64 and N % bn:
            continue   # 96-wide tiles: only where they divide N (BERT's 768 / 2304 / 3072)
        tiles = -(-M // bm) * -(-N // bn)
        for s in (1, 2, 4, 8, 16):
            if s > 1 and (no_split or nk // s < 2 or tiles >= 1024 or tiles * s > 4096):
                continue
            out.append((cfg, s))
    return out


_CACHE_STATE = {"loaded": False, "entries": 0}
_CACHE_LOCK = threading.Lock()


def _ensure_cache() -> None:
    if not _CACHE_STATE["loaded"]:
        with _CACHE_LOCK:
            if not _CACHE_STATE["loaded"]:
                _CACHE_STATE["loaded"] = True
                if AUTOTUNE:
                    _CACHE_STATE["entries"] = load_tuned_cache()


_REGIME = threading.local()


@contextlib.contextmanager
def tuning_regime(conc: int):
    """Tile picks made inside the block are for ``conc`` batches in flight at
    once (the serving regime of a loaded server: each lane replays its graph on
    its own stream).  Such picks live under their own keys (``key + (("conc",
    conc),)``), so the isolated-replay picks of the same shapes stay separate,
    and a candidate is ranked by its throughput with ``conc`` streams running
    it concurrently: a few large tiles that leave CUs idle alone can win there,
    because the idle CUs run the other streams' kernels
    (scripts/conc_sweep.py: the stage-4 3x3 layer 17.3 -> 11.9 us per launch
    at 3 streams with the concurrent pick, profiles/round5/s2/conc.log).

    Measured, not adopted (off unless TFSERVE_CONC_TUNE=1): picks made this
    way lost in the real serving regime, where the concurrent kernels are
    different layers -- ResNet-50 b32 at 4 in flight 0.659 ms per batch and
    47.8k RPC/s against 0.59 / 52.4k with the isolated screen + whole-graph
    concurrent tuner (profiles/round5/s3/).  Big-LDS tiles that pair up well
    with copies of themselves block other layers' workgroups from the CUs."""
    prev = getattr(_REGIME, "conc", 1)
    _REGIME.conc = max(1, int(conc)) if CONC_TUNE else 1
    try:
        yield
    finally:
        _REGIME.conc = prev


def regime_key(key: Tuple) -> Tuple:
    c = getattr(_REGIME, "conc", 1)
    return key if c <= 1 else tuple(key) + (("conc", c),)


CONC_TUNE = os.environ.get("TFSERVE_CONC_TUNE", "0") == "1"
CONC_TUNE_MAX = int(os.environ.get("TFSERVE_CONC_TUNE_MAX", "24"))     # candidates timed concurrently
CONC_TUNE_RATIO = float(os.environ.get("TFSERVE_CONC_TUNE_RATIO", "3.0"))


def _time_concurrent(launch: Callable[[int, int], None], cands, conc: int, flush: torch.Tensor,
                     reps: int = 6, trials: int = 3) -> List[Tuple[float, Tuple[int, int]]]:
    """Per-launch ms of each candidate at ``conc`` streams: every stream
    replays a graph of ``reps`` launches at once (graphs, so the host's
    launch cost is not in the sample), L2 flushed before each trial.  The
    launches of all streams write the same output (identical values)."""
    streams = [torch.cuda.Stream() for _ in range(conc)]
    cur = torch.cuda.current_stream()
    out = []
    for c, s in cands:
        graphs = []
        try:
            for st in streams:
                g = torch.cuda.CUDAGraph()
                st.wait_stream(cur)
                with capture_owner(g), torch.cuda.stream(st):
                    g.capture_begin(capture_error_mode="thread_local")
                    try:
                        for _ in range(reps):
                            launch(c, s)
                    finally:
                        g.capture_end()
                graphs.append(g)
            for g, st in zip(graphs, streams):
                with torch.cuda.stream(st):
                    g.replay()
            torch.cuda.synchronize()
            samples = []
            for _ in range(trials):
                flush.zero_()
                start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                start.record(cur)
                for g, st in zip(graphs, streams):
                    st.wait_event(start)
                    with torch.cuda.stream(st):
                        g.replay()
                for st in streams:
                    cur.wait_stream(st)
                end.record(cur)
                end.synchronize()
                samples.append(start.elapsed_time(end) / (reps * conc))
            samples.sort()
            out.append((samples[len(samples) // 2], (c, s)))
        except RuntimeError:
            torch.cuda.synchronize()
        finally:
            del graphs
    return sorted(out)


def tuned_config(key: Tuple, M: int, N: int, launch: Callable[[int, int], None], K: int = 64,
                 dma: bool = True, aligned64: bool = False, cgemm_only: bool = False,
                 halo: bool = False, no_split: bool = False, stem: bool = False,
                 ln: bool = False) -> Tuple[int, int]:
    """Pick the fastest (tile config, split-K) for ``key`` by timing each
    candidate (eager only — never during HIP-graph capture, where the
    heuristic is used).  Inside ``tuning_regime(k > 1)`` the pick is the
    best aggregate throughput at k concurrent streams, under its own key."""
    key = regime_key(key)
    conc = getattr(_REGIME, "conc", 1)
    rec = getattr(_REC, "keys", None)
    if rec is not None:
        rec[key] = rec.get(key, 0) + 1
    _ensure_cache()
    hit = _TUNED.get(key)
    if hit is not None:
        return hit
    remote = _REMOTE.get(repr(key)) if _REMOTE else None
    if remote is not None:
        with _TUNE_LOCK:
            _TUNED[key] = remote
            _GRAPH_TUNED.add(key)          # the leader already graph-tuned it
        return remote
    if not AUTOTUNE or torch.cuda.is_current_stream_capturing():
        c = (36 if no_split else 42) if cgemm_only else heuristic_config(M, N)
        return c, 1 if no_split else heuristic_splits(M, N, K, c)
    with _TUNE_LOCK:
        hit = _TUNED.get(key)
        if hit is not None:
            return hit
        best, best_t = None, float("inf")
        times = []
        flush = _flush_buffer()
        cands = candidates(M, N, K, dma, aligned64, cgemm_only, halo, no_split, stem, ln)
        for c, s in cands:
            try:
                launch(c, s)   # warm (also sets the kernel's LDS attribute)
            except RuntimeError:
                # a host-side launch rejection (an operand mode the config does
                # not take): not a candidate.  Device faults are not caught here
                # -- they surface at the synchronize below and end the tuning.
                continue
            samples = []
            for _rep in range(5):
                # evict the L2s first: inside the serving graph a layer's weights
                # arrive cold and its neighbours' activations have moved through
                # the caches, so one cold launch is the representative sample.
                # (Timing warm back-to-back bursts instead picked configs that
                # lost in the graph, e.g. BERT FFN1 on 64x64 tiles.)
                flush.zero_()
                # keep the GPU busy while the host records the start event and
                # issues the launch, so the sample is the kernel's own time, as
                # in a graph replay, not the host's per-launch work (which is
                # larger for split-K candidates: workspace, counter slice)
                torch.cuda._sleep(_HOST_SHADOW_CYCLES)
                start = torch.cuda.Event(enable_timing=True)
                end = torch.cuda.Event(enable_timing=True)
                start.record()
                launch(c, s)
                end.record()
                end.synchronize()
                samples.append(start.elapsed_time(end))
            samples.sort()
            t = samples[len(samples) // 2]
            times.append((t, (c, s)))
            if t < best_t:
                best, best_t = (c, s), t
        times.sort()
        if best is None:
            raise RuntimeError(f"no tile config could launch {key} (M={M} N={N} K={K})")
        if conc > 1 and times:
            # the serving regime: rank the plausible candidates (isolated time
            # within CONC_TUNE_RATIO of the best, at most CONC_TUNE_MAX) by
            # their throughput at `conc` concurrent streams
            pool = [cs for t, cs in times if t <= times[0][0] * CONC_TUNE_RATIO][:CONC_TUNE_MAX]
            ctimes = _time_concurrent(launch, pool, conc, flush)
            if ctimes:
                times = ctimes
                best = ctimes[0][1]
        _TUNE_TIMES[key] = times
        _TUNED[key] = best
        return best


def tuned_choice(key: Tuple, options: Dict[int, Callable[[], None]], default: int) -> int:
    """Pick the fastest of a few whole implementations of one op (e.g. a
    chained two-conv kernel vs the two convs) for ``key`` -- timed like
    tuned_config (cold L2, median of 5 single launches), stored with the tile
    picks (``(option, 1)``: the committed table, the replicas' shared table and
    graph_tune, which re-times the options inside the whole replay, all apply).
    Options that raise RuntimeError are skipped; ``default`` during capture or
    without autotuning."""
    key = regime_key(key)
    rec = getattr(_REC, "keys", None)
    if rec is not None:
        rec[key] = rec.get(key, 0) + 1
    _ensure_cache()
    hit = _TUNED.get(key)
    if hit is not None:
        return hit[0]
    remote = _REMOTE.get(repr(key)) if _REMOTE else None
    if remote is not None:
        with _TUNE_LOCK:
            _TUNED[key] = remote
            _GRAPH_TUNED.add(key)
        return remote[0]
    if not AUTOTUNE or torch.cuda.is_current_stream_capturing():
        return default
    ok = {}
    for o, fn in options.items():
        try:
            fn()            # warm: the option's own tile picks are made here, outside the lock
            ok[o] = fn
        except RuntimeError:
            continue
    if not ok:
        raise RuntimeError(f"no implementation could run {key}")
    with _TUNE_LOCK:
        hit = _TUNED.get(key)
        if hit is not None:
            return hit[0]
        flush = _flush_buffer()
        times = []
        for o, fn in ok.items():
            samples = []
            for _rep in range(5):
                flush.zero_()
                torch.cuda._sleep(_HOST_SHADOW_CYCLES)
                start = torch.cuda.Event(enable_timing=True)
                end = torch.cuda.Event(enable_timing=True)
                start.record()
                fn()
                end.record()
                end.synchronize()
                samples.append(start.elapsed_time(end))
            samples.sort()
            times.append((samples[len(samples) // 2], (o, 1)))
        times.sort()
        _TUNE_TIMES[key] = times
        _TUNED[key] = times[0][1]
        return times[0][1][0]


@contextlib.contextmanager
def record_tuned_keys():
    """Collect {key: uses} of every tuned_config lookup made on this thread
    inside the block (one program run -> the tunable launches it makes)."""
    keys: Dict[Tuple, int] = {}
    prev = getattr(_REC, "keys", None)
    _REC.keys = keys
    try:
        yield keys
    finally:
        _REC.keys = prev


def graph_tune_params(bucket: int) -> dict:
    """graph_tune knobs (env overrides for experiments): TFSERVE_GRAPH_TUNE_TOP,
    _RATIO, _MIN_US."""
    out = {}
    if os.environ.get("TFSERVE_GRAPH_TUNE_TOP"):
        out["top"] = int(os.environ["TFSERVE_GRAPH_TUNE_TOP"])
    if os.environ.get("TFSERVE_GRAPH_TUNE_RATIO"):
        out["ratio"] = float(os.environ["TFSERVE_GRAPH_TUNE_RATIO"])
    if os.environ.get("TFSERVE_GRAPH_TUNE_MIN_US"):
        out["min_ms"] = float(os.environ["TFSERVE_GRAPH_TUNE_MIN_US"]) / 1e3
    return out


def graph_tune(keys: Dict[Tuple, int], time_fn: Callable[[], float], top: int = 4, ratio: float = 1.35,
               min_ms: float = 0.012) -> Dict[Tuple, Tuple[int, int]]:
    """Re-pick tile configs by timing the WHOLE program (``time_fn`` captures
    and replays it, returning ms) instead of one cold launch per kernel: inside
    a replay a GEMM's operands arrive from the previous kernel and its
    neighbours' tails overlap it, which the isolated timings do not see.

    Coordinate descent over ``keys`` (largest estimated share first); each key
    tries its ``top`` fastest isolated candidates within ``ratio`` of the best.
    Keys whose isolated time is under ``min_ms`` (launch-floor bound) or that
    were already graph-tuned are skipped.  Returns the changed picks."""
    todo = []
    for k, uses in keys.items():
        times = _TUNE_TIMES.get(k)
        if k in _GRAPH_TUNED or not times or times[0][0] < min_ms:
            continue
        cands = [c for t, c in times[:top] if t <= times[0][0] * ratio]
        if len(cands) > 1:
            todo.append((times[0][0] * uses, k, cands))
    changed: Dict[Tuple, Tuple[int, int]] = {}
    if not todo:
        _GRAPH_TUNED.update(keys)
        return changed
    todo.sort(key=lambda x: -x[0])
    time_fn()                            # first capture/replay runs slow: discard it
    base = time_fn()
    for _w, k, cands in todo:
        cur = _TUNED[k]
        best_t, best_c = base, cur
        for c in cands:
            if c == cur:
                continue
            _TUNED[k] = c
            t = time_fn()
            if t < best_t * 0.995:       # ignore sub-noise wins
                best_t, best_c = t, c
        _TUNED[k] = best_c
        if best_c != cur:
            changed[k] = best_c
            base = best_t
    _GRAPH_TUNED.update(keys)
    return changed


FIXUP_MAX_BUCKET = 8     # batch buckets up to this finish split-K in-kernel


@contextlib.contextmanager
def splitk_fixup_for_bucket(bucket: int):
    """Around a bucket's tuning + capture: in-kernel split-K (no reduce launch)
    for the small buckets, the separate reduce for the large ones (see
    kernels/bindings.cpp split_fixup_mode for the measurements)."""
    try:
        h = hip()
    except KernelsUnavailable:
        yield
        return
    # thread-local in the extension (the capture runs on this thread); the
    # previous mode is restored, so nested / re-entrant use composes
    prev = h.set_splitk_fixup(1 if bucket <= FIXUP_MAX_BUCKET else 0)
    try:
        yield
    finally:
        h.set_splitk_fixup(-1 if prev is None else int(prev))


_HEAD_ROWS = threading.local()


@contextlib.contextmanager
def head_host_rows(rows):
    """Around a serving lane's capture: ``rows`` = (probs_ptr, probs_width,
    classes_ptr) of the lane's pinned output rows (0 = none), or None.  A
    one-launch classifier head captured inside stores its rows there too and
    tags its outputs (``_tfs_host``), so the lane can drop their D2H copies
    (two ~4.5-us blit kernels at batch 1).  TFSERVE_HEAD_HOST=0: off."""
    prev = getattr(_HEAD_ROWS, "rows", None)
    _HEAD_ROWS.rows = rows if os.environ.get("TFSERVE_HEAD_HOST", "1") != "0" else None
    try:
        yield
    finally:
        _HEAD_ROWS.rows = prev


def current_head_host_rows():
    return getattr(_HEAD_ROWS, "rows", None)


_OWNER_SEQ = itertools.count(1)
_GC_HOLD = [0]
_GC_LOCK = threading.Lock()


@contextlib.contextmanager
def _no_gc():
    """Python's cyclic GC off while a capture runs on this thread: a
    collection there can finalize an unreachable server's CUDAGraph, whose
    destructor frees its private pool (hipFree) on the capturing thread --
    illegal mid-capture, and the C++ error inside a destructor aborts the
    process (seen once in the GPU suite: abort under "Garbage-collecting" in a
    fast-path test's capture).  Counted, since captures on several threads
    overlap; torch.cuda.graph's own gc.collect() still runs before capture."""
    with _GC_LOCK:
        _GC_HOLD[0] += 1
        if _GC_HOLD[0] == 1:
            _GC_HOLD.append(gc.isenabled())
            gc.disable()
    try:
        yield
    finally:
        with _GC_LOCK:
            _GC_HOLD[0] -= 1
            if _GC_HOLD[0] == 0 and _GC_HOLD.pop():
                gc.enable()


@contextlib.contextmanager
def capture_owner(graph, replay_streams: Sequence = ()):
    """Around a HIP-graph capture: the split-K arrival counters its launches
    take (the split-K fixup) belong to ``graph`` and go back to the pool
    when the graph object is collected, so tuning candidates and reload
    cycles do not use the counter pool up (kernels/counters.cpp).  The
    return is stream-ordered: the capturing stream (recorded by the pool)
    and ``replay_streams`` (other streams the graph will replay on) each get
    a fence; the slices are zeroed on the lane's stream and reused only after
    every fence and that memset have completed.  Python's GC is held off for
    the capture (``_no_gc``)."""
    with _no_gc():
        try:
            h = hip()
        except KernelsUnavailable:
            yield None
            return
        # released slices whose fences have completed come back zeroed before
        # this capture can take them; the rest stay pending (never blocks)
        if hasattr(h, "splitk_counters_reclaim"):
            h.splitk_counters_reclaim()
        tok = next(_OWNER_SEQ)
        h.splitk_counters_set_owner(tok)
        for st in replay_streams:
            h.splitk_counters_add_stream(tok, int(st.cuda_stream))
        try:
            yield tok
        finally:
            h.splitk_counters_set_owner(0)
            weakref.finalize(graph, h.splitk_counters_release, tok)


_FLUSH: Dict[int, torch.Tensor] = {}


_HOST_SHADOW_CYCLES = 150_000      # ~60 us of GPU spin: longer than the host's launch path


def _flush_buffer() -> torch.Tensor:
    """64 MB scratch per device (> the 8 x 4 MB L2 of an MI355X)."""
    dev = torch.cuda.current_device()
    buf = _FLUSH.get(dev)
    if buf is None:
        buf = _FLUSH[dev] = torch.empty(64 << 20, dtype=torch.uint8, device=f"cuda:{dev}")
    return buf


def tuned_table() -> Dict[Tuple, int]:
    return dict(_TUNED)
