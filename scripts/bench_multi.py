"""BASELINE config 5: multi-model hot reload -- ResNet-50 + BERT-base
co-resident on every GPU, ResNet traffic continuous, BERT dropped and re-added
by HandleReloadConfigRequest ``--reload-cycles`` times.

Run through ``bench.py --model multi`` (same launcher, placement and rank
layout as the headline benchmark).  What it reports (rank 0's JSON line; all
ranks' numbers aggregated):

* ``value``: ResNet-50 Predict RPC/s over the whole run (reload windows
  included), summed over ranks;
* ``bert_rps``: BERT-base Predict RPC/s while it is loaded;
* ``resnet_p99_ms_steady`` / ``resnet_p99_ms_during_reload``: ResNet latency
  outside / inside the reload windows (a reload compiles, tunes and captures
  BERT on the same GPU while ResNet batches keep running);
* ``reload_to_available_s``: per cycle, from the re-adding reload RPC to
  BERT AVAILABLE (get_model_status.proto:44-53); ``unload_s``: the dropping
  reload until BERT is gone (UNLOADING before unavailable, model_service.proto:19-21);
* ``device_mem_high_water_gb``: peak device memory in use (hipMemGetInfo,
  sampled) and the caching allocator's peak reservation;
* ``errors``: failed ResNet calls (must be 0) and failed BERT calls sent
  while BERT was AVAILABLE (must be 0).

The reference could not do this at all: its reload example is commented out
because the sample config made the model unavailable (examples/model_info.rs:41-57).
"""
from __future__ import annotations

import asyncio
import json
import os
import threading
import time

import numpy as np

PREDICT = "/tensorflow.serving.PredictionService/Predict"


def _cfg(models):
    from rust_tensorflow_serving2_amd.schema import serving
    cfg = serving.ModelServerConfig()
    for name, base in models:
        mc = cfg.model_config_list.config.add()
        mc.name = name
        mc.base_path = base
        mc.model_platform = "tensorflow"
    return cfg


def run(args, rank, world, device, on_gpu, dist, topology, placement, pinned):
    import torch
    from rust_tensorflow_serving2_amd import _C, native
    from rust_tensorflow_serving2_amd.client import TensorflowServing
    from rust_tensorflow_serving2_amd.models import bert, resnet
    from rust_tensorflow_serving2_amd.server.server import ModelServer, ServerOptions
    from rust_tensorflow_serving2_amd.server.servable import ServableOptions
    import tempfile

    root = os.path.join(tempfile.gettempdir(), f"tfserve_bench_{os.environ.get('MASTER_PORT', 'solo')}", "multi")
    base_r, base_b = os.path.join(root, "resnet"), os.path.join(root, "bert")
    if rank == 0:
        if not os.path.exists(os.path.join(base_r, "1", "saved_model.pb")):
            if args.image_size == 224:
                resnet.export(os.path.join(base_r, "1"), seed=0)
            else:      # CPU test mode: same graph vocabulary, tiny
                resnet.export(os.path.join(base_r, "1"), seed=0, image_size=args.image_size, blocks=(1, 1, 1, 1),
                              width=8, num_classes=1001)
        if not os.path.exists(os.path.join(base_b, "1", "saved_model.pb")):
            bc = bert.BertConfig(seq_len=args.seq_len) if on_gpu else \
                bert.BertConfig(vocab_size=1000, seq_len=args.seq_len, layers=2, hidden=128, heads=2,
                                intermediate=256)
            bert.export(os.path.join(base_b, "1"), bc, seed=0)
    if world > 1:
        dist.barrier()
    both = _cfg([("resnet", base_r), ("bert", base_b)])
    only_r = _cfg([("resnet", base_r)])

    weight_source = None
    if world > 1:
        from rust_tensorflow_serving2_amd.parallel.weights import ReplicatedWeightSource
        weight_source = ReplicatedWeightSource(dist.distributed_c10d._get_default_store(), device=device)
    sopts = ServableOptions(device=str(device), max_batch_size=args.batch, lanes=args.lanes,
                            allowed_batch_sizes=tuple(sorted({1, 2, 4, 8, 16, args.batch})))
    server = ModelServer(ServerOptions(port=0, host="127.0.0.1", model_config=both, device=str(device),
                                       transport="native", servable=sopts, io_threads=args.io_threads,
                                       batch_timeout_us=args.batch_timeout_us, file_system_poll_wait_seconds=0,
                                       weight_source=weight_source, monitoring=False))
    t_load = time.perf_counter()
    server.start()
    t_load = time.perf_counter() - t_load
    tr = server.transports[0]

    def endpoints():
        return set(k.split("/")[0] for k in tr.stats().get("endpoints", {}))

    def wait_eps(want, timeout=900.0):
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < timeout:
            if want(endpoints()):
                return time.perf_counter() - t0
            time.sleep(0.01)
        raise SystemExit(f"endpoints never became {want}: {endpoints()}")
    wait_eps(lambda e: {"resnet", "bert"} <= e)

    rng = np.random.default_rng(1234 + rank)
    spec_r = native.spec_tuple("resnet", None, None, "serving_default")
    spec_b = native.spec_tuple("bert", None, None, "serving_default")
    S = args.seq_len
    bodies_r = [native.encode_predict_request(
        spec_r, {"input": rng.random((1, args.image_size, args.image_size, 3), dtype=np.float32)})
        for _ in range(args.distinct_requests)]
    bodies_b = []
    for _ in range(16):
        ids = rng.integers(0, 30522 if on_gpu else 1000, (1, S)).astype(np.int32)
        mask = np.ones((1, S), np.int32)
        seg = np.zeros((1, S), np.int32)
        bodies_b.append(native.encode_predict_request(spec_b, {"input_ids": ids, "input_mask": mask,
                                                               "segment_ids": seg}))
    conc = args.concurrency or 4 * args.batch
    lg_r = _C.LoadGen("127.0.0.1", server.port, PREDICT, bodies_r, conc, args.connections, args.client_threads)
    lg_b = _C.LoadGen("127.0.0.1", server.port, PREDICT, bodies_b, min(conc, 64), 4, 1)

    # ResNet: continuous windows on a background thread (time-stamped)
    windows = []                     # (t_start, t_end, ok, errors, latencies)
    stop = threading.Event()
    chunk = max(32, args.batch * 4)

    def resnet_traffic():
        lg_r.start()
        while not stop.is_set():
            t = time.perf_counter()
            r = lg_r.window(chunk, 600.0)
            windows.append((t, time.perf_counter(), r["ok"], r["errors"], r["latency_us"], r["first_error"]))
        lg_r.stop(30.0)

    mem = {"used_max": 0.0}

    def sample_mem():
        if on_gpu:
            free, total = torch.cuda.mem_get_info(device)
            mem["used_max"] = max(mem["used_max"], (total - free) / 2 ** 30)

    def bert_window(n):
        r = lg_b.run(n, 300.0)
        return r["ok"], r["errors"], r["elapsed_s"], r["first_error"]

    async def reload(cfg):
        c = await TensorflowServing.new().hostname("127.0.0.1").port(server.port).build()
        resp = await c.reload(cfg.model_config_list.config)
        return resp.status.error_code, resp.status.error_message

    def status_bert():
        from rust_tensorflow_serving2_amd.client import TFServingError

        async def go():
            c = await TensorflowServing.new().hostname("127.0.0.1").port(server.port).build()
            try:
                r = await c.model_status("bert")
                return [int(v.state) for v in r.model_version_status]
            except TFServingError:
                return []
        return asyncio.run(go())

    def mem_sampler():
        while not stop.wait(0.05):
            sample_mem()

    th = threading.Thread(target=resnet_traffic, name="tfs-bench-r", daemon=True)
    th.start()
    thm = threading.Thread(target=mem_sampler, name="tfs-bench-mem", daemon=True)
    thm.start()
    t_run0 = time.perf_counter()
    bert_ok = bert_err = 0
    bert_s = 0.0
    first_errs = []
    lg_b.run(max(16, args.batch), 120.0)           # warm BERT's connections
    time.sleep(args.prewarm_s)
    reload_windows = []
    cycles = []
    for cyc in range(args.reload_cycles + 1):
        sample_mem()
        ok, err, el, fe = bert_window(args.bert_requests)
        bert_ok, bert_err, bert_s = bert_ok + ok, bert_err + err, bert_s + el
        if fe:
            first_errs.append(fe)
        sample_mem()
        if cyc == args.reload_cycles:
            break
        if world > 1:
            dist.barrier()
        # drop BERT (the new config supersedes: model_service.proto:19-21)
        t0 = time.perf_counter()
        # (each rank is its own server here: every rank reloads in lockstep,
        # so the replicas load BERT in the same order for the weight broadcast)
        code, msg = asyncio.run(reload(only_r))
        if code:
            raise SystemExit(f"reload (drop) failed: {code} {msg}")
        wait_eps(lambda e: "bert" not in e)
        t_unload = time.perf_counter() - t0
        st_after_drop = status_bert()
        if world > 1:
            dist.barrier()
        # re-add it: load, compile, tune, capture while ResNet keeps serving
        t1 = time.perf_counter()
        code, msg = asyncio.run(reload(both))
        if code:
            raise SystemExit(f"reload (re-add) failed: {code} {msg}")
        wait_eps(lambda e: "bert" in e)
        t_avail = time.perf_counter() - t1
        reload_windows.append((t0, time.perf_counter()))
        cycles.append({"unload_s": round(t_unload, 3), "reload_to_available_s": round(t_avail, 3),
                       "bert_states_after_drop": st_after_drop})
        sample_mem()
    stop.set()
    th.join(timeout=120)
    thm.join(timeout=5)
    t_run = time.perf_counter() - t_run0

    ok_r = sum(w[2] for w in windows)
    err_r = sum(w[3] for w in windows)
    first_errs += [w[5] for w in windows if w[5]]
    t_span = (windows[-1][1] - windows[0][0]) if windows else 1.0

    def in_reload(w):
        return any(w[0] < b and w[1] > a for a, b in reload_windows)
    lat_reload = np.concatenate([np.asarray(w[4], np.float64) for w in windows if in_reload(w)] or [np.zeros(0)])
    lat_steady = np.concatenate([np.asarray(w[4], np.float64) for w in windows if not in_reload(w)] or
                                [np.zeros(0)])
    mine = {
        "rank": rank, "resnet_ok": ok_r, "resnet_errors": err_r, "resnet_span_s": t_span,
        "resnet_p50_ms_steady": float(np.percentile(lat_steady, 50)) / 1e3 if lat_steady.size else None,
        "resnet_p99_ms_steady": float(np.percentile(lat_steady, 99)) / 1e3 if lat_steady.size else None,
        "resnet_p99_ms_during_reload": float(np.percentile(lat_reload, 99)) / 1e3 if lat_reload.size else None,
        "resnet_calls_during_reload": int(lat_reload.size),
        "bert_ok": bert_ok, "bert_errors": bert_err, "bert_s": bert_s, "cycles": cycles,
        "device_mem_used_gb_max": round(mem["used_max"], 2),
        "allocator_reserved_gb_max": round(torch.cuda.max_memory_reserved(device) / 2 ** 30, 2) if on_gpu else None,
        "first_errors": first_errs[:3], "load_s": round(t_load, 2), "run_s": round(t_run, 2),
        "placement": dict(placement.as_dict(), pinned=pinned),
    }
    if world > 1:
        allr = [None] * world
        dist.all_gather_object(allr, mine)
    else:
        allr = [mine]
    if rank == 0:
        rps = sum(r["resnet_ok"] / max(r["resnet_span_s"], 1e-9) for r in allr)
        bert_rps = sum(r["bert_ok"] / max(r["bert_s"], 1e-9) for r in allr)
        p99r = [r["resnet_p99_ms_during_reload"] for r in allr if r["resnet_p99_ms_during_reload"] is not None]
        p99s = [r["resnet_p99_ms_steady"] for r in allr if r["resnet_p99_ms_steady"] is not None]
        out = {
            "metric": "Multi-model hot reload (HandleReloadConfigRequest): ResNet-50 + BERT-base co-resident, "
                      "ResNet Predict RPCs/sec during BERT drop/re-add cycles",
            "value": round(rps, 1), "unit": "Predict RPCs/s (ResNet-50)", "n_gpus": world,
            "higher_is_better": True, "dtype": "bf16" if on_gpu else "fp32 (cpu test mode)",
            "data": "synthetic 224x224x3 f32 images + int32 token ids, random-init ResNet-50 v1.5 and BERT-base",
            "config": {"models": ["ResNet-50 v1.5", f"BERT-base seq {S}"], "server_batch": args.batch,
                       "reload_cycles": args.reload_cycles, "parallelism": f"dp{world}"},
            "bert_rps": round(bert_rps, 1),
            "resnet_p99_ms_steady": round(max(p99s), 3) if p99s else None,
            "resnet_p99_ms_during_reload": round(max(p99r), 3) if p99r else None,
            "reload_to_available_s": [c["reload_to_available_s"] for c in allr[0]["cycles"]],
            "unload_s": [c["unload_s"] for c in allr[0]["cycles"]],
            "device_mem_high_water_gb": max(r["device_mem_used_gb_max"] for r in allr),
            "allocator_reserved_gb_max": allr[0]["allocator_reserved_gb_max"],
            "errors": int(sum(r["resnet_errors"] + r["bert_errors"] for r in allr)),
            "per_rank": allr,
        }
        print(json.dumps(out), flush=True)
    server.stop()
