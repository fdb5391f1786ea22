"""``python -m rust_tensorflow_serving2_amd.server`` — the model server binary.

Replaces the stock container the reference starts with
``docker run -p 9000:8500 -p 9001:8501 -v $(pwd)/models:/models/resnet
-e MODEL_NAME=resnet tensorflow/serving`` (``serving/rundocker.sh:15``).  Flag
names follow TensorFlow Serving's ``tensorflow_model_server`` so existing
launch scripts keep working::

    python -m rust_tensorflow_serving2_amd.server --port=8500 --rest_api_port=8501 \\
        --model_name=resnet --model_base_path=/models/resnet --num_gpus=8

``--num_gpus N`` (N > 1, or 0 = every visible GPU) starts one replica process
per GPU (``parallel/replicas.py``): all replicas share the gRPC/REST ports via
SO_REUSEPORT, weights are read once and broadcast over RCCL, and reload
requests are replicated to every GPU.  The same entry point runs under
``torchrun`` (it honours RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*).
"""
from __future__ import annotations

import argparse
import logging
import os
import signal
import sys
import threading
import time
from typing import List, Optional

log = logging.getLogger("tfserve.cli")


def _bool(v: str) -> bool:
    return str(v).lower() in ("1", "true", "yes", "on")


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="python -m rust_tensorflow_serving2_amd.server",
                                 description="MI355X-native TensorFlow-Serving-compatible model server")
    a = ap.add_argument
    a("--port", type=int, default=8500, help="gRPC port (PredictionService + ModelService)")
    a("--rest_api_port", type=int, default=0, help="REST/HTTP port (0 = disabled)")
    a("--host", "--grpc_host", default="0.0.0.0", dest="host")
    # MODEL_NAME / MODEL_BASE_PATH env: the tensorflow/serving container convention
    # (serving/rundocker.sh:15 passes -e MODEL_NAME=resnet)
    a("--model_name", default=os.environ.get("MODEL_NAME", "default"))
    a("--model_base_path", default=os.environ.get("MODEL_BASE_PATH", ""))
    a("--model_config_file", default="", help="text-format ModelServerConfig (supersedes --model_name/base_path)")
    a("--model_config_file_poll_wait_seconds", type=float, default=0.0)
    a("--file_system_poll_wait_seconds", type=float, default=1.0)
    a("--enable_batching", type=_bool, nargs="?", const=True, default=False)
    a("--batching_parameters_file", default="", help="text-format BatchingParameters")
    a("--enable_model_warmup", type=_bool, nargs="?", const=True, default=True)
    a("--monitoring", type=_bool, nargs="?", const=True, default=True,
      help="Prometheus metrics at /monitoring/prometheus/metrics on the REST port")
    # MI355X-specific
    a("--device", default="auto", help="auto | cpu | cuda[:i] (replicas always use cuda:LOCAL_RANK)")
    a("--num_gpus", type=int, default=1, help="replica processes, one per GPU (0 = all visible GPUs)")
    a("--transport", default="native", choices=["native", "grpc"],
      help="native = C++ HTTP/2 front end with the Predict fast path; grpc = grpcio server")
    a("--io_threads", type=int, default=4, help="native transport epoll threads (per replica)")
    a("--batch_timeout_us", type=int, default=2000, help="fast-path batch window when batching params unset")
    a("--idle_dispatch", type=_bool, nargs="?", const=True, default=True,
      help="fast path: run a partly filled batch immediately when no batch of its model is executing "
           "(batch-1 latency without the batch window; under load batches still fill)")
    a("--max_batch_size", type=int, default=32, help="fast-path GPU batch (HIP-graph bucket) limit")
    a("--hip_graphs", type=_bool, nargs="?", const=True, default=True)
    a("--dtype", default="bf16", choices=["bf16", "fp32"],
      help="GPU compute dtype: bf16 = fused MFMA kernels; fp32 = unfused fp32 reference path")
    a("--trace_dir", default="", help="write request/batch timelines (JSON lines) here")
    a("--health_failure_threshold", type=int, default=8,
      help="consecutive failed batches after which a servable is reloaded (0 = no health monitor)")
    a("--health_max_recoveries", type=int, default=3, help="reloads of one version before it is quarantined")
    a("--route_streams", type=_bool, nargs="?", const=True, default=True,
      help="replicas: route individual Predicts to the least-loaded replica over shared memory "
           "(one client connection still uses every GPU)")
    a("--log_level", default="INFO")
    return ap


def _read_text_proto(path: str, msg):
    from google.protobuf import text_format
    with open(path) as f:
        text_format.Parse(f.read(), msg)
    return msg


def make_server(args, rank: int = 0, world: int = 1):
    """Build a ModelServer for this process (replica ``rank`` of ``world``)."""
    import torch
    from ..schema import serving
    from .servable import ServableOptions
    from .server import ModelServer, ServerOptions

    if world > 1:
        device = f"cuda:{int(os.environ.get('LOCAL_RANK', rank))}" if args.device in ("auto", "cuda") or \
            args.device.startswith("cuda") else "cpu"
    elif args.device == "auto":
        device = "cuda:0" if torch.cuda.is_available() else "cpu"
    elif args.device == "cuda":
        device = "cuda:0"
    else:
        device = args.device
    batching = None
    if args.enable_batching and args.batching_parameters_file:
        batching = _read_text_proto(args.batching_parameters_file, serving.BatchingParameters())
    weight_source = replicas = router = None
    if world > 1:
        import torch.distributed as dist
        from ..parallel.replicas import ReplicaControl
        from ..parallel.weights import ReplicatedWeightSource
        dev = torch.device(device)
        if dev.type == "cuda":
            torch.cuda.set_device(dev)
        restarts = int(os.environ.get("TFSERVE_RESTARTS", "0"))
        store_addr = os.environ.get("TFSERVE_STORE", "")
        store = None
        if store_addr:
            # the supervisor's store (parallel/replicas.py launch): outlives any replica
            from datetime import timedelta
            host, sport = store_addr.rsplit(":", 1)
            store = dist.TCPStore(host, int(sport), is_master=False, timeout=timedelta(seconds=120))
        from datetime import timedelta
        if restarts == 0:
            if not dist.is_initialized():
                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                backend = "nccl" if dev.type == "cuda" else "gloo"
                kw = {"device_id": dev} if dev.type == "cuda" else {}
                # bounded: a collective whose peer died must fail, not hang the replica
                kw["timeout"] = timedelta(seconds=300)
                if store is not None:
                    dist.init_process_group(backend, store=dist.PrefixStore("tfs/pg", store), rank=rank,
                                            world_size=world, **kw)
                else:
                    dist.init_process_group(backend, **kw)
            if store is None:
                store = dist.distributed_c10d._get_default_store()
        # a replacement replica (restarted by the supervisor) joins the group of
        # the current generation at the leader's next load; the models the group
        # already holds it reads from disk
        if store is not None:
            weight_source = ReplicatedWeightSource(store, device=dev, rank=rank, world=world,
                                                   restarted=restarts > 0)
        replicas = ReplicaControl(store, rank, world, restarted=restarts > 0)
        router = (os.environ.get("TFSERVE_ROUTE_GROUP") or f"p{os.environ.get('MASTER_PORT', '0')}", rank, world)
    sopts = ServableOptions(device=device, hip_graphs=args.hip_graphs, warmup=args.enable_model_warmup,
                            max_batch_size=args.max_batch_size, compute_dtype=args.dtype,
                            fuse=False if args.dtype == "fp32" else None)
    opts = ServerOptions(port=args.port, rest_api_port=args.rest_api_port, host=args.host,
                         model_name=args.model_name, model_base_path=args.model_base_path,
                         model_config_file=args.model_config_file,
                         model_config_file_poll_wait_seconds=args.model_config_file_poll_wait_seconds,
                         device=device, enable_batching=args.enable_batching, batching_parameters=batching,
                         transport=args.transport, file_system_poll_wait_seconds=args.file_system_poll_wait_seconds,
                         io_threads=args.io_threads, batch_timeout_us=args.batch_timeout_us,
                         idle_dispatch=args.idle_dispatch, servable=sopts,
                         monitoring=args.monitoring, weight_source=weight_source, replicas=replicas,
                         trace_dir=args.trace_dir, health_failure_threshold=args.health_failure_threshold,
                         health_max_recoveries=args.health_max_recoveries,
                         router=router if args.route_streams else None)
    return ModelServer(opts)


def _write_stats(server, stats_dir: str, rank: int):
    """Per-replica counters at shutdown (TFSERVE_STATS_DIR; multi-replica tests)."""
    import json
    d = {"rank": rank, "pid": os.getpid(), "restarts": int(os.environ.get("TFSERVE_RESTARTS", "0"))}
    for t in server.transports:
        if hasattr(t, "srv") and hasattr(t.srv, "router_stats"):
            st = t.srv.stats()
            rs = dict(t.srv.router_stats())
            d["requests"] = st["requests"]
            d["router"] = rs
            d["served"] = st["requests"] - rs.get("forwarded", 0)   # answered by this replica's device
    ws = getattr(server.opts, "weight_source", None)
    if ws is not None:
        d["weights"] = {k: v for k, v in ws.stats.items() if isinstance(v, (int, float))}
        d["weights"]["gen"] = ws.gen
    os.makedirs(stats_dir, exist_ok=True)
    path = os.path.join(stats_dir, f"replica{rank}.{os.getpid()}.json")
    with open(path + ".tmp", "w") as f:
        json.dump(d, f)
    os.replace(path + ".tmp", path)


def serve(args, rank: int = 0, world: int = 1, ready: Optional[threading.Event] = None,
          stop: Optional[threading.Event] = None) -> int:
    server = make_server(args, rank, world)
    server.start()
    log.info("replica %d/%d serving gRPC on %s:%d%s", rank, world, args.host, server.port,
             f", REST on {server.rest_port}" if getattr(server, "rest_port", None) else "")
    print(f"[tfserve] replica {rank}/{world} ready: pid={os.getpid()} grpc={server.port}"
          + (f" rest={server.rest_port}" if getattr(server, "rest_port", None) else ""), flush=True)
    stop = stop or threading.Event()
    signalled = []
    if threading.current_thread() is threading.main_thread():
        # the handler only flips a flag: Event.set() from a signal handler can
        # deadlock against the main thread's own Event.wait() (same lock)
        for s in (signal.SIGINT, signal.SIGTERM):
            signal.signal(s, lambda *_: signalled.append(1))
    if ready is not None:
        ready.set()
    stats_dir = os.environ.get("TFSERVE_STATS_DIR")
    n = 0
    while not signalled and not stop.is_set():
        time.sleep(0.1)
        n += 1
        if stats_dir and n % 5 == 0:
            _write_stats(server, stats_dir, rank)
    if stats_dir:
        _write_stats(server, stats_dir, rank)
    server.stop()
    if world > 1:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()
    return 0


def main(argv: Optional[List[str]] = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    import faulthandler
    faulthandler.register(signal.SIGUSR1, all_threads=True)     # `kill -USR1 <pid>` dumps stacks
    args = build_parser().parse_args(argv)
    logging.basicConfig(level=getattr(logging, args.log_level.upper(), logging.INFO),
                        format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env > 1:                       # a replica (launched by us or by torchrun)
        return serve(args, int(os.environ.get("RANK", "0")), world_env)
    n = args.num_gpus
    if n == 0:
        # sysfs KFD topology: the supervisor never initialises the HIP runtime
        from ..parallel.replicas import count_gpus
        n = max(1, count_gpus())
    if n > 1:
        from ..parallel.replicas import launch
        return launch(argv, n)
    return serve(args)


if __name__ == "__main__":
    sys.exit(main())
