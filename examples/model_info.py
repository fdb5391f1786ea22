"""Model status + metadata, then a working reload (``examples/model_info.rs``).

    python examples/model_info.py -m resnet [--hostname 127.0.0.1] [--port 9000] [--reload-base-path /models/resnet]

The reference leaves its reload commented out because its sample config used
``base_path: "/"``, which made the model unavailable after the reload
superseded the config (``examples/model_info.rs:41-57``).  Here the reload is
opt-in and uses the real base path, so the model stays AVAILABLE.
"""
import argparse
import asyncio
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from rust_tensorflow_serving2_amd.client import ModelConfig, TensorflowServing, unpack_signature_defs  # noqa: E402


def parse(argv=None):
    ap = argparse.ArgumentParser(prog="model_info")
    ap.add_argument("-m", "--model", required=True)
    ap.add_argument("--hostname", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=9000)
    ap.add_argument("--reload-base-path", default=None,
                    help="if set, send HandleReloadConfigRequest with this base_path and show the new status")
    return ap.parse_args(argv)


async def main(argv=None):
    opts = parse(argv)
    client = await TensorflowServing.new().hostname(opts.hostname).port(opts.port).build()
    status = await client.model_status(opts.model)
    print(status)
    metadata = await client.model_metadata(opts.model)
    print(metadata.model_spec)
    for name, sig in sorted(unpack_signature_defs(metadata).items()):
        print(f"signature {name!r}: method={sig.method_name} inputs={sorted(sig.inputs)} outputs={sorted(sig.outputs)}")
    if opts.reload_base_path:
        cfg = ModelConfig(name=opts.model, base_path=opts.reload_base_path, model_platform="tensorflow")
        print(await client.reload([cfg]))
        print(await client.model_status(opts.model))
    return status, metadata


if __name__ == "__main__":
    asyncio.run(main())
