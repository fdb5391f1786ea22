"""Concurrent status + metadata on cloned clients (``examples/async.rs``).

    python examples/async_requests.py -m resnet [--hostname 127.0.0.1] [--port 9000]

Clones share one HTTP/2 channel (``src/lib.rs:148-156``); both RPCs are in
flight at once as multiplexed streams, then joined (``examples/async.rs:29-52``).
(Named ``async_requests.py`` because ``async`` is a Python keyword and could
not be imported as a module.)
"""
import argparse
import asyncio
import logging
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from rust_tensorflow_serving2_amd.client import TensorflowServing  # noqa: E402


def parse(argv=None):
    ap = argparse.ArgumentParser(prog="async")
    ap.add_argument("-m", "--model", required=True)
    ap.add_argument("--hostname", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=9000)
    return ap.parse_args(argv)


async def main(argv=None):
    logging.basicConfig(level=os.environ.get("LOGLEVEL", "WARNING"))
    opts = parse(argv)
    client = await TensorflowServing.new().hostname(opts.hostname).port(opts.port).build()
    c1, c2 = client.clone(), client.clone()
    results = await asyncio.gather(c1.model_status(opts.model), c2.model_metadata(opts.model),
                                   return_exceptions=True)
    for r in results:
        if isinstance(r, BaseException):
            print(f"task failed: {r}", file=sys.stderr)
        else:
            print(r)
    return results


if __name__ == "__main__":
    asyncio.run(main())
