"""Predict one image (``examples/prediction.rs``).

    python examples/prediction.py image.jpg -m resnet [--version 1] [--hostname 127.0.0.1] [--port 9000]

Same flags and defaults as the reference example (``examples/prediction.rs:5-17``);
preprocessing is ``value / 255.`` (``:43``) and the response is pretty-printed (``:46``).
"""
import argparse
import asyncio
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from rust_tensorflow_serving2_amd.client import ModelDescription, TensorflowServing, to_image  # noqa: E402


def parse(argv=None):
    ap = argparse.ArgumentParser(prog="prediction")
    ap.add_argument("image")
    ap.add_argument("-m", "--model", required=True)
    ap.add_argument("--version", type=int, default=None)
    ap.add_argument("--hostname", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=9000)
    return ap.parse_args(argv)


async def main(argv=None):
    opts = parse(argv)
    img = to_image(opts.image)
    client = await TensorflowServing.new().hostname(opts.hostname).port(opts.port).build()
    model = ModelDescription(opts.model, opts.version)
    resp = await client.predict_with_preprocessing(img, model, lambda v: v / 255.0)
    print(resp)
    return resp


if __name__ == "__main__":
    asyncio.run(main())
