"""Synthesize the model repository (``serving/fetch.sh`` equivalent, no network).

The reference downloads ``resnet_v2_fp32_savedmodel_NHWC`` and copies version
``1538687283`` into ``models/1/`` plus an ``example.jpg`` (``serving/fetch.sh:7-31``).
Offline, we write random-init SavedModels of the same architectures in the
same ``<root>/<name>/<version>/`` layout:

    python serving/make_models.py --root serving/models [--models resnet,resnet_v2,bert,half_plus_two]

* ``resnet``        ResNet-50 v1.5 (NHWC, alias "input", outputs classes/probabilities)
* ``resnet_v2``     ResNet-50 v2 pre-activation (the fetch.sh model's architecture)
* ``bert``          BERT-base seq 128 (input_ids / input_mask / segment_ids)
* ``half_plus_two`` TF Serving's canonical test model

and ``example.jpg`` (a synthetic 224x224 RGB image).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--root", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "models"))
    ap.add_argument("--models", default="resnet,half_plus_two")
    ap.add_argument("--version", type=int, default=1)
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args(argv)
    import numpy as np
    from rust_tensorflow_serving2_amd.models import half_plus_two, resnet
    for m in [m.strip() for m in args.models.split(",") if m.strip()]:
        out = os.path.join(args.root, m, str(args.version))
        if os.path.exists(os.path.join(out, "saved_model.pb")):
            print(f"exists: {out}")
            continue
        if m == "resnet":
            resnet.export(out, seed=args.seed)
        elif m == "resnet_v2":
            resnet.export(out, seed=args.seed, version="v2")
        elif m == "bert":
            from rust_tensorflow_serving2_amd.models import bert
            bert.export(out, bert.BertConfig(), seed=args.seed)
        elif m == "half_plus_two":
            half_plus_two.export(out)
        else:
            raise SystemExit(f"unknown model {m}")
        print(f"wrote {out}")
    from PIL import Image
    rng = np.random.default_rng(args.seed)
    img = os.path.join(args.root, "example.jpg")
    Image.fromarray(rng.integers(0, 256, (224, 224, 3), dtype=np.uint8)).save(img)
    print(f"wrote {img}")


if __name__ == "__main__":
    main()
