"""Print the compiled (folded + CSE + fused) program of a synthetic model on a
device: op histogram and the ops that did not fuse (they run as PyTorch ops).

    python scripts/program_ops.py --model bert-base --device cuda:0
"""
import argparse
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="bert-base", choices=["bert-base", "resnet50"])
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--fuse", action="store_true", help="run the fusion passes on a CPU device too")
    a = ap.parse_args()
    from rust_tensorflow_serving2_amd.models import bert, resnet
    from rust_tensorflow_serving2_amd.server.servable import Servable, ServableOptions
    path = os.path.join(tempfile.mkdtemp(), "1")
    if a.model == "bert-base":
        bert.export(path, seed=0)
        ins, outs = ["input_ids", "input_mask", "segment_ids"], ["pooled_output", "probabilities"]
    else:
        resnet.export(path, seed=0)
        ins, outs = ["input"], ["classes", "probabilities"]
    s = Servable(a.model, 1, path, ServableOptions(device=a.device, max_batch_size=4,
                                                       fuse=True if a.fuse else None))
    r = s.runner("serving_default", ins, outs)
    prog = r.program
    print(sorted(prog.op_histogram().items(), key=lambda x: -x[1]))
    for _fn, node, _i, _o in prog.steps:
        if not node.op.startswith("_"):
            print(f"  {node.op:16s} {node.name}  <- {[f'{n}:{i}' for n, i in node.inputs]}")


if __name__ == "__main__":
    main()
