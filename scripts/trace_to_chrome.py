"""Convert --trace_dir JSON lines into a chrome://tracing / Perfetto file.

    python scripts/trace_to_chrome.py /tmp/traces/trace-1234.jsonl out.json
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tensorflow_serving2_amd.utils.tracing import load, to_chrome  # noqa: E402

if __name__ == "__main__":
    with open(sys.argv[2], "w") as f:
        json.dump(to_chrome(load(sys.argv[1])), f)
