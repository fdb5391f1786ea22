#!/bin/bash
# Start the model server the way serving/rundocker.sh starts the TF Serving
# container (gRPC 8500 -> host 9000, REST 8501 -> host 9001, MODEL_NAME=resnet,
# models under ./models).  No container: the server runs on the local MI355X
# GPUs, one replica per GPU (NUM_GPUS, default 1; 0 = all visible).
set -euo pipefail
cd "$(dirname "$0")"
MODEL_NAME="${MODEL_NAME:-resnet}"
NUM_GPUS="${NUM_GPUS:-1}"
[ -d "models/${MODEL_NAME}" ] || python3 make_models.py --root models --models "${MODEL_NAME}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
export PYTHONPATH="$(cd .. && pwd):${PYTHONPATH:-}"
exec python3 -m rust_tensorflow_serving2_amd.server --port=9000 --rest_api_port=9001 \
  --model_name="${MODEL_NAME}" --model_base_path="$(pwd)/models/${MODEL_NAME}" --num_gpus="${NUM_GPUS}" "$@"
