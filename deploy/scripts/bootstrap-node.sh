#!/bin/bash
# Single-node bootstrap for an MI355X host (the reference's infrastructure/user-data-cpu.sh, re-targeted):
# checks the ROCm stack and GPUs, creates the working directories, and starts the pipelines API and
# model server as local processes (no Kubernetes required). Run as the service user.
set -euo pipefail
ROOT=${MIFX_ROOT:-/var/lib/mifx}
REPO=${MIFX_REPO:-$(cd "$(dirname "$0")/../.." && pwd)}
command -v rocm-smi >/dev/null && rocm-smi --showproductname || echo "warning: rocm-smi not found"
python3 -c "import torch; print('GPUs:', torch.cuda.device_count())"
mkdir -p "$ROOT"/{pipelines,models,experiments}
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH="$REPO${PYTHONPATH:+:$PYTHONPATH}"
python3 -c "from mifx.ops.build import build_all; build_all()"
nohup python3 -m mifx.kfp.server --port 8888 --root "$ROOT/pipelines" > "$ROOT/pipelines-api.log" 2>&1 &
echo "pipelines API on :8888 (pid $!)"
if [ -d "$ROOT/models/taxi" ]; then
  nohup python3 -m mifx.serving.server --model_name taxi --model_base_path "$ROOT/models/taxi" \
    --rest_api_port 8500 > "$ROOT/model-server.log" 2>&1 &
  echo "model server on :8500 (pid $!)"
fi
