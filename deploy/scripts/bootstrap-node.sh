#!/bin/bash
# Single-node bootstrap for an MI355X host (the reference's infrastructure/user-data-cpu.sh:72-163, re-targeted).
#
#   bootstrap-node.sh [--k8s] [--no-services]
#
# 1. checks the ROCm stack: rocm-smi, the 8 GPUs and their xGMI links, the ROCm-enabled torch, dmabuf IPC mode;
# 2. builds every gfx950 HIP library in-tree (python -m mifx.ops.build) and creates the working directories;
# 3. default (no Kubernetes): starts the stack as local processes -- central dashboard, pipelines API, metadata
#    service, scalar dashboard, notebook runner, training-job operator (local CR directory), RESP tensor store, and
#    the model server (REST 8500 + gRPC 9000) when a model is exported -- behind deploy/nginx.conf if nginx exists;
# 4. --k8s: on a cluster whose kubeconfig kubectl already uses (the reference's kubeadm / weave / openebs steps are
#    cluster-provider specific and stay with the provider): installs the MIFXJob CRD, creates the kubeflow namespace,
#    labels this node for the AMD GPU device plugin, and applies the whole stack with `kubectl apply -k deploy/k8s`
#    (device plugin, pipelines API, metadata, artifact store, model server, dashboards, operator, jobs), then waits
#    for the device plugin to advertise amd.com/gpu.
set -euo pipefail
ROOT=${MIFX_ROOT:-/var/lib/mifx}
REPO=${MIFX_REPO:-$(cd "$(dirname "$0")/../.." && pwd)}
K8S=0
SERVICES=1
for a in "$@"; do
  case "$a" in
    --k8s) K8S=1 ;;
    --no-services) SERVICES=0 ;;
    *) echo "unknown option $a" >&2; exit 2 ;;
  esac
done
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH="$REPO${PYTHONPATH:+:$PYTHONPATH}"

# ---- 1. ROCm / GPUs
if command -v rocm-smi >/dev/null; then
  rocm-smi --showproductname || true
  rocm-smi --showtopotype 2>/dev/null | head -20 || true   # XGMI between every GPU pair on an MI355X node
else
  echo "warning: rocm-smi not found (is ROCm >= 7.0 installed?)" >&2
fi
python3 - <<'PY'
import torch
n = torch.cuda.device_count()
print(f"torch {torch.__version__} hip {torch.version.hip}: {n} GPU(s)")
assert torch.version.hip, "this torch build is not ROCm-enabled"
PY

# ---- 2. build + directories
mkdir -p "$ROOT"/{pipelines,models,experiments,jobs,logs,board,metadata}
python3 -m mifx.ops.build

# ---- 4. Kubernetes
if [ "$K8S" = 1 ]; then
  command -v kubectl >/dev/null || { echo "kubectl not found" >&2; exit 1; }
  kubectl get namespace kubeflow >/dev/null 2>&1 || kubectl create namespace kubeflow
  kubectl apply -f "$REPO/deploy/crd/mifxjob-crd.yaml"
  kubectl apply -f "$REPO/deploy/crd/studyjob-notebook-crds.yaml"
  kubectl label node "$(hostname)" amd.com/gpu.present=true --overwrite || true
  kubectl apply -k "$REPO/deploy/k8s"
  for i in $(seq 1 60); do
    n=$(kubectl get node "$(hostname)" -o jsonpath='{.status.allocatable.amd\.com/gpu}' 2>/dev/null || true)
    [ -n "$n" ] && [ "$n" != "0" ] && { echo "amd.com/gpu allocatable: $n"; break; }
    sleep 5
  done
  exit 0
fi

# ---- 3. local services
[ "$SERVICES" = 1 ] || exit 0
start() {  # name, command...
  local name=$1; shift
  nohup "$@" > "$ROOT/logs/$name.log" 2>&1 &
  echo "$name (pid $!)"
}
start dashboard python3 -m mifx.dashboard --port 8082
start pipelines-api python3 -m mifx.kfp.server --port 8888 --root "$ROOT/pipelines"
start metadata python3 -m mifx.metadata.server --port 8080 --db "$ROOT/metadata/metadata.db"
start board python3 -m mifx.board --port 6006 --logdir "$ROOT/board"
start notebooks python3 -m mifx.notebook_server --port 8889
start operator python3 -m mifx.launch.operator --local "$ROOT/jobs"
# the tensor store loads models it is sent: loopback only, and a password because nginx proxies :9736 to it
mkdir -p "$ROOT/secrets" && chmod 700 "$ROOT/secrets"
[ -s "$ROOT/secrets/resp_password" ] || (umask 077; head -c 24 /dev/urandom | od -An -tx1 | tr -d ' \n' > "$ROOT/secrets/resp_password")
MIFX_RESP_PASSWORD="$(cat "$ROOT/secrets/resp_password")" start tensor-store python3 -m mifx.serving.resp_server \
  --host 127.0.0.1 --port 6379 --model-root "$ROOT/models"
if [ -d "$ROOT/models/taxi" ]; then
  start model-server python3 -m mifx.serving.server --model_name taxi --model_base_path "$ROOT/models/taxi" \
    --rest_api_port 8500 --port 9000
fi
if command -v nginx >/dev/null; then
  nginx -c "$REPO/deploy/nginx.conf" && echo "reverse proxy on :80 (deploy/nginx.conf)"
fi
