#!/usr/bin/env bash
# Multi-node torchrun launcher for MI355X nodes (8 GPUs each, RCCL over xGMI
# inside a node).  Provider-agnostic equivalent of the reference's cloud-init
# launch logic (infrastructure/nebius/cluster/scripts/cloud-init.tftpl:18-78):
# workers wait for the master's rendezvous port, then every node runs torchrun
# with its node rank.  Also builds the gfx950 extension in-tree first
# (idempotent: hash-stamped), so a fresh checkout launches with one command.
#
#   NNODES=2 NODE_RANK=0 scripts/launch_multinode.sh                 # on the master
#   NNODES=2 NODE_RANK=1 MASTER_ADDR=10.0.0.5 scripts/launch_multinode.sh
#   ... scripts/launch_multinode.sh 10 2 --batch_size 32          # legacy CLI args pass through
#
# Environment (defaults):
#   NNODES (1)  NODE_RANK (0)  MASTER_ADDR (this host on rank 0; required otherwise)
#   MASTER_PORT (29500)  NPROC_PER_NODE (GPUs seen by rocm-smi/torch, else 8)
#   ENTRY (src/multigpu_multi_node.py)  MAX_RESTARTS (unset: static, like the reference)
#   WAIT_ATTEMPTS (30)  WAIT_SECONDS (10)  SKIP_BUILD (0)  DRY_RUN (0: print the command)
set -euo pipefail

cd "$(dirname "$0")/.."

NNODES=${NNODES:-1}
NODE_RANK=${NODE_RANK:-0}
MASTER_PORT=${MASTER_PORT:-29500}
ENTRY=${ENTRY:-src/multigpu_multi_node.py}
WAIT_ATTEMPTS=${WAIT_ATTEMPTS:-30}
WAIT_SECONDS=${WAIT_SECONDS:-10}
DRY_RUN=${DRY_RUN:-0}

if [ -z "${MASTER_ADDR:-}" ]; then
  if [ "$NODE_RANK" = "0" ]; then
    MASTER_ADDR=$(hostname -I 2>/dev/null | awk '{print $1}')
    MASTER_ADDR=${MASTER_ADDR:-127.0.0.1}
  else
    echo "launch_multinode: MASTER_ADDR is required on worker nodes" >&2
    exit 2
  fi
fi

if [ -z "${NPROC_PER_NODE:-}" ]; then
  # count devices without initialising HIP in this shell's children that outlive us
  NPROC_PER_NODE=$(python3 -c "import torch; print(torch.cuda.device_count() or 8)" 2>/dev/null || echo 8)
fi

# dmabuf IPC (needed by RCCL / CUDA-tensor sharing on hosts without legacy IPC)
export HSA_ENABLE_IPC_MODE_LEGACY=${HSA_ENABLE_IPC_MODE_LEGACY:-0}
export TORCH_NCCL_ASYNC_ERROR_HANDLING=${TORCH_NCCL_ASYNC_ERROR_HANDLING:-1}
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"

wait_for_master() {
  local attempt=1
  while [ "$attempt" -le "$WAIT_ATTEMPTS" ]; do
    if (exec 3<>"/dev/tcp/$MASTER_ADDR/$MASTER_PORT") 2>/dev/null; then
      return 0
    fi
    echo "launch_multinode: attempt $attempt: waiting for master $MASTER_ADDR:$MASTER_PORT ..."
    sleep "$WAIT_SECONDS"
    attempt=$((attempt + 1))
  done
  return 1
}

CMD=(python3 -m torch.distributed.run
     --nnodes="$NNODES" --node_rank="$NODE_RANK"
     --master_addr="$MASTER_ADDR" --master_port="$MASTER_PORT"
     --nproc_per_node="$NPROC_PER_NODE")
if [ -n "${MAX_RESTARTS:-}" ]; then
  CMD+=(--max-restarts="$MAX_RESTARTS")
fi
CMD+=("$ENTRY" "$@")

if [ "$DRY_RUN" = "1" ]; then
  printf '%q ' "${CMD[@]}"
  echo
  exit 0
fi

if [ "${SKIP_BUILD:-0}" != "1" ]; then
  python3 -m distributed_training_amd.ops._build
fi

if [ "$NODE_RANK" != "0" ] && [ "$NNODES" -gt 1 ]; then
  if ! wait_for_master; then
    echo "launch_multinode: master $MASTER_ADDR:$MASTER_PORT unreachable after $WAIT_ATTEMPTS attempts" >&2
    exit 1
  fi
fi

exec "${CMD[@]}"
