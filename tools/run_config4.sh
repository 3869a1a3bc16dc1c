#!/usr/bin/env bash
# BASELINE config 4 launcher: 8 islands on 8 MI355X (one rank per GPU, one island per rank), RCCL elite
# all-gather every 50 generations, FunSearch programs JIT-compiled and replayed on each rank's own card.
# Elastic: torchrun restarts a crashed group (--max-restarts) and every restart resumes from the per-rank
# checkpoints (--resume re-shards them onto whatever world size comes back).
#   NPROC=8 GENS=2000 bash tools/run_config4.sh
# CPU rehearsal (gloo ranks, CPU engines; tools/collective_wait.py reads the per-rank logs):
#   NPROC=8 GENS=60 FKS_DIST_BACKEND=gloo CONFIG=configs/config4_rehearsal.json DEVICE_ARGS="--device cpu" \
#     RUN_DIR=runs/c4r OMP_NUM_THREADS=1 bash tools/run_config4.sh
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD HSA_ENABLE_IPC_MODE_LEGACY=0
NPROC=${NPROC:-8}
GENS=${GENS:-2000}
PORT=${PORT:-29541}
RUN_DIR=${RUN_DIR:-runs/config4}
CONFIG=${CONFIG:-configs/config4.json}
DEVICE_ARGS=${DEVICE_ARGS:-}
mkdir -p "$RUN_DIR"
python -m torch.distributed.run --nnodes=1 --nproc-per-node="$NPROC" --max-restarts="${RESTARTS:-2}" \
  --rdzv-backend=c10d --rdzv-endpoint="127.0.0.1:$PORT" --local-addr=127.0.0.1 \
  -m funsearch_kubernetes_simulator_amd.funsearch --config "$CONFIG" --generations "$GENS" --resume $DEVICE_ARGS \
  --checkpoint-dir "$RUN_DIR" --metrics-log "$RUN_DIR/metrics.jsonl" --save "$RUN_DIR/top5.json"
