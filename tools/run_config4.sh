#!/usr/bin/env bash
# BASELINE config 4 launcher: 8 islands on 8 MI355X (one rank per GPU, one island per rank), RCCL elite
# all-gather every 50 generations, FunSearch programs JIT-compiled and replayed on each rank's own card.
# Elastic: torchrun restarts a crashed group (--max-restarts) and every restart resumes from the per-rank
# checkpoints (--resume re-shards them onto whatever world size comes back).
#   NPROC=8 GENS=2000 bash tools/run_config4.sh
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD HSA_ENABLE_IPC_MODE_LEGACY=0
NPROC=${NPROC:-8}
GENS=${GENS:-2000}
PORT=${PORT:-29541}
RUN_DIR=${RUN_DIR:-runs/config4}
mkdir -p "$RUN_DIR"
python -m torch.distributed.run --nnodes=1 --nproc-per-node="$NPROC" --max-restarts="${RESTARTS:-2}" \
  --rdzv-backend=c10d --rdzv-endpoint="127.0.0.1:$PORT" --local-addr=127.0.0.1 \
  -m funsearch_kubernetes_simulator_amd.funsearch --config configs/config4.json --generations "$GENS" --resume \
  --checkpoint-dir "$RUN_DIR" --metrics-log "$RUN_DIR/metrics.jsonl" --save "$RUN_DIR/top5.json"
