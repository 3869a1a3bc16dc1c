# BASELINE config 3 on the device: 4 pipelined islands, FunSearch programs JIT-compiled and replayed on the
# MI355X (k_replay_native), seeds = first-fit + best-fit only (configs/config3_native.json).  Runs in parts of G
# generations, resuming from the checkpoint staged in runs/config3_native (copied into gpurun_out/c3n).
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CFG=${CFG:-configs/config3_native.json}
RUN=${RUN:-runs/config3_native}
mkdir -p gpurun_out/c3n
cp $RUN/islands_rank0.json $RUN/metrics.jsonl gpurun_out/c3n/ 2>/dev/null
G=${G:-100}
T=${T:-1100}
timeout -k 10 $T python -u -m funsearch_kubernetes_simulator_amd.funsearch --config $CFG \
  --generations $G --resume --checkpoint-dir gpurun_out/c3n --log gpurun_out/c3n/metrics.jsonl \
  --save gpurun_out/c3n/top5.json > gpurun_out/c3n/run.log 2>&1
rc=$?
echo "rc=$rc"; tail -2 gpurun_out/c3n/run.log | cut -c1-600; grep '"kind": "generation"' gpurun_out/c3n/metrics.jsonl | tail -1 | cut -c1-700
