# BASELINE config 3: program-level FunSearch, 4 islands x 2,000 generations on one MI355X
# (offline mutation LLM backend, device bytecode VM), resumable from gpurun_out/c3 checkpoints.
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c3
G=${G:-2000}
R=${RESUME:-}
timeout -k 10 1050 python -u -m funsearch_kubernetes_simulator_amd.funsearch --config configs/config3_islands.json \
  --generations $G $R --verbose --checkpoint-dir gpurun_out/c3 --log gpurun_out/c3/metrics.jsonl \
  --save gpurun_out/c3/top5.json > gpurun_out/c3/run.log 2>&1
rc=$?
echo "rc=$rc"; tail -2 gpurun_out/c3/run.log | cut -c1-400
