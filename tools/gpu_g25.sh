# BASELINE config 3 continued: resume the 4-island program-level FunSearch run from the
# checkpoint staged in runs/config3 (copied into gpurun_out/c3 so the box returns it).
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c3
cp runs/config3/islands_rank0.json runs/config3/metrics.jsonl gpurun_out/c3/
G=${G:-550}
timeout -k 10 1100 python -u -m funsearch_kubernetes_simulator_amd.funsearch --config configs/config3_islands.json \
  --generations $G --resume --verbose --checkpoint-dir gpurun_out/c3 --log gpurun_out/c3/metrics.jsonl \
  --save gpurun_out/c3/top5.json > gpurun_out/c3/run.log 2>&1
rc=$?
echo "rc=$rc"; tail -2 gpurun_out/c3/metrics.jsonl | cut -c1-400
