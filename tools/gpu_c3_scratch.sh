# BASELINE config 3 from scratch: 4 islands x 2,000 generations on one MI355X, seeds = first-fit + best-fit
# only (configs/config3_scratch.json).  Runs in parts of G generations; each part resumes from the checkpoint
# staged in runs/config3_scratch (copied into gpurun_out/c3s so the box returns it).
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c3s
cp runs/config3_scratch/islands_rank0.json runs/config3_scratch/metrics.jsonl gpurun_out/c3s/ 2>/dev/null
G=${G:-1000}
timeout -k 10 1100 python -u -m funsearch_kubernetes_simulator_amd.funsearch --config configs/config3_scratch.json \
  --generations $G --resume --verbose --checkpoint-dir gpurun_out/c3s --log gpurun_out/c3s/metrics.jsonl \
  --save gpurun_out/c3s/top5.json > gpurun_out/c3s/run.log 2>&1
rc=$?
echo "rc=$rc"; tail -1 gpurun_out/c3s/metrics.jsonl | cut -c1-400
