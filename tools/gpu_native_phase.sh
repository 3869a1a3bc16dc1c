# Native programs: phase split of the row kernel in the latency regime + throughput bench.
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/np
timeout -k 10 200 python -u tools/native_phase.py --programs 48 > gpurun_out/np/phase.jsonl 2>&1 \
  || { echo "phase failed"; tail -20 gpurun_out/np/phase.jsonl; exit 1; }
cat gpurun_out/np/phase.jsonl
timeout -k 10 300 python -u tools/native_bench.py --batch 64 --batches 2 --cpu --single 5 > gpurun_out/np/native_bench.jsonl 2>&1 \
  || { echo "native bench failed"; tail -20 gpurun_out/np/native_bench.jsonl; exit 1; }
cat gpurun_out/np/native_bench.jsonl
