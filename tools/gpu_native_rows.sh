# Native programs on the row kernel: GPU tests + native bench (latency per event, batch throughput).
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/nr
timeout -k 10 300 python -u -m pytest tests/test_gpu_native.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/nr/tests.txt 2>&1 || { echo "tests failed"; tail -40 gpurun_out/nr/tests.txt; exit 1; }
tail -12 gpurun_out/nr/tests.txt
timeout -k 10 300 python -u tools/native_bench.py --batch 64 --batches 3 --cpu --single 6 > gpurun_out/nr/native_bench.jsonl 2>&1 \
  || { echo "native bench failed"; tail -20 gpurun_out/nr/native_bench.jsonl; exit 1; }
cat gpurun_out/nr/native_bench.jsonl
