# Round-2 checkpoint on a fresh MI355X box: GPU tests, smoke, short bench, native-program bench.
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/r2/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r2/gpu_tests.txt; exit 1; }
tail -3 gpurun_out/r2/gpu_tests.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2/smoke.txt 2>&1 \
  || { echo "smoke failed"; tail -20 gpurun_out/r2/smoke.txt; exit 1; }
tail -1 gpurun_out/r2/smoke.txt
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/r2/bench.json 2> gpurun_out/r2/bench.err \
  || { echo "bench failed"; tail -20 gpurun_out/r2/bench.err; exit 1; }
cut -c1-600 gpurun_out/r2/bench.json
timeout -k 10 300 python -u tools/native_bench.py --batch 64 --batches 3 --cpu --single 6 > gpurun_out/r2/native_bench.jsonl 2>&1 \
  || { echo "native bench failed"; tail -20 gpurun_out/r2/native_bench.jsonl; exit 1; }
cat gpurun_out/r2/native_bench.jsonl
