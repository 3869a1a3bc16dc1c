# End-of-session check on a fresh box: every GPU test, smoke, then a rocprofv3 kernel trace of the native
# program path (two-wave kernel) and of the 256-node config-5 bench.
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fin
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/fin/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/fin/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/fin/gpu_tests.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin/smoke.txt 2>&1 \
  || { echo "smoke failed"; tail -20 gpurun_out/fin/smoke.txt; exit 1; }
tail -1 gpurun_out/fin/smoke.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/fin/prof_native -o run -- python3 tools/native_bench.py --batch 64 --batches 2 \
  > gpurun_out/fin/prof_native.log 2>&1 || { echo "native profile failed"; tail -20 gpurun_out/fin/prof_native.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fin/prof_c5 -o run -- python3 bench.py --trace synthetic --candidates 1536 --steps 2 --warmup 1 --programs 0 \
  > gpurun_out/fin/prof_c5.log 2>&1 || { echo "c5 profile failed"; tail -20 gpurun_out/fin/prof_c5.log; exit 1; }
find gpurun_out/fin -name "*.db" -o -name "*kernel_stats.csv" | head
