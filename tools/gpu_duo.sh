# Two-wave native kernel (replay_duo.hip.h): native GPU tests first (exactness vs the CPU VM, every layout),
# then the native-program bench with the two-wave kernel and with the one-wave row kernel.
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/duo
timeout -k 10 300 python -u -m pytest tests/test_gpu_native.py -x -v --timeout 150 --timeout-method thread \
  > gpurun_out/duo/tests.txt 2>&1 || { echo "native tests failed"; tail -40 gpurun_out/duo/tests.txt; exit 1; }
tail -3 gpurun_out/duo/tests.txt
timeout -k 10 200 python -u tools/native_bench.py --batch 64 --batches 3 --single 6 > gpurun_out/duo/bench_duo.jsonl 2>&1 \
  || { echo "duo bench failed"; tail -20 gpurun_out/duo/bench_duo.jsonl; exit 1; }
timeout -k 10 200 python -u tools/native_bench.py --batch 64 --batches 3 --single 6 --options '{"native_duo": false}' \
  > gpurun_out/duo/bench_rows1.jsonl 2>&1 || { echo "rows1 bench failed"; tail -20 gpurun_out/duo/bench_rows1.jsonl; exit 1; }
echo "== duo"; grep '^{' gpurun_out/duo/bench_duo.jsonl | cut -c1-260
echo "== rows1"; grep '^{' gpurun_out/duo/bench_rows1.jsonl | cut -c1-260
