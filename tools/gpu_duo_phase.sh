# two-wave kernel: exactness (layouts + reference programs), phase split, native bench
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/dp2
timeout -k 10 300 python -u -m pytest tests/test_gpu_native.py -x -q --timeout 150 --timeout-method thread \
  > gpurun_out/dp2/tests.txt 2>&1 || { echo "native tests failed"; tail -30 gpurun_out/dp2/tests.txt; exit 1; }
tail -1 gpurun_out/dp2/tests.txt
timeout -k 10 300 python -u tools/duo_phase.py --programs 48 > gpurun_out/dp2/duo_phase.jsonl 2>&1 \
  || { echo "phase failed"; tail -20 gpurun_out/dp2/duo_phase.jsonl; exit 1; }
grep '^{' gpurun_out/dp2/duo_phase.jsonl | cut -c1-420
timeout -k 10 200 python -u tools/native_bench.py --batch 64 --batches 3 --single 6 > gpurun_out/dp2/bench.jsonl 2>&1 \
  || { echo "bench failed"; tail -20 gpurun_out/dp2/bench.jsonl; exit 1; }
grep '^{' gpurun_out/dp2/bench.jsonl | cut -c1-200
