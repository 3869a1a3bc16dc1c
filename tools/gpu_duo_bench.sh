# native-program bench only (two-wave kernel), for build-knob A/B runs
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/db
timeout -k 10 300 python -u -m pytest tests/test_gpu_native.py -x -q --timeout 150 --timeout-method thread -k "layouts or reference" \
  > gpurun_out/db/tests.txt 2>&1 || { echo "native tests failed"; tail -30 gpurun_out/db/tests.txt; exit 1; }
tail -1 gpurun_out/db/tests.txt
timeout -k 10 200 python -u tools/native_bench.py --batch 64 --batches 3 --single 6 > gpurun_out/db/bench.jsonl 2>&1 \
  || { echo "bench failed"; tail -20 gpurun_out/db/bench.jsonl; exit 1; }
grep '^{' gpurun_out/db/bench.jsonl | cut -c1-230
