# GPU tests on a fresh box, then a part of the config-3 native run (only if the tests pass).
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/chk
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/chk/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/chk/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/chk/gpu_tests.txt
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --programs 0 > gpurun_out/chk/bench.json 2> gpurun_out/chk/bench.err \
  || { echo "bench failed"; tail -20 gpurun_out/chk/bench.err; exit 1; }
cut -c1-400 gpurun_out/chk/bench.json
G=${G:-800} T=${T:-800} bash tools/gpu_c3_native.sh
