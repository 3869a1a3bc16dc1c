#!/bin/bash
# Round-3 re-entry check on a fresh box: GPU tests, smoke, default bench, rocprofv3 kernel stats of the
# default bench (family row kernel) for the headline.
set -o pipefail
export PYTHONPATH=$PWD FKS_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3d
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/r3d/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r3d/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r3d/gpu_tests.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3d/smoke.txt 2>&1 \
  || { echo "smoke failed"; tail -20 gpurun_out/r3d/smoke.txt; exit 1; }
tail -1 gpurun_out/r3d/smoke.txt
timeout -k 10 240 python -u bench.py > gpurun_out/r3d/bench.json 2> gpurun_out/r3d/bench.err \
  || { echo "bench failed"; tail -20 gpurun_out/r3d/bench.err; exit 1; }
cut -c1-600 gpurun_out/r3d/bench.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r3d/prof -o run -- python3 bench.py --steps 3 --warmup 1 --programs 0 --novel 0 \
  > gpurun_out/r3d/prof.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/r3d/prof.log; exit 1; }
find gpurun_out/r3d/prof -name "*kernel_stats.csv" | head
