#!/bin/bash
# Closing check of the round-3 tree after the wave-kernel changes: every GPU test, smoke, driver-default
# bench (with program_path), rocprofv3 kernel stats of the bench, config 5 at 4,096 candidates.
set -o pipefail
export PYTHONPATH=$PWD FKS_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3z
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1 \
  || { echo "gpu tests failed"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 1 --programs 0 --novel 0 \
  > $O/prof.log 2>&1 || { echo "profile failed"; tail -20 $O/prof.log; exit 1; }
timeout -k 10 300 python -u bench.py --trace synthetic --candidates 4096 --steps 3 --warmup 1 --programs 0 > $O/c5_4096.json 2> $O/c5_4096.err \
  || { echo "c5 failed"; tail -20 $O/c5_4096.err; exit 1; }
cut -c1-200 $O/c5_4096.json
