#!/bin/bash
# Register diet (hash/threshold in LDS, 16-bit waiting counters, generic-pointer heap copy): tests, 4 vs 5 waves/SIMD.
set -o pipefail
export PYTHONPATH=$PWD FKS_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3m
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_native.py -x -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 \
  || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for wv in 4 5 4; do
  timeout -k 10 200 python -u bench.py --programs 0 --novel 0 --row-composite-waves $wv > $O/b_$wv.json 2> $O/b_$wv.err \
    || { echo "bench $wv failed"; tail -20 $O/b_$wv.err; exit 1; }
  echo "waves $wv: $(cut -c70-170 $O/b_$wv.json)"
done
