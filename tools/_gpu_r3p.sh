#!/bin/bash
# Feasibility-prologue skip in the native kernels: native + gcn + engine tests, duo phase split and native bench
# with / without the skip, then the default bench (5-wave composite row kernel).
set -o pipefail
export PYTHONPATH=$PWD FKS_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3p
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_native.py tests/test_gpu_gcn.py tests/test_gpu_engine.py -x -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 \
  || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for sk in 1 0; do
  FKS_FEAS_SKIP=$sk timeout -k 10 300 python -u tools/duo_phase.py --programs 48 > $O/duo_phase_skip$sk.jsonl 2>&1 \
    || { echo "phase $sk failed"; tail -20 $O/duo_phase_skip$sk.jsonl; exit 1; }
  echo "skip=$sk"; grep '^{' $O/duo_phase_skip$sk.jsonl | cut -c1-330
  FKS_FEAS_SKIP=$sk timeout -k 10 200 python -u tools/native_bench.py --batch 64 --batches 2 > $O/native_skip$sk.jsonl 2>&1 \
    || { echo "native bench $sk failed"; tail -20 $O/native_skip$sk.jsonl; exit 1; }
  grep '^{"batch' $O/native_skip$sk.jsonl | cut -c1-160
done
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
timeout -k 10 300 python -u bench.py --programs 0 --novel 0 --row-composite-waves 4 > $O/bench_w4.json 2> $O/bench_w4.err || { echo "bench w4 failed"; tail -20 $O/bench_w4.err; exit 1; }
echo "w4: $(cut -c70-170 $O/bench_w4.json)"
