#!/bin/bash
# Final check of the round-3 tree: every GPU test, smoke, driver-default bench (with program_path), rocprofv3 kernel
# stats of the bench, native batches with / without the feasibility-prologue skip, then a 180 s config-3 steady run.
set -o pipefail
export PYTHONPATH=$PWD FKS_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3t
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
for sk in 1 0; do
  FKS_FEAS_SKIP=$sk timeout -k 10 200 python -u tools/native_bench.py --batch 256 --batches 2 > $O/nb_256_$sk.jsonl 2>&1 \
    || { echo "nb $sk failed"; tail -20 $O/nb_256_$sk.jsonl; exit 1; }
  echo "batch=256 skip=$sk: $(grep '^{"batch": 1' $O/nb_256_$sk.jsonl | cut -c1-200)"
done
timeout -k 10 400 python -u -m funsearch_kubernetes_simulator_amd.funsearch --config configs/config3_steady.json \
  --verbose --wall-s 180 --save $O/top5.json --checkpoint-dir $O/ck --metrics-log $O/metrics.jsonl > $O/steady.log 2>&1 \
  || { echo "steady failed"; tail -20 $O/steady.log; exit 1; }
grep steady_final $O/steady.log | cut -c1-300
