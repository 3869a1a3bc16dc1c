#!/bin/bash
# Flat vs exec-masked heap accesses in the row kernels: engine + native tests, bench A/B, phase split.
set -o pipefail
export PYTHONPATH=$PWD FKS_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3g
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_native.py -x -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 \
  || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for v in "flat:" "split:--row-split-heap" "flat2:"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --programs 0 --novel 0 $a > $O/b_$n.json 2> $O/b_$n.err \
    || { echo "bench $n failed"; tail -20 $O/b_$n.err; exit 1; }
  echo "$n: $(cut -c1-230 $O/b_$n.json)"
done
timeout -k 10 200 python -u tools/phase_rows.py 12288 composite_linear > $O/phase.jsonl 2> $O/phase.err \
  || { echo "phase failed"; tail -20 $O/phase.err; exit 1; }
cat $O/phase.jsonl
timeout -k 10 200 python -u tools/native_bench.py --batch 64 --batches 2 > $O/native.jsonl 2> $O/native.err \
  || { echo "native bench failed"; tail -20 $O/native.err; exit 1; }
tail -3 $O/native.jsonl | cut -c1-300
