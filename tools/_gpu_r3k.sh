#!/bin/bash
# Row kernel: LDS node divisors, single-compare trunc, stranded/tg tweaks -- engine + native tests, bench x2, phase.
set -o pipefail
export PYTHONPATH=$PWD FKS_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3k
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_native.py -x -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 \
  || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for n in 1 2; do
  timeout -k 10 200 python -u bench.py --programs 0 --novel 0 > $O/b$n.json 2> $O/b$n.err \
    || { echo "bench $n failed"; tail -20 $O/b$n.err; exit 1; }
  echo "b$n: $(cut -c70-170 $O/b$n.json)"
done
timeout -k 10 200 python -u tools/phase_rows.py 12288 composite_linear > $O/phase.jsonl 2> $O/phase.err \
  || { echo "phase failed"; tail -20 $O/phase.err; exit 1; }
cat $O/phase.jsonl
