#!/bin/bash
# Composite row kernel with reciprocal divisions: engine tests, then bench at 4 and 5 waves per SIMD, phase split.
set -o pipefail
export PYTHONPATH=$PWD FKS_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3f
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 \
  || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for wv in 4 5; do
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --programs 0 --novel 0 --row-composite-waves $wv > $O/b$wv.json 2> $O/b$wv.err \
    || { echo "bench $wv failed"; tail -20 $O/b$wv.err; exit 1; }
  echo "waves $wv: $(cut -c1-260 $O/b$wv.json)"
done
timeout -k 10 200 python -u tools/phase_rows.py 12288 composite_linear > $O/phase.jsonl 2> $O/phase.err \
  || { echo "phase failed"; tail -20 $O/phase.err; exit 1; }
cat $O/phase.jsonl
