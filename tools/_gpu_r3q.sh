#!/bin/bash
# Full check + config 5 with reciprocal divisions / bit-pattern argmax in the wave kernel's composite instance.
set -o pipefail
export PYTHONPATH=$PWD FKS_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3q
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1 \
  || { echo "gpu tests failed"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
for c in 4096 1536; do
  timeout -k 10 300 python -u bench.py --trace synthetic --candidates $c --steps 3 --warmup 1 --programs 0 --novel 0 > $O/c5_$c.json 2> $O/c5_$c.err \
    || { echo "c5 $c failed"; tail -20 $O/c5_$c.err; exit 1; }
  echo "c5 $c: $(cut -c70-170 $O/c5_$c.json)"
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 1 --programs 0 --novel 0 \
  > $O/prof.log 2>&1 || { echo "profile failed"; tail -20 $O/prof.log; exit 1; }
echo done
