# Config 5 (65,536 pods / 256 nodes): full-shape exactness test, phase split, bench at two batch sizes.
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c5
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -k "config5" -x -v --timeout 250 --timeout-method thread \
  > gpurun_out/c5/tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/c5/tests.txt; exit 1; }
tail -4 gpurun_out/c5/tests.txt
for c in ${CANDS:-1536 4096}; do
  timeout -k 10 300 python -u bench.py --trace synthetic --candidates $c --steps 3 --warmup 1 --programs 0 > gpurun_out/c5/bench_$c.json 2> gpurun_out/c5/bench_$c.err \
    || { echo "bench $c failed"; tail -20 gpurun_out/c5/bench_$c.err; exit 1; }
  cut -c1-300 gpurun_out/c5/bench_$c.json
done
