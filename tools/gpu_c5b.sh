# Config 5 after the occupancy change: full-shape exactness test, then the bench at two batch sizes.
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c5b
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -k "config5" -x -v --timeout 250 --timeout-method thread \
  > gpurun_out/c5b/tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/c5b/tests.txt; exit 1; }
tail -2 gpurun_out/c5b/tests.txt
for c in ${CANDS:-1536 4096}; do
  timeout -k 10 300 python -u bench.py --trace synthetic --candidates $c --steps 3 --warmup 1 --programs 0 $EXTRA > gpurun_out/c5b/c5_$c.json 2> gpurun_out/c5b/c5_$c.err \
    || { echo "bench $c failed"; tail -20 gpurun_out/c5b/c5_$c.err; exit 1; }
  cut -c1-200 gpurun_out/c5b/c5_$c.json
done
