# Wave kernel: one wave argmax per creation event (lane-local best over node slots).
# Engine GPU tests (exactness of every wave / row path), then config 5 at two batch sizes.
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3u
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_native.py -m gpu -x -v --timeout 250 --timeout-method thread \
  > gpurun_out/r3u/tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r3u/tests.txt; exit 1; }
tail -2 gpurun_out/r3u/tests.txt
for c in 1536 4096; do
  timeout -k 10 300 python -u bench.py --trace synthetic --candidates $c --steps 3 --warmup 1 --programs 0 > gpurun_out/r3u/c5_$c.json 2> gpurun_out/r3u/c5_$c.err \
    || { echo "bench $c failed"; tail -20 gpurun_out/r3u/c5_$c.err; exit 1; }
  cut -c1-200 gpurun_out/r3u/c5_$c.json
done
