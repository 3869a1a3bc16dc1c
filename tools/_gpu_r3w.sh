# Wave kernel pop path: heap top / last slot / first pop round as plain LDS or HBM loads.
# Phase split at the config-5 shape, engine GPU tests, then config 5 at two batch sizes.
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${TAG:-r3w}
mkdir -p $D
timeout -k 10 300 python -u tools/wave_phase_c5.py 2048 > $D/phase.json 2> $D/phase.err || { echo "phase failed"; tail -20 $D/phase.err; exit 1; }
cat $D/phase.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_native.py -m gpu -x -v --timeout 250 --timeout-method thread \
  > $D/tests.txt 2>&1 || { echo "tests failed"; tail -30 $D/tests.txt; exit 1; }
tail -1 $D/tests.txt
for c in 1536 4096; do
  timeout -k 10 300 python -u bench.py --trace synthetic --candidates $c --steps 3 --warmup 1 --programs 0 > $D/c5_$c.json 2> $D/c5_$c.err \
    || { echo "bench $c failed"; tail -20 $D/c5_$c.err; exit 1; }
  cut -c1-200 $D/c5_$c.json
done
