# Config 5 with the 256-node wave kernels built for 4 waves/SIMD (FKS_NP4_WAVES=4: 128 VGPRs, spills).
set -o pipefail
export PYTHONPATH=$PWD FKS_NP4_WAVES=4 FKS_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r3zb
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -k "config5 or 256_nodes" -m gpu -x -v --timeout 250 --timeout-method thread \
  > $D/tests.txt 2>&1 || { echo "tests failed"; tail -30 $D/tests.txt; exit 1; }
tail -1 $D/tests.txt
for c in 1536 4096; do
  timeout -k 10 300 python -u bench.py --trace synthetic --candidates $c --steps 3 --warmup 1 --programs 0 > $D/c5_$c.json 2> $D/c5_$c.err \
    || { echo "bench $c failed"; tail -20 $D/c5_$c.err; exit 1; }
  cut -c1-200 $D/c5_$c.json
done
