# One GPU-milli total per node (NodeRegs::gmt1): every GPU test (all kernels read node registers), then
# config 5 (256 nodes, NPASS=4 kernels now compiled for 3 waves/SIMD) and the default headline bench.
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/np4
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/np4/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/np4/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/np4/gpu_tests.txt
for c in ${CANDS:-1536 4096}; do
  timeout -k 10 300 python -u bench.py --trace synthetic --candidates $c --steps 3 --warmup 1 --programs 0 > gpurun_out/np4/c5_$c.json 2> gpurun_out/np4/c5_$c.err \
    || { echo "bench $c failed"; tail -20 gpurun_out/np4/c5_$c.err; exit 1; }
  cut -c1-200 gpurun_out/np4/c5_$c.json
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/np4/bench.json 2> gpurun_out/np4/bench.err \
  || { echo "bench failed"; tail -20 gpurun_out/np4/bench.err; exit 1; }
cut -c1-200 gpurun_out/np4/bench.json
