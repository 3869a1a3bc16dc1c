# Native programs with LDS-staged constant blocks: GPU tests, phase split, bench, short config-3 run.
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/kc
timeout -k 10 300 python -u -m pytest tests/test_gpu_native.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/kc/tests.txt 2>&1 || { echo "tests failed"; tail -40 gpurun_out/kc/tests.txt; exit 1; }
tail -3 gpurun_out/kc/tests.txt
timeout -k 10 200 python -u tools/native_phase.py --programs 48 > gpurun_out/kc/phase.jsonl 2>&1 \
  || { echo "phase failed"; tail -20 gpurun_out/kc/phase.jsonl; exit 1; }
cat gpurun_out/kc/phase.jsonl
timeout -k 10 300 python -u tools/native_bench.py --batch 64 --batches 3 --cpu --single 5 > gpurun_out/kc/native_bench.jsonl 2>&1 \
  || { echo "native bench failed"; tail -20 gpurun_out/kc/native_bench.jsonl; exit 1; }
cat gpurun_out/kc/native_bench.jsonl
G=${G:-40} T=${T:-400} bash tools/gpu_c3_native.sh
