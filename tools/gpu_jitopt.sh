# A/B of clang's optimisation level for JIT-compiled programs (FKS_JIT_OPT): native tests at -O1, then the
# native-program bench at -O3 and -O1 (compile time vs replay latency).
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/jo
FKS_JIT_OPT=-O1 timeout -k 10 300 python -u -m pytest tests/test_gpu_native.py -x -q --timeout 150 --timeout-method thread \
  > gpurun_out/jo/tests_O1.txt 2>&1 || { echo "native tests (-O1) failed"; tail -30 gpurun_out/jo/tests_O1.txt; exit 1; }
tail -1 gpurun_out/jo/tests_O1.txt
for o in -O3 -O1; do
  FKS_JIT_OPT=$o timeout -k 10 200 python -u tools/native_bench.py --batch 64 --batches 3 --single 6 > gpurun_out/jo/bench$o.jsonl 2>&1 \
    || { echo "bench $o failed"; tail -20 gpurun_out/jo/bench$o.jsonl; exit 1; }
  echo "== $o"; grep '^{' gpurun_out/jo/bench$o.jsonl | cut -c1-230
done
