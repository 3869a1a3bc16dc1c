# Large native batches: two-wave kernel (one program per 128-thread workgroup) vs the row kernel with four
# programs per wave, at 128 / 256 / 512 programs per batch (cached shapes; device time only).
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/dvr
for b in 128 256 512; do
  for opt in '{"native_rows": 1, "native_duo": true}' '{"native_rows": 4}'; do
    timeout -k 10 240 python -u tools/native_bench.py --batch $b --batches 2 --options "$opt" > gpurun_out/dvr/b${b}_$(echo $opt | tr -dc 'a-z0-9').jsonl 2>&1 \
      || { echo "bench $b $opt failed"; exit 1; }
    echo "batch=$b $opt"; grep '"batch": 1' gpurun_out/dvr/b${b}_$(echo $opt | tr -dc 'a-z0-9').jsonl | cut -c1-220
  done
done
