# Very large native batches (polish-sized): two-wave kernel (forced) vs four programs per wave at 1,024 / 2,048 programs
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/dbig
for b in 1024 2048; do
  for opt in '{"native_rows": 1, "native_duo": true}' '{"native_rows": 4}'; do
    f=gpurun_out/dbig/b${b}_$(echo $opt | tr -dc 'a-z0-9').jsonl
    timeout -k 10 300 python -u tools/native_bench.py --batch $b --batches 2 --options "$opt" > $f 2>&1 || { echo "bench $b $opt failed"; exit 1; }
    echo "batch=$b $opt"; grep '"batch": 1' $f | cut -c1-220
  done
done
