# MFMA screening A/B at equal wall-clock (60 s per arm) + kernel stats of a screened run.
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/screen
for k in 1 4; do
  timeout -k 10 200 python -u bench.py --warmup 2 --time-budget ${B:-60} --screen $k --programs 0 --seed 7 \
    > gpurun_out/screen/k$k.json 2> gpurun_out/screen/k$k.err || { echo "k=$k failed"; tail -20 gpurun_out/screen/k$k.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/screen/k$k.json')); print($k, d['steps'], d['value'], d['best_score'], d.get('screen'))"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/screen/prof -o run -- python3 -u bench.py --warmup 1 --steps 4 --screen 4 --programs 0 \
  > gpurun_out/screen/prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/screen/prof.log; exit 1; }
find gpurun_out/screen/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cut -d, -f1-8 {} | head -12
