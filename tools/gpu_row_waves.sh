# Row-kernel occupancy A/B: rebuild the extension on the box with FKS_ROW_HEAVY_WAVES = 4 / 5 / 6
# (composite / feature families) and run the default bench for each build.
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/rw
for hw in ${HWS:-4 5 6}; do
  FKS_ROW_HEAVY_WAVES=$hw timeout -k 10 300 python -c "from funsearch_kubernetes_simulator_amd.ops.build import build_hip; build_hip(force=True)" \
    > gpurun_out/rw/build_$hw.log 2>&1 || { echo "build $hw failed"; tail -20 gpurun_out/rw/build_$hw.log; exit 1; }
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --programs 0 > gpurun_out/rw/bench_$hw.json 2> gpurun_out/rw/bench_$hw.err \
    || { echo "bench $hw failed"; tail -20 gpurun_out/rw/bench_$hw.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/rw/bench_$hw.json')); print('heavy_waves', $hw, d['value'], d['ms_per_step'], d['best_score'])"
done
