set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/screen_bench.py > gpurun_out/g15_screen.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof15 -o run -- python3 bench.py --steps 10 --warmup 2 > gpurun_out/g15_prof_bench.log 2>&1 && \
timeout -k 10 600 python bench.py --trace synthetic --steps 3 --warmup 1 > gpurun_out/g15_syn.log 2>&1
echo "rc=$?"; cat gpurun_out/g15_screen.log; tail -1 gpurun_out/g15_prof_bench.log | cut -c1-300; tail -1 gpurun_out/g15_syn.log | cut -c1-400; find gpurun_out/prof15 -name "*stats*" | head
