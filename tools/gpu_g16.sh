set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="timeout -k 10 300 python bench.py --steps 20 --warmup 2"
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/g16_tests.log 2>&1 && \
$B > gpurun_out/g16_cl.log 2>&1 && \
$B --family random_linear > gpurun_out/g16_rl.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof16 -o run -- python3 bench.py --steps 10 --warmup 2 > gpurun_out/g16_prof.log 2>&1
echo "rc=$?"; tail -2 gpurun_out/g16_tests.log
for f in g16_cl g16_rl; do python -c "
import json,sys; d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d.get('events_per_s'), d['best_score'])"; done
