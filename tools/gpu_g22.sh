set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g22_tests.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/g22_default.log 2>&1 && \
timeout -k 10 300 python bench.py --family random_linear > gpurun_out/g22_rl.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof22 -o run -- python3 bench.py --steps 5 --warmup 1 > gpurun_out/g22_prof.log 2>&1
echo "rc=$?"; tail -2 gpurun_out/g22_tests.log
for f in g22_default g22_rl; do python -c "
import json,sys; d=json.loads([l for l in open('gpurun_out/$f.log').read().strip().splitlines() if l.startswith('{')][-1]); print('$f', d['value'], d['ms_per_step'], d.get('events_per_s'), d['best_score'])" || true; done
