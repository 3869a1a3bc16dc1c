set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="timeout -k 10 300 python bench.py"
$B > gpurun_out/g24_a.log 2>&1 && \
$B --family random_linear > gpurun_out/g24_rl.log 2>&1 && \
$B --seed 7 > gpurun_out/g24_b.log 2>&1 && \
$B --steps 20 > gpurun_out/g24_s20.log 2>&1
echo "rc=$?"
for f in g24_a g24_b g24_s20 g24_rl; do python -c "
import json,sys; d=json.loads([l for l in open('gpurun_out/$f.log').read().strip().splitlines() if l.startswith('{')][-1]); print('$f', d['value'], d['ms_per_step'], d.get('events_per_s'), d['best_score'])" || true; done
