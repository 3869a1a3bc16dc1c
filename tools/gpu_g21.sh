set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="timeout -k 10 300 python bench.py --steps 10 --warmup 2"
$B --row-wave-share 1.5 > gpurun_out/g21_s150.log 2>&1 && \
$B --row-wave-share 2.0 > gpurun_out/g21_s200.log 2>&1 && \
$B --row-wave-share 1.0 > gpurun_out/g21_s100.log 2>&1 && \
$B --row-wave-share 1.5 --family random_linear > gpurun_out/g21_s150_rl.log 2>&1
echo "rc=$?"
for f in g21_s100 g21_s150 g21_s200 g21_s150_rl; do python -c "
import json,sys; d=json.loads([l for l in open('gpurun_out/$f.log').read().strip().splitlines() if l.startswith('{')][-1]); print('$f', d['value'], d['ms_per_step'], d.get('events_per_s'), d['best_score'])" || true; done
