set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="timeout -k 10 300 python bench.py --steps 10 --warmup 2"
$B --row-wave-share 0.5 > gpurun_out/g20_s050.log 2>&1 && \
$B --row-wave-share 0.25 > gpurun_out/g20_s025.log 2>&1 && \
$B --row-wave-share 0.5 --candidates 4096 > gpurun_out/g20_s050_c4096.log 2>&1 && \
$B --row-wave-share 0.5 --family random_linear > gpurun_out/g20_s050_rl.log 2>&1 && \
$B --row-wave-share 1.0 > gpurun_out/g20_s100.log 2>&1
echo "rc=$?"
for f in g20_s100 g20_s050 g20_s025 g20_s050_c4096 g20_s050_rl; do python -c "
import json,sys; d=json.loads([l for l in open('gpurun_out/$f.log').read().strip().splitlines() if l.startswith('{')][-1]); print('$f', d['value'], d['ms_per_step'], d.get('events_per_s'), d['best_score'])" || true; done
