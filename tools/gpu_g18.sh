set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="timeout -k 10 300 python bench.py --steps 10 --warmup 2"
$B --candidates 16384 > gpurun_out/g18_c16384.log 2>&1 && \
$B --candidates 24576 > gpurun_out/g18_c24576.log 2>&1 && \
$B --candidates 12288 --family random_linear > gpurun_out/g18_rl12288.log 2>&1 && \
$B --candidates 16384 --family random_linear > gpurun_out/g18_rl16384.log 2>&1
echo "rc=$?"
for f in g18_c16384 g18_c24576 g18_rl12288 g18_rl16384; do python -c "
import json,sys; d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d.get('events_per_s'), d['best_score'])" || true; done
