set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="timeout -k 10 300 python bench.py --steps 10 --warmup 2"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g17_tests.log 2>&1 && \
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/g17_smoke.log 2>&1 && \
$B > gpurun_out/g17_c4096.log 2>&1 && \
$B --candidates 8192 > gpurun_out/g17_c8192.log 2>&1 && \
$B --candidates 12288 > gpurun_out/g17_c12288.log 2>&1 && \
$B --candidates 8192 --family random_linear > gpurun_out/g17_rl8192.log 2>&1
echo "rc=$?"; tail -2 gpurun_out/g17_tests.log; tail -1 gpurun_out/g17_smoke.log
for f in g17_c4096 g17_c8192 g17_c12288 g17_rl8192; do python -c "
import json,sys; d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d.get('events_per_s'), d['best_score'])" || true; done
