set -o pipefail
export PYTHONPATH=$PWD
B="timeout -k 10 300 python bench.py --steps 20 --warmup 2"
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/g13_tests.log 2>&1 && \
$B --family random_linear > gpurun_out/g13_rl.log 2>&1 && \
$B > gpurun_out/g13_cl.log 2>&1 && \
timeout -k 10 300 python tools/phase_profile.py > gpurun_out/g13_phase.log 2>&1 && \
timeout -k 10 300 python tools/heap_bench.py > gpurun_out/g13_heap.log 2>&1
echo "rc=$?"; tail -2 gpurun_out/g13_tests.log; cat gpurun_out/g13_phase.log; tail -5 gpurun_out/g13_heap.log
for f in g13_rl g13_cl; do python -c "
import json,sys; d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d.get('events_per_s'), d['best_score'])"; done
