set -o pipefail
export PYTHONPATH=$PWD
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/g3_tests.log 2>&1 && \
timeout -k 10 300 python tools/heap_top_sweep.py 4096 > gpurun_out/g3_sweep.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 40 --warmup 2 > gpurun_out/g3_cl_async.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 40 --warmup 2 --sync-islands > gpurun_out/g3_cl_sync.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 2 --family random_linear > gpurun_out/g3_rl_async.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 2 --family random_linear --islands 8 --candidates 512 > gpurun_out/g3_rl_async8.log 2>&1
echo "rc=$?"; tail -3 gpurun_out/g3_tests.log; cat gpurun_out/g3_sweep.log
for f in g3_cl_async g3_cl_sync g3_rl_async g3_rl_async8; do python -c "
import json,sys; d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d.get('events_per_s'), d['best_score'])"; done
