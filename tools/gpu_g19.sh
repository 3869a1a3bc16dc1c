set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py > gpurun_out/g19_default.log 2>&1 && \
timeout -k 10 300 python bench.py --family random_linear > gpurun_out/g19_rl.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof19 -o run -- python3 bench.py --steps 5 --warmup 1 > gpurun_out/g19_prof.log 2>&1 && \
FKS_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/g19_two_ranks.log 2>&1
echo "rc=$?"
for f in g19_default g19_rl g19_two_ranks; do python -c "
import json,sys; d=json.loads([l for l in open('gpurun_out/$f.log').read().strip().splitlines() if l.startswith('{')][-1]); print('$f', d['value'], d['n_gpus'], d['ms_per_step'], d.get('events_per_s'), d['best_score'], d['config']['global_batch'])" || true; done
find gpurun_out/prof19 -name "*kernel_stats.csv" | head -2
