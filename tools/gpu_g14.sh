set -o pipefail
export PYTHONPATH=$PWD
FKS_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 6 --warmup 1 --migrate-every 2 > gpurun_out/g14_2rank.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 2 > gpurun_out/g14_cl.log 2>&1
echo "rc=$?"; grep '^{' gpurun_out/g14_2rank.log | tail -1 | cut -c1-400; tail -1 gpurun_out/g14_cl.log | cut -c1-300
