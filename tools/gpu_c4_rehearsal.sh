# Config-4 rehearsal on a one-GPU box: the multi-rank program-island search (2 ranks x 4 islands,
# elite migration every 25 generations) with gloo collectives, both ranks sharing device 0; then the
# scaling harness at N=1 on the card.
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c4
FKS_DIST_BACKEND=gloo timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
  --master-addr 127.0.0.1 --master-port 29533 -m funsearch_kubernetes_simulator_amd.funsearch \
  --config configs/offline_islands.json --generations 100 --migrate-every 25 --verbose \
  --checkpoint-dir gpurun_out/c4 --metrics-log gpurun_out/c4/metrics.jsonl --save gpurun_out/c4/top5.json \
  > gpurun_out/c4/run.log 2>&1 || { echo "c4 rc=$?"; tail -20 gpurun_out/c4/run.log; exit 1; }
tail -1 gpurun_out/c4/metrics.rank0.jsonl | cut -c1-300
tail -1 gpurun_out/c4/metrics.rank1.jsonl | cut -c1-300
timeout -k 10 300 python -u -m funsearch_kubernetes_simulator_amd.bench.scaling --gpus 1,2 -- --steps 5 --warmup 1 \
  > gpurun_out/c4/scaling.txt 2>&1
echo "scaling rc=$?"; cat gpurun_out/c4/scaling.txt | cut -c1-300
