set -o pipefail
export PYTHONPATH=$PWD
B="timeout -k 10 300 python bench.py --steps 20 --warmup 2"
$B --family random_linear > gpurun_out/g11_rl_w4.log 2>&1 && \
$B > gpurun_out/g11_cl_w4.log 2>&1 && \
FKS_LIGHT_WAVES=5 FKS_HEAVY_WAVES=4 timeout -k 10 600 python -c "from funsearch_kubernetes_simulator_amd.ops import build; build.build_hip(force=True)" > gpurun_out/g11_build5.log 2>&1 && \
$B --family random_linear > gpurun_out/g11_rl_w5.log 2>&1 && \
$B --family random_linear --candidates 1280 > gpurun_out/g11_rl_w5_1280.log 2>&1 && \
$B > gpurun_out/g11_cl_w4h.log 2>&1
echo "rc=$?"
for f in g11_rl_w4 g11_cl_w4 g11_rl_w5 g11_rl_w5_1280 g11_cl_w4h; do python -c "
import json,sys; d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d.get('events_per_s'), d['best_score'])"; done
