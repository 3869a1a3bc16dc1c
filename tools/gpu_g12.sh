set -o pipefail
export PYTHONPATH=$PWD
B="timeout -k 10 300 python bench.py --steps 20 --warmup 2"
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/g12_tests.log 2>&1 && \
$B --family random_linear > gpurun_out/g12_rl.log 2>&1 && \
$B > gpurun_out/g12_cl.log 2>&1 && \
timeout -k 10 600 python tools/vm_bench.py > gpurun_out/g12_vm.log 2>&1 && \
timeout -k 10 300 python tools/phase_profile.py > gpurun_out/g12_phase.log 2>&1 && \
FKS_LIGHT_WAVES=5 FKS_HEAVY_WAVES=4 timeout -k 10 600 python -c "from funsearch_kubernetes_simulator_amd.ops import build; build.build_hip(force=True)" > gpurun_out/g12_build5.log 2>&1 && \
$B --family random_linear > gpurun_out/g12_rl5.log 2>&1 && \
$B > gpurun_out/g12_cl4.log 2>&1
echo "rc=$?"; tail -2 gpurun_out/g12_tests.log; cat gpurun_out/g12_vm.log gpurun_out/g12_phase.log
for f in g12_rl g12_cl g12_rl5 g12_cl4; do python -c "
import json,sys; d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d.get('events_per_s'), d['best_score'])"; done
