set -o pipefail
export PYTHONPATH=$PWD
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/g4_tests.log 2>&1 && \
timeout -k 10 600 python tools/vm_bench.py > gpurun_out/g4_vm.log 2>&1 && \
timeout -k 10 300 python tools/phase_profile.py > gpurun_out/g4_phase.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 2 --family random_linear --candidates 1280 > gpurun_out/g4_rl1280.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 2 --family random_linear --candidates 1536 > gpurun_out/g4_rl1536.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 2 --family random_linear --islands 2 --candidates 2048 > gpurun_out/g4_rl2x2048.log 2>&1
echo "rc=$?"; tail -3 gpurun_out/g4_tests.log; cat gpurun_out/g4_vm.log gpurun_out/g4_phase.log
for f in g4_rl1280 g4_rl1536 g4_rl2x2048; do python -c "
import json,sys; d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d.get('events_per_s'), d['best_score'])"; done
