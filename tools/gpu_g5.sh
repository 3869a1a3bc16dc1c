set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/g5_tests.log 2>&1 && \
timeout -k 10 300 python tools/phase_profile.py > gpurun_out/g5_phase.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 2 --family random_linear --candidates 1536 > gpurun_out/g5_rl1536.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 2 --candidates 1536 > gpurun_out/g5_cl1536.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM -d gpurun_out/pmc1 -o run --output-format csv -- python3 tools/pmc_driver.py random_linear 4096 > gpurun_out/g5_pmc1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pmc2 -o run --output-format csv -- python3 tools/pmc_driver.py random_linear 4096 > gpurun_out/g5_pmc2.log 2>&1
echo "rc=$?"; tail -3 gpurun_out/g5_tests.log; cat gpurun_out/g5_phase.log
for f in g5_rl1536 g5_cl1536; do python -c "
import json,sys; d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d.get('events_per_s'), d['best_score'])"; done
find gpurun_out/pmc1 gpurun_out/pmc2 -name "*.csv" | head; tail -2 gpurun_out/g5_pmc1.log
