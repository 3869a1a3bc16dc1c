# Push-ancestor prefetch: exactness tests (row + wave kernels), default bench, config-5 bench, row-kernel PMC,
# then a FKS_ROW_HEAVY_WAVES=5 rebuild + bench (occupancy A/B).
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pf
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_native.py -x -q --timeout 250 --timeout-method thread \
  > gpurun_out/pf/tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pf/tests.txt; exit 1; }
tail -2 gpurun_out/pf/tests.txt
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --programs 0 > gpurun_out/pf/bench.json 2> gpurun_out/pf/bench.err \
  || { echo "bench failed"; tail -20 gpurun_out/pf/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/pf/bench.json')); print('default', d['value'], d['ms_per_step'])"
timeout -k 10 200 python -u bench.py --trace synthetic --candidates 1536 --steps 2 --warmup 1 --programs 0 > gpurun_out/pf/c5.json 2> gpurun_out/pf/c5.err \
  || { echo "c5 failed"; tail -20 gpurun_out/pf/c5.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/pf/c5.json')); print('config5', d['value'], d['ms_per_step'])"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  --kernel-trace -d gpurun_out/pf/pmc_a -o run --output-format csv -- python3 tools/pmc_driver.py composite_linear 49152 \
  > gpurun_out/pf/pmc_a.log 2>&1 || { echo "pmc a failed"; tail -5 gpurun_out/pf/pmc_a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH \
  --kernel-trace -d gpurun_out/pf/pmc_b -o run --output-format csv -- python3 tools/pmc_driver.py composite_linear 49152 \
  > gpurun_out/pf/pmc_b.log 2>&1 || { echo "pmc b failed"; tail -5 gpurun_out/pf/pmc_b.log; exit 1; }
grep '"events"' gpurun_out/pf/pmc_a.log | cut -c1-120
HWS="5" bash tools/gpu_row_waves.sh
