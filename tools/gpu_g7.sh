set -o pipefail
export PYTHONPATH=$PWD
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/g7_tests.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM -d gpurun_out/pmc_vm1 -o run --output-format csv -- python3 tools/pmc_vm_driver.py 1024 hbm > gpurun_out/g7_pmc1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY -d gpurun_out/pmc_vm2 -o run --output-format csv -- python3 tools/pmc_vm_driver.py 1024 hbm > gpurun_out/g7_pmc2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_IFETCH SQ_WAIT_INST_LDS -d gpurun_out/pmc_vm3 -o run --output-format csv -- python3 tools/pmc_vm_driver.py 1024 hbm > gpurun_out/g7_pmc3.log 2>&1 && \
timeout -k 10 600 python bench.py --trace synthetic --steps 3 --warmup 1 --candidates 512 > gpurun_out/g7_syn.log 2>&1
echo "rc=$?"; tail -3 gpurun_out/g7_tests.log; grep '"P"' gpurun_out/g7_pmc1.log; tail -3 gpurun_out/g7_pmc3.log; tail -1 gpurun_out/g7_syn.log
