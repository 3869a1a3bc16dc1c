set -o pipefail
export PYTHONPATH=$PWD
timeout -k 10 600 python -m pytest tests/test_gpu_vm.py tests/test_gpu_engine.py -x -q > gpurun_out/g8_tests.log 2>&1 && \
timeout -k 10 600 python tools/vm_bench.py > gpurun_out/g8_vm.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH -d gpurun_out/pmc_vm8 -o run --output-format csv -- python3 tools/pmc_vm_driver.py 1024 hbm > gpurun_out/g8_pmc.log 2>&1
echo "rc=$?"; tail -3 gpurun_out/g8_tests.log; cat gpurun_out/g8_vm.log
