set -o pipefail
export PYTHONPATH=$PWD
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/g6_tests.log 2>&1 && \
timeout -k 10 600 python tools/vm_bench.py > gpurun_out/g6_vm.log 2>&1 && \
timeout -k 10 300 python tools/phase_profile.py > gpurun_out/g6_phase.log 2>&1
echo "rc=$?"; tail -3 gpurun_out/g6_tests.log; cat gpurun_out/g6_vm.log gpurun_out/g6_phase.log
