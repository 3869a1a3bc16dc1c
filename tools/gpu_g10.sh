set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out/c3
timeout -k 10 600 python -m pytest tests/test_gpu_vm.py -x -q > gpurun_out/g10_tests.log 2>&1 && \
timeout -k 10 600 python tools/vm_bench.py > gpurun_out/g10_vm.log 2>&1 && \
timeout -k 10 900 python -m funsearch_kubernetes_simulator_amd.funsearch --config configs/config3_islands.json --generations 150 --checkpoint-dir gpurun_out/c3 --log gpurun_out/c3/metrics.jsonl --save gpurun_out/c3/top5.json > gpurun_out/g10_c3.log 2>&1
echo "rc=$?"; tail -3 gpurun_out/g10_tests.log; cat gpurun_out/g10_vm.log; tail -1 gpurun_out/g10_c3.log; tail -1 gpurun_out/c3/metrics.jsonl
