set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out/c3a gpurun_out/c3b
timeout -k 10 600 python -m funsearch_kubernetes_simulator_amd.funsearch --config configs/config3_islands.json --generations 8 --checkpoint-dir gpurun_out/c3a --log gpurun_out/c3a/metrics.jsonl > gpurun_out/g9_c3_cpu.log 2>&1 && \
timeout -k 10 600 python -m funsearch_kubernetes_simulator_amd.funsearch --config configs/config3_islands.json --generations 8 --device-min-batch 1 --checkpoint-dir gpurun_out/c3b --log gpurun_out/g9_c3b_metrics.jsonl > gpurun_out/g9_c3_dev.log 2>&1 && \
timeout -k 10 600 python tools/vm_bench.py > gpurun_out/g9_vm.log 2>&1
echo "rc=$?"; tail -1 gpurun_out/g9_c3_cpu.log; tail -1 gpurun_out/g9_c3_dev.log; tail -2 gpurun_out/c3a/metrics.jsonl; tail -2 gpurun_out/g9_c3b_metrics.jsonl; cat gpurun_out/g9_vm.log
