#!/bin/bash
# overlap probe (JIT load vs replaying slots), GPU JIT-tier tests, short steady config-3 run
set -o pipefail
export FKS_NO_AUTOBUILD=1
mkdir -p gpurun_out/r3b
timeout -k 10 300 python -u tools/gcn_probe.py overlap > gpurun_out/r3b/overlap.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_gcn.py tests/test_gpu_native.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r3b/pytest.log 2>&1 && \
timeout -k 10 400 python -u -m funsearch_kubernetes_simulator_amd.funsearch --config configs/config3_steady.json \
  --verbose --wall-s 180 --save gpurun_out/r3b/top5.json --checkpoint-dir gpurun_out/r3b/ck \
  --metrics-log gpurun_out/r3b/metrics.jsonl > gpurun_out/r3b/steady.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/r3b/bench.json 2> gpurun_out/r3b/bench.err
rc=$?
grep -v amdgpu.ids gpurun_out/r3b/overlap.log | tail -3
tail -3 gpurun_out/r3b/pytest.log
grep steady_final gpurun_out/r3b/steady.log | cut -c1-600
cut -c1-300 gpurun_out/r3b/bench.json
exit $rc
