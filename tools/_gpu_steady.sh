#!/bin/bash
# BASELINE config 3 in steady-state island mode on one MI355X (FF/BF seeds only).
set -o pipefail
mkdir -p gpurun_out/steady
timeout -k 10 700 python -u -m funsearch_kubernetes_simulator_amd.funsearch --config configs/config3_steady.json \
  --verbose --save gpurun_out/steady/top5.json --checkpoint-dir gpurun_out/steady/ck \
  --metrics-log gpurun_out/steady/metrics.jsonl > gpurun_out/steady/run.log 2>&1
rc=$?
tail -5 gpurun_out/steady/run.log
exit $rc
