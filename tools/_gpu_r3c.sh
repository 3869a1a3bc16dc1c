#!/bin/bash
# steady config 3 (phase breakdown), config-5 copy trace, MFMA screening A/B
set -o pipefail
export FKS_NO_AUTOBUILD=1
mkdir -p gpurun_out/r3c
timeout -k 10 300 python -u -m funsearch_kubernetes_simulator_amd.funsearch --config configs/config3_steady.json \
  --verbose --wall-s 120 --checkpoint-dir gpurun_out/r3c/ck \
  --metrics-log gpurun_out/r3c/metrics.jsonl > gpurun_out/r3c/steady.log 2>&1 && \
grep steady_final gpurun_out/r3c/steady.log | cut -c1-3000 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/r3c/c5prof -o c5 -- \
  python3 bench.py --trace synthetic --candidates 1536 --steps 2 --warmup 1 --programs 0 --novel 0 \
  > gpurun_out/r3c/c5.json 2> gpurun_out/r3c/c5.err && \
BUDGET=45 bash tools/screen_ab.sh
rc=$?
find gpurun_out/r3c/c5prof -name "*stats*" | head
exit $rc
