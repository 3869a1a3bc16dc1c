#!/bin/bash
# BASELINE config 3 steady-state islands (FF/BF seeds): feasibility-prologue skip on vs off, 90 s each.
set -o pipefail
export PYTHONPATH=$PWD FKS_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3r
mkdir -p $O
for sk in 1 0; do
  FKS_FEAS_SKIP=$sk timeout -k 10 300 python -u -m funsearch_kubernetes_simulator_amd.funsearch --config configs/config3_steady.json \
    --verbose --wall-s 90 --save $O/top5_skip$sk.json --checkpoint-dir $O/ck$sk \
    --metrics-log $O/metrics_skip$sk.jsonl > $O/steady_skip$sk.log 2>&1 || { echo "steady $sk failed"; tail -20 $O/steady_skip$sk.log; exit 1; }
  echo "skip=$sk: $(grep steady_final $O/steady_skip$sk.log | cut -c1-260)"
done
