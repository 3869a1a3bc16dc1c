# BASELINE config 3 from FF/BF seeds with the family coupler (configs/config3_coupled.json): 4 pipelined
# program islands evaluated natively on the MI355X, plus a random_linear / feature_linear family search on its
# own HIP slot whose champions are injected into the program islands as program text.  Runs in parts of G
# generations, resuming from the checkpoint staged in runs/config3_coupled (copied into gpurun_out/c3c).
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CFG=${CFG:-configs/config3_coupled.json}
RUN=${RUN:-runs/config3_coupled}
mkdir -p gpurun_out/c3c
cp $RUN/islands_rank0.json $RUN/metrics.jsonl gpurun_out/c3c/ 2>/dev/null
G=${G:-1000}
T=${T:-1100}
timeout -k 10 $T python -u -m funsearch_kubernetes_simulator_amd.funsearch --config $CFG \
  --generations $G --resume --verbose --checkpoint-dir gpurun_out/c3c --log gpurun_out/c3c/metrics.jsonl \
  --save gpurun_out/c3c/top5.json > gpurun_out/c3c/run.log 2>&1
rc=$?
echo "rc=$rc"; tail -2 gpurun_out/c3c/run.log | cut -c1-600
grep '"kind": "coupling"' gpurun_out/c3c/metrics.jsonl | tail -4 | cut -c1-400
grep '"kind": "generation"' gpurun_out/c3c/metrics.jsonl | tail -1 | cut -c1-700
exit $rc
