#!/bin/bash
# Deterministic A/B of the feasibility-prologue skip: the same offline-mutation programs in batches of 64 and 256.
set -o pipefail
export PYTHONPATH=$PWD FKS_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3s
mkdir -p $O
for b in 256 64; do
  for sk in 1 0 1 0; do
    FKS_FEAS_SKIP=$sk timeout -k 10 200 python -u tools/native_bench.py --batch $b --batches 2 > $O/nb_${b}_$sk.jsonl 2>&1 \
      || { echo "nb $b $sk failed"; tail -20 $O/nb_${b}_$sk.jsonl; exit 1; }
    echo "batch=$b skip=$sk: $(grep '^{"batch": 1' $O/nb_${b}_$sk.jsonl | cut -c1-200)"
  done
done
