#!/bin/bash
# Config 5 A/B: HBM-heap wave kernels with flat heap accesses (default build) vs exec-masked (rebuilt here with
# FKS_WAVE_FLAT=0; the knob is part of the source hash, so the import check accepts that build under the same env).
set -o pipefail
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3o
mkdir -p $O
for c in 4096 1536; do
  FKS_NO_AUTOBUILD=1 timeout -k 10 300 python -u bench.py --trace synthetic --candidates $c --steps 3 --warmup 1 --programs 0 --novel 0 > $O/flat_$c.json 2> $O/flat_$c.err \
    || { echo "flat $c failed"; tail -20 $O/flat_$c.err; exit 1; }
  echo "flat c5 $c: $(cut -c70-170 $O/flat_$c.json)"
done
FKS_WAVE_FLAT=0 timeout -k 10 400 python -c "from funsearch_kubernetes_simulator_amd.ops.build import build_hip; build_hip(jobs=16)" > $O/build.log 2>&1 \
  || { echo "build failed"; tail -20 $O/build.log; exit 1; }
for c in 4096 1536; do
  FKS_WAVE_FLAT=0 FKS_NO_AUTOBUILD=1 timeout -k 10 300 python -u bench.py --trace synthetic --candidates $c --steps 3 --warmup 1 --programs 0 --novel 0 > $O/split_$c.json 2> $O/split_$c.err \
    || { echo "split $c failed"; tail -20 $O/split_$c.err; exit 1; }
  echo "split c5 $c: $(cut -c70-170 $O/split_$c.json)"
done
