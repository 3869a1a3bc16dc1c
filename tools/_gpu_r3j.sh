#!/bin/bash
# Persistent-wave share sweep with asynchronous islands (rows drain more than one policy per launch below 1.0).
set -o pipefail
export PYTHONPATH=$PWD FKS_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3j
mkdir -p $O
for s in 1.0 0.5 0.34 0.25 0.75; do
  timeout -k 10 200 python -u bench.py --programs 0 --novel 0 --row-wave-share $s > $O/share_$s.json 2> $O/share_$s.err \
    || { echo "share $s failed"; tail -20 $O/share_$s.err; exit 1; }
  echo "share $s: $(cut -c70-160 $O/share_$s.json)"
done
