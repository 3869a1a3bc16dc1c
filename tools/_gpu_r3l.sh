#!/bin/bash
# Occupancy sensitivity of the composite row kernel: pad LDS per wave to 12 / 16 / 20 KiB (13 / 10 / 8 waves per CU).
set -o pipefail
export PYTHONPATH=$PWD FKS_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3l
mkdir -p $O
for l in 0 12288 16384 20480; do
  timeout -k 10 200 python -u bench.py --programs 0 --novel 0 --steps 5 --warmup 1 --row-min-lds $l > $O/lds_$l.json 2> $O/lds_$l.err \
    || { echo "lds $l failed"; tail -20 $O/lds_$l.err; exit 1; }
  echo "lds $l: $(cut -c70-170 $O/lds_$l.json)"
done
for c in 1536 4096; do
  timeout -k 10 300 python -u bench.py --trace synthetic --candidates $c --steps 2 --warmup 1 --programs 0 --novel 0 > $O/c5_$c.json 2> $O/c5_$c.err \
    || { echo "c5 $c failed"; tail -20 $O/c5_$c.err; exit 1; }
  echo "c5 $c: $(cut -c70-170 $O/c5_$c.json)"
done
