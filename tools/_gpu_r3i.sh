#!/bin/bash
# Continuous asynchronous islands in bench.py (no epoch barrier): driver-default bench, short bench, no-migration bench.
set -o pipefail
export PYTHONPATH=$PWD FKS_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3i
mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/default.json 2> $O/default.err || { echo "default failed"; tail -20 $O/default.err; exit 1; }
echo "default: $(cut -c1-200 $O/default.json)"
timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --programs 0 --novel 0 > $O/s5.json 2> $O/s5.err || { echo "s5 failed"; tail -20 $O/s5.err; exit 1; }
echo "s5: $(cut -c1-200 $O/s5.json)"
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --programs 0 --novel 0 --migrate-every 0 > $O/nomig.json 2> $O/nomig.err || { echo "nomig failed"; tail -20 $O/nomig.err; exit 1; }
echo "nomig: $(cut -c1-200 $O/nomig.json)"
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --programs 0 --novel 0 --sync-islands > $O/sync.json 2> $O/sync.err || { echo "sync failed"; tail -20 $O/sync.err; exit 1; }
echo "sync: $(cut -c1-200 $O/sync.json)"
