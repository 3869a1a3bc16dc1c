#!/bin/bash
# Full check of the current tree: every GPU test, smoke, driver-default bench, rocprofv3 kernel stats of the bench
# (family row kernel) and one PMC pass of the row kernel.
set -o pipefail
export PYTHONPATH=$PWD FKS_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3n
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1 \
  || { echo "gpu tests failed"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 1 --programs 0 --novel 0 \
  > $O/prof.log 2>&1 || { echo "profile failed"; tail -20 $O/prof.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE \
  -d $O/pmc1 -o run --output-format csv -- python3 tools/pmc_driver.py composite_linear 49152 > $O/pmc1.log 2>&1 \
  || { echo "pmc1 failed"; tail -20 $O/pmc1.log; exit 1; }
echo done
