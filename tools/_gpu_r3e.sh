#!/bin/bash
# Row-kernel diagnosis: phase split, occupancy sensitivity (persistent-wave share), family cost, PMC passes.
set -o pipefail
export PYTHONPATH=$PWD FKS_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 200 python -u tools/phase_rows.py 12288 composite_linear random_linear > $O/phase.jsonl 2> $O/phase.err \
  || { echo "phase failed"; tail -20 $O/phase.err; exit 1; }
cat $O/phase.jsonl
for s in 0.75 0.5; do
  timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --programs 0 --novel 0 --row-wave-share $s > $O/share_$s.json 2> $O/share_$s.err \
    || { echo "share $s failed"; tail -20 $O/share_$s.err; exit 1; }
  echo "share $s: $(cut -c1-200 $O/share_$s.json)"
done
timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --programs 0 --novel 0 --family random_linear > $O/rl.json 2> $O/rl.err \
  || { echo "rl failed"; tail -20 $O/rl.err; exit 1; }
echo "random_linear: $(cut -c1-200 $O/rl.json)"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE \
  -d $O/pmc1 -o run --output-format csv -- python3 tools/pmc_driver.py composite_linear 49152 > $O/pmc1.log 2>&1 \
  || { echo "pmc1 failed"; tail -20 $O/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_WAVES TCC_HIT_sum TCC_MISS_sum \
  -d $O/pmc2 -o run --output-format csv -- python3 tools/pmc_driver.py composite_linear 49152 > $O/pmc2.log 2>&1 \
  || { echo "pmc2 failed"; tail -20 $O/pmc2.log; exit 1; }
find $O -name "*counter_collection*" | head
