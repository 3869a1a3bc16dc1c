#!/bin/bash
# Row kernel: engine tests, bench x2, phase split, PMC pass (per policy-event VALU / SALU / waits).
set -o pipefail
export PYTHONPATH=$PWD FKS_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3h
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 \
  || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for n in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --programs 0 --novel 0 > $O/b$n.json 2> $O/b$n.err \
    || { echo "bench $n failed"; tail -20 $O/b$n.err; exit 1; }
  echo "b$n: $(cut -c1-200 $O/b$n.json)"
done
timeout -k 10 200 python -u tools/phase_rows.py 12288 composite_linear > $O/phase.jsonl 2> $O/phase.err \
  || { echo "phase failed"; tail -20 $O/phase.err; exit 1; }
cat $O/phase.jsonl
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE \
  -d $O/pmc1 -o run --output-format csv -- python3 tools/pmc_driver.py composite_linear 49152 > $O/pmc1.log 2>&1 \
  || { echo "pmc1 failed"; tail -20 $O/pmc1.log; exit 1; }
tail -1 $O/pmc1.log
for c in 1536 4096; do
  timeout -k 10 300 python -u bench.py --trace synthetic --candidates $c --steps 2 --warmup 1 --programs 0 --novel 0 > $O/c5_$c.json 2> $O/c5_$c.err \
    || { echo "c5 $c failed"; tail -20 $O/c5_$c.err; exit 1; }
  echo "c5 $c: $(cut -c1-200 $O/c5_$c.json)"
done
