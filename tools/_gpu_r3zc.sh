# PMC pass of the late round-3 256-node composite wave kernel (config-5 shape, 2,048 policies).
set -o pipefail
export PYTHONPATH=$PWD FKS_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3zc
mkdir -p $O
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE \
  -d $O/pmc1 -o run --output-format csv -- python3 tools/pmc_c5_driver.py 2048 > $O/pmc1.log 2>&1 \
  || { echo "pmc1 failed"; tail -20 $O/pmc1.log; exit 1; }
grep '"events"' $O/pmc1.log
