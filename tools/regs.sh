#!/bin/bash
# Register / occupancy summary of one replay unit: tools/regs.sh <KIND> [extra hipcc flags]
cd "$(dirname "$0")/.."
F=$(python -c "from funsearch_kubernetes_simulator_amd.ops.build import _hip_flags; print(' '.join(_hip_flags()))")
/opt/rocm/bin/hipcc $F -DFKS_KIND=${1:-3} -DFKS_NPASS=1 "${@:2}" -c csrc/hip/replay_kernels.hip -o /tmp/regs_probe.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 tools/regs_summary.py
