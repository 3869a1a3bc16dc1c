// Host-side launch API of the replay kernels.
//
// The kernels are compiled in separate translation units (one per NPASS and
// kind, see replay_kernels.hip and ops/build.py) so the many template
// instances build in parallel; module.hip only sees these launchers.
#pragma once

#include <hip/hip_runtime.h>

#include "replay.hip.h"
#include "vm_dev.hip.h"
#include "replay_rows.hip.h"
#include "replay_wave_duo.hip.h"

// waves per SIMD of the 256-node (NPASS 4) wave kernels; the host sizes their
// LDS share to match (build knob for A/B runs)
#ifndef FKS_NP4_WAVES
#define FKS_NP4_WAVES 4     // packed GPU milli + node constants on demand: <= 128 VGPRs
#endif
// waves per SIMD of the two-wave (heap wave + scoring wave) NPASS-4 kernel: 5 (96 VGPRs, a few
// spills) measured above 4 (124 VGPRs), profiles/r5_config5_wave_duo_ab.txt
#ifndef FKS_NP4_DUO_WAVES
#define FKS_NP4_DUO_WAVES 5
#endif

namespace fksk {

using fksd::DevProgramTable;
using fksd::DevResult;
using fksd::DevWorkload;

struct BuiltinArgs {
  DevWorkload W;
  const DevWorkload* Wc;  // the same workload struct, resident in HBM (cold fields)
  const int32_t* fam;     // [P] family id per policy
  const double* weights;  // [P, kWeights] (pinned host memory, device-mapped)
  double* wdev;           // [P, kWeights] device copy written by the kernel prologue
  DevResult* out;
  uint64_t* gheap;        // HBM heap slices (GHEAP) or nullptr
  uint64_t* prof;         // [P, 8] phase cycles (profiling launches only)
  double* table = nullptr;  // row kernels: [P, 13] result table written by the kernel (k_eval_reduce fused)
};

struct VmArgs {
  DevWorkload W;
  const DevWorkload* Wc;
  DevProgramTable T;
  DevResult* out;
  int64_t budget;
  int32_t nregs;          // max virtual registers over the batch's programs
  uint64_t* gheap;
  uint64_t* prof;
};

// Native programs (FKS_KIND 4): fn[p] = device address of policy p's
// JIT-compiled scorer (jit_abi.h ProgFn), kc + koff[p] its constant block.
struct NativeArgs {
  DevWorkload W;
  const DevWorkload* Wc;
  const uint64_t* fn;     // [P] function pointers (pinned host memory, device-mapped)
  const int64_t* kc;      // concatenated constant blocks
  const int32_t* koff;    // [P] offsets into kc
  DevResult* out;
  uint64_t* gheap;
};

// One set of launchers per NPASS (1, 2, 4), named *_np<NPASS>.
// fam_spec >= 0: every policy of the batch has that family (specialised
// kernel); -1: mixed batch.
#define FKS_DECLARE_NPASS(N)                                                                          \
  hipError_t launch_builtin_np##N(bool gheap, int fam_spec, int P, size_t lds, hipStream_t s,         \
                                  const BuiltinArgs& a);                                              \
  hipError_t launch_vm_np##N(bool gheap, int P, size_t lds, hipStream_t s, const VmArgs& a);          \
  hipError_t set_builtin_attrs_np##N(int max_lds);                                                    \
  hipError_t set_vm_attrs_np##N(int max_lds);                                                         \
  hipError_t launch_native_np##N(bool gheap, int P, size_t lds, hipStream_t s, const NativeArgs& a);  \
  hipError_t set_native_attrs_np##N(int max_lds);
FKS_DECLARE_NPASS(1)
FKS_DECLARE_NPASS(2)
FKS_DECLARE_NPASS(4)
#undef FKS_DECLARE_NPASS
// NPASS 4, HBM heap: one policy per 128-thread workgroup of a heap wave and a
// scoring wave (replay_wave_duo.hip.h); lds includes fksd::wave_duo_box_bytes()
hipError_t launch_builtin_duo_np4(int fam_spec, int P, size_t lds, hipStream_t s, const BuiltinArgs& a);

// row kernels: 4 policies per wave (clusters of <= 16 nodes, replay_rows.hip.h)
// `waves` persistent waves drain the P-policy queue: claims are
// atomicAdd(queue) - qbase (the counter runs on across launches; a launch
// makes exactly P + 4 * waves claims).
hipError_t launch_builtin_rows(int fam_spec, int P, int waves, uint32_t* queue, uint32_t qbase, size_t lds, hipStream_t s,
                              const BuiltinArgs& a);
// s_memtime phase-profiled variant (random_linear / composite_linear / mixed); a.prof: [waves, 8]
hipError_t launch_builtin_rows_prof(int fam_spec, int P, int waves, uint32_t* queue, uint32_t qbase, size_t lds, hipStream_t s,
                                   const BuiltinArgs& a);
// resident row-kernel waves per CU for a family's instance at `lds` bytes (-1: error)
int rows_waves_per_cu(int fam_spec, size_t lds);
hipError_t set_rows_attrs(int max_lds);

// row kernel over natively compiled programs (fn / kc / koff as in NativeArgs);
// rows_active rows per wave claim programs, so a launch makes P + rows_active * waves claims;
// a.prof != nullptr: the s_memtime phase-profiled build ([waves, 8] cycles)
hipError_t launch_native_rows(int P, int waves, int rows_active, uint32_t* queue, uint32_t qbase, size_t lds,
                              hipStream_t s, const BuiltinArgs& a, const fksd::RowNativeArgs& nat);
hipError_t set_native_rows_attrs(int max_lds);
// two-wave native replay (replay_duo.hip.h): one program per 128-thread workgroup;
// a.prof != nullptr: the s_memtime phase-profiled build ([P, 2, 8] cycles)
hipError_t launch_native_duo(int P, size_t lds, hipStream_t stream, const BuiltinArgs& a,
                             const fksd::RowNativeArgs& nat);
hipError_t set_native_duo_attrs(int max_lds);
int native_rows_waves_per_cu(size_t lds);
int native_duo_blocks_per_cu(size_t lds);   // resident two-wave workgroups per CU
// the resident program service (replay_kernels.hip k_native_service): its one
// kernel argument, read back through the kernarg segment pointer
struct ServiceArgs {
  BuiltinArgs a;
  fksd::RowNativeArgs nat;
  fksd::ServiceCtl c;
};
static_assert(offsetof(ServiceArgs, a) == 0, "BuiltinArgs (and its DevWorkload) must open the service arguments");
hipError_t launch_native_service(int blocks, size_t lds, hipStream_t stream, const ServiceArgs& s);
hipError_t set_native_service_attrs(int max_lds);
int native_service_blocks_per_cu(size_t lds);

// addresses of the native programs' runtime library (fks_rt_binop, fks_rt_unop, register floor)
hipError_t native_rt_table(uint64_t* dev_out, hipStream_t s);
// glibc_math.h on the device (tests): fn 0 exp, 1 log, 2 pow; n arguments, one per lane
hipError_t launch_gm_batch(int fn, const double* x, const double* y, double* out, int32_t* st, int64_t n);

// phase-profiled variants (NPASS = 1)
hipError_t launch_builtin_prof(bool gheap, int P, size_t lds, hipStream_t s, const BuiltinArgs& a);
hipError_t launch_vm_prof(bool gheap, int P, size_t lds, hipStream_t s, const VmArgs& a);
// composite family, 4 node slots per lane, HBM heap (config-5 shape)
hipError_t launch_c5_prof(int P, size_t lds, hipStream_t s, const BuiltinArgs& a);
hipError_t set_prof_attrs(int max_lds);

}  // namespace fksk
