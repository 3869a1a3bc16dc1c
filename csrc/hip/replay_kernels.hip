// Replay kernels: one wave64 workgroup per candidate policy.
//
// Compiled once per (FKS_KIND, FKS_NPASS) by ops/build.py:
//   FKS_KIND 0 -> built-in family kernels for FKS_NPASS (one instance per family + a mixed one)
//   FKS_KIND 1 -> bytecode-VM kernels for FKS_NPASS
//   FKS_KIND 2 -> phase-profiled diagnostics kernels (NPASS = 1)
//   FKS_KIND 3 -> row kernels (4 policies per wave, <= 16 nodes; replay_rows.hip.h)
//   FKS_KIND 4 -> native-program kernels (JIT-compiled scorers called through
//                 function pointers; jit_abi.h) for FKS_NPASS
// Each unit defines the matching launchers of launch.h.
#include <hip/hip_runtime.h>

#include "launch.h"
#include "replay.hip.h"
#include "scorers.hip.h"
#include "vm_dev.hip.h"
#include "replay_rows.hip.h"
#include "replay_duo.hip.h"
#include "replay_wave_duo.hip.h"

namespace {
// The launch's workload struct as the kernel received it: every kernel's
// first parameter is an argument struct whose first member is the
// DevWorkload, so it sits at offset 0 of the kernarg segment.  The kernels
// re-read their cold fields from there with scalar loads -- no per-slot HBM
// copy, hence no copy kernel that would have to wait for a CU slot behind
// the other slots' persistent replay waves (~1 s at config-5 shape).
// (`&a.W` would not do: taking a by-value parameter's address makes clang
// copy the struct to scratch.)
__device__ __forceinline__ const fksd::DevWorkload* kernarg_workload() {
  // constant (4) -> flat: the same 64-bit address (the kernarg segment is ordinary global memory)
  return reinterpret_cast<const fksd::DevWorkload*>((uintptr_t)__builtin_amdgcn_kernarg_segment_ptr());
}
static_assert(offsetof(fksk::BuiltinArgs, W) == 0, "DevWorkload must open the kernel arguments");
static_assert(offsetof(fksk::VmArgs, W) == 0, "DevWorkload must open the kernel arguments");
static_assert(offsetof(fksk::NativeArgs, W) == 0, "DevWorkload must open the kernel arguments");
}  // namespace
#include "jit_abi.h"

#ifndef FKS_KIND
#define FKS_KIND 0
#endif
#ifndef FKS_NPASS
#define FKS_NPASS 1
#endif
#ifndef FKS_WAVE_FLAT
#define FKS_WAVE_FLAT 1   // HBM-heap wave kernels: flat heap accesses (heap_wave.h WaveHeapT)
#endif

using namespace fksd;

namespace {

// Where a policy's heap, deletion bitmap and VM registers live.
//   GHEAP = false: LDS = heap | bitmap | vregs (2 policies/CU on the 8k trace)
//   GHEAP = true : heap in its HBM slice, LDS = bitmap | heap top (W.heap_top
//                  slots) | vregs (16 policies/CU)
struct Slot {
  FKS_LDS double* w;       // builtin policy weights, copied in by the prologue
  FKS_GLOBAL uint64_t* h;
  FKS_LDS uint64_t* top;
  int T;
  FKS_LDS uint32_t* delmap;
  uint64_t* vregs;
  FKS_LDS int32_t* inv;   // invariant-check scratch (debug; unused when off)
};
template <bool GHEAP>
__device__ __forceinline__ Slot policy_slot(const DevWorkload& W, uint64_t* gheap, int p) {
  extern __shared__ uint64_t lds_raw[];
  FKS_LDS uint64_t* lds0 = lds_ptr(lds_raw);
  // [invariant scratch | builtin weights (kWeights doubles) | policy layout]
  FKS_LDS uint64_t* lds = lds0 + W.inv_words + kWeights;
  const int N = W.n_pods;
  Slot s;
  s.inv = reinterpret_cast<FKS_LDS int32_t*>(lds0);
  s.w = reinterpret_cast<FKS_LDS double*>(lds0 + W.inv_words);
  if (GHEAP) {
    // the deletion bitmap covers the first W.delmap_slots slots (a multiple of 64)
    const int dw = W.delmap_slots >> 5;
    s.h = global_ptr(gheap + (size_t)p * lds_heap_entries(N));
    s.delmap = reinterpret_cast<FKS_LDS uint32_t*>(lds);
    s.top = lds + dw / 2;
    s.T = W.heap_top;
    s.vregs = lds_raw + W.inv_words + kWeights + dw / 2 + W.heap_top;
  } else {
    s.h = global_ptr(gheap);   // never dereferenced: T covers the whole heap
    s.top = lds;
    s.T = lds_heap_entries(N);
    s.delmap = reinterpret_cast<FKS_LDS uint32_t*>(lds + lds_heap_entries(N));
    s.vregs = lds_raw + W.inv_words + kWeights + lds_vreg_offset(N);
  }
  return s;
}

// Waves per SIMD the kernel is compiled for: the LDS-heap variant is LDS-bound at
// 2 waves/CU anyway; the HBM-heap variant trades registers for occupancy.
#define FKS_BOUNDS(G) __launch_bounds__(64, (G) ? 4 : 1)
// The VM keeps its hot virtual registers in VGPRs (vm_dev.hip.h): 2 waves/SIMD.
#define FKS_VM_BOUNDS(G) __launch_bounds__(64, (G) ? 2 : 1)

// Prologue: the batch's family ids / weights live in pinned host memory
// (zero-copy, no copy kernel queued behind busy CUs); each policy moves its 16
// weights into its slot of a device buffer once, which the scorer then reads
// through the scalar cache.
template <int FAM>
__device__ __forceinline__ void load_policy(BuiltinScorerDev<FAM>& sc, const Slot&, const fksk::BuiltinArgs& a,
                                            int p) {
  const int lane = lane_id();
  double* wd = a.wdev + (size_t)p * kWeights;
  if (lane < kWeights) wd[lane] = a.weights[(size_t)p * kWeights + lane];
  const int fam = uni(lane == 0 ? a.fam[p] : 0);
  __threadfence();   // stores visible to the scalar loads that follow
  sc.load(fam, wd);
  sc.zp = a.W.node_recip;
  sc.capz = kernarg_workload()->cap_recip;
}

template <class T>
hipError_t raise_lds(T* f, int max_lds) {
  return hipFuncSetAttribute(reinterpret_cast<const void*>(f), hipFuncAttributeMaxDynamicSharedMemorySize, max_lds);
}

#if FKS_KIND == 0
// the feature families carry ~40 more live values through scoring: 3 waves/SIMD
// without spills beats 4 with scratch traffic
// without spills beats 4 with scratch traffic; 128 / 256 nodes (NPASS 2 / 4)
// hold 2 / 4 node slots per lane: 3 / 2 waves per SIMD.
#ifndef FKS_LIGHT_WAVES
#define FKS_LIGHT_WAVES 4   // first-fit / best-fit / random_linear (build-time knob for A/B runs)
#endif
#ifndef FKS_HEAVY_WAVES
#define FKS_HEAVY_WAVES 3   // feature / composite families and mixed batches
#endif
#define FKS_FAM_BOUNDS(G, F, NP)                                               \
  __launch_bounds__(64, !(G) ? 1 : (NP) >= 4 ? FKS_NP4_WAVES : (NP) == 2 ? 3   \
                           : (((F) == 3 || (F) == 4 || (F) < 0) ? FKS_HEAVY_WAVES : FKS_LIGHT_WAVES))
template <int NPASS, bool GHEAP, int FAM>
__global__ FKS_FAM_BOUNDS(GHEAP, FAM, NPASS) void k_replay_builtin(fksk::BuiltinArgs a) {
  const int p = blockIdx.x;
  const Slot s = policy_slot<GHEAP>(a.W, a.gheap, p);
  BuiltinScorerDev<FAM> sc;
  load_policy<FAM>(sc, s, a, p);
  replay_one<NPASS, BuiltinScorerDev<FAM>, NoProf, GHEAP && FKS_WAVE_FLAT>(a.W, kernarg_workload(), sc, s.h, s.top, s.T,
                                                                           s.delmap, s.inv, a.out + p);
}

template <int NPASS, bool GHEAP>
hipError_t launch_g(int fam, int P, size_t lds, hipStream_t st, const fksk::BuiltinArgs& a) {
#define FKS_CASE(F) \
  case F: hipLaunchKernelGGL((k_replay_builtin<NPASS, GHEAP, F>), dim3(P), dim3(64), lds, st, a); break;
  switch (fam) {
    FKS_CASE(FAM_FIRST_FIT)
    FKS_CASE(FAM_BEST_FIT)
    FKS_CASE(FAM_RANDOM_LINEAR)
    FKS_CASE(FAM_FEATURE_LINEAR)
    FKS_CASE(FAM_COMPOSITE_LINEAR)
    default: hipLaunchKernelGGL((k_replay_builtin<NPASS, GHEAP, -1>), dim3(P), dim3(64), lds, st, a);
  }
#undef FKS_CASE
  return hipGetLastError();
}

template <int NPASS, bool GHEAP>
hipError_t attrs_g(int mx) {
  hipError_t e = hipSuccess;
  for (hipError_t r : {raise_lds(&k_replay_builtin<NPASS, GHEAP, -1>, mx),
                       raise_lds(&k_replay_builtin<NPASS, GHEAP, FAM_FIRST_FIT>, mx),
                       raise_lds(&k_replay_builtin<NPASS, GHEAP, FAM_BEST_FIT>, mx),
                       raise_lds(&k_replay_builtin<NPASS, GHEAP, FAM_RANDOM_LINEAR>, mx),
                       raise_lds(&k_replay_builtin<NPASS, GHEAP, FAM_FEATURE_LINEAR>, mx),
                       raise_lds(&k_replay_builtin<NPASS, GHEAP, FAM_COMPOSITE_LINEAR>, mx)})
    if (r != hipSuccess) e = r;
  return e;
}
#endif

#if FKS_KIND == 0 && FKS_NPASS == 4
// 256-node clusters, HBM heap: heap wave + scoring wave per policy
// (replay_wave_duo.hip.h); both waves share the register allocation of the
// scoring wave, FKS_NP4_DUO_WAVES waves per SIMD (launch.h)
template <int FAM>
__global__ __launch_bounds__(128, FKS_NP4_DUO_WAVES) void k_replay_builtin_duo(fksk::BuiltinArgs a) {
  const int p = blockIdx.x;
  const Slot s = policy_slot<true>(a.W, a.gheap, p);
  BuiltinScorerDev<FAM> sc;
  if (threadIdx.x >= kWave) load_policy<FAM>(sc, s, a, p);   // the scoring wave's weights
  FKS_LDS DuoBox* box = reinterpret_cast<FKS_LDS DuoBox*>(lds_ptr(s.vregs));
  replay_wave_duo<4, BuiltinScorerDev<FAM>, FKS_WAVE_FLAT>(a.W, kernarg_workload(), sc, s.h, s.top, s.T, s.delmap,
                                                            box, a.out + p);
}

hipError_t launch_duo4(int fam, int P, size_t lds, hipStream_t st, const fksk::BuiltinArgs& a) {
#define FKS_CASE(F) \
  case F: hipLaunchKernelGGL((k_replay_builtin_duo<F>), dim3(P), dim3(128), lds, st, a); break;
  switch (fam) {
    FKS_CASE(FAM_FIRST_FIT)
    FKS_CASE(FAM_BEST_FIT)
    FKS_CASE(FAM_RANDOM_LINEAR)
    FKS_CASE(FAM_FEATURE_LINEAR)
    FKS_CASE(FAM_COMPOSITE_LINEAR)
    default: hipLaunchKernelGGL((k_replay_builtin_duo<-1>), dim3(P), dim3(128), lds, st, a);
  }
#undef FKS_CASE
  return hipGetLastError();
}

hipError_t attrs_duo4(int mx) {
  hipError_t e = hipSuccess;
  for (hipError_t r : {raise_lds(&k_replay_builtin_duo<-1>, mx), raise_lds(&k_replay_builtin_duo<FAM_FIRST_FIT>, mx),
                       raise_lds(&k_replay_builtin_duo<FAM_BEST_FIT>, mx),
                       raise_lds(&k_replay_builtin_duo<FAM_RANDOM_LINEAR>, mx),
                       raise_lds(&k_replay_builtin_duo<FAM_FEATURE_LINEAR>, mx),
                       raise_lds(&k_replay_builtin_duo<FAM_COMPOSITE_LINEAR>, mx)})
    if (r != hipSuccess) e = r;
  return e;
}
#endif

#if FKS_KIND == 1
template <int NPASS, bool GHEAP>
__global__ FKS_VM_BOUNDS(GHEAP) void k_replay_vm(fksk::VmArgs a) {
  const int p = blockIdx.x;
  const Slot s = policy_slot<GHEAP>(a.W, a.gheap, p);
  VmScorerDev sc;
  sc.init(a.T, p, a.W, a.budget, s.vregs);
  replay_one<NPASS>(a.W, kernarg_workload(), sc, s.h, s.top, s.T, s.delmap, s.inv, a.out + p);
}
#endif

#if FKS_KIND == 2
template <bool GHEAP>
__global__ FKS_BOUNDS(GHEAP) void k_replay_builtin_prof(fksk::BuiltinArgs a) {
  const int p = blockIdx.x;
  const Slot s = policy_slot<GHEAP>(a.W, a.gheap, p);
  BuiltinScorerDev<-1> sc;
  load_policy<-1>(sc, s, a, p);
  replay_one<1, BuiltinScorerDev<-1>, PhaseProf>(a.W, kernarg_workload(), sc, s.h, s.top, s.T, s.delmap, s.inv, a.out + p,
                                                 a.prof + (size_t)p * 8);
}

// 256-node clusters: the production composite instance (4 node slots per
// lane, HBM heap, same launch bounds) with the s_memtime phase profiler
__global__ __launch_bounds__(64, FKS_NP4_WAVES) void k_replay_c5_prof(fksk::BuiltinArgs a) {
  const int p = blockIdx.x;
  const Slot s = policy_slot<true>(a.W, a.gheap, p);
  BuiltinScorerDev<FAM_COMPOSITE_LINEAR> sc;
  load_policy<FAM_COMPOSITE_LINEAR>(sc, s, a, p);
  replay_one<4, BuiltinScorerDev<FAM_COMPOSITE_LINEAR>, PhaseProf, FKS_WAVE_FLAT>(
      a.W, kernarg_workload(), sc, s.h, s.top, s.T, s.delmap, s.inv, a.out + p, a.prof + (size_t)p * 8);
}

template <bool GHEAP>
__global__ FKS_VM_BOUNDS(GHEAP) void k_replay_vm_prof(fksk::VmArgs a) {
  const int p = blockIdx.x;
  const Slot s = policy_slot<GHEAP>(a.W, a.gheap, p);
  VmScorerDev sc;
  sc.init(a.T, p, a.W, a.budget, s.vregs);
  replay_one<1, VmScorerDev, PhaseProf>(a.W, kernarg_workload(), sc, s.h, s.top, s.T, s.delmap, s.inv, a.out + p, a.prof + (size_t)p * 8);
}
#endif


#if FKS_KIND == 3
// Row kernels: the LDS share per wave (4 heap tops + bitmaps) is what bounds
// residency; registers are capped so LDS, not VGPRs, stays the limit.
#ifndef FKS_ROW_WAVES
#define FKS_ROW_WAVES 5        // first-fit / best-fit / random_linear
#endif
#ifndef FKS_ROW_HEAVY_WAVES
#define FKS_ROW_HEAVY_WAVES 4  // feature / composite families (composite: only loop-invariant snapshot
                               // divisors spill, reloaded on the rare snapshot path)
#endif
template <int FAM>
__global__ __launch_bounds__(64, FAM < 0 ? 2 : (FAM == 3 || FAM == 4) ? FKS_ROW_HEAVY_WAVES : FKS_ROW_WAVES) void k_replay_rows(fksk::BuiltinArgs a, int P, uint32_t* queue, uint32_t qbase) {
  replay_rows<FAM>(a.W, kernarg_workload(), a.fam, a.weights, a.gheap, a.out, P, queue, qbase, nullptr,
                   RowNativeArgs{nullptr, nullptr, nullptr}, kRowsPerWave, a.table);
}
#endif

#if FKS_KIND == 3
// The composite instance at 5 waves per SIMD (<= 96 VGPRs, a few loop-invariant
// spills): host family code kRowCompositeW5 (`row_composite_waves` option).
__global__ __launch_bounds__(64, 5) void k_replay_rows_c5(fksk::BuiltinArgs a, int P, uint32_t* queue, uint32_t qbase) {
  replay_rows<FAM_COMPOSITE_LINEAR>(a.W, kernarg_workload(), a.fam, a.weights, a.gheap, a.out, P, queue, qbase, nullptr,
                                    RowNativeArgs{nullptr, nullptr, nullptr}, kRowsPerWave, a.table);
}
__global__ __launch_bounds__(64, FKS_ROW_HEAVY_WAVES) void k_replay_rows_split(fksk::BuiltinArgs a, int P, uint32_t* queue,
                                                                               uint32_t qbase) {
  replay_rows<FAM_COMPOSITE_LINEAR, RowNoProf, false>(a.W, kernarg_workload(), a.fam, a.weights, a.gheap, a.out, P, queue,
                                                      qbase, nullptr, RowNativeArgs{nullptr, nullptr, nullptr}, kRowsPerWave,
                                                      a.table);
}
template <int FAM>
__global__ __launch_bounds__(64, FAM < 0 ? 2 : (FAM == 3 || FAM == 4) ? FKS_ROW_HEAVY_WAVES : FKS_ROW_WAVES)
void k_replay_rows_prof(fksk::BuiltinArgs a, int P, uint32_t* queue, uint32_t qbase) {
  replay_rows<FAM, RowProf>(a.W, kernarg_workload(), a.fam, a.weights, a.gheap, a.out, P, queue, qbase, a.prof,
                            RowNativeArgs{nullptr, nullptr, nullptr}, kRowsPerWave, a.table);
}
#endif


#if FKS_KIND == 4
// Scorer of natively compiled programs: one indirect call per node pass to the
// policy's JIT function (wave-uniform pointer -> a plain s_swappc).
struct NativeScorerDev {
  ProgFn fn;
  bool feas;             // the program opens with the feasibility prologue (jit_abi.h kFnFeasBit):
                         // called for feasible nodes only -- its JIT code may lack the prologue
  const int64_t* gmem;   // [node][kGmax] GPU memory MiB
  KcPtr kc;              // the policy's [budget, constants...], staged in LDS
  template <int NPASS, bool GP>
  __device__ int64_t score(int ps, const NodeRegs<NPASS, GP>& nr, const PodView& pod, int& exc) {
    if (feas && !feasible<NPASS, GP>(ps, nr, pod)) return 0;
    const int node = ps * kWave + lane_id();
    int32_t gl[kGmax], gt[kGmax];
#pragma unroll
    for (int g = 0; g < kGmax; ++g) {
      gl[g] = nr.g(ps, g);
      gt[g] = nr.gt(ps, g);
    }
    const int64_t r = fn(nr.cpu_left[ps], nr.ctot(ps), nr.mem_left[ps], nr.mtot(ps),
                         pack_gpu_ng(nr.gpu_left[ps], nr.ngp(ps)), gl[0], gl[1], gl[2], gl[3], gl[4], gl[5], gl[6], gl[7], gt[0], gt[1], gt[2], gt[3],
                         gt[4], gt[5], gt[6], gt[7], gmem + (size_t)node * kGmax, pod.cpu, pod.mem,
                         pod.gmilli | (pod.ngpu << 16), pod.ctime, pod.dur, kc);
    if (r < 0) { exc = (int)(-r); return 0; }
    return r;
  }
};

// Register floor: an address-taken function touching v127 / s101 raises this
// unit's amdgpu.max_num_vgpr / max_num_sgpr, and with them the allocation of
// every kernel here that makes an indirect call, to what JIT-compiled
// programs may use (kJitVgprs / kJitSgprs, checked by ops/jit.py).
__device__ __noinline__ int64_t fks_reg_floor(int64_t a) {
  asm volatile("" ::: "v127", "s101");
  return a;
}

// Runtime library of native programs (jit_abi.h rt_binop / rt_unop): the
// exact float //, %, **, math.log / exp / sqrt / pow of the device VM.
extern "C" __device__ __noinline__ Ret2 fks_rt_binop(int op, int64_t ab, int32_t afl, int64_t bb, int32_t bfl) {
  return d_binop_s(op, ab, afl, bb, bfl);
}
extern "C" __device__ __noinline__ Ret2 fks_rt_unop(int op, int64_t ab, int32_t afl) { return d_unop_s(op, ab, afl); }

__global__ void k_native_rt_table(uint64_t* out) {
  if (threadIdx.x == 0) {
    out[0] = (uint64_t)&fks_rt_binop;
    out[1] = (uint64_t)&fks_rt_unop;
    out[2] = (uint64_t)&fks_reg_floor;
    out[3] = 0;
  }
}

#if FKS_NPASS == 1
// Row kernel with natively compiled programs (replay_rows.hip.h, kFamNative):
// clusters of <= 16 nodes; `rows_active` rows per wave claim programs (1 for
// latency-bound LLM-sized batches, 4 for large ones).
__global__ __launch_bounds__(64, 1) void k_replay_rows_native(fksk::BuiltinArgs a, RowNativeArgs nat, int P,
                                                             uint32_t* queue, uint32_t qbase, int rows_active) {
  replay_rows<kFamNative>(a.W, kernarg_workload(), nullptr, nullptr, a.gheap, a.out, P, queue, qbase, nullptr, nat, rows_active,
                          a.table);
}
// s_memtime phase-profiled build (diagnostics): a.prof = [waves, 8] cycles
__global__ __launch_bounds__(64, 1) void k_replay_rows_native_prof(fksk::BuiltinArgs a, RowNativeArgs nat, int P,
                                                                  uint32_t* queue, uint32_t qbase, int rows_active) {
  replay_rows<kFamNative, RowProf>(a.W, kernarg_workload(), nullptr, nullptr, a.gheap, a.out, P, queue, qbase, a.prof, nat,
                                   rows_active, a.table);
}
// Two waves per program (wave 0: heap, wave 1: scoring; replay_duo.hip.h).
__global__ __launch_bounds__(128, 1) void k_replay_native_duo(fksk::BuiltinArgs a, RowNativeArgs nat) {
  replay_duo<false>(a.W, kernarg_workload(), a.gheap, a.out, nat, a.table);
}
// s_memtime-profiled build (diagnostics): a.prof = [blocks, 2 waves, 8] cycles
__global__ __launch_bounds__(128, 1) void k_replay_native_duo_prof(fksk::BuiltinArgs a, RowNativeArgs nat) {
  replay_duo<true>(a.W, kernarg_workload(), a.gheap, a.out, nat, a.table, a.prof);
}
// The resident program service (replay_duo.hip.h native_service): one workgroup
// per resident two-wave slot, programs from the host's ring until told to stop.
// ----------------------------------------------------------------------------
// k_native_service: a resident pool of two-wave workgroups that replays
// native programs from a ring the host keeps filling, one program after the
// other per workgroup -- a program's replay ends, its workgroup takes the next
// one.  A batch launch instead holds every one of its CU slots until its
// longest replay is done (the tail of a launch: ~40% mean occupancy on evolved
// programs, and one slow program pinned a 512-program slot in the steady loop).
//
// Host <-> device protocol (host memory: fine-grained, mapped; `claimed` in HBM):
//   the host writes program i into a free data slot s (fn, kc block, koff),
//   qslot[i % nq] = s, then publishes `published` = i + 1 (release); a
//   workgroup claims the next index from `claimed` (atomic), waits until it is
//   published, reads s, marks started[i % nq] = i + 1, replays slot s, writes
//   its result row and then done[s] = i + 1 (system-scope release).  The host
//   frees a slot when it consumed the row, and reuses a queue entry only once
//   it is marked started -- a straggler holds its slot, nothing else.
//   Exit: `stop` set and nothing left to claim, or `max_idle_polls` polls with
//   nothing published (a lost host: the whole grid drains instead of spinning
//   on; the host relaunches it from the lowest unstarted index).
//
// The replay is a call (service_replay, not inlined): inlined into the service
// loop, values of its prologue and epilogue were hoisted out of the loop and
// kept live across every event -- 144-156 VGPRs (6 workgroups per CU) against
// the 128 of k_replay_native_duo.  Called, it reads every argument from the
// kernarg segment afresh and the kernel holds the two-wave kernel's 8 per CU
// (a 224 B stack frame: the callee-saved registers, saved once per program).
constexpr uint32_t kServiceExit = 0xFFFFFFFFu;

// The kernarg segment pointer exists in the kernel only (a callee reading
// __builtin_amdgcn_kernarg_segment_ptr gets null): the kernel passes it down,
// the callees make it wave-uniform again (scalar loads of the arguments).
__device__ __forceinline__ const FKS_CONST fksk::ServiceArgs* service_args(uint64_t kp) {
  return (const FKS_CONST fksk::ServiceArgs*)uniu64(kp);
}

__device__ __forceinline__ void service_replay_body(uint64_t kp, int slot) {
  const FKS_CONST fksk::ServiceArgs* A = service_args(kp);
  const fksd::DevWorkload& W = *(const fksd::DevWorkload*)&A->a.W;
  const RowNativeArgs nat{A->nat.fn, A->nat.kc, A->nat.koff, A->nat.abort, A->nat.max_events};
  replay_duo<false>(W, (const fksd::DevWorkload*)uniu64(kp), A->a.gheap, A->a.out, nat, A->a.table, nullptr, slot,
                    (int)blockIdx.x);
}

// Claim the next index and wait until it is published.  Only the workgroups
// at the front (within kServiceFront of the HBM mirror of `published`) read
// the host's counter -- thousands of waiting workgroups polling host memory
// (one PCIe read each) starved the link and the replays' own host traffic --
// and advance the mirror; the rest poll the mirror (HBM, device scope),
// sleeping longer the further their index lies ahead.  Every index below the
// mirror is published, and the lowest unprocessed index is always claimed by
// a front workgroup (claims are handed out in order), so the mirror advances
// whenever the host publishes.  `stop` propagates the same way.
constexpr uint32_t kServiceFront = 2;

__device__ __noinline__ void service_replay(uint64_t kp, int slot) { service_replay_body(kp, slot); }

// The queued program's data slot (its index-queue entry, then marked started
// so the host may reuse the entry), or kServiceExit; an index a previous
// launch already started (a relaunch after an idle drain) is skipped.
__device__ __forceinline__ uint32_t service_entry(const FKS_CONST ServiceCtl& c, uint32_t idx, uint32_t* slot) {
  const uint32_t e = idx % c.nq;
  if (__hip_atomic_load(&c.started[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == idx + 1u) return 0u;
  *slot = __hip_atomic_load(&c.qslot[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&c.started[e], idx + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return 1u;
}

__device__ __noinline__ uint32_t service_claim(uint64_t kp, uint32_t* slot) {
  const FKS_CONST ServiceCtl& c = service_args(kp)->c;
  uint32_t* mirror = c.claimed + 32;   // HBM: published (lower bound), then stop
  uint32_t* stopd = c.claimed + 64;
  uint32_t idx = __hip_atomic_fetch_add(c.claimed, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint32_t polls = 0;
  for (;;) {
    uint32_t pub = __hip_atomic_load(mirror, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    if ((int32_t)(idx - pub) < 0) {   // published (wrap-safe)
      // (the mirror's acquire orders this after the host's queue writes: the
      // front workgroup that advanced it acquired them at system scope)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      if (service_entry(c, idx, slot)) return idx;
      idx = __hip_atomic_fetch_add(c.claimed, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      continue;
    }
    if (__hip_atomic_load(stopd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return kServiceExit;
    if (idx - pub < kServiceFront) {
      const uint32_t hp = __hip_atomic_load(c.published, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
      if ((int32_t)(hp - pub) > 0) {
        __hip_atomic_fetch_max(mirror, hp, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        continue;   // published now: take it through the path above
      }
      if (__hip_atomic_load(c.stop, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) {
        __hip_atomic_store(stopd, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return kServiceExit;
      }
    }
    const uint32_t d = idx - pub + 1u < 32u ? idx - pub + 1u : 32u;
    for (uint32_t z = d; z > 0; --z) __builtin_amdgcn_s_sleep(127);
    polls += d;
    if (polls > c.max_idle_polls) {
      // idle drain, all or nothing: every workgroup leaves (the stop mirror),
      // so the grid ends as a whole and the host's revive relaunches from the
      // lowest index no workgroup started -- an index claimed by a workgroup
      // that left while others stayed resident would never start
      __hip_atomic_store(stopd, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return kServiceExit;
    }
  }
}

__global__ __launch_bounds__(128, 1) void k_native_service(fksk::ServiceArgs) {
  __shared__ uint32_t claim[2];   // index, data slot
  __shared__ uint64_t t_start;    // s_memtime when the program was claimed
  for (;;) {
    uint64_t kp = (uint64_t)(uintptr_t)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(kp));   // re-derived per program, not held across the replay
    if (threadIdx.x == 0) {
      uint32_t slot = 0;
      claim[0] = service_claim(kp, &slot);
      claim[1] = slot;
      t_start = __builtin_amdgcn_s_memtime();
    }
    __syncthreads();
    const uint32_t idx = claim[0];
    if (idx == kServiceExit) return;   // (uniform across the workgroup)
    service_replay(kp, (int)claim[1]);
    if (threadIdx.x >= kWave) {
      const FKS_CONST ServiceCtl& c = service_args((uint64_t)(uintptr_t)__builtin_amdgcn_kernarg_segment_ptr())->c;
      if (threadIdx.x == kWave) {
        // the replay's device cost (the search's parent sampling and bloat
        // control read it; never the score), covered by the release below
        const uint64_t dt = __builtin_amdgcn_s_memtime() - t_start;
        __hip_atomic_store(&c.cost[claim[1]], dt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      // the scoring wave wrote the result row: make it visible to the host, then flag it
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      if (threadIdx.x == kWave)
        __hip_atomic_store(&c.done[claim[1]], claim[0] + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __syncthreads();   // both waves are done with the LDS (and with `claim`) before the next program
  }
}
// glibc-exact exp / log / pow (glibc_math.h) on device, one argument per lane:
// the device side of tests/test_gpu_glibc_math.py
__global__ __launch_bounds__(256) void k_gm_batch(int fn, const double* x, const double* y, double* out, int32_t* st,
                                                  int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double o = 0.0;
  int s = 0;
  if (fn == 0) s = gm::exp(x[i], o);
  else if (fn == 1) s = gm::log(x[i], o);
  else s = gm::pow(x[i], y[i], o);
  out[i] = o;
  st[i] = s;
}
#endif

template <int NPASS, bool GHEAP>
__global__ __launch_bounds__(64, GHEAP ? 2 : 1) void k_replay_native(fksk::NativeArgs a) {
  const int p = blockIdx.x;
  const Slot s = policy_slot<GHEAP>(a.W, a.gheap, p);
  NativeScorerDev sc;
  sc.fn = prog_of(uniu64(a.fn[p]));
  sc.feas = prog_feas(uniu64(a.fn[p]));
  sc.gmem = a.W.gmem_total;
  // the constant block moves into the slot's register area (the host reserves
  // kKcLds / 64 VM registers for it; the allocation is padded by kKcLds entries,
  // so the fixed-size copy never reads past it)
  const FKS_GLOBAL int64_t* ksrc = global_ptr(a.kc + a.koff[p]);
  FKS_LDS int64_t* kl = reinterpret_cast<FKS_LDS int64_t*>(lds_ptr(s.vregs));
  for (int i = lane_id(); i < kKcLds; i += kWave) kl[i] = ksrc[i];
  sc.kc = kl;
  replay_one<NPASS>(a.W, kernarg_workload(), sc, s.h, s.top, s.T, s.delmap, s.inv, a.out + p);
}
#endif

}  // namespace

namespace fksk {

#define FKS_CAT2(a, b) a##b
#define FKS_CAT(a, b) FKS_CAT2(a, b)

#if FKS_KIND == 0
hipError_t FKS_CAT(launch_builtin_np, FKS_NPASS)(bool gheap, int fam, int P, size_t lds, hipStream_t s, const BuiltinArgs& a) {
  return gheap ? launch_g<FKS_NPASS, true>(fam, P, lds, s, a) : launch_g<FKS_NPASS, false>(fam, P, lds, s, a);
}
hipError_t FKS_CAT(set_builtin_attrs_np, FKS_NPASS)(int mx) {
  hipError_t e = attrs_g<FKS_NPASS, true>(mx);
#if FKS_NPASS == 4
  if (e == hipSuccess) e = attrs_duo4(mx);
#endif
  return e != hipSuccess ? e : attrs_g<FKS_NPASS, false>(mx);
}
#if FKS_NPASS == 4
hipError_t launch_builtin_duo_np4(int fam, int P, size_t lds, hipStream_t s, const BuiltinArgs& a) {
  return launch_duo4(fam, P, lds, s, a);
}
#endif
#endif

#if FKS_KIND == 1
hipError_t FKS_CAT(launch_vm_np, FKS_NPASS)(bool gheap, int P, size_t lds, hipStream_t s, const VmArgs& a) {
  if (gheap) hipLaunchKernelGGL((k_replay_vm<FKS_NPASS, true>), dim3(P), dim3(64), lds, s, a);
  else hipLaunchKernelGGL((k_replay_vm<FKS_NPASS, false>), dim3(P), dim3(64), lds, s, a);
  return hipGetLastError();
}
hipError_t FKS_CAT(set_vm_attrs_np, FKS_NPASS)(int mx) {
  const hipError_t e = raise_lds(&k_replay_vm<FKS_NPASS, true>, mx);
  return e != hipSuccess ? e : raise_lds(&k_replay_vm<FKS_NPASS, false>, mx);
}
#endif

#if FKS_KIND == 2
hipError_t launch_builtin_prof(bool gheap, int P, size_t lds, hipStream_t s, const BuiltinArgs& a) {
  if (gheap) hipLaunchKernelGGL(k_replay_builtin_prof<true>, dim3(P), dim3(64), lds, s, a);
  else hipLaunchKernelGGL(k_replay_builtin_prof<false>, dim3(P), dim3(64), lds, s, a);
  return hipGetLastError();
}
hipError_t launch_c5_prof(int P, size_t lds, hipStream_t s, const BuiltinArgs& a) {
  hipLaunchKernelGGL(k_replay_c5_prof, dim3(P), dim3(64), lds, s, a);
  return hipGetLastError();
}
hipError_t launch_vm_prof(bool gheap, int P, size_t lds, hipStream_t s, const VmArgs& a) {
  if (gheap) hipLaunchKernelGGL(k_replay_vm_prof<true>, dim3(P), dim3(64), lds, s, a);
  else hipLaunchKernelGGL(k_replay_vm_prof<false>, dim3(P), dim3(64), lds, s, a);
  return hipGetLastError();
}
hipError_t set_prof_attrs(int mx) {
  hipError_t e = hipSuccess;
  for (hipError_t r : {raise_lds(&k_replay_builtin_prof<true>, mx), raise_lds(&k_replay_builtin_prof<false>, mx),
                       raise_lds(&k_replay_vm_prof<true>, mx), raise_lds(&k_replay_vm_prof<false>, mx),
                       raise_lds(&k_replay_c5_prof, mx)})
    if (r != hipSuccess) e = r;
  return e;
}
#endif


#if FKS_KIND == 3
hipError_t launch_builtin_rows(int fam, int P, int waves, uint32_t* queue, uint32_t qbase, size_t lds, hipStream_t st,
                              const BuiltinArgs& a) {
  const dim3 grid(waves);
#define FKS_CASE(F) \
  case F: hipLaunchKernelGGL((k_replay_rows<F>), grid, dim3(64), lds, st, a, P, queue, qbase); break;
  switch (fam) {
    FKS_CASE(FAM_FIRST_FIT)
    FKS_CASE(FAM_BEST_FIT)
    FKS_CASE(FAM_RANDOM_LINEAR)
    FKS_CASE(FAM_FEATURE_LINEAR)
    FKS_CASE(FAM_COMPOSITE_LINEAR)
    case kRowCompositeW5: hipLaunchKernelGGL(k_replay_rows_c5, grid, dim3(64), lds, st, a, P, queue, qbase); break;
    case kRowCompositeSplit: hipLaunchKernelGGL(k_replay_rows_split, grid, dim3(64), lds, st, a, P, queue, qbase); break;
    default: hipLaunchKernelGGL((k_replay_rows<-1>), grid, dim3(64), lds, st, a, P, queue, qbase);
  }
#undef FKS_CASE
  return hipGetLastError();
}
int rows_waves_per_cu(int fam, size_t lds) {
  int n = 0;
  hipError_t e;
  switch (fam) {
    case FAM_FIRST_FIT: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_replay_rows<FAM_FIRST_FIT>, 64, lds); break;
    case FAM_BEST_FIT: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_replay_rows<FAM_BEST_FIT>, 64, lds); break;
    case FAM_RANDOM_LINEAR:
      e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_replay_rows<FAM_RANDOM_LINEAR>, 64, lds); break;
    case FAM_FEATURE_LINEAR:
      e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_replay_rows<FAM_FEATURE_LINEAR>, 64, lds); break;
    case FAM_COMPOSITE_LINEAR:
      e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_replay_rows<FAM_COMPOSITE_LINEAR>, 64, lds); break;
    case kRowCompositeW5: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_replay_rows_c5, 64, lds); break;
    case kRowCompositeSplit: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_replay_rows_split, 64, lds); break;
    default: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_replay_rows<-1>, 64, lds);
  }
  return e == hipSuccess ? n : -1;
}
hipError_t launch_builtin_rows_prof(int fam, int P, int waves, uint32_t* queue, uint32_t qbase, size_t lds, hipStream_t st,
                                   const BuiltinArgs& a) {
  const dim3 grid(waves);
  if (fam == FAM_RANDOM_LINEAR) hipLaunchKernelGGL((k_replay_rows_prof<FAM_RANDOM_LINEAR>), grid, dim3(64), lds, st, a, P, queue, qbase);
  else if (fam == FAM_COMPOSITE_LINEAR || fam == kRowCompositeW5 || fam == kRowCompositeSplit)
    hipLaunchKernelGGL((k_replay_rows_prof<FAM_COMPOSITE_LINEAR>), grid, dim3(64), lds, st, a, P, queue, qbase);
  else hipLaunchKernelGGL((k_replay_rows_prof<-1>), grid, dim3(64), lds, st, a, P, queue, qbase);
  return hipGetLastError();
}
hipError_t set_rows_attrs(int mx) {
  hipError_t e = hipSuccess;
  for (hipError_t r : {raise_lds(&k_replay_rows_prof<-1>, mx), raise_lds(&k_replay_rows_prof<FAM_RANDOM_LINEAR>, mx),
                       raise_lds(&k_replay_rows_prof<FAM_COMPOSITE_LINEAR>, mx)})
    if (r != hipSuccess) e = r;
  for (hipError_t r : {raise_lds(&k_replay_rows<-1>, mx), raise_lds(&k_replay_rows<FAM_FIRST_FIT>, mx),
                       raise_lds(&k_replay_rows<FAM_BEST_FIT>, mx), raise_lds(&k_replay_rows<FAM_RANDOM_LINEAR>, mx),
                       raise_lds(&k_replay_rows<FAM_FEATURE_LINEAR>, mx),
                       raise_lds(&k_replay_rows<FAM_COMPOSITE_LINEAR>, mx), raise_lds(&k_replay_rows_c5, mx),
                       raise_lds(&k_replay_rows_split, mx)})
    if (r != hipSuccess) e = r;
  return e;
}
#endif


#if FKS_KIND == 4
hipError_t FKS_CAT(launch_native_np, FKS_NPASS)(bool gheap, int P, size_t lds, hipStream_t s, const NativeArgs& a) {
  if (gheap) hipLaunchKernelGGL((k_replay_native<FKS_NPASS, true>), dim3(P), dim3(64), lds, s, a);
  else hipLaunchKernelGGL((k_replay_native<FKS_NPASS, false>), dim3(P), dim3(64), lds, s, a);
  return hipGetLastError();
}
hipError_t FKS_CAT(set_native_attrs_np, FKS_NPASS)(int mx) {
  const hipError_t e = raise_lds(&k_replay_native<FKS_NPASS, true>, mx);
  return e != hipSuccess ? e : raise_lds(&k_replay_native<FKS_NPASS, false>, mx);
}
#if FKS_NPASS == 1
hipError_t launch_native_rows(int P, int waves, int rows_active, uint32_t* queue, uint32_t qbase, size_t lds,
                              hipStream_t st, const BuiltinArgs& a, const fksd::RowNativeArgs& nat) {
  if (a.prof) hipLaunchKernelGGL(k_replay_rows_native_prof, dim3(waves), dim3(64), lds, st, a, nat, P, queue, qbase, rows_active);
  else hipLaunchKernelGGL(k_replay_rows_native, dim3(waves), dim3(64), lds, st, a, nat, P, queue, qbase, rows_active);
  return hipGetLastError();
}
hipError_t set_native_rows_attrs(int mx) {
  const hipError_t e = raise_lds(&k_replay_rows_native, mx);
  return e != hipSuccess ? e : raise_lds(&k_replay_rows_native_prof, mx);
}
hipError_t launch_native_duo(int P, size_t lds, hipStream_t st, const BuiltinArgs& a, const fksd::RowNativeArgs& nat) {
  if (a.prof) hipLaunchKernelGGL(k_replay_native_duo_prof, dim3(P), dim3(128), lds, st, a, nat);
  else hipLaunchKernelGGL(k_replay_native_duo, dim3(P), dim3(128), lds, st, a, nat);
  return hipGetLastError();
}
hipError_t set_native_duo_attrs(int mx) {
  const hipError_t e = raise_lds(&k_replay_native_duo, mx);
  return e != hipSuccess ? e : raise_lds(&k_replay_native_duo_prof, mx);
}
hipError_t launch_native_service(int blocks, size_t lds, hipStream_t st, const ServiceArgs& s) {
  hipLaunchKernelGGL(k_native_service, dim3(blocks), dim3(128), lds, st, s);
  return hipGetLastError();
}
// (the kernel's static LDS -- the claim word -- counts against the 160 KiB too)
hipError_t set_native_service_attrs(int mx) { return raise_lds(&k_native_service, mx - 64); }
int native_service_blocks_per_cu(size_t lds) {
  int n = 0;
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_native_service, 128, lds) == hipSuccess ? n : -1;
}
int native_duo_blocks_per_cu(size_t lds) {
  int n = 0;
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_replay_native_duo, 128, lds) == hipSuccess ? n : -1;
}
int native_rows_waves_per_cu(size_t lds) {
  int n = 0;
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_replay_rows_native, 64, lds) == hipSuccess ? n : -1;
}
hipError_t native_rt_table(uint64_t* dev_out, hipStream_t s) {
  hipLaunchKernelGGL(k_native_rt_table, dim3(1), dim3(64), 0, s, dev_out);
  return hipGetLastError();
}
hipError_t launch_gm_batch(int fn, const double* x, const double* y, double* out, int32_t* st, int64_t n) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_gm_batch, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, fn, x, y, out, st, n);
  return hipGetLastError();
}
#endif
#endif

}  // namespace fksk
