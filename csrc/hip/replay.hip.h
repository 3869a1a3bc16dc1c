// k_replay: batched exact replay of the OpenB event trace on MI355X.
//
// One workgroup = one wave64 = one candidate policy.  Per policy:
//   * the event heap lives in LDS as packed u64 keys
//       key = time << (RB+LB) | rank << LB | gpu_mask << (2+NB) | node << 2 | kind
//     compared on (key >> LB) = (time, pod rank): exactly the reference's
//     (time, pod_id) tuple order (simulator/event_simulator.py:16-17), and
//     manipulated with CPython's heapq algorithms -- wave-parallel, see
//     heap_wave.h -- so the array layout, which the repush rule observes, is
//     bit-identical to the reference's;
//   * lanes = nodes (64 x NPASS nodes); each lane keeps its node's cpu / mem /
//     GPU-count / per-GPU-milli state in VGPRs, so scoring, the placement
//     argmax (DPP wave max + ballot/ffs for the first-node tie-break),
//     best-fit GPU selection, fragmentation sums and active-node counts are
//     register-only;
//   * the waiting-pod multiset needed by the fragmentation metric is a
//     per-lane histogram over the distinct gpu_milli classes, its minimum a
//     ballot; membership is carried by the heap entry itself (kind 1 =
//     re-queued creation = the pod is waiting);
//   * snapshot triggers come from a host-precomputed schedule (the same IEEE
//     `processed / total >= threshold`, `threshold += 0.05` sequence), and the
//     evaluator's means are accumulated in exact 128-bit fixed point and
//     finished by k_eval_reduce.
// LDS per policy: heap (N padded to 64) | deletion bitmap | [VM registers].
// The scorer (built-in families, or the bytecode VM) is a template argument.
#pragma once

#include "device_common.h"
#include "exc_codes.h"
#include "heap_wave.h"

namespace fksd {

constexpr int kGmax = 8;        // GPUs per node held in registers
constexpr int kFresh = 0, kRetry = 1, kDelete = 2;


struct DevWorkload {
  int32_t n_nodes, n_pods, n_classes, n_fire;
  const int32_t* cpu_total;   // [64*NPASS]
  const int32_t* cpu_left0;
  const int32_t* mem_total;
  const int32_t* mem_left0;
  const int32_t* gpu_left0;
  const int32_t* ngpus;
  const int32_t* gml_total;   // [node][kGmax]
  const int32_t* gml_left0;   // [node][kGmax]
  const int64_t* gmem_total;  // [node][kGmax] (GPU memory MiB, read-only field)
  const int4* pod;            // by rank: {cpu, mem, dur, gmilli | ngpu<<16 | cls<<24}
  const int32_t* pod_ctime;   // by rank: original creation time
  const uint64_t* heap0;      // initial heapified keys
  const int32_t* class_value; // ascending distinct gpu_milli of GPU pods
  const int64_t* snap_fire;   // processed-event counts that trigger snapshots 0..n_fire-1
  int64_t tot_cpu, tot_mem, tot_gcnt, tot_gmilli;
  int64_t used_cpu0, used_mem0, used_gcnt0, used_gmilli0;
  int32_t rank_bits, node_bits, low_bits, time_bits;
  double snapshot_interval;
  double thr_after_fire;      // threshold value after the last precomputed snapshot
  int32_t repush_earliest, first_fit_alloc, truncate;
  int32_t heap_top;           // heap slots kept in LDS when the heap lives in HBM
  int32_t check_every;        // k_check_invariants cadence in events (0: off)
  int32_t inv_words;          // LDS u64 words reserved for the invariant check (0: off)
  int32_t trace_hash;         // 1: fold every event into DevResult.hash (cross-engine trace check)
  const uint64_t* heap0p;     // initial heap shifted by one slot (row kernel layout: address = slot + 1)
  const int4* node_c4;        // [64*NPASS] {cpu_total, mem_total, ngpus, gml_total of GPU 0} per node slot
  int32_t delmap_slots;       // wave kernels: heap slots the LDS deletion bitmap covers (WaveHeapT::M)
  // Row-kernel composite scorer (scorers.hip.h composite_row): host-verified
  // reciprocals RN(1/d) of the node-constant divisors max(cpu_total, 1),
  // max(mem_total, 1), max(ngpus, 1) ([node][3]) and of 1000 (z1000), valid
  // for every numerator a replay can form (fast_div = 1 iff all verified),
  // and pod.cpu / max(pod.mem, 1) by rank.
  const double* node_recip;
  const double* pod_cm;
  double z1000;
  int32_t fast_div;
  // composite GPU utilisation: every GPU node has per-GPU milli total
  // cap_milli; cap_recip[k] = RN(1 / max(k * cap_milli, 1)), k = 0..8,
  // verified on |numerators| <= 8 * cap_milli (all 0 when not uniform)
  int32_t cap_milli;
  double cap_recip[kGmax + 1];
  // fragmentation: RN(1 / tot_gmilli) verified on [0, tot_gmilli] (0: divide)
  double z_tg;
  double tot_gmilli_d;        // (double)tot_gmilli
};

// RN(n / d) from z = RN(1/d) with one remainder step (Markstein): exact for
// the numerators the host checked (fks_recip_verified), not in general.
__host__ __device__ __forceinline__ double div_by_recip(double n, double d, double z) {
  const double q = n * z;
  const double r = __builtin_fma(-q, d, n);
  return __builtin_fma(r, z, q);
}

struct DevResult {
  int64_t n_events, n_snap, n_frag, n_unplaced, n_repush, max_nodes;
  uint64_t hash;
  int32_t exc, inexact;
  uint64_t acc_lo[5];
  uint64_t acc_hi[5];
};

// LDS layout helpers (in u64 units)
__host__ __device__ inline int lds_heap_entries(int n_pods) { return (n_pods + 63) & ~63; }
__host__ __device__ inline int lds_delmap_words(int n_pods) { return (((n_pods + 31) >> 5) + 63) & ~63; }
__host__ __device__ inline int lds_vreg_offset(int n_pods) {
  return lds_heap_entries(n_pods) + lds_delmap_words(n_pods) / 2;
}

// Per-lane view of node state handed to a scorer.  A node's GPUs are one
// model (one CSV row per node in the trace format), so their milli totals are
// one value per node (`gmt1`; the host checks it): 1 register per node slot
// instead of kGmax -- 28 VGPRs on 256-node clusters, the difference between 2
// and 3 waves per SIMD there.  gt(ps, j) is the per-GPU view (0 past ngpus,
// like the zero padding of the host table).
// GP (on 256-node clusters, NPASS = 4, and in the row kernels) packs the
// per-GPU milli left of two GPUs into one register (16-bit halves; the host
// refuses GPU milli totals >= 2^16 there): 16 VGPRs instead of 32 for the four
// node slots, 4 instead of 8 per row lane.  Updates are plain 32-bit adds of
// the shifted delta -- a GPU never holds less than it gives back or more than
// its total, so a half never borrows from or carries into the other.
template <int NPASS, bool GP = (NPASS >= 4)>
struct NodeRegs {
  static constexpr bool kPack = GP;
  static constexpr bool kCst = NPASS >= 4;   // node constants re-read from `cst`
  static constexpr int kGW = kPack ? kGmax / 2 : kGmax;
  int32_t cpu_left[NPASS], mem_left[NPASS], gpu_left[NPASS];
  int32_t gw[NPASS][kGW];
  // node constants: registers, or (kCst) re-read from the workload's int4
  // table {cpu_total, mem_total, ngpus, gmt1} where used -- 16 VGPRs less
  // through the pop / push phases, which need none of them
  static constexpr int kCR = kCst ? 1 : NPASS;
  int32_t cpu_total[kCR], mem_total[kCR], ngpus[kCR], gmt1[kCR];
  const int4* cst;   // kCst: DevWorkload::node_c4, [slot * 64 + lane]
  __device__ __forceinline__ int4 c4(int ps) const { return cst[ps * kWave + lane_id()]; }
  __device__ __forceinline__ int32_t ctot(int ps) const { if constexpr (kCst) return c4(ps).x; else return cpu_total[ps]; }
  __device__ __forceinline__ int32_t mtot(int ps) const { if constexpr (kCst) return c4(ps).y; else return mem_total[ps]; }
  __device__ __forceinline__ int32_t ngp(int ps) const { if constexpr (kCst) return c4(ps).z; else return ngpus[ps]; }
  __device__ __forceinline__ int32_t gmt(int ps) const { if constexpr (kCst) return c4(ps).w; else return gmt1[ps]; }
  __device__ __forceinline__ int32_t gt(int ps, int j) const { return j < ngp(ps) ? gmt(ps) : 0; }
  // GPU j's milli left on node slot ps
  __device__ __forceinline__ int32_t g(int ps, int j) const {
    if constexpr (kPack) return (int32_t)(((uint32_t)gw[ps][j >> 1] >> ((j & 1) * 16)) & 0xFFFFu);
    else return gw[ps][j];
  }
  __device__ __forceinline__ void g_add(int ps, int j, int32_t d) {
    if constexpr (kPack) gw[ps][j >> 1] += (int32_t)((uint32_t)d << ((j & 1) * 16));
    else gw[ps][j] += d;
  }
  __device__ __forceinline__ void g_init(int ps, int j, int32_t v) {
    if constexpr (kPack) {
      if (j & 1) gw[ps][j >> 1] |= (int32_t)((uint32_t)v << 16);
      else gw[ps][j >> 1] = v;
    } else {
      gw[ps][j] = v;
    }
  }
};

struct PodView {
  int32_t cpu, mem, dur, gmilli, ngpu, cls;
  int64_t ctime;  // current creation time (event time)
  int32_t rank;
  double cm;      // cpu / max(mem, 1) (DevWorkload::pod_cm; set where a scorer reads it)
};

// the scorers' feasibility test (scorers.hip.h), used by the diagnostics build
template <int NPASS, bool GP>
__device__ __forceinline__ bool feasible(int ps, const NodeRegs<NPASS, GP>& nr, const PodView& pod);

// Scorer contract:  score<NPASS>(pass, node_regs, pod, exc) -> int64 priority
// after int(max(0, s)) truncation (>= 0), exceptions reported through `exc`.

// ----------------------------------------------------------------------------
// Phase profiler (s_memtime deltas; compiled out with NoProf).
struct NoProf {
  static constexpr bool kOn = false;
  __device__ void start() {}
  __device__ void mark(int) {}
  __device__ void count(int, uint64_t) {}
  __device__ void flush(uint64_t*) {}
};
struct PhaseProf {
  static constexpr bool kOn = true;
  uint64_t acc[8];
  uint64_t last;
  // acc[6] / acc[7]: counters, not cycles (feasible node slots / creation events)
  __device__ void count(int k, uint64_t v) { acc[k] += v; }
  __device__ void start() {
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0;
    last = __builtin_amdgcn_s_memtime();
  }
  __device__ void mark(int ph) {
    const uint64_t now = __builtin_amdgcn_s_memtime();
    acc[ph] += now - last;
    last = now;
  }
  __device__ void flush(uint64_t* o) {
    if (lane_id() == 0)
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = acc[k];
  }
};
enum Phase { PH_POP = 0, PH_DELETE = 1, PH_SCORE = 2, PH_FAIL = 3, PH_COMMIT = 4, PH_EVAL = 5 };

// GPU pick on one node (lane-local): mask of the `need` tightest-fitting
// eligible GPUs (stable: ties by index) or the first `need` eligible GPUs.
template <int NPASS, bool GP>
__device__ __forceinline__ int pick_gpus(const NodeRegs<NPASS, GP>& nr, int ps, int gm, int need, bool first_fit,
                                         int& ok) {
  const int ng = nr.ngp(ps);
  int cnt = 0;
#pragma unroll
  for (int j = 0; j < kGmax; ++j) cnt += (j < ng && nr.g(ps, j) >= gm);
  ok = cnt >= need;
  int mask = 0;
  if (need == 1 && !first_fit) {
    int best = -1, bv = 0;
#pragma unroll
    for (int j = 0; j < kGmax; ++j) {
      const int l = nr.g(ps, j);
      if (j < ng && l >= gm && (best < 0 || l < bv)) { best = j; bv = l; }
    }
    mask = best >= 0 ? (1 << best) : 0;
    return mask;
  }
#pragma unroll
  for (int j = 0; j < kGmax; ++j) {
    const bool vj = j < ng && nr.g(ps, j) >= gm;
    int r = 0;
#pragma unroll
    for (int i = 0; i < kGmax; ++i) {
      const bool vi = i < ng && nr.g(ps, i) >= gm;
      r += first_fit ? (vi && i < j)
                     : (vi && (nr.g(ps, i) < nr.g(ps, j) || (nr.g(ps, i) == nr.g(ps, j) && i < j)));
    }
    if (vj && r < need) mask |= 1 << j;
  }
  return mask;
}

// ----------------------------------------------------------------------------
// Debug check (the reference's `_validate_cluster_invariants`,
// simulator/main.py:201-272): every node's / GPU's remaining capacity lies in
// [0, total] and equals total minus what the pods with a pending DELETION in
// the heap hold.  Per-node "used" sums are built with LDS atomics from the
// heap's deletion keys (node, GPU mask and pod rank are packed in the key).
constexpr int kInvCols = 3 + kGmax;   // cpu, mem, gpu count, per-GPU milli
__host__ __device__ inline int inv_words_for(int npass) { return (kWave * npass * kInvCols * 4 + 7) / 8; }

template <int NPASS, class Heap, bool GP>
__device__ bool invariants_hold(const DevWorkload& W, const Heap& heap, int n, const NodeRegs<NPASS, GP>& nr,
                                FKS_LDS int32_t* inv, int lane) {
  for (int i = lane; i < kWave * NPASS * kInvCols; i += kWave) inv[i] = 0;
  __syncthreads();
  const int lb = W.low_bits, nb = W.node_bits, rb = W.rank_bits;
  for (int i = lane; i < n; i += kWave) {
    const uint64_t k = heap.ld(i);
    if ((int)(k & 3) != kDelete) continue;
    const int node = (int)((k >> 2) & ((1u << nb) - 1));
    const int mask = (int)((k >> (2 + nb)) & 0xFF);
    const int rank = (int)((k >> lb) & ((1ull << rb) - 1));
    const int4 pr = W.pod[rank];
    FKS_LDS int32_t* row = inv + node * kInvCols;
    __hip_atomic_fetch_add(&row[0], pr.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_add(&row[1], pr.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_add(&row[2], (pr.w >> 16) & 0xFF, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
    for (int j = 0; j < kGmax; ++j)
      if ((mask >> j) & 1) __hip_atomic_fetch_add(&row[3 + j], pr.w & 0xFFFF, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __syncthreads();
  bool bad = false;
#pragma unroll
  for (int ps = 0; ps < NPASS; ++ps) {
    const int node = ps * kWave + lane;
    if (node >= W.n_nodes) continue;
    const FKS_LDS int32_t* row = inv + node * kInvCols;
    const int32_t cl = nr.cpu_left[ps], ml = nr.mem_left[ps], gl = nr.gpu_left[ps];
    bad |= cl < 0 || cl > nr.ctot(ps) || row[0] + cl != nr.ctot(ps);
    bad |= ml < 0 || ml > nr.mtot(ps) || row[1] + ml != nr.mtot(ps);
    bad |= gl < 0 || gl > nr.ngp(ps) || row[2] + gl != nr.ngp(ps);
#pragma unroll
    for (int j = 0; j < kGmax; ++j)
      if (j < nr.ngp(ps)) {
        const int32_t l = nr.g(ps, j), t = nr.gt(ps, j);
        bad |= l < 0 || l > t || row[3 + j] + l != t;
      }
  }
  __syncthreads();
  return ballot(bad) == 0;
}

// ----------------------------------------------------------------------------
template <int NPASS, class Scorer, class Prof = NoProf, bool FLAT = false>
__device__ void replay_one(const DevWorkload& W, const DevWorkload* Wcold, Scorer& scorer, FKS_GLOBAL uint64_t* hbuf,
                           FKS_LDS uint64_t* htop, int T, FKS_LDS uint32_t* delmap, FKS_LDS int32_t* inv,
                           DevResult* out,
                           uint64_t* prof_out = nullptr) {
  // W: the kernel-argument copy (hot fields, kept in SGPRs); Wcold: the same
  // struct in global memory for the fields only snapshots / failures / commits
  // of multi-GPU pods need.  Its address is made opaque once per event so the
  // compiler re-loads those fields (scalar-cache hits) where they are used
  // instead of pinning ~30 SGPRs for the whole loop and spilling them.
  // hbuf: the policy's heap array -- LDS (fast, 2 policies/CU on the 8k trace)
  // or its private slice of an HBM buffer (any trace length, 16 policies/CU);
  // slots [0, T) are held in LDS at htop instead (T >= N: all of it)
  Prof prof;
  const int lane = lane_id();
  const int lb = W.low_bits, nb = W.node_bits;
  const int rb = W.rank_bits;
  const int tshift = rb + lb;
  const uint64_t time_max = (W.time_bits >= 63) ? ~0ull : ((1ull << W.time_bits) - 1);
  const int N = W.n_pods;

  WaveHeapT<FLAT> heap;
  heap.h = hbuf;
  heap.top = htop;
  heap.bind();
  heap.T = T;
  heap.delmap = delmap;
  heap.M = W.delmap_slots;
  heap.lb = lb;
  for (int i = lane; i < N; i += kWave) heap.st(i, W.heap0[i]);
  for (int i = lane; i < (W.delmap_slots >> 5); i += kWave) heap.delmap[i] = 0u;

  NodeRegs<NPASS> nr;
  nr.cst = W.node_c4;
#pragma unroll
  for (int ps = 0; ps < NPASS; ++ps) {
    const int node = ps * kWave + lane;
    nr.cpu_left[ps] = W.cpu_left0[node];
    nr.mem_left[ps] = W.mem_left0[node];
    nr.gpu_left[ps] = W.gpu_left0[node];
    if constexpr (!NodeRegs<NPASS>::kCst) {
      nr.cpu_total[ps] = W.cpu_total[node];
      nr.mem_total[ps] = W.mem_total[node];
      nr.ngpus[ps] = W.ngpus[node];
      nr.gmt1[ps] = W.gml_total[node * kGmax];
    }
#pragma unroll
    for (int j = 0; j < kGmax; ++j) nr.g_init(ps, j, W.gml_left0[node * kGmax + j]);
  }
  // waiting histogram over gpu_milli classes: class k -> lane k%64, slot k/64
  constexpr int KP = 4;  // up to 256 classes
  int32_t wcnt[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) wcnt[k] = 0;

  int64_t used_cpu = W.used_cpu0, used_mem = W.used_mem0, used_gcnt = W.used_gcnt0, used_gml = W.used_gmilli0;
  LaneAcc acc;   // accumulators 0-3: utilisation snapshots, 4: fragmentation
  acc.init();
  int64_t processed = 0, n_repush = 0, n_dropped = 0;
  int ksnap = 0;
  const int n_fire = W.n_fire;
  int64_t next_fire = n_fire > 0 ? W.snap_fire[0] : INT64_MAX;
  double thr = W.thr_after_fire;   // used once the precomputed schedule is exhausted
  uint64_t hsh = 0xcbf29ce484222325ull;
  int32_t exc = EXC_NONE;
  int n = N;
  __syncthreads();
  prof.start();

  heap.lane = lane;
  while (n > 0) {
    const DevWorkload* Wg = reinterpret_cast<const DevWorkload*>(uniu64(reinterpret_cast<uint64_t>(Wcold)));
    asm volatile("" : "+s"(Wg));
    const FKS_CONST DevWorkload* Wc = const_ptr(Wg);   // scalar loads (read-only during the launch)
    // Lane-derived predicates (subtree slots of the heap walk, "GPU j exists")
    // are loop-invariant; hoisted they become dozens of live 64-bit lane masks
    // in SGPRs that get spilled every event.  Opaque copies are recomputed per
    // event with a few VALU compares instead.
    {
      int ol = lane;
      asm volatile("" : "+v"(ol));
      heap.lane = ol;
      if constexpr (!NodeRegs<NPASS>::kCst) {
#pragma unroll
        for (int ps = 0; ps < NPASS; ++ps) asm volatile("" : "+v"(nr.ngpus[ps]));
      } else {
        // re-derived per event (uniform, opaque): the constant loads are not hoisted out of the loop
        const int4* c = reinterpret_cast<const int4*>(uniu64(reinterpret_cast<uint64_t>(nr.cst)));
        asm volatile("" : "+s"(c));
        nr.cst = c;
      }
    }
    // ---------------- pop (pod record load issued first, consumed after the sift)
    const uint64_t top = uniu64(heap.ld_u(0));
    const int rank = (int)((top >> lb) & ((1ull << rb) - 1));
    const int4 precv = load_vgpr(&W.pod[rank]);
    const uint64_t last = uniu64(heap.ld_u(n - 1));
    --n;
    if (n > 0) heap.pop_reinsert(n, last);

    const int kind = (int)(top & 3);
    const int64_t t = (int64_t)(top >> tshift);
    PodView pod;
    const int pw = uni(precv.w);
    pod.cpu = uni(precv.x); pod.mem = uni(precv.y); pod.dur = uni(precv.z);
    pod.gmilli = pw & 0xFFFF; pod.ngpu = (pw >> 16) & 0xFF; pod.cls = (pw >> 24) & 0xFF;
    pod.ctime = t; pod.rank = rank;
    pod.cm = W.pod_cm[rank];   // scalar load (dropped by the compiler where no scorer reads it)
    prof.mark(PH_POP);

    if (kind == kDelete) {
      const int node = (int)((top >> 2) & ((1u << nb) - 1));
      const int mask = (int)((top >> (2 + nb)) & 0xFF);
#pragma unroll
      for (int ps = 0; ps < NPASS; ++ps) {
        if (ps * kWave + lane == node) {
          nr.cpu_left[ps] += pod.cpu;
          nr.mem_left[ps] += pod.mem;
          nr.gpu_left[ps] += pod.ngpu;
#pragma unroll
          for (int j = 0; j < kGmax; ++j)
            if ((mask >> j) & 1) nr.g_add(ps, j, pod.gmilli);
        }
      }
      used_cpu -= pod.cpu; used_mem -= pod.mem; used_gcnt -= pod.ngpu;
      used_gml -= (int64_t)pod.gmilli * __builtin_popcount(mask);
      if (W.trace_hash) hsh = mix_event(hsh, ((uint64_t)(uint32_t)rank << 2) | 1, (uint64_t)t);
      prof.mark(PH_DELETE);
    } else {
      // ---------------- creation: score all nodes, argmax (first node wins ties)
      // Each lane keeps the best of its node slots (strict >: the lowest slot
      // wins ties) and its first exception; ONE wave max per event then finds
      // the winning score, and the lowest node index holding it is the lowest
      // slot whose ballot hits -- the same node as a pass-by-pass argmax, with
      // NPASS - 1 fewer DPP reductions.  A score of 0 never places.
      if constexpr (Prof::kOn) {   // how many node slots the scorer finds feasible (diagnostics build)
        uint64_t nf = 0;
#pragma unroll
        for (int ps = 0; ps < NPASS; ++ps)
          nf += __popcll(ballot((ps * kWave + lane) < W.n_nodes && feasible<NPASS>(ps, nr, pod)));
        prof.count(6, nf);
        prof.count(7, 1);
        prof.mark(PH_POP);   // (the count's own cycles go to the pop phase)
      }
      uint64_t lbest = 0;
      // packed per-lane state (one VGPR): bits 0-1 slot of lbest, bits 2-3
      // slot of the first exception, bits 8+ its code (EXC_NONE = 0)
      int lst = 0;
#pragma unroll
      for (int ps = 0; ps < NPASS; ++ps) {
        const bool valid = (ps * kWave + lane) < W.n_nodes;
        int lexc = EXC_NONE;
        const uint64_t s = valid ? (uint64_t)scorer.template score<NPASS>(ps, nr, pod, lexc) : 0;   // >= 0
        if (valid && lexc != EXC_NONE && (lst >> 8) == 0) lst |= (lexc << 8) | (ps << 2);
        if (s > lbest) { lbest = s; lst = (lst & ~3) | ps; }
      }
      if (ballot((lst >> 8) != 0)) {
        // the first raising node in node order (slot-major, then lane); the
        // slots after an exception were scored too, which has no side effects
#pragma unroll
        for (int ps = 0; ps < NPASS; ++ps) {
          const uint64_t b = ballot((lst >> 8) != 0 && ((lst >> 2) & 3) == ps);
          if (b) { exc = readlane(lst >> 8, first_lane(b)); break; }
        }
        break;
      }
      int best_node = -1;
      const uint64_t m = wave_max_u64(lbest);
      if (m > 0) {
#pragma unroll
        for (int ps = NPASS - 1; ps >= 0; --ps) {
          const uint64_t b = ballot(lbest == m && (lst & 3) == ps);
          if (b) best_node = ps * kWave + first_lane(b);
        }
      }
      prof.mark(PH_SCORE);

      if (best_node < 0) {
        // ---------------- failed placement
        if (kind == kFresh && pod.ngpu > 0) {
#pragma unroll
          for (int k = 0; k < KP; ++k)
            if (k * kWave + lane == pod.cls) wcnt[k] += 1;
        }
        // fragmentation: min gpu_milli over waiting GPU pods, stranded milli below it
        double frag = 0.0;
        int mcls = -1;
#pragma unroll
        for (int k = 0; k < KP; ++k) {
          const uint64_t b = ballot(wcnt[k] > 0);
          if (mcls < 0 && b) mcls = k * kWave + first_lane(b);
        }
        if (mcls >= 0) {
          const int m = const_ptr(Wc->class_value)[mcls];
          int64_t stranded = 0;
#pragma unroll
          for (int ps = 0; ps < NPASS; ++ps)
#pragma unroll
            for (int j = 0; j < kGmax; ++j) {
              const int l = nr.g(ps, j);
              if (j < nr.ngp(ps) && 0 < l && l < m) stranded += l;
            }
          stranded = wave_sum_i64(stranded);
          const int64_t tg = Wc->tot_gmilli;
          frag = tg > 0 ? (double)stranded / (double)tg : 0.0;
        }
        acc.add(4, frag);
        // repush: first DELETION in heap-array order (or the earliest one)
        int64_t anchor = -1;
        if (!Wc->repush_earliest) {
          const int f = heap.first_deletion(n);
          if (f >= 0) anchor = (int64_t)(uniu64(heap.ld(f)) >> tshift);
        } else {
          uint64_t mn = ~0ull;
          for (int base = 0; base < n; base += kWave) {
            const int i = base + lane;
            uint64_t tv = ~0ull;
            if (i < n) { const uint64_t k = heap.ld(i); if ((k & 3) == kDelete) tv = k >> tshift; }
            tv = ~wave_max_u64(~tv);
            mn = tv < mn ? tv : mn;
          }
          anchor = mn == ~0ull ? -1 : (int64_t)mn;
        }
        if (anchor >= 0) {
          const uint64_t nt = (uint64_t)(anchor + 1);
          if (nt > time_max) { exc = EXC_UNSUPPORTED; break; }
          heap.push(n, (nt << tshift) | ((uint64_t)rank << lb) | kRetry);
          ++n;
          ++n_repush;
        } else {
          ++n_dropped;
        }
        if (W.trace_hash) hsh = mix_event(hsh, ((uint64_t)(uint32_t)rank << 2) | 2, (uint64_t)t);
        prof.mark(PH_FAIL);
      } else {
        // ---------------- commit on best_node
        const int bp = best_node / kWave, bl = best_node % kWave;
        int gmask = 0;
        int ok = 1;
        if (pod.ngpu > 0) {
          int mymask = 0, myok = 1;
#pragma unroll
          for (int ps = 0; ps < NPASS; ++ps)
            if (ps == bp) mymask = pick_gpus<NPASS>(nr, ps, pod.gmilli, pod.ngpu, Wc->first_fit_alloc != 0, myok);
          gmask = readlane(mymask, bl);
          ok = readlane(myok, bl);
        }
        if (!ok) { exc = EXC_ALLOC; break; }
#pragma unroll
        for (int ps = 0; ps < NPASS; ++ps) {
          if (ps == bp && lane == bl) {
            nr.cpu_left[ps] -= pod.cpu;
            nr.mem_left[ps] -= pod.mem;
            nr.gpu_left[ps] -= pod.ngpu;
#pragma unroll
            for (int j = 0; j < kGmax; ++j)
              if ((gmask >> j) & 1) nr.g_add(ps, j, -pod.gmilli);
          }
        }
        used_cpu += pod.cpu; used_mem += pod.mem; used_gcnt += pod.ngpu;
        used_gml += (int64_t)pod.gmilli * __builtin_popcount(gmask);
        if (kind == kRetry && pod.ngpu > 0) {
#pragma unroll
          for (int k = 0; k < KP; ++k)
            if (k * kWave + lane == pod.cls) wcnt[k] -= 1;
        }
        const uint64_t dt = (uint64_t)(t + pod.dur);
        if (t + pod.dur < 0 || dt > time_max) { exc = EXC_UNSUPPORTED; break; }
        heap.push(n, (dt << tshift) | ((uint64_t)rank << lb) | ((uint64_t)gmask << (2 + nb)) |
                         ((uint64_t)best_node << 2) | kDelete);
        ++n;
        if (W.trace_hash) hsh = mix_event(hsh, ((uint64_t)(uint32_t)rank << 2), ((uint64_t)t << 8) ^ (uint64_t)best_node);
        prof.mark(PH_COMMIT);
      }
    }

    // ---------------- evaluator hook (snapshot schedule precomputed on the host)
    ++processed;
    bool fire;
    if (ksnap < n_fire) fire = processed >= next_fire;
    else fire = (double)processed / (double)N >= thr;
    if (fire) {
      const int64_t t0 = Wc->tot_cpu, t1 = Wc->tot_mem, t2 = Wc->tot_gcnt, t3 = Wc->tot_gmilli;
      const double r0 = t0 > 0 ? (double)used_cpu / (double)t0 : 0.0;
      const double r1 = t1 > 0 ? (double)used_mem / (double)t1 : 0.0;
      const double r2 = t2 > 0 ? (double)used_gcnt / (double)t2 : 0.0;
      const double r3 = t3 > 0 ? (double)used_gml / (double)t3 : 0.0;
      acc.add(0, r0); acc.add(1, r1); acc.add(2, r2); acc.add(3, r3);
      if (ksnap >= n_fire) thr += Wc->snapshot_interval;
      ++ksnap;
      next_fire = ksnap < n_fire ? const_ptr(Wc->snap_fire)[ksnap] : INT64_MAX;
    }
    // (the reference's max_nodes counter feeds no metric: not tracked)
    if (W.check_every > 0 && (processed % W.check_every == 0 || n == 0) &&
        !invariants_hold<NPASS>(W, heap, n, nr, inv, lane)) {
      exc = EXC_INVARIANT;
      break;
    }
    prof.mark(PH_EVAL);
  }
  if (prof_out) prof.flush(prof_out);

  const int64_t n_snap = readlane64(acc.count, 0), n_frag = readlane64(acc.count, 4);
  const int inexact = ballot(lane < 5 && acc.inexact != 0) != 0;
  if (lane < 5) {
    out->acc_lo[lane] = (uint64_t)(u128)acc.sum;
    out->acc_hi[lane] = (uint64_t)((u128)acc.sum >> 64);
  }
  if (lane == 0) {
    out->n_events = processed;
    out->n_snap = n_snap;
    out->n_frag = n_frag;
    out->n_unplaced = n_dropped;
    out->n_repush = n_repush;
    out->max_nodes = 0;
    out->hash = hsh;
    out->exc = exc;
    out->inexact = inexact;
  }
}

}  // namespace fksd
