// k_replay_rows: four candidate policies per wave64 for clusters of <= 16 nodes.
//
// The wave kernel (replay.hip.h) maps one policy onto a whole wave with lanes =
// nodes, so on the 16-node OpenB cluster 48 of 64 lanes idle through every
// VALU instruction, and the per-event dependency chain (heap walk, ballots,
// reductions) is paid once per policy.  Here the wave is split into its four
// DPP rows of 16 lanes and each row replays its own policy:
//   * lane (r, j) holds node j of policy r in VGPRs; everything a policy needs
//     wave-uniform in the wave kernel (event key, pod record, heap size,
//     counters, utilisation totals) is row-uniform here and lives in VGPRs;
//   * row collectives: per-row ballots (16-bit slice of the wave ballot),
//     butterfly max / sum over the row with DPP row_ror (no LDS round trip),
//     row_read = ds_bpermute inside the row;
//   * the CPython-exact heap per policy: slot i at address i+1 so a node's two
//     children are one aligned 16-byte pair; a pop gathers the 4-level subtree
//     under the current path end (15 child pairs, one per lane) per round, a
//     push gathers all 16 ancestors at once; the top 2^k-1 slots of each heap
//     sit in LDS, the rest in the policy's HBM slice;
//   * divergence between the four policies (deletion vs creation, placement vs
//     failure) is ordinary exec masking: every branch condition is
//     row-uniform, so a row is always wholly active or wholly masked.
// Same semantics and arithmetic as replay_one (bit-identical results; checked
// against the CPU oracle in tests/test_gpu_engine.py); the invariant checker
// and the opt-in "earliest deletion" repush rule stay on the wave kernel.
#pragma once

#include "replay.hip.h"
#include "scorers.hip.h"
#include "jit_abi.h"

namespace fksd {

// heap slot accesses through flat (generic) addresses: RowHeapT<FLAT>
#ifndef FKS_ROW_FLAT
#define FKS_ROW_FLAT 1
#endif
// FAM value of the native-program instance: every row calls its own
// JIT-compiled scorer (jit_abi.h ProgFn) instead of a built-in family.
constexpr int kFamNative = 100;
// host family codes of composite row-kernel variants: built for 5 waves per
// SIMD; with exec-masked LDS / HBM heap accesses instead of flat ones
constexpr int kRowCompositeW5 = 5;
constexpr int kRowCompositeSplit = 6;
struct RowNativeArgs {
  const uint64_t* fn;     // [P] device addresses of the programs' scorers
  const int64_t* kc;      // concatenated constant blocks
  const int32_t* koff;    // [P] offset of policy p's block in kc
  const uint32_t* abort = nullptr;   // host flag (two-wave kernel): nonzero ends replays early, EXC_TIMEOUT
  uint32_t max_events = 0;           // two-wave kernel: a replay past this many events ends, EXC_EVENTS (0: none)
};
// Control block of the resident program service (replay_kernels.hip k_native_service)
struct ServiceCtl {
  uint32_t* claimed;            // HBM: [0] next index to claim, [32] mirror of published, [64] of stop
  const uint32_t* published;    // host: indexes < published are queued
  const uint32_t* stop;         // host: 1 = leave once nothing is left to claim
  uint32_t* done;               // host: [slots] index + 1 once the slot's row is written
  const uint32_t* qslot;        // host: [nq] data slot of index i (entry i % nq)
  uint32_t* started;            // host: [nq] index + 1 once a workgroup read entry i % nq
  uint32_t nq;
  uint32_t max_idle_polls;
  uint64_t* cost;               // host: [slots] s_memtime cycles of the slot's replay (written before done)
};

constexpr int kRow = 16;            // lanes per DPP row = max nodes per policy
constexpr int kRowsPerWave = 4;
constexpr int kRowClassSlots = 4;   // waiting-class histogram: 64 gpu_milli classes
constexpr int kRowMaxHeap = (1 << 17) - 2;   // push gathers <= 16 ancestors

__host__ __device__ inline int row_heap_entries(int n_pods) { return (n_pods + 2 + 63) & ~63; }

// ---- row collectives ---------------------------------------------------------
__device__ __forceinline__ uint32_t row_ballot(bool p, int rbase) {
  return (uint32_t)(ballot(p) >> rbase) & 0xFFFFu;
}
template <int N>
__device__ __forceinline__ uint32_t row_ror32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x120 + N, 0xF, 0xF, false);
}
template <int N>
__device__ __forceinline__ uint64_t row_ror64(uint64_t v) {
  return ((uint64_t)row_ror32<N>((uint32_t)(v >> 32)) << 32) | row_ror32<N>((uint32_t)v);
}
__device__ __forceinline__ uint64_t row_max_u64(uint64_t v) {
  uint64_t o;
  o = row_ror64<8>(v); v = o > v ? o : v;
  o = row_ror64<4>(v); v = o > v ? o : v;
  o = row_ror64<2>(v); v = o > v ? o : v;
  o = row_ror64<1>(v); v = o > v ? o : v;
  return v;
}
__device__ __forceinline__ int64_t row_sum_i64(int64_t v) {
  uint64_t u = (uint64_t)v;
  u += row_ror64<8>(u);
  u += row_ror64<4>(u);
  u += row_ror64<2>(u);
  u += row_ror64<1>(u);
  return (int64_t)u;
}
// value of lane k (row-uniform) of my row
__device__ __forceinline__ int row_read(int v, int rbase, int k) {
  return __builtin_amdgcn_ds_bpermute((rbase + k) << 2, v);
}

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

// ---- one policy's heap, driven by the 16 lanes of its row ---------------------
template <bool FLAT = FKS_ROW_FLAT != 0>
struct RowHeapT {
  FKS_GLOBAL uint64_t* h;     // HBM slice (address = slot + 1)
  FKS_LDS uint64_t* top;      // LDS copy of addresses [0, T + 1)
  int T;                      // slots [0, T) in LDS, T = 2^k - 1
  FKS_LDS uint32_t* delmap;   // bit p set <=> slot p holds a deletion
  int lb;
  int j, rbase;               // lane within the row, first lane of the row
  uint32_t anc, dir;          // subtree node j: BFS indices of its ancestors / of those stepping right

  // FLAT: slot i through one generic (flat) address -- the LDS aperture
  // below T, the HBM slice above: one flat_load / flat_store per access
  // instead of an exec-masked ds_* / global_* pair (a subtree or ancestor
  // gather often straddles T within a row, which ran both sides, the LDS
  // side behind a vmcnt(0) for the shared destination registers).
  uint64_t* gtop;   // generic address of `top`
  uint64_t* gh;     // generic address of `h`
  __device__ __forceinline__ void bind() {   // after setting top and h
    gtop = (uint64_t*)top;
    gh = (uint64_t*)h;
  }
  __device__ __forceinline__ uint64_t* slot(int i) const { return (i < T ? gtop : gh) + (i + 1); }
  __device__ __forceinline__ uint64_t ld(int i) const {
    if constexpr (FLAT) return *slot(i);
    else return i < T ? top[i + 1] : h[i + 1];
  }
  __device__ __forceinline__ void st(int i, uint64_t v) const {
    if constexpr (FLAT) {
      *slot(i) = v;
    } else {
      if (i < T) top[i + 1] = v;
      else h[i + 1] = v;
    }
  }
  // children (c, c + 1) of a node, c odd: one aligned 16-byte pair, never
  // split between LDS and HBM (T is odd)
  __device__ __forceinline__ u64x2 ld_pair(int c) const {
    if constexpr (FLAT) return *reinterpret_cast<const u64x2*>(slot(c));
    if (c < T) return *reinterpret_cast<const FKS_LDS u64x2*>(top + c + 1);
    return *reinterpret_cast<const FKS_GLOBAL u64x2*>(h + c + 1);
  }
  // bit `pos` of the deletion bitmap := (v is a DELETION): one LDS masked-OR
  // atomic (word = (word & ~bit) | data), safe when several lanes of the row
  // hit the same word in one instruction.  LDS operations of a wave complete
  // in order, so later bitmap reads see it without an extra wait.
  __device__ __forceinline__ void mark(int pos, uint64_t v) const {
    const uint32_t bit = 1u << (pos & 31);
    const uint32_t data = (v & 3) == kDelKind ? bit : 0u;
    const uint32_t addr = (uint32_t)(uintptr_t)(delmap + (pos >> 5));
    asm volatile("ds_mskor_b32 %0, %1, %2" ::"v"(addr), "v"(bit), "v"(data) : "memory");
  }

  // Keys compare as plain u64: a pod has at most one entry in the heap, so two
  // entries never share (time, rank) and the payload bits below `lb` never
  // decide an order.
  // CPython heappop's re-insertion of `last` (= old h[n]) at the root of a
  // heap of n >= 1 items: same algorithm as WaveHeap::pop_reinsert with
  // 4-level rounds (lane j < 15 = the j-th node, BFS order, of the 4-level
  // subtree under the path end, holding that node's child pair).
  __device__ void pop_reinsert(int n, uint64_t last) const {
    const int k = j == 0 ? 0 : j < 3 ? 1 : j < 7 ? 2 : 3;   // depth of node j in the subtree
    const int ki = j - ((1 << k) - 1);
    // The path values grow downwards, so the bubble-up of `last` ends at the
    // first path entry greater than it: rounds above that entry move their
    // path up as soon as they are walked (nothing is carried between rounds),
    // the round holding it moves the entries before it and places `last` on
    // its parent, and the walk stops there -- the entries below keep their
    // slots, exactly as after CPython's full descent and bubble-up.
    constexpr int kRounds = 5;   // 20 levels (host guarantees n < 2^17)
    int pos = 0, target = -1;
#pragma unroll
    for (int rd = 0; rd < kRounds; ++rd) {
      if (2 * pos + 1 >= n) break;   // pos is a leaf
      const int q = ((pos + 1) << k) - 1 + ki;
      const int c = 2 * q + 1;
      const bool valid = j < 15 && c < n;
      uint64_t vl = ~0ull, vr = ~0ull;
      if (valid) {
        const u64x2 pr = ld_pair(c);
        vl = pr.x;
        vr = pr.y;
      }
      const bool go_r = valid && (c + 1 < n) && !(vl < vr);
      const uint32_t m = row_ballot(go_r, rbase);
      // node j is on the path iff every ancestor in the subtree chooses the
      // child towards j (lane constants anc / dir), and it is a path *parent*
      // iff it has children itself: no serial walk.  (A valid node's
      // ancestors are valid: their child pairs sit at smaller heap indices.)
      const bool on = valid && ((m ^ dir) & anc) == 0;
      const uint32_t onm = row_ballot(on, rbase);
      const uint64_t v = go_r ? vr : vl;
      const uint32_t g = row_ballot(on && last < v, rbase);
      const int jl = g ? __ffs(g) - 1 : kRow;
      if (on && j < jl) {   // moves up one level
        st(q, v);
        mark(q, v);
      }
      if (g) {   // `last` lands on the slot of the first path entry greater than it
        target = row_read(q, rbase, jl);
        break;
      }
      // the deepest path parent jd hands over its chosen child (the new path
      // end) and its depth in the subtree (levels descended this round - 1)
      const int jd = 31 - __clz(onm);
      const int nk = row_read(((c + (int)go_r) << 2) | k, rbase, jd);
      pos = nk >> 2;
      if ((nk & 3) < 3) break;   // reached a leaf
    }
    if (target < 0) target = pos;
    if (j == 0) { st(target, last); mark(target, last); }
  }

  // CPython heappush on a heap of n items
  __device__ void push(int n, uint64_t item) const {
    const int l = j + 1;
    const int anc = ((n + 1) >> l) - 1;
    const bool valid = n > 0 && anc >= 0;
    const uint64_t v = valid ? ld(anc) : 0;
    const bool gt = valid && item < v;
    const int J = __popc(row_ballot(gt, rbase));
    const int dst = ((n + 1) >> (l - 1)) - 1;
    if (gt) { st(dst, v); mark(dst, v); }
    const int aJ = J == 0 ? n : ((n + 1) >> J) - 1;
    if (j == 0) { st(aJ, item); mark(aJ, item); }
  }

  // index of the first DELETION in slots [0, n), or -1
  __device__ int first_deletion(int n) const {
    const int words = (n + 31) >> 5;
    for (int base = 0; base < words; base += kRow) {
      const int wi = base + j;
      uint32_t w = wi < words ? delmap[wi] : 0u;
      if (wi == words - 1 && (n & 31)) w &= (1u << (n & 31)) - 1;
      const uint32_t b = row_ballot(w != 0, rbase);
      if (b) {
        const int fl = __ffs(b) - 1;
        const uint32_t fw = (uint32_t)row_read((int)w, rbase, fl);
        return ((base + fl) << 5) + (__ffs(fw) - 1);
      }
    }
    return -1;
  }
};
using RowHeap = RowHeapT<>;

// Exact fixed-point accumulators 0-4 on lanes 0-4 of the row: sum of v * 2^96
// over the added doubles (LaneAcc's grid and contract).  Everything the row
// kernel accumulates -- utilisation ratios and fragmentation -- is >= +0.0,
// so the sum is an unsigned 128-bit pair (lo, hi) and the conversion is a
// two-word shift; a negative, subnormal, non-finite or off-grid value marks
// the replay inexact (the host then re-runs it on the CPU oracle).
struct RowAcc {
  uint64_t lo, hi;
  int32_t count;
  int32_t inexact;
  __device__ void init() { lo = hi = 0; count = 0; inexact = 0; }
  __device__ void add(int k, double v, int j) {
    const bool mine = j == k;
    const uint64_t bits = (uint64_t)__double_as_longlong(v);
    if (mine) ++count;
    if (bits == 0) return;                                   // +0.0
    const int E = (int)(bits >> 52);                         // sign bit set -> E >= 2048
    const uint64_t M = (bits & ((1ull << 52) - 1)) | (1ull << 52);
    const int shift = E - 979;                               // v * 2^96 = M << shift
    bool bad = E == 0 || E >= 0x7FF || shift > 126 - 53;
    uint64_t tl, th;
    if (shift >= 0) {
      tl = shift < 64 ? M << shift : 0ull;
      th = shift == 0 ? 0ull : shift < 64 ? M >> (64 - shift) : M << (shift - 64);
    } else {
      bad = bad || shift <= -53 || (M & ((1ull << (-shift)) - 1)) != 0;
      tl = M >> (-shift & 63);
      th = 0;
    }
    if (bad) {
      if (mine) inexact = 1;
      return;
    }
    if (mine) {
      lo += tl;
      hi += th + (lo < tl);
      if (hi >> 62) inexact = 1;   // keep LaneAcc's 2^126 headroom
    }
  }
  // add() for a quotient n / d of integers 0 <= n <= d < 2^31 (utilisation
  // ratios, fragmentation): +0.0 or 2^-31 <= v <= 1, so v * 2^96 = M << s
  // with s in [13, 44] -- always on the grid, no range or sign cases (a value
  // outside that band still marks the replay inexact)
  __device__ void add_unit(int k, double v, int j) {
    const bool mine = j == k;
    const uint64_t bits = (uint64_t)__double_as_longlong(v);
    if (mine) ++count;
    if (bits == 0) return;
    const int s = (int)(bits >> 52) - 979;
    const uint64_t M = (bits & ((1ull << 52) - 1)) | (1ull << 52);
    const uint64_t tl = M << (s & 63), th = M >> ((64 - s) & 63);
    if (mine) {
      if (s < 13 || s > 44) inexact = 1;
      lo += tl;
      hi += th + (lo < tl);
    }
  }
};

// LDS per wave: [4 x 16 weights | 64 class values | 16 x 4 node constants |
// 16 x 3 node reciprocals | 10 GPU-capacity reciprocals] then per row
// [deletion bitmap | heap top].
constexpr int kNodeConsts = 4;   // cpu_total, mem_total, ngpus, per-GPU milli total
constexpr int kNodeRecips = 6;   // DevWorkload::node_recip (3), then the same divisors as doubles
constexpr int kCapRecips = 10;   // DevWorkload::cap_recip (9) + pad
constexpr int kRowClassBytes =
    (kRow * kRowClassSlots * 4 + kRow * kNodeConsts * 4 + kRow * kNodeRecips * 8 + kCapRecips * 8 + 15) & ~15;
__device__ __forceinline__ FKS_LDS double* row_node_recips(FKS_LDS int32_t* ntab) {
  return reinterpret_cast<FKS_LDS double*>(ntab + kRow * kNodeConsts);
}
__device__ __forceinline__ FKS_LDS double* row_cap_recips(FKS_LDS int32_t* ntab) {
  return row_node_recips(ntab) + kRow * kNodeRecips;
}
// sum over the row of a per-lane int32 (|total| < 2^31)
__device__ __forceinline__ int32_t row_sum_i32(int32_t v) {
  v += (int32_t)row_ror32<8>((uint32_t)v);
  v += (int32_t)row_ror32<4>((uint32_t)v);
  v += (int32_t)row_ror32<2>((uint32_t)v);
  v += (int32_t)row_ror32<1>((uint32_t)v);
  return v;
}
__device__ __forceinline__ uint32_t row_min_u32(uint32_t v) {
  v = min(v, row_ror32<8>(v));
  v = min(v, row_ror32<4>(v));
  v = min(v, row_ror32<2>(v));
  v = min(v, row_ror32<1>(v));
  return v;
}
// max of two non-NaN doubles: one v_max_f64 (fmax() adds two canonicalising
// v_max_f64 for IEEE NaN quieting, which scores never need)
__device__ __forceinline__ double max_nn(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// row maximum of finite scores
__device__ __forceinline__ double row_max_f64(double v) {
  v = max_nn(v, __longlong_as_double((long long)row_ror64<8>((uint64_t)__double_as_longlong(v))));
  v = max_nn(v, __longlong_as_double((long long)row_ror64<4>((uint64_t)__double_as_longlong(v))));
  v = max_nn(v, __longlong_as_double((long long)row_ror64<2>((uint64_t)__double_as_longlong(v))));
  v = max_nn(v, __longlong_as_double((long long)row_ror64<1>((uint64_t)__double_as_longlong(v))));
  return v;
}
// the node tables (lanes < 16 of one wave)
__device__ __forceinline__ void fill_node_tables(const DevWorkload& W, FKS_LDS int32_t* ntab, int lane) {
  if (lane < kRow) {
    ntab[lane * kNodeConsts + 0] = W.cpu_total[lane];
    ntab[lane * kNodeConsts + 1] = W.mem_total[lane];
    ntab[lane * kNodeConsts + 2] = W.ngpus[lane];
    ntab[lane * kNodeConsts + 3] = W.gml_total[lane * kGmax];
    FKS_LDS double* z = row_node_recips(ntab);
#pragma unroll
    for (int k = 0; k < 3; ++k) z[lane * kNodeRecips + k] = W.node_recip[lane * 3 + k];
    // max(cpu_total, 1), max(mem_total, 1), max(ngpus, 1) as doubles: an LDS read
    // per creation event instead of an int -> f64 conversion on the VALU
    const int32_t ct = W.cpu_total[lane], mt = W.mem_total[lane], ng = W.ngpus[lane];
    z[lane * kNodeRecips + 3] = (double)(ct > 1 ? ct : 1);
    z[lane * kNodeRecips + 4] = (double)(mt > 1 ? mt : 1);
    z[lane * kNodeRecips + 5] = (double)(ng > 1 ? ng : 1);
  }
  if (lane <= kGmax) row_cap_recips(ntab)[lane] = W.cap_recip[lane];
}
// per row: deletion bitmap | heap top (T + 1 slots) | cold state (trace hash,
// snapshot threshold beyond the host's schedule: read rarely, so kept out of
// the registers the 4- and 5-waves-per-SIMD register budgets are tight on)
constexpr int kRowColdBytes = 32;   // hash, threshold, repush / dropped / snapshot counters
__host__ __device__ inline size_t rows_row_bytes(int n_pods, int T) {
  return (size_t)lds_delmap_words(n_pods) * 4 + (size_t)(T + 1) * 8 + kRowColdBytes;
}
// native programs (kc = true) also stage each active row's constant block
// (kKcLds int64) after the rows' heap areas
__host__ __device__ inline size_t rows_lds_bytes(int n_pods, int T, int rows = kRowsPerWave, bool kc = false) {
  return (size_t)kRowsPerWave * kWeights * 8 + kRowClassBytes + (size_t)rows * rows_row_bytes(n_pods, T) +
         (kc ? (size_t)rows * kKcLds * 8 : 0);
}

// Wave-level phase profiler for the row kernel (diagnostics build only): each
// instrumented region, whenever the wave executes it (for any of its rows),
// charges the s_memtime cycles since the previous mark to its phase.  The
// counters live in the wave's LDS tail so masked-off rows do not matter.
struct RowNoProf {
  __device__ void start(FKS_LDS uint64_t*) {}
  __device__ void mark(int) {}
  __device__ void kinds(int) {}
  __device__ void flush(uint64_t*) {}
};
// s_memtime phase split, plus a histogram of the event kinds a wave-step's
// rows executed: the row kernel runs the union of its four rows' paths under
// exec masks, so the mix decides how much of the issued work is masked off
struct RowProf {
  FKS_LDS uint64_t* c;   // [0, 8): phase cycles, [8]: last timestamp, [8 + m]: wave-steps with kind set m
  __device__ void start(FKS_LDS uint64_t* at) {
    c = at;
    if (lane_id() < 16) c[lane_id()] = lane_id() == 8 ? __builtin_amdgcn_s_memtime() : 0;
  }
  __device__ void mark(int ph) {
    const uint64_t now = __builtin_amdgcn_s_memtime();
    if (lane_id() == __builtin_amdgcn_readfirstlane(lane_id())) {
      c[ph] += now - c[8];
      c[8] = now;
    }
  }
  // cat: this row's event -- 0 none (no policy), 1 deletion, 2 creation
  // placed, 3 creation failed; m = the set of kinds present (bit cat - 1)
  __device__ void kinds(int cat) {
    const int m = (ballot(cat == 1) != 0 ? 1 : 0) | (ballot(cat == 2) != 0 ? 2 : 0) | (ballot(cat == 3) != 0 ? 4 : 0);
    if (m != 0 && lane_id() == __builtin_amdgcn_readfirstlane(lane_id())) c[8 + m] += 1;
  }
  __device__ void flush(uint64_t* o) {
    if (lane_id() < 16) o[lane_id()] = lane_id() == 8 ? 0 : c[lane_id()];
  }
};
constexpr int kRowProfBytes = 128;
constexpr int kRowProfWords = 16;   // per wave in the host's profile buffer

// The row kernel body: a persistent work queue of policies.  Every row claims
// policies with atomicAdd(queue, 1); a row that finishes its replay (or
// aborts on a policy exception) writes the result and claims the next one, so
// the four rows of a wave stay busy until the batch is drained instead of
// idling behind their wave's longest replay, and waves that only become
// resident once others exit find the queue empty and leave at once.  fam: per-policy family ids (FAM = -1), weights: [P, kWeights]
// (device-mapped pinned host memory), gheap: [4 * gridDim.x,
// row_heap_entries(N)] HBM heap slices (one per row slot), heap0p: the
// initial heap shifted by one slot (address = slot + 1).
//
// FAM == kFamNative: natively compiled programs (`nat`), one per row; only
// rows < rows_active claim policies, so small batches can run one program per
// wave (the whole heap in LDS, no other row's divergence in the event loop).
template <int FAM, class Prof = RowNoProf, bool FLAT = FKS_ROW_FLAT != 0>
__device__ void replay_rows(const DevWorkload& W, const DevWorkload* Wdev, const int32_t* fam, const double* weights,
                            uint64_t* gheap, DevResult* out, int P, uint32_t* queue, uint32_t qbase,
                            uint64_t* prof_out = nullptr, RowNativeArgs nat = RowNativeArgs{nullptr, nullptr, nullptr},
                            int rows_active = kRowsPerWave, double* table = nullptr) {
  constexpr bool kNative = FAM == kFamNative;
  const int ra = kNative ? rows_active : kRowsPerWave;
  // W: the kernel-argument copy, read once for the hot scalars below; every
  // other field is re-read where it is used through an opaque pointer to the
  // HBM copy (scalar loads), so the loop carries no spilled SGPR copies of it
  auto cold = [&]() {
    const DevWorkload* g = reinterpret_cast<const DevWorkload*>(uniu64(reinterpret_cast<uint64_t>(Wdev)));
    asm volatile("" : "+s"(g));
    return const_ptr(g);
  };
  extern __shared__ uint64_t lds_raw[];
  const int lane = lane_id();
  const int row = lane >> 4;
  const int rbase = lane & 48;
  const int slot = blockIdx.x * kRowsPerWave + row;
  const int N = W.n_pods;
  const int T = W.heap_top;
  const int lb = W.low_bits, nb = W.node_bits, rb = W.rank_bits;
  const int tshift = rb + lb;
  const uint64_t time_max = (W.time_bits >= 63) ? ~0ull : ((1ull << W.time_bits) - 1);
  int jv = lane & 15;
  const bool node_valid = jv < W.n_nodes;

  FKS_LDS uint64_t* lds = lds_ptr(lds_raw);
  FKS_LDS double* wl = reinterpret_cast<FKS_LDS double*>(lds) + row * kWeights;
  FKS_LDS int32_t* cls_lds = reinterpret_cast<FKS_LDS int32_t*>(lds + kRowsPerWave * kWeights);
  FKS_LDS char* rowbase = reinterpret_cast<FKS_LDS char*>(lds + kRowsPerWave * kWeights) + kRowClassBytes +
                          (size_t)row * rows_row_bytes(N, T);
  // the waiting-class values (gpu_milli of each class) for the fragmentation minimum
  if (lane < W.n_classes) cls_lds[lane] = *global_ptr(&W.class_value[lane]);
  // per-node constants shared by the four rows: cpu / mem totals, GPU count,
  // per-GPU milli totals -- read back only by creation events, so they hold no
  // registers through the pop
  FKS_LDS int32_t* ntab = cls_lds + kRow * kRowClassSlots;
  fill_node_tables(W, ntab, lane);
  RowHeapT<FLAT> heap;
  heap.delmap = reinterpret_cast<FKS_LDS uint32_t*>(rowbase);
  heap.top = reinterpret_cast<FKS_LDS uint64_t*>(rowbase + (size_t)lds_delmap_words(N) * 4);
  heap.h = global_ptr(gheap + (size_t)slot * row_heap_entries(N));
  heap.bind();
  heap.T = T;
  heap.lb = lb;
  heap.j = jv;
  heap.rbase = rbase;
  heap.anc = heap.dir = 0;
  for (int x = jv; x > 0 && x < 15; x = (x - 1) >> 1) {
    const int a = (x - 1) >> 1;
    heap.anc |= 1u << a;
    if ((x & 1) == 0) heap.dir |= 1u << a;   // even BFS index = right child
  }
  const FKS_GLOBAL u64x2* heap_src = reinterpret_cast<const FKS_GLOBAL u64x2*>(global_ptr(W.heap0p));

  auto claim = [&]() {
    // the counter is never reset: this launch's claims start at qbase (the
    // host adds every launch's P + rows claims), so no fill kernel has to
    // queue for a CU slot before the replay can start
    if (kNative && row >= ra) return P;   // idle row: never claims
    const int c = jv == 0 ? (int)(__hip_atomic_fetch_add(queue, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - qbase) : 0;
    return row_read(c, rbase, 0);
  };
  // per-policy state (row-uniform except the node registers / lane-owned slots)
  int p = claim();
  int family = FAM;
  NodeRegs<1, !kNative> nr;   // builtin families: two GPUs per register (host: GPU milli totals < 2^16)
  auto load_consts = [&]() {
    const FKS_LDS int32_t* e = ntab + jv * kNodeConsts;
    nr.cpu_total[0] = e[0];
    nr.mem_total[0] = e[1];
    nr.ngpus[0] = e[2];
    nr.gmt1[0] = e[3];
  };
  // waiting-class histogram, two 16-bit counters per register (slot sl in
  // word sl / 2, half sl % 2; the host allows the row kernel only when every
  // class has fewer than 2^16 GPU pods)
  uint32_t wcp[kRowClassSlots / 2];
  auto wcount = [&](int sl) -> uint32_t { return (wcp[sl >> 1] >> (16 * (sl & 1))) & 0xFFFFu; };
  RowAcc acc;
  int32_t processed = 0, next_fire = INT32_MAX;
  int n = 0;
  FKS_LDS uint64_t* rcs = heap.top + (T + 1);   // [0] trace hash, [1] threshold bits
  // [0] repushes, [1] dropped pods, [2] snapshots taken (per-row counters)
  FKS_LDS uint32_t* rcn = reinterpret_cast<FKS_LDS uint32_t*>(rcs + 2);
  auto bump = [&](int k) {   // one lane of the row adds 1
    if (jv == 0) __hip_atomic_fetch_add(&rcn[k], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  int32_t exc = EXC_NONE;
  ProgFn prog = nullptr;          // native: the row's scorer
  bool feas_pro = false;          // native: it opens with the feasibility prologue (call feasible nodes only)
  // native: its constant block, staged in LDS after the active rows' heap areas
  FKS_LDS int64_t* kcp = reinterpret_cast<FKS_LDS int64_t*>(
      reinterpret_cast<FKS_LDS char*>(lds + kRowsPerWave * kWeights) + kRowClassBytes +
      (size_t)ra * rows_row_bytes(N, T)) + (size_t)row * kKcLds;

  // start policy p on this row: weights, heap image, bitmap, node state, counters
  auto begin = [&]() {
    if constexpr (kNative) {
      const uint64_t fne = *global_ptr(&nat.fn[p]);
      prog = prog_of(fne);
      feas_pro = prog_feas(fne);
      // fixed-size copy: the host pads the kc allocation by kKcLds entries
      const FKS_GLOBAL int64_t* ksrc = global_ptr(nat.kc + *global_ptr(&nat.koff[p]));
      for (int i = jv; i < kKcLds; i += kRow) kcp[i] = ksrc[i];
    } else {
      wl[jv] = *global_ptr(&weights[(size_t)p * kWeights + jv]);
      if (FAM < 0) family = *global_ptr(&fam[p]);
    }
    const int words = row_heap_entries(N) / 2;   // 16-byte pairs of the shifted heap
    for (int i = jv; i < words; i += kRow) {
      const u64x2 v = heap_src[i];
      if constexpr (FLAT) {
        // through the generic addresses the event loop uses (no separate
        // LDS / HBM pointers held live across the loop)
        *reinterpret_cast<u64x2*>((2 * i < T + 1 ? heap.gtop : heap.gh) + 2 * i) = v;
      } else {
        if (2 * i < T + 1) *reinterpret_cast<FKS_LDS u64x2*>(heap.top + 2 * i) = v;
        else *reinterpret_cast<FKS_GLOBAL u64x2*>(heap.h + 2 * i) = v;
      }
    }
    for (int i = jv; i < lds_delmap_words(N); i += kRow) heap.delmap[i] = 0u;
    const FKS_CONST DevWorkload* Wb = cold();
    nr.cpu_left[0] = Wb->cpu_left0[jv];
    nr.mem_left[0] = Wb->mem_left0[jv];
    nr.gpu_left[0] = Wb->gpu_left0[jv];
#pragma unroll
    for (int g = 0; g < kGmax; ++g) {
      nr.g_init(0, g, Wb->gml_left0[jv * kGmax + g]);
    }
#pragma unroll
    for (int k = 0; k < kRowClassSlots / 2; ++k) wcp[k] = 0u;
    acc.init();
    processed = 0;
    rcn[0] = 0u; rcn[1] = 0u; rcn[2] = 0u;
    const double thr = Wb->thr_after_fire;
    rcs[1] = (uint64_t)__double_as_longlong(thr);
    if (Wb->n_fire > 0) {
      next_fire = (int32_t)*global_ptr(&Wb->snap_fire[0]);
    } else {
      int32_t c = 1;
      while ((double)c / (double)N < thr) ++c;
      next_fire = c;
    }
    rcs[0] = 0xcbf29ce484222325ull;
    exc = EXC_NONE;
    n = N;
    __builtin_amdgcn_s_waitcnt(0);   // heap image stored before the first pop reads it
  };

  Prof prof;
  prof.start(reinterpret_cast<FKS_LDS uint64_t*>(reinterpret_cast<FKS_LDS char*>(lds) + rows_lds_bytes(N, T, ra, kNative)));
  bool have = p < P;
  if (have) begin();
  prof.mark(PH_EVAL);

  while (have) {
    // opaque lane id: keeps the lane-derived subtree predicates out of SGPRs
    asm volatile("" : "+v"(jv));
    heap.j = jv;
    int ecat = 0;   // (profiled build: the event's kind for the wave-step histogram)
    do {   // one event; `break` = abort the replay (exc set) or end of the event
      // ---------------- pop
      const uint64_t top = heap.ld(0);
      const int rank = (int)((top >> lb) & ((1ull << rb) - 1));
      typedef int v4i __attribute__((ext_vector_type(4)));
      const v4i precv = *reinterpret_cast<const FKS_GLOBAL v4i*>(global_ptr(&W.pod[rank]));
      const uint64_t last = heap.ld(n - 1);
      --n;
      if (n > 0) heap.pop_reinsert(n, last);
      const int kind = (int)(top & 3);
      const int64_t t = (int64_t)(top >> tshift);
      PodView pod;
      pod.cpu = precv.x; pod.mem = precv.y; pod.dur = precv.z;
      pod.gmilli = precv.w & 0xFFFF; pod.ngpu = (precv.w >> 16) & 0xFF; pod.cls = (precv.w >> 24) & 0xFF;
      pod.ctime = t; pod.rank = rank;
      prof.mark(PH_POP);

      if (kind == kDelete) {
        const int node = (int)((top >> 2) & ((1u << nb) - 1));
        const int mask = (int)((top >> (2 + nb)) & 0xFF);
        if (jv == node) {
          nr.cpu_left[0] += pod.cpu;
          nr.mem_left[0] += pod.mem;
          nr.gpu_left[0] += pod.ngpu;
#pragma unroll
          for (int g = 0; g < kGmax; ++g)
            if ((mask >> g) & 1) nr.g_add(0, g, pod.gmilli);
        }
        if (cold()->trace_hash) rcs[0] = mix_event(rcs[0], ((uint64_t)(uint32_t)rank << 2) | 1, (uint64_t)t);
        ecat = 1;
        prof.mark(PH_DELETE);
      } else {
        // ---------------- creation: score the row's nodes, first maximum wins
        // composite: composite_row (the host runs this instance only on
        // finite weights and verified reciprocals, engine_host stage_builtin)
        constexpr bool kComp = FAM == FAM_COMPOSITE_LINEAR;
        double pcm = 0.0;   // the pod's cpu / mem quotient
        if (kComp) pcm = *global_ptr(&W.pod_cm[rank]);
        load_consts();
        int lexc = EXC_NONE;
        int64_t s = 0;
        double sd = 0.0;   // composite: the truncated score as a double (trunc_score_f)
        if constexpr (kNative) {
          // the program holds the template's feasibility prologue itself; one
          // that opens with it is not called for nodes feasible() rejects
          if (node_valid && (!feas_pro || feasible<1>(0, nr, pod))) {
            const int32_t* gl = nr.gw[0];   // NPASS 1: unpacked
            int32_t gt[kGmax];
#pragma unroll
            for (int g = 0; g < kGmax; ++g) gt[g] = nr.gt(0, g);
            s = prog(nr.cpu_left[0], nr.cpu_total[0], nr.mem_left[0], nr.mem_total[0], pack_gpu_ng(nr.gpu_left[0], nr.ngpus[0]),
                     gl[0], gl[1], gl[2], gl[3], gl[4], gl[5], gl[6], gl[7], gt[0], gt[1], gt[2], gt[3], gt[4], gt[5],
                     gt[6], gt[7], cold()->gmem_total + (size_t)jv * kGmax, pod.cpu, pod.mem,
                     pod.gmilli | (pod.ngpu << 16), pod.ctime, pod.dur, kcp);
            if (s < 0) { lexc = (int)(-s); s = 0; }
          }
        } else if (node_valid && feasible<1>(0, nr, pod)) {
          // weights read from LDS where each term uses them (no 32-VGPR weight vector)
          const FKS_LDS double* wq = wl;
          if constexpr (kComp) {
            const FKS_LDS double* z = row_node_recips(ntab) + jv * kNodeRecips;
            const double zcap = pod.ngpu > 0 ? row_cap_recips(ntab)[nr.gpu_left[0]] : 0.0;
            const typename BuiltinScorerDev<FAM>::RowRecip rz{z[0], z[1], z[2], W.z1000, pcm, zcap, z[3], z[4], z[5]};
            sd = trunc_score_f(BuiltinScorerDev<FAM>::composite_row(nr, pod, wq, rz), lexc);
          } else {
            s = BuiltinScorerDev<FAM>::template score_weights<1>(family, wq, 0, nr, pod, lexc);
          }
          if (lexc != EXC_NONE) { s = 0; sd = 0.0; }
        }
        const uint32_t bad = row_ballot(lexc != EXC_NONE, rbase);
        if (bad) {
          exc = row_read(lexc, rbase, __ffs(bad) - 1);
          break;
        }
        int best_node;
        if constexpr (kComp) {
          const double md = row_max_f64(sd);   // scores are >= 0
          best_node = md > 0.0 ? __ffs(row_ballot(sd == md, rbase)) - 1 : -1;
        } else {
          const int64_t m = (int64_t)row_max_u64((uint64_t)s);   // scores are >= 0
          best_node = m > 0 ? __ffs(row_ballot(s == m, rbase)) - 1 : -1;
        }
        uint64_t push_item = 0;   // never 0 for a real entry: keys hold the pod rank's time > 0 or kind
        prof.mark(PH_SCORE);

        if (best_node < 0) {
          // ---------------- failed placement
          if (kind == kFresh && pod.ngpu > 0) {
#pragma unroll
            for (int sl = 0; sl < kRowClassSlots; ++sl)
              if (sl == (pod.cls >> 4) && jv == (pod.cls & 15)) wcp[sl >> 1] += 1u << (16 * (sl & 1));
          }
          double frag = 0.0;
          // smallest waiting class: each lane offers its lowest nonempty slot's
          // class (sl * 16 + j), the row takes the minimum (64: none waits)
          uint32_t nzs = 0;
#pragma unroll
          for (int sl = kRowClassSlots - 1; sl >= 0; --sl) nzs = wcount(sl) > 0 ? (uint32_t)sl : nzs;
          bool any = false;
#pragma unroll
          for (int k = 0; k < kRowClassSlots / 2; ++k) any = any || wcp[k] != 0u;
          const int mcls = (int)row_min_u32(any ? nzs * kRow + (uint32_t)jv : 64u);
          if (mcls < 64) {
            const int mv = cls_lds[mcls];
            int32_t stranded = 0;   // the cluster's GPU milli total < 2^31 (host-checked)
#pragma unroll
            for (int g = 0; g < kGmax; ++g) {
              const int l = nr.g(0, g);
              if (0 < l && l < mv) stranded += l;   // GPUs past ngpus hold 0 milli (host padding)
            }
            stranded = row_sum_i32(node_valid ? stranded : 0);
            const int64_t tg = cold()->tot_gmilli;
            // stranded in [0, tg]: W.z_tg is verified there
            frag = tg <= 0 ? 0.0 : W.z_tg != 0.0 ? div_by_recip((double)stranded, W.tot_gmilli_d, W.z_tg)
                                                 : (double)stranded / W.tot_gmilli_d;
          }
          acc.add_unit(4, frag, jv);
          const int f = heap.first_deletion(n);
          if (f >= 0) {
            const uint64_t nt = (heap.ld(f) >> tshift) + 1;
            if (nt > time_max) { exc = EXC_UNSUPPORTED; break; }
            push_item = (nt << tshift) | ((uint64_t)rank << lb) | kRetry;
            bump(0);
          } else {
            bump(1);
          }
          if (cold()->trace_hash) rcs[0] = mix_event(rcs[0], ((uint64_t)(uint32_t)rank << 2) | 2, (uint64_t)t);
          ecat = 3;
          prof.mark(PH_FAIL);
        } else {
          // ---------------- commit on best_node
          int gmask = 0, ok = 1;
          if (pod.ngpu > 0) {
            int myok = 1;
            const int mymask = pick_gpus<1>(nr, 0, pod.gmilli, pod.ngpu, cold()->first_fit_alloc != 0, myok);
            const int packed = row_read(mymask | (myok << 8), rbase, best_node);
            gmask = packed & 0xFF;
            ok = packed >> 8;
          }
          if (!ok) { exc = EXC_ALLOC; break; }
          if (jv == best_node) {
            nr.cpu_left[0] -= pod.cpu;
            nr.mem_left[0] -= pod.mem;
            nr.gpu_left[0] -= pod.ngpu;
#pragma unroll
            for (int g = 0; g < kGmax; ++g)
              if ((gmask >> g) & 1) nr.g_add(0, g, -pod.gmilli);
          }
          if (kind == kRetry && pod.ngpu > 0) {
#pragma unroll
            for (int sl = 0; sl < kRowClassSlots; ++sl)
              if (sl == (pod.cls >> 4) && jv == (pod.cls & 15)) wcp[sl >> 1] -= 1u << (16 * (sl & 1));
          }
          const uint64_t dt = (uint64_t)(t + pod.dur);
          if (t + pod.dur < 0 || dt > time_max) { exc = EXC_UNSUPPORTED; break; }
          push_item = (dt << tshift) | ((uint64_t)rank << lb) | ((uint64_t)gmask << (2 + nb)) |
                      ((uint64_t)best_node << 2) | kDelete;
          if (cold()->trace_hash)
            rcs[0] = mix_event(rcs[0], ((uint64_t)(uint32_t)rank << 2), ((uint64_t)t << 8) ^ (uint64_t)best_node);
          ecat = 2;
          prof.mark(PH_COMMIT);
        }
        // one heappush for both outcomes (re-queued creation or deletion): rows
        // that placed and rows that failed share the ancestor gather
        if (push_item != 0) {
          heap.push(n, push_item);
          ++n;
        }
      }

      // ---------------- evaluator hook (host-precomputed snapshot schedule)
      ++processed;
      if (processed >= next_fire) {
        const FKS_CONST DevWorkload* Ws = cold();
        // cluster usage = totals minus the row's sums of what is left (nodes past
        // n_nodes and GPUs past ngpus hold 0): no per-event used counters
        int32_t gl_sum = 0;
#pragma unroll
        for (int g = 0; g < kGmax; ++g) gl_sum += nr.g(0, g);
        const int32_t used_cpu = (int32_t)Ws->tot_cpu - row_sum_i32(nr.cpu_left[0]);
        const int32_t used_mem = (int32_t)Ws->tot_mem - row_sum_i32(nr.mem_left[0]);
        const int32_t used_gcnt = (int32_t)Ws->tot_gcnt - row_sum_i32(nr.gpu_left[0]);
        const int32_t used_gml = (int32_t)Ws->tot_gmilli - row_sum_i32(gl_sum);   // host: totals < 2^31
        const double r0 = Ws->tot_cpu > 0 ? (double)used_cpu / (double)Ws->tot_cpu : 0.0;
        const double r1 = Ws->tot_mem > 0 ? (double)used_mem / (double)Ws->tot_mem : 0.0;
        const double r2 = Ws->tot_gcnt > 0 ? (double)used_gcnt / (double)Ws->tot_gcnt : 0.0;
        const double r3 = Ws->tot_gmilli > 0 ? (double)used_gml / (double)Ws->tot_gmilli : 0.0;
        acc.add_unit(0, r0, jv); acc.add_unit(1, r1, jv); acc.add_unit(2, r2, jv); acc.add_unit(3, r3, jv);
        bump(2);
        const int ksnap = (int)rcn[2];
        if (ksnap < Ws->n_fire) {
          next_fire = (int32_t)*global_ptr(&Ws->snap_fire[ksnap]);
        } else {
          // past the host's precomputed schedule: the next count c > processed
          // with c / N >= thr (the evaluator's IEEE test), thr += interval after
          // every snapshot beyond it (simulator/evaluator.py:55-67)
          double thr = __longlong_as_double((long long)rcs[1]);
          if (ksnap > Ws->n_fire) {
            thr += Ws->snapshot_interval;
            rcs[1] = (uint64_t)__double_as_longlong(thr);
          }
          int32_t c = processed + 1;
          while ((double)c / (double)N < thr) ++c;
          next_fire = c;
        }
      }
      prof.mark(PH_EVAL);
    } while (0);
    prof.kinds(ecat);

    if (n > 0 && exc == EXC_NONE) continue;
    // ---------------- replay done (or aborted): result, then the next policy
    const int n_dropped = (int)rcn[1];
    const int64_t n_snap = row_read(acc.count, rbase, 0);
    const int64_t n_frag = row_read(acc.count, rbase, 4);
    const int inexact = row_ballot(jv < 5 && acc.inexact != 0, rbase) != 0;
    DevResult* o = out + p;
    if (jv < 5) {
      o->acc_lo[jv] = acc.lo;
      o->acc_hi[jv] = acc.hi;
    }
    if (jv == 0) {
      o->n_events = processed;
      o->n_snap = n_snap;
      o->n_frag = n_frag;
      o->n_unplaced = n_dropped;
      o->n_repush = (int64_t)rcn[0];
      o->max_nodes = 0;
      o->hash = rcs[0];
      o->exc = exc;
      o->inexact = inexact;
    }
    if (table) {
      // the evaluator (k_eval_reduce's arithmetic, fused): lane k < 5 turns its
      // own accumulator into the exact mean (its count is that accumulator's),
      // the row gathers the five means, and lane c < 13 writes column c
      double av = 0.0;
      if (jv < 5 && acc.count > 0)
        av = fixed_div_round_dev((i128)(((u128)acc.hi << 64) | acc.lo), (uint64_t)acc.count);
      const uint64_t ab = (uint64_t)__double_as_longlong(av);
      double avg[5];
#pragma unroll
      for (int k = 0; k < 5; ++k)
        avg[k] = __longlong_as_double((long long)(((uint64_t)(uint32_t)row_read((int)(ab >> 32), rbase, k) << 32) |
                                                  (uint32_t)row_read((int)(uint32_t)ab, rbase, k)));
      double score = 0.0;
      if (exc == EXC_NONE && n_snap > 0 && n_dropped == 0) {
        const double overall = (avg[0] + avg[1] + avg[2] + avg[3]) / 4.0;
        const double pen = avg[4] < 0.1 ? avg[4] : 0.1;
        double sc = overall - pen;
        sc = sc < 1.0 ? sc : 1.0;
        score = sc > 0.0 ? sc : 0.0;
      }
      const bool ok = exc == EXC_NONE;   // an aborted replay reports only its exception class
      double v = 0.0;
      switch (jv) {
        case 0: v = score; break;
        case 1: case 2: case 3: case 4: case 5: v = avg[jv - 1]; break;
        case 6: v = (double)n_snap; break;
        case 7: v = (double)n_frag; break;
        case 8: v = (double)processed; break;
        case 9: v = (double)n_dropped; break;
        case 10: v = (double)exc; break;
        case 11: v = (double)inexact; break;
        case 12: v = (double)(rcs[0] >> 11); break;
        default: break;
      }
      if (!ok && jv != 10) v = 0.0;
      if (jv < 13) table[(size_t)p * 13 + jv] = v;
    }
    p = claim();
    have = p < P;
    if (have) begin();
    prof.mark(PH_EVAL + 1);   // result write-back + next policy's prologue
  }
  if (prof_out) prof.flush(prof_out + (size_t)blockIdx.x * kRowProfWords);
}

}  // namespace fksd
