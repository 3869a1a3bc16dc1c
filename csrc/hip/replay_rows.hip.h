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

namespace fksd {

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
struct RowHeap {
  FKS_GLOBAL uint64_t* h;     // HBM slice (address = slot + 1)
  FKS_LDS uint64_t* top;      // LDS copy of addresses [0, T + 1)
  int T;                      // slots [0, T) in LDS, T = 2^k - 1
  FKS_LDS uint32_t* delmap;   // bit p set <=> slot p holds a deletion
  int lb;
  int j, rbase;               // lane within the row, first lane of the row

  __device__ __forceinline__ uint64_t ld(int i) const { return i < T ? top[i + 1] : h[i + 1]; }
  __device__ __forceinline__ void st(int i, uint64_t v) const {
    if (i < T) top[i + 1] = v;
    else h[i + 1] = v;
  }
  // children (c, c + 1) of a node, c odd: one aligned 16-byte pair, never
  // split between LDS and HBM (T is odd)
  __device__ __forceinline__ u64x2 ld_pair(int c) const {
    if (c < T) return *reinterpret_cast<const FKS_LDS u64x2*>(top + c + 1);
    return *reinterpret_cast<const FKS_GLOBAL u64x2*>(h + c + 1);
  }
  __device__ __forceinline__ void mark(int pos, uint64_t v) const {
    const uint32_t bit = 1u << (pos & 31);
    if ((v & 3) == kDelKind) __hip_atomic_fetch_or(&delmap[pos >> 5], bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else __hip_atomic_fetch_and(&delmap[pos >> 5], ~bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }

  // CPython heappop's re-insertion of `last` (= old h[n]) at the root of a
  // heap of n >= 1 items: same algorithm as WaveHeap::pop_reinsert with
  // 4-level rounds (lane j < 15 = the j-th node, BFS order, of the 4-level
  // subtree under the path end, holding that node's child pair).
  __device__ void pop_reinsert(int n, uint64_t last) const {
    const int k = j == 0 ? 0 : j < 3 ? 1 : j < 7 ? 2 : 3;   // depth of node j in the subtree
    const int ki = j - ((1 << k) - 1);
    constexpr int kRounds = 5;   // 20 levels: n < 2^20 (host guarantees n < 2^17)
    uint64_t val[kRounds];
    int par[kRounds];
    bool on[kRounds];
    int start[kRounds];
    int pos = 0;
    bool leaf = false;
#pragma unroll
    for (int rd = 0; rd < kRounds; ++rd) {
      start[rd] = pos;
      val[rd] = 0; par[rd] = 0; on[rd] = false;
      if (leaf || 2 * pos + 1 >= n) { leaf = true; continue; }
      const int q = ((pos + 1) << k) - 1 + ki;
      const int c = 2 * q + 1;
      const bool valid = j < 15 && c < n;
      uint64_t vl = ~0ull, vr = ~0ull;
      if (valid) {
        const u64x2 pr = ld_pair(c);
        vl = pr.x;
        vr = pr.y;
      }
      const bool go_r = valid && (c + 1 < n) && !key_lt(vl, vr, lb);
      const uint32_t m = row_ballot(go_r, rbase);
      const uint32_t ex = row_ballot(valid, rbase);
      int cj = 0, taken = 0, idx = 0;
      uint32_t onm = 0;
#pragma unroll
      for (int lv = 0; lv < 4; ++lv) {
        if (taken == lv && ((ex >> cj) & 1)) {
          onm |= 1u << cj;
          idx = 2 * (cj - ((1 << lv) - 1)) + (int)((m >> cj) & 1);
          cj = (1 << (lv + 1)) - 1 + idx;
          taken = lv + 1;
        }
      }
      on[rd] = (onm >> j) & 1;
      val[rd] = go_r ? vr : vl;
      par[rd] = q;
      pos = ((pos + 1) << taken) - 1 + idx;
      if (taken < 4) leaf = true;
    }
    // bubble `last` up: the first path entry (path order = round, then lane)
    // with last < v and everything below keep their slots; `last` lands on
    // that entry's parent, the entries above move up one level
    int jr = -1, jl = 0, target = pos;
#pragma unroll
    for (int rd = 0; rd < kRounds; ++rd) {
      const uint32_t g = row_ballot(on[rd] && key_lt(last, val[rd], lb), rbase);
      if (jr < 0 && g) {
        jr = rd;
        jl = __ffs(g) - 1;
        const int kk = jl == 0 ? 0 : jl < 3 ? 1 : jl < 7 ? 2 : 3;
        target = ((start[rd] + 1) << kk) - 1 + (jl - ((1 << kk) - 1));
      }
    }
#pragma unroll
    for (int rd = 0; rd < kRounds; ++rd) {
      const bool above = jr < 0 || rd < jr || (rd == jr && j < jl);
      if (on[rd] && above) {
        st(par[rd], val[rd]);
        mark(par[rd], val[rd]);
      }
    }
    if (j == 0) { st(target, last); mark(target, last); }
  }

  // CPython heappush on a heap of n items
  __device__ void push(int n, uint64_t item) const {
    const int l = j + 1;
    const int anc = ((n + 1) >> l) - 1;
    const bool valid = n > 0 && anc >= 0;
    const uint64_t v = valid ? ld(anc) : 0;
    const bool gt = valid && key_lt(item, v, lb);
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

// Exact fixed-point accumulators 0-4 on lanes 0-4 of the row (LaneAcc's
// arithmetic, lane-within-row ownership).
struct RowAcc {
  i128 sum;
  int64_t count;
  int32_t inexact;
  __device__ void init() { sum = 0; count = 0; inexact = 0; }
  __device__ void add(int k, double v, int j) {
    const bool mine = j == k;
    const uint64_t bits = (uint64_t)__double_as_longlong(v);
    const int E = (int)((bits >> 52) & 0x7FF);
    const uint64_t frac = bits & ((1ull << 52) - 1);
    if (mine) ++count;
    if (E == 0 && frac == 0) return;
    bool bad = (E == 0x7FF || E == 0);
    uint64_t M = frac | (1ull << 52);
    int shift = E - 979;
    if (!bad && shift < 0) {
      if (shift <= -53 || (M & ((1ull << (-shift)) - 1))) bad = true;
      else { M >>= (-shift); shift = 0; }
    }
    if (!bad && shift > 126 - 53) bad = true;
    if (bad) { if (mine) inexact = 1; return; }
    i128 t = (i128)(u128)M << shift;
    if (bits >> 63) t = -t;
    if (mine) {
      sum += t;
      const u128 mag = sum < 0 ? (u128)(-sum) : (u128)sum;
      if (mag >> 126) inexact = 1;
    }
  }
};

// LDS per wave: [4 x 16 weights] then per row [deletion bitmap | heap top].
__host__ __device__ inline size_t rows_row_bytes(int n_pods, int T) {
  return (size_t)lds_delmap_words(n_pods) * 4 + (size_t)(T + 1) * 8;
}
__host__ __device__ inline size_t rows_lds_bytes(int n_pods, int T) {
  return (size_t)kRowsPerWave * kWeights * 8 + kRowsPerWave * rows_row_bytes(n_pods, T);
}

// The row kernel body.  P policies, wave w replays policies 4w .. 4w+3.
// fam: per-policy family ids (FAM = -1), weights: [P, kWeights] (device-mapped
// pinned host memory), gheap: [P, row_heap_entries(N)] HBM heap slices,
// heap0p: the initial heap shifted by one slot (address = slot + 1).
template <int FAM>
__device__ void replay_rows(const DevWorkload& W, const int32_t* fam, const double* weights, uint64_t* gheap,
                            DevResult* out, int P) {
  extern __shared__ uint64_t lds_raw[];
  const int lane = lane_id();
  const int row = lane >> 4;
  const int rbase = lane & 48;
  const int p = blockIdx.x * kRowsPerWave + row;
  const bool live = p < P;
  const int N = W.n_pods;
  const int T = W.heap_top;
  const int lb = W.low_bits, nb = W.node_bits, rb = W.rank_bits;
  const int tshift = rb + lb;
  const uint64_t time_max = (W.time_bits >= 63) ? ~0ull : ((1ull << W.time_bits) - 1);
  int jv = lane & 15;

  FKS_LDS uint64_t* lds = lds_ptr(lds_raw);
  FKS_LDS double* wl = reinterpret_cast<FKS_LDS double*>(lds) + row * kWeights;
  FKS_LDS char* rowbase = reinterpret_cast<FKS_LDS char*>(lds + kRowsPerWave * kWeights) +
                          (size_t)row * rows_row_bytes(N, T);
  RowHeap heap;
  heap.delmap = reinterpret_cast<FKS_LDS uint32_t*>(rowbase);
  heap.top = reinterpret_cast<FKS_LDS uint64_t*>(rowbase + (size_t)lds_delmap_words(N) * 4);
  heap.h = global_ptr(gheap + (size_t)(live ? p : 0) * row_heap_entries(N));
  heap.T = T;
  heap.lb = lb;
  heap.j = jv;
  heap.rbase = rbase;

  // ---- prologue: weights, heap image, bitmap, node state
  int family = FAM;
  if (live) {
    wl[jv] = *global_ptr(&weights[(size_t)p * kWeights + jv]);
    if (FAM < 0) family = fam[p];
    const int words = row_heap_entries(N) / 2;   // 16-byte pairs of the shifted heap
    const FKS_GLOBAL u64x2* src = reinterpret_cast<const FKS_GLOBAL u64x2*>(global_ptr(W.heap0p));
    for (int i = jv; i < words; i += kRow) {
      const u64x2 v = src[i];
      if (2 * i < T + 1) *reinterpret_cast<FKS_LDS u64x2*>(heap.top + 2 * i) = v;
      else *reinterpret_cast<FKS_GLOBAL u64x2*>(heap.h + 2 * i) = v;
    }
    for (int i = jv; i < lds_delmap_words(N); i += kRow) heap.delmap[i] = 0u;
  }
  NodeRegs<1> nr;
  nr.cpu_left[0] = W.cpu_left0[jv];
  nr.mem_left[0] = W.mem_left0[jv];
  nr.gpu_left[0] = W.gpu_left0[jv];
  nr.cpu_total[0] = W.cpu_total[jv];
  nr.mem_total[0] = W.mem_total[jv];
  nr.ngpus[0] = W.ngpus[jv];
#pragma unroll
  for (int g = 0; g < kGmax; ++g) {
    nr.gml[0][g] = W.gml_left0[jv * kGmax + g];
    nr.gmt[0][g] = W.gml_total[jv * kGmax + g];
  }
  const bool node_valid = jv < W.n_nodes;
  int32_t wcnt[kRowClassSlots];
#pragma unroll
  for (int s = 0; s < kRowClassSlots; ++s) wcnt[s] = 0;

  int64_t used_cpu = W.used_cpu0, used_mem = W.used_mem0, used_gcnt = W.used_gcnt0, used_gml = W.used_gmilli0;
  RowAcc acc;
  acc.init();
  int64_t processed = 0;
  int n_repush = 0, n_dropped = 0;
  int ksnap = 0;
  const int n_fire = W.n_fire;
  int64_t next_fire = n_fire > 0 ? W.snap_fire[0] : INT64_MAX;
  double thr = W.thr_after_fire;
  uint64_t hsh = 0xcbf29ce484222325ull;
  int32_t exc = EXC_NONE;
  int n = live ? N : 0;
  __syncthreads();

  while (n > 0) {
    // opaque lane id: keeps the lane-derived subtree predicates out of SGPRs
    asm volatile("" : "+v"(jv));
    heap.j = jv;
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

    if (kind == kDelete) {
      const int node = (int)((top >> 2) & ((1u << nb) - 1));
      const int mask = (int)((top >> (2 + nb)) & 0xFF);
      if (jv == node) {
        nr.cpu_left[0] += pod.cpu;
        nr.mem_left[0] += pod.mem;
        nr.gpu_left[0] += pod.ngpu;
#pragma unroll
        for (int g = 0; g < kGmax; ++g)
          if ((mask >> g) & 1) nr.gml[0][g] += pod.gmilli;
      }
      used_cpu -= pod.cpu; used_mem -= pod.mem; used_gcnt -= pod.ngpu;
      used_gml -= (int64_t)pod.gmilli * __popc(mask);
      if (W.trace_hash) hsh = mix_event(hsh, ((uint64_t)(uint32_t)rank << 2) | 1, (uint64_t)t);
    } else {
      // ---------------- creation: score the row's nodes, first maximum wins
      int lexc = EXC_NONE;
      int64_t s = 0;
      if (node_valid && feasible<1>(0, nr, pod)) {
        double w[kWeights];
#pragma unroll
        for (int q = 0; q < kWeights; ++q) w[q] = q < family_weights(FAM) ? wl[q] : 0.0;
        s = BuiltinScorerDev<FAM>::template score_weights<1>(family, w, 0, nr, pod, lexc);
        if (lexc != EXC_NONE) s = 0;
      }
      const uint32_t bad = row_ballot(lexc != EXC_NONE, rbase);
      if (bad) {
        exc = row_read(lexc, rbase, __ffs(bad) - 1);
        break;
      }
      const int64_t m = (int64_t)row_max_u64((uint64_t)s);   // scores are >= 0
      const int best_node = m > 0 ? __ffs(row_ballot(s == m, rbase)) - 1 : -1;

      if (best_node < 0) {
        // ---------------- failed placement
        if (kind == kFresh && pod.ngpu > 0) {
#pragma unroll
          for (int sl = 0; sl < kRowClassSlots; ++sl)
            if (sl == (pod.cls >> 4) && jv == (pod.cls & 15)) wcnt[sl] += 1;
        }
        double frag = 0.0;
        int mcls = -1;
#pragma unroll
        for (int sl = 0; sl < kRowClassSlots; ++sl) {
          const uint32_t b = row_ballot(wcnt[sl] > 0, rbase);
          if (mcls < 0 && b) mcls = sl * kRow + __ffs(b) - 1;
        }
        if (mcls >= 0) {
          const int mv = *global_ptr(&W.class_value[mcls]);
          int64_t stranded = 0;
#pragma unroll
          for (int g = 0; g < kGmax; ++g) {
            const int l = nr.gml[0][g];
            if (g < nr.ngpus[0] && 0 < l && l < mv) stranded += l;
          }
          stranded = row_sum_i64(node_valid ? stranded : 0);
          const int64_t tg = W.tot_gmilli;
          frag = tg > 0 ? (double)stranded / (double)tg : 0.0;
        }
        acc.add(4, frag, jv);
        const int f = heap.first_deletion(n);
        if (f >= 0) {
          const uint64_t nt = (heap.ld(f) >> tshift) + 1;
          if (nt > time_max) { exc = EXC_UNSUPPORTED; break; }
          heap.push(n, (nt << tshift) | ((uint64_t)rank << lb) | kRetry);
          ++n;
          ++n_repush;
        } else {
          ++n_dropped;
        }
        if (W.trace_hash) hsh = mix_event(hsh, ((uint64_t)(uint32_t)rank << 2) | 2, (uint64_t)t);
      } else {
        // ---------------- commit on best_node
        int gmask = 0, ok = 1;
        if (pod.ngpu > 0) {
          int myok = 1;
          const int mymask = pick_gpus<1>(nr, 0, pod.gmilli, pod.ngpu, W.first_fit_alloc != 0, myok);
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
            if ((gmask >> g) & 1) nr.gml[0][g] -= pod.gmilli;
        }
        used_cpu += pod.cpu; used_mem += pod.mem; used_gcnt += pod.ngpu;
        used_gml += (int64_t)pod.gmilli * __popc(gmask);
        if (kind == kRetry && pod.ngpu > 0) {
#pragma unroll
          for (int sl = 0; sl < kRowClassSlots; ++sl)
            if (sl == (pod.cls >> 4) && jv == (pod.cls & 15)) wcnt[sl] -= 1;
        }
        const uint64_t dt = (uint64_t)(t + pod.dur);
        if (t + pod.dur < 0 || dt > time_max) { exc = EXC_UNSUPPORTED; break; }
        heap.push(n, (dt << tshift) | ((uint64_t)rank << lb) | ((uint64_t)gmask << (2 + nb)) |
                         ((uint64_t)best_node << 2) | kDelete);
        ++n;
        if (W.trace_hash) hsh = mix_event(hsh, ((uint64_t)(uint32_t)rank << 2), ((uint64_t)t << 8) ^ (uint64_t)best_node);
      }
    }

    // ---------------- evaluator hook (host-precomputed snapshot schedule)
    ++processed;
    bool fire;
    if (ksnap < n_fire) fire = processed >= next_fire;
    else fire = (double)processed / (double)N >= thr;
    if (fire) {
      const double r0 = W.tot_cpu > 0 ? (double)used_cpu / (double)W.tot_cpu : 0.0;
      const double r1 = W.tot_mem > 0 ? (double)used_mem / (double)W.tot_mem : 0.0;
      const double r2 = W.tot_gcnt > 0 ? (double)used_gcnt / (double)W.tot_gcnt : 0.0;
      const double r3 = W.tot_gmilli > 0 ? (double)used_gml / (double)W.tot_gmilli : 0.0;
      acc.add(0, r0, jv); acc.add(1, r1, jv); acc.add(2, r2, jv); acc.add(3, r3, jv);
      if (ksnap >= n_fire) thr += W.snapshot_interval;
      ++ksnap;
      next_fire = ksnap < n_fire ? *global_ptr(&W.snap_fire[ksnap]) : INT64_MAX;
    }
  }
  if (!live) return;

  const int64_t n_snap = (int64_t)(((uint64_t)(uint32_t)row_read((int)(acc.count >> 32), rbase, 0) << 32) |
                                   (uint32_t)row_read((int)acc.count, rbase, 0));
  const int64_t n_frag = (int64_t)(((uint64_t)(uint32_t)row_read((int)(acc.count >> 32), rbase, 4) << 32) |
                                   (uint32_t)row_read((int)acc.count, rbase, 4));
  const int inexact = row_ballot(jv < 5 && acc.inexact != 0, rbase) != 0;
  DevResult* o = out + p;
  if (jv < 5) {
    o->acc_lo[jv] = (uint64_t)(u128)acc.sum;
    o->acc_hi[jv] = (uint64_t)((u128)acc.sum >> 64);
  }
  if (jv == 0) {
    o->n_events = processed;
    o->n_snap = n_snap;
    o->n_frag = n_frag;
    o->n_unplaced = n_dropped;
    o->n_repush = n_repush;
    o->max_nodes = 0;
    o->hash = hsh;
    o->exc = exc;
    o->inexact = inexact;
  }
}

}  // namespace fksd
