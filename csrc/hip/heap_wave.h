// Wave-parallel CPython heapq on an LDS-resident u64 key array.
//
// CPython's heappop/_siftup walks root->leaf always taking the smaller child
// (the right one when !(left < right)), moves each chosen child up one
// level, drops the last element at the leaf and bubbles it up (_siftdown).
// The chosen path depends only on the ORIGINAL array, so the wave gathers
// whole 5-level subtrees below the current path end (62 lanes, one
// ds_read_b64), decides every left/right choice of the subtree at once
// (sibling exchange by DPP + one ballot) and follows the path with a few
// scalar bit operations; the final bubble-up position is a ballot over the
// path values and all writes land in one parallel store.  heappush's bubble-up
// likewise gathers all ancestors at once: their values are sorted along the
// path, so the insertion depth is a popcount.
//
// The resulting array is bit-identical to CPython's after every operation
// (the repush rule observes the layout), verified against the serial code
// and the CPU oracle.  A parallel bitmap marks the slots holding DELETION
// events so "first deletion in array order" is a ballot over 64-word chunks.
//
// Placement: slots [0, T) live in LDS (`top`), slots [T, n) in the policy's
// HBM slice (`h`).  With the whole heap in LDS T covers everything; with an
// HBM heap the top levels (the hottest: every pop walks root -> leaf) stay in
// LDS so only the last round of a pop and the tail of a push touch HBM.
#pragma once

#include "device_common.h"

namespace fksd {

constexpr int kDelKind = 2;

__device__ __forceinline__ bool key_lt(uint64_t a, uint64_t b, int lb) { return (a >> lb) < (b >> lb); }

// FLAT (HBM heaps with an LDS top): slot i through one generic address --
// one flat_load / flat_store instead of an exec-masked ds_* / global_* pair,
// which ran both sides whenever a gather straddled T (and the LDS side waited
// for the HBM side: same destination registers).
template <bool FLAT = false>
struct WaveHeapT {
  FKS_GLOBAL uint64_t* h;   // keys (slots >= T), the policy's HBM slice
  FKS_LDS uint64_t* top;    // LDS copy of slots [0, T)
  int T;
  FKS_LDS uint32_t* delmap; // bit p set <=> slot p (< M) holds a deletion
  int M;              // slots the bitmap covers (a multiple of 32; >= n: all of them)
  int lb;             // low (payload) bits below the (time, rank) compare key
  int lane;           // this lane's id, refreshed (opaquely) per event by the caller
  uint64_t* gtop;     // FLAT: generic addresses of top / h (bind())
  uint64_t* gh;

  __device__ __forceinline__ void bind() {   // after setting top and h
    gtop = (uint64_t*)top;
    gh = (uint64_t*)h;
  }
  __device__ __forceinline__ uint64_t ld(int i) const {
    if constexpr (FLAT) return *((i < T ? gtop : gh) + i);
    if (i < T) return top[i];
    return h[i];
  }
  // Slot i with i uniform: a ds_read or a global_load behind a scalar branch.
  // A flat load counts in both vmcnt and lgkmcnt, so an LDS read issued after
  // a flat HBM load waits for it; these wait on their own counter only.
  __device__ __forceinline__ uint64_t ld_u(int i) const {
    if (i < T) return top[i];
    return h[i];
  }
  __device__ __forceinline__ void st(int i, uint64_t v) const {
    if constexpr (FLAT) {
      *((i < T ? gtop : gh) + i) = v;
    } else {
      if (i < T) top[i] = v;
      else h[i] = v;
    }
  }

  __device__ __forceinline__ void mark(int pos, uint64_t v) const {
    if (pos >= M) return;   // beyond the bitmap: first_deletion reads the keys themselves
    const uint32_t bit = 1u << (pos & 31);
    if ((v & 3) == kDelKind) __hip_atomic_fetch_or(&delmap[pos >> 5], bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else __hip_atomic_fetch_and(&delmap[pos >> 5], ~bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }

  // Removes the root of a heap that holds n+1 items; `last` (= old h[n]) is
  // re-inserted (CPython: heap.pop(); heap[0] = last; _siftup(heap, 0)).
  // n = new size (>= 1).
  __device__ void pop_reinsert(int n, uint64_t last) const {
    // lane l in [0, 62): subtree level r (1..5), index i within the level
    const int r = lane < 2 ? 1 : lane < 6 ? 2 : lane < 14 ? 3 : lane < 30 ? 4 : 5;
    const int i = lane - ((1 << r) - 2);
    // Up to 4 rounds of 5 levels (depth <= 20, n < 2^20): each round keeps its
    // gathered values; a lane is ON the path when its subtree index equals the
    // path choice at its level (computed with scalar bit ops from one ballot).
    constexpr int kRounds = 4;
    uint64_t val[kRounds];
    int posv[kRounds];
    bool on[kRounds];
    int start[kRounds + 1];  // path-end position entering each round
    int lev[kRounds];        // levels taken in each round
    int pos = 0, rounds = 0;
#pragma unroll
    for (int rd = 0; rd < kRounds; ++rd) {
      start[rd] = pos;
      val[rd] = 0; posv[rd] = 0; on[rd] = false; lev[rd] = 0;
      if (rd > 0 && (lev[rd - 1] < 5 || rounds < rd)) continue;   // previous round hit a leaf
      if (2 * pos + 1 >= n) continue;
      rounds = rd + 1;
      const int idx = ((pos + 1) << r) - 1 + i;
      const bool valid = lane < 62 && idx < n;
      // the first round (slots < 63) is LDS-resident whenever T >= 63: ds_read
      const uint64_t v = !valid ? ~0ull : (FLAT && rd == 0 && T >= 63) ? top[idx] : ld(idx);
      const uint64_t sib = swap_pairs64(v);
      const bool go_right = ((lane & 1) == 0) && valid && (idx + 1 < n) && !key_lt(v, sib, lb);
      const uint64_t right_mask = ballot(go_right);
      // scalar walk: path index per level, bit-packed (cur at level lv in bits)
      int cur = 0, taken = 0;
      uint32_t path_code = 0;  // 5 bits per level: index within level
#pragma unroll
      for (int lv = 1; lv <= 5; ++lv) {
        const int left_idx = ((pos + 1) << lv) - 1 + 2 * cur;
        if (taken == lv - 1 && left_idx < n) {
          const int left_lane = (1 << lv) - 2 + 2 * cur;
          cur = 2 * cur + (int)((right_mask >> left_lane) & 1);
          path_code |= (uint32_t)cur << (5 * (lv - 1));
          taken = lv;
        }
      }
      lev[rd] = taken;
      const int my_cur = (int)((path_code >> (5 * (r - 1))) & 31);
      on[rd] = lane < 62 && r <= taken && i == my_cur;
      val[rd] = v;
      posv[rd] = idx;
      pos = ((pos + 1) << taken) - 1 + cur;   // new path end
    }
    // bubble `last` up: first path entry (in path order) with last < v; it
    // and everything below keep their values, `last` lands on its parent slot
    int jr = -1, jl = 0;   // round / lane of the first such entry
#pragma unroll
    for (int rd = 0; rd < kRounds; ++rd) {
      const uint64_t g = ballot(on[rd] && key_lt(last, val[rd], lb));
      if (jr < 0 && g) { jr = rd; jl = first_lane(g); }
    }
    // moves: every path entry ABOVE the first greater one moves to its parent
    int target;  // slot receiving `last`
    if (jr < 0) {
      target = pos;  // last path entry (leaf) -- all entries moved up
    } else {
      const int lvl = jl < 2 ? 1 : jl < 6 ? 2 : jl < 14 ? 3 : jl < 30 ? 4 : 5;
      const int idx_j = ((start[jr] + 1) << lvl) - 1 + (jl - ((1 << lvl) - 2));
      target = (idx_j - 1) >> 1;   // its parent: path entry j-1 (or the root)
    }
#pragma unroll
    for (int rd = 0; rd < kRounds; ++rd) {
      const bool above = jr < 0 || rd < jr || (rd == jr && lane < jl);
      if (on[rd] && above) {
        const int parent = (posv[rd] - 1) >> 1;
        st(parent, val[rd]);
        mark(parent, val[rd]);
      }
    }
    if (lane == 0) { st(target, last); mark(target, last); }
  }

  // CPython heappush on a heap of n items (item lands at index <= n).
  __device__ void push(int n, uint64_t item) const {
    // ancestors a_l = ((n+1) >> l) - 1, l >= 1, exist while (n+1) >> l >= 1
    const int l = lane + 1;
    const int anc = lane < 30 ? ((n + 1) >> l) - 1 : -1;
    const bool valid = anc >= 0 && n > 0;
    const uint64_t v = valid ? ld(anc) : 0;
    const bool gt = valid && key_lt(item, v, lb);
    const int J = __popcll(ballot(gt));        // sorted path: a prefix from the bottom
    // moves: v_l -> a_{l-1} (a_0 = n) for l <= J ; item -> a_J
    const int dst = lane < 30 ? ((n + 1) >> (l - 1)) - 1 : 0;
    if (gt) { st(dst, v); mark(dst, v); }
    const int aJ = J == 0 ? n : ((n + 1) >> J) - 1;
    if (lane == 0) { st(aJ, item); mark(aJ, item); }
  }

  // index of the first DELETION in h[0, n), or -1: the bitmap for slots below
  // M, then (rarely: a deletion usually sits near the root, its time being
  // close) the keys themselves, 64 slots per step
  __device__ int first_deletion(int n) const {
    const int nb = n < M ? n : M;
    const int words = (nb + 31) >> 5;
    for (int base = 0; base < words; base += kWave) {
      const int wi = base + lane;
      uint32_t w = wi < words ? delmap[wi] : 0u;
      if (wi == words - 1 && (nb & 31)) w &= (1u << (nb & 31)) - 1;   // stale bits past the end
      const uint64_t b = ballot(w != 0);
      if (b) {
        const int fl = first_lane(b);
        const uint32_t fw = (uint32_t)readlane((int)w, fl);
        return ((base + fl) << 5) + (__ffs(fw) - 1);
      }
    }
    for (int base = nb; base < n; base += kWave) {
      const int i = base + lane;
      const uint64_t b = ballot(i < n && (ld(i) & 3) == (uint64_t)kDelKind);
      if (b) return base + first_lane(b);
    }
    return -1;
  }
};
using WaveHeap = WaveHeapT<false>;

}  // namespace fksd
