// k_replay_native_duo: one natively compiled program per workgroup of TWO
// waves that split a replay's dependency chain (latency regime: LLM-sized
// batches of a few dozen programs on <= 16 nodes).
//
// In the one-program-per-wave row kernel every event runs pop -> sift of the
// heap's last entry -> score -> commit -> push back to back on one wave,
// although the sift and the scoring are independent (s_memtime split:
// ~3.2k cycles of pop/sift, 2.9k-9.2k of scoring per event).  Here
//   * wave H owns the CPython heap (LDS top + HBM tail, RowHeap) and its
//     deletion bitmap: it pops an event, publishes the key in an LDS ring,
//     then sifts; a DELETION needs nothing back, so H runs ahead through
//     deletions (bounded by the ring); for a creation it waits for S's
//     verdict and pushes (the deletion entry of a placement, or -- after
//     computing the first-deletion repush time itself -- the re-queued pod);
//   * wave S owns the node registers, the waiting-class histogram, the
//     utilisation totals, the exact accumulators and the program: it replays
//     the events in order (node updates, scoring through the JIT function
//     pointer, argmax, GPU pick, snapshot schedule) and answers creations.
// The two waves of a workgroup are co-resident, and each waits on the other
// through LDS counters with release/acquire ordering and a bounded spin (a
// lost partner ends the replay with EXC_TIMEOUT instead of hanging).
// Event order, heap operations and arithmetic are exactly those of
// replay_rows (bit-identical results; tests/test_gpu_native.py).
#pragma once

#include "replay_rows.hip.h"

namespace fksd {

constexpr int kDuoRing = 64;                  // events H may run ahead of S
#ifndef FKS_DUO_SLEEP
#define FKS_DUO_SLEEP 1                       // s_sleep argument of a poll (0: busy poll)
#endif
constexpr uint32_t kDuoSpinCap = 1u << 26;    // polls before a wait is declared lost
enum DuoReply : int32_t { DUO_NONE = 0, DUO_PLACED = 1, DUO_FAIL = 2, DUO_ABORT = 3 };

struct DuoBox {
  uint64_t ev[kDuoRing];   // popped keys, ring (H -> S)
  uint64_t item;           // S -> H: heap entry to push after a placement
  uint32_t head;           // events published by H
  uint32_t tail;           // events consumed by S
  uint32_t rseq;           // creations answered by S (the event index + 1)
  int32_t code;            // DuoReply of the last answer
  uint32_t term;           // H: no more events
  uint32_t sabort;         // S: the replay was aborted (RowNativeArgs::abort) -- H stops too
  int32_t h_exc, n_repush, n_dropped;
};
// Scoring-wave state kept in LDS between events (16 lanes): the mutable node
// registers and waiting-class counters (16 int32 per lane) and the exact
// accumulators (RowAcc, 32 B per lane).  Nothing of it is live across the
// program call then: the JIT program may use every caller-saved VGPR below
// kJitVgprs, so whatever the scoring wave keeps in registers across the call
// must sit in the callee-saved blocks -- in registers this state pushed the
// kernel to 169 VGPRs (2 waves/SIMD: 4 programs per CU); in LDS it stays at
// the 128-VGPR floor (4 waves/SIMD: 8 programs per CU, 2,048 in flight).
constexpr int kDuoNodeInts = 16;   // cpu_left, mem_left, gpu_left, -, gml[8], wcnt[4]
constexpr size_t kDuoSBytes = (size_t)kRow * kDuoNodeInts * 4 + (size_t)kRow * 32;
__host__ __device__ inline size_t duo_lds_bytes(int n_pods, int T) {
  return rows_lds_bytes(n_pods, T, 1, true) + ((sizeof(DuoBox) + 15) & ~size_t(15)) + kDuoSBytes;
}

__device__ __forceinline__ uint32_t duo_ld(FKS_LDS uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void duo_st(FKS_LDS uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// CPython heappop's re-insertion of `last` at the root of a heap of n >= 1
// items, walked by a whole wave: lane j < 63 is node j (BFS order) of the
// 6-level subtree under the path end and holds that node's child pair, so a
// round descends six levels (the 16-lane RowHeap::pop_reinsert: four) -- the
// 8k-entry heap of the OpenB trace in two rounds instead of three.  anc / dir:
// BFS indices of node j's ancestors in the subtree / of those stepping right.
// Same moves and stores as RowHeap::pop_reinsert (bit-identical heap arrays).
__device__ void pop_reinsert64(const RowHeap& hp, int n, uint64_t last, int j, uint64_t anc, uint64_t dir) {
  const int k = 31 - __clz(j + 1);   // depth of node j in the subtree
  const int ki = j - ((1 << k) - 1);
  constexpr int kRounds = 4;          // 24 levels (host guarantees n < 2^20)
  int pos = 0, target = -1;
#pragma unroll
  for (int rd = 0; rd < kRounds; ++rd) {
    if (2 * pos + 1 >= n) break;     // pos is a leaf
    const int q = ((pos + 1) << k) - 1 + ki;
    const int c = 2 * q + 1;
    const bool valid = j < 63 && c < n;
    uint64_t vl = ~0ull, vr = ~0ull;
    if (valid) {
      const u64x2 pr = hp.ld_pair(c);
      vl = pr.x;
      vr = pr.y;
    }
    const bool go_r = valid && (c + 1 < n) && !(vl < vr);
    const uint64_t m = ballot(go_r);
    const uint64_t ex = ballot(valid);
    const bool on = valid && (ex & anc) == anc && ((m ^ dir) & anc) == 0;
    const uint64_t onm = ballot(on);
    const int jd = 63 - __clzll((long long)onm);   // deepest path parent
    const int kd = 31 - __clz(jd + 1);
    const int taken = kd + 1;                       // levels descended this round
    const int qd = ((pos + 1) << kd) - 1 + (jd - ((1 << kd) - 1));
    const int next = 2 * qd + 1 + (int)((m >> jd) & 1);
    const uint64_t v = go_r ? vr : vl;
    const uint64_t g = ballot(on && last < v);
    const int jl = g ? __ffsll((long long)g) - 1 : 64;
    if (on && j < jl) {   // moves up one level
      hp.st(q, v);
      hp.mark(q, v);
    }
    if (g) {
      const int kk = 31 - __clz(jl + 1);
      target = ((pos + 1) << kk) - 1 + (jl - ((1 << kk) - 1));
      break;
    }
    pos = next;
    if (taken < 6) break;   // reached a leaf
  }
  if (target < 0) target = pos;
  if (j == 0) { hp.st(target, last); hp.mark(target, last); }
}

// PROF: s_memtime phase split (diagnostics build), per wave into
// prof_out[16 * blockIdx.x + 8 * wave + phase] (H: pop, ring, sift, wait, push;
// S: wait, pod, score, verdict, delete, eval, args, call; `score` is the
// argmax after the call, `args` the node-state load, `call` the feasibility
// test, argument set-up and the program call)
// slot: the program's index into nat / out / table (the block index of a batch
// launch; a ring slot under k_native_service); hslot: the HBM heap slice used
// (per program in a batch, per resident workgroup in the service)
template <bool PROF = false>
__device__ void replay_duo(const DevWorkload& W, const DevWorkload* Wdev, uint64_t* gheap, DevResult* out,
                           RowNativeArgs nat, double* table, uint64_t* prof_out = nullptr, int slot = -1,
                           int hslot = -1) {
  uint64_t pacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t plast = 0;
  auto mark = [&](int ph) {
    if constexpr (PROF) {
      const uint64_t now = __builtin_amdgcn_s_memtime();
      pacc[ph] += now - plast;
      plast = now;
    }
  };
  auto flush = [&](int wv) {
    if constexpr (PROF) {
      if (lane_id() < 8) {
        uint64_t v = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) v = lane_id() == i ? pacc[i] : v;
        prof_out[16 * (size_t)blockIdx.x + 8 * wv + lane_id()] = v;
      }
    }
  };
  auto cold = [&]() {
    const DevWorkload* g = reinterpret_cast<const DevWorkload*>(uniu64(reinterpret_cast<uint64_t>(Wdev)));
    asm volatile("" : "+s"(g));
    return const_ptr(g);
  };
  extern __shared__ uint64_t lds_raw[];
  const int lane = lane_id();
  const int wave = (int)(threadIdx.x >> 6);   // 0: H (heap), 1: S (scoring)
  const int p = slot >= 0 ? slot : (int)blockIdx.x;
  const int hs = hslot >= 0 ? hslot : p;
  const int N = W.n_pods;
  const int T = W.heap_top;
  const int lb = W.low_bits, nb = W.node_bits, rb = W.rank_bits;
  const int tshift = rb + lb;
  const uint64_t time_max = (W.time_bits >= 63) ? ~0ull : ((1ull << W.time_bits) - 1);
  int jv = lane & 15;
  const bool node_valid = jv < W.n_nodes;

  // LDS: [weights area (unused) | class values | node constants | bitmap | heap top | constant block | box]
  FKS_LDS uint64_t* lds = lds_ptr(lds_raw);
  FKS_LDS int32_t* cls_lds = reinterpret_cast<FKS_LDS int32_t*>(lds + kRowsPerWave * kWeights);
  FKS_LDS char* rowbase = reinterpret_cast<FKS_LDS char*>(lds + kRowsPerWave * kWeights) + kRowClassBytes;
  FKS_LDS int32_t* ntab = cls_lds + kRow * kRowClassSlots;
  FKS_LDS int64_t* kcp = reinterpret_cast<FKS_LDS int64_t*>(rowbase + rows_row_bytes(N, T));
  FKS_LDS DuoBox* box = reinterpret_cast<FKS_LDS DuoBox*>(reinterpret_cast<FKS_LDS char*>(lds) + rows_lds_bytes(N, T, 1, true));
  FKS_LDS int32_t* sstate = reinterpret_cast<FKS_LDS int32_t*>(reinterpret_cast<FKS_LDS char*>(box) +
                                                                ((sizeof(DuoBox) + 15) & ~size_t(15)));
  FKS_LDS uint64_t* sacc = reinterpret_cast<FKS_LDS uint64_t*>(sstate + kRow * kDuoNodeInts);

  if (wave == 0) {
    if (lane < W.n_classes) cls_lds[lane] = *global_ptr(&W.class_value[lane]);
    fill_node_tables(W, ntab, lane);
    if (lane == 0) {
      box->item = 0; box->head = 0; box->tail = 0; box->rseq = 0; box->code = DUO_NONE; box->term = 0;
      box->sabort = 0;
      box->h_exc = EXC_NONE; box->n_repush = 0; box->n_dropped = 0;
    }
  } else {
    const FKS_GLOBAL int64_t* ksrc = global_ptr(nat.kc + *global_ptr(&nat.koff[p]));
    for (int i = lane; i < kKcLds; i += kWave) kcp[i] = ksrc[i];
  }
  __syncthreads();
  // H uses all 64 lanes for the pop's subtree walk (its 16-lane heap routines
  // run duplicated on the other rows: same values, same stores); rows 1-3 of S
  // take no part (no barrier follows)
  if (wave == 1 && lane >= kRow) return;

  if (wave == 0) {
    // ================= H: the heap
    RowHeap heap;
    heap.delmap = reinterpret_cast<FKS_LDS uint32_t*>(rowbase);
    heap.top = reinterpret_cast<FKS_LDS uint64_t*>(rowbase + (size_t)lds_delmap_words(N) * 4);
    heap.h = global_ptr(gheap + (size_t)hs * row_heap_entries(N));
    heap.bind();
    heap.T = T;
    heap.lb = lb;
    heap.j = jv;
    heap.rbase = 0;
    heap.anc = heap.dir = 0;   // (RowHeap::pop_reinsert is not used here)
    uint64_t anc64 = 0, dir64 = 0;
    for (int x = lane; x > 0 && x < 63; x = (x - 1) >> 1) {
      const int a = (x - 1) >> 1;
      anc64 |= 1ull << a;
      if ((x & 1) == 0) dir64 |= 1ull << a;   // even BFS index = right child
    }
    const FKS_GLOBAL u64x2* heap_src = reinterpret_cast<const FKS_GLOBAL u64x2*>(global_ptr(W.heap0p));
    for (int i = lane; i < row_heap_entries(N) / 2; i += kWave) {
      const u64x2 v = heap_src[i];
      if (2 * i < T + 1) *reinterpret_cast<FKS_LDS u64x2*>(heap.top + 2 * i) = v;
      else *reinterpret_cast<FKS_GLOBAL u64x2*>(heap.h + 2 * i) = v;
    }
    for (int i = lane; i < lds_delmap_words(N); i += kWave) heap.delmap[i] = 0u;
    __builtin_amdgcn_s_waitcnt(0);
    int n = N, n_repush = 0, n_dropped = 0;
    int32_t hexc = EXC_NONE;
    uint32_t k = 0, tail_seen = 0;
    // publish event k (a free ring slot first: S consumes in order; the
    // consumer count is re-read only when the last value seen says the ring
    // may be full)
    auto publish = [&](uint64_t key) -> bool {
      uint32_t spins = 0;
      while (k - tail_seen >= (uint32_t)kDuoRing) {
        tail_seen = duo_ld(&box->tail);
        if (k - tail_seen < (uint32_t)kDuoRing) break;
        if (duo_ld(&box->sabort)) return false;
        __builtin_amdgcn_s_sleep(FKS_DUO_SLEEP);
        if (++spins > kDuoSpinCap) { hexc = EXC_TIMEOUT; return false; }
      }
      if (lane == 0) box->ev[k % kDuoRing] = key;
      if (lane == 0) duo_st(&box->head, k + 1);
      return true;
    };
    bool published = false;   // event k already published (the previous push's forecast)
    uint64_t top = 0;
    if constexpr (PROF) plast = __builtin_amdgcn_s_memtime();
    while (n > 0) {
      asm volatile("" : "+v"(jv));
      heap.j = jv;
      if (!published) {
        top = heap.ld(0);
        mark(0);
        if (!publish(top)) break;   // published before `last` is even read
      }
      published = false;
      const uint64_t last = heap.ld(n - 1);
      --n;
      mark(1);
      if (n > 0) pop_reinsert64(heap, n, last, lane, anc64, dir64);
      mark(2);
      if ((int)(top & 3) != kDelete) {
        uint32_t spins = 0;
        while (duo_ld(&box->rseq) != k + 1) {
          if (duo_ld(&box->sabort)) { hexc = EXC_TIMEOUT; break; }
          __builtin_amdgcn_s_sleep(FKS_DUO_SLEEP);
          if (++spins > kDuoSpinCap) { hexc = EXC_TIMEOUT; break; }
        }
        if (hexc != EXC_NONE) break;
        mark(3);
        const int code = box->code;
        if (code == DUO_ABORT) break;   // S holds the exception
        uint64_t item = box->item;
        if (code == DUO_FAIL) {
          item = 0;
          const int rank = (int)((top >> lb) & ((1ull << rb) - 1));
          const int f = heap.first_deletion(n);
          if (f >= 0) {
            const uint64_t nt = (heap.ld(f) >> tshift) + 1;
            if (nt > time_max) { hexc = EXC_UNSUPPORTED; break; }
            item = (nt << tshift) | ((uint64_t)rank << lb) | kRetry;
            ++n_repush;
          } else {
            ++n_dropped;
          }
        }
        if (item != 0) {
          // the next pop returns min(root, item) (keys are unique): publish it
          // before the push itself, so S starts the next event meanwhile
          const uint64_t root = n > 0 ? heap.ld(0) : ~0ull;
          const uint64_t next = item < root ? item : root;
          ++k;
          if (!publish(next)) break;
          published = true;
          top = next;
          heap.push(n, item);
          ++n;
          mark(4);
          continue;
        }
        mark(4);
      }
      ++k;
    }
    flush(0);
    if (lane == 0) {
      box->h_exc = hexc;
      box->n_repush = n_repush;
      box->n_dropped = n_dropped;
      duo_st(&box->term, 1u);
    }
    return;
  }

  // ================= S: nodes, program, evaluator
  // wave-uniform by construction (one program per workgroup): read it into
  // SGPRs so the call is a single direct s_swappc -- a VGPR-held pointer
  // (the service path loads `nat` through the ring) makes LLVM wrap the
  // call in a readfirstlane waterfall loop
  const uint64_t fne = uniu64(*global_ptr(&nat.fn[p]));
  const ProgFn prog = prog_of(fne);
  const bool feas_pro = prog_feas(fne);   // call only for feasible nodes
  // this lane's node state and accumulators in LDS (kDuoSBytes above)
  typedef int v4i __attribute__((ext_vector_type(4)));
  FKS_LDS v4i* my = reinterpret_cast<FKS_LDS v4i*>(sstate + jv * kDuoNodeInts);
  FKS_LDS uint64_t* myacc = sacc + jv * 4;
  {
    const FKS_CONST DevWorkload* Wb = cold();
    v4i a = {Wb->cpu_left0[jv], Wb->mem_left0[jv], Wb->gpu_left0[jv], 0};
    v4i g0 = {Wb->gml_left0[jv * kGmax + 0], Wb->gml_left0[jv * kGmax + 1], Wb->gml_left0[jv * kGmax + 2],
              Wb->gml_left0[jv * kGmax + 3]};
    v4i g1 = {Wb->gml_left0[jv * kGmax + 4], Wb->gml_left0[jv * kGmax + 5], Wb->gml_left0[jv * kGmax + 6],
              Wb->gml_left0[jv * kGmax + 7]};
    my[0] = a; my[1] = g0; my[2] = g1; my[3] = v4i{0, 0, 0, 0};
    myacc[0] = 0; myacc[1] = 0; myacc[2] = 0; myacc[3] = 0;
  }
  const FKS_LDS int32_t* ncon = ntab + jv * kNodeConsts;
  // node registers of this lane, fresh from LDS (constants from the node table)
  auto load_nr = [&]() {
    NodeRegs<1> r;
    const v4i a = my[0], g0 = my[1], g1 = my[2];
    r.cpu_left[0] = a.x; r.mem_left[0] = a.y; r.gpu_left[0] = a.z;
    r.gw[0][0] = g0.x; r.gw[0][1] = g0.y; r.gw[0][2] = g0.z; r.gw[0][3] = g0.w;
    r.gw[0][4] = g1.x; r.gw[0][5] = g1.y; r.gw[0][6] = g1.z; r.gw[0][7] = g1.w;
    r.cpu_total[0] = ncon[0]; r.mem_total[0] = ncon[1]; r.ngpus[0] = ncon[2]; r.gmt1[0] = ncon[3];
    return r;
  };
  auto store_nr = [&](const NodeRegs<1>& r) {
    my[0] = v4i{r.cpu_left[0], r.mem_left[0], r.gpu_left[0], 0};
    my[1] = v4i{r.gw[0][0], r.gw[0][1], r.gw[0][2], r.gw[0][3]};
    my[2] = v4i{r.gw[0][4], r.gw[0][5], r.gw[0][6], r.gw[0][7]};
  };
  auto load_acc = [&]() {
    RowAcc a;
    a.lo = myacc[0]; a.hi = myacc[1];
    a.count = (int32_t)(uint32_t)myacc[2]; a.inexact = (int32_t)(uint32_t)myacc[3];
    return a;
  };
  auto store_acc = [&](const RowAcc& a) {
    myacc[0] = a.lo; myacc[1] = a.hi;
    myacc[2] = (uint64_t)(uint32_t)a.count; myacc[3] = (uint64_t)(uint32_t)a.inexact;
  };
  FKS_LDS int32_t* wcnt = sstate + jv * kDuoNodeInts + 12;   // waiting-class counters
  int32_t used_cpu = (int32_t)cold()->used_cpu0, used_mem = (int32_t)cold()->used_mem0;
  int32_t used_gcnt = (int32_t)cold()->used_gcnt0, used_gml = (int32_t)cold()->used_gmilli0;
  int32_t processed = 0, next_fire = INT32_MAX;
  int ksnap = 0;
  double thr = cold()->thr_after_fire;
  // per-event flags / pointers of the scoring path, read once (the scoring wave
  // carries far fewer live values than the row kernel, so they stay in SGPRs)
  const bool trace_hash = cold()->trace_hash != 0;
  const bool first_fit_alloc = cold()->first_fit_alloc != 0;
  const int64_t* gmem_node = cold()->gmem_total + (size_t)jv * kGmax;
  if (cold()->n_fire > 0) {
    next_fire = (int32_t)*global_ptr(&cold()->snap_fire[0]);
  } else {
    int32_t c = 1;
    while ((double)c / (double)N < thr) ++c;
    next_fire = c;
  }
  uint64_t hsh = 0xcbf29ce484222325ull;
  int32_t exc = EXC_NONE;
  auto reply = [&](int code, uint64_t item, uint32_t k) {
    if (jv == 0) {
      box->item = item;
      box->code = code;
      duo_st(&box->rseq, k + 1);
    }
  };
  uint32_t k = 0;
  if constexpr (PROF) plast = __builtin_amdgcn_s_memtime();
  for (;;) {
    asm volatile("" : "+v"(jv));
    if ((k & 1023u) == 1023u) {
      if (nat.abort != nullptr && __hip_atomic_load(nat.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) {
        exc = EXC_TIMEOUT;   // the host gave up on the replays in flight (a stopping run)
        if (jv == 0) duo_st(&box->sabort, 1u);
        break;
      }
      if (nat.max_events != 0u && k >= nat.max_events) {
        // past the caller's event budget (a resource limit: a policy whose failed
        // placements re-queue for millions of events holds a workgroup for tens
        // of seconds); the row says so and carries no score
        exc = EXC_EVENTS;
        if (jv == 0) duo_st(&box->sabort, 1u);
        break;
      }
    }
    // next event, or the end of the replay
    uint32_t spins = 0;
    bool have = false;
    for (;;) {
      if (duo_ld(&box->head) > k) { have = true; break; }
      if (duo_ld(&box->term)) { have = duo_ld(&box->head) > k; break; }
      __builtin_amdgcn_s_sleep(FKS_DUO_SLEEP);
      if (++spins > kDuoSpinCap) { exc = EXC_TIMEOUT; break; }
    }
    if (!have) break;
    mark(0);
    // the event and its pod are wave-uniform: SGPRs, not VGPRs across the call
    const uint64_t top = uniu64(box->ev[k % kDuoRing]);
    if (jv == 0) duo_st(&box->tail, k + 1);
    const int rank = (int)((top >> lb) & ((1ull << rb) - 1));
    const v4i precv = *reinterpret_cast<const FKS_GLOBAL v4i*>(global_ptr(&W.pod[rank]));
    const int kind = (int)(top & 3);
    const int64_t t = (int64_t)(top >> tshift);
    PodView pod;
    const int pw = uni(precv.w);
    pod.cpu = uni(precv.x); pod.mem = uni(precv.y); pod.dur = uni(precv.z);
    pod.gmilli = pw & 0xFFFF; pod.ngpu = (pw >> 16) & 0xFF; pod.cls = (pw >> 24) & 0xFF;
    pod.ctime = t; pod.rank = rank;
    if constexpr (PROF) __builtin_amdgcn_s_waitcnt(0);
    mark(1);

    if (kind == kDelete) {
      const int node = (int)((top >> 2) & ((1u << nb) - 1));
      const int mask = (int)((top >> (2 + nb)) & 0xFF);
      if (jv == node) {
        NodeRegs<1> nr = load_nr();
        nr.cpu_left[0] += pod.cpu;
        nr.mem_left[0] += pod.mem;
        nr.gpu_left[0] += pod.ngpu;
#pragma unroll
        for (int g = 0; g < kGmax; ++g)
          if ((mask >> g) & 1) nr.g_add(0, g, pod.gmilli);
        store_nr(nr);
      }
      used_cpu -= pod.cpu; used_mem -= pod.mem; used_gcnt -= pod.ngpu;
      used_gml -= pod.gmilli * __popc(mask);
      if (trace_hash) hsh = mix_event(hsh, ((uint64_t)(uint32_t)rank << 2) | 1, (uint64_t)t);
      mark(4);
    } else {
      int lexc = EXC_NONE;
      int64_t s = 0;
      const NodeRegs<1> na = load_nr();   // call arguments; dead after the call
      mark(6);
      if (node_valid && (!feas_pro || feasible<1>(0, na, pod))) {
        const NodeRegs<1>& nr = na;
        const int32_t* gl = nr.gw[0];   // NPASS 1: unpacked
        int32_t gt[kGmax];
#pragma unroll
        for (int g = 0; g < kGmax; ++g) gt[g] = nr.gt(0, g);
        s = prog(nr.cpu_left[0], nr.cpu_total[0], nr.mem_left[0], nr.mem_total[0], pack_gpu_ng(nr.gpu_left[0], nr.ngpus[0]),
                 gl[0], gl[1], gl[2], gl[3], gl[4], gl[5], gl[6], gl[7], gt[0], gt[1], gt[2], gt[3], gt[4], gt[5],
                 gt[6], gt[7], gmem_node, pod.cpu, pod.mem,
                 pod.gmilli | (pod.ngpu << 16), pod.ctime, pod.dur, kcp);
        if (s < 0) { lexc = (int)(-s); s = 0; }
      }
      mark(7);
      NodeRegs<1> nr = load_nr();         // re-read after the call (nothing kept across it)
      const uint32_t bad = row_ballot(lexc != EXC_NONE, 0);
      if (bad) {
        exc = row_read(lexc, 0, __ffs(bad) - 1);
        reply(DUO_ABORT, 0, k);
        break;
      }
      const int64_t m = (int64_t)row_max_u64((uint64_t)s);
      const int best_node = m > 0 ? __ffs(row_ballot(s == m, 0)) - 1 : -1;
      mark(2);
      if (best_node < 0) {
        // failed placement: S keeps the metrics, H computes the repush
        if (kind == kFresh && pod.ngpu > 0 && jv == (pod.cls & 15)) wcnt[pod.cls >> 4] += 1;
        reply(DUO_FAIL, 0, k);   // H's first-deletion scan overlaps the fragmentation sum
        double frag = 0.0;
        int mcls = -1;
        const v4i wc = *reinterpret_cast<FKS_LDS v4i*>(wcnt);
#pragma unroll
        for (int sl = 0; sl < kRowClassSlots; ++sl) {
          const int32_t w = sl == 0 ? wc.x : sl == 1 ? wc.y : sl == 2 ? wc.z : wc.w;
          const uint32_t b = row_ballot(w > 0, 0);
          if (mcls < 0 && b) mcls = sl * kRow + __ffs(b) - 1;
        }
        if (mcls >= 0) {
          const int mv = cls_lds[mcls];
          int64_t stranded = 0;
#pragma unroll
          for (int g = 0; g < kGmax; ++g) {
            const int l = nr.g(0, g);
            if (g < nr.ngpus[0] && 0 < l && l < mv) stranded += l;
          }
          stranded = row_sum_i64(node_valid ? stranded : 0);
          const int64_t tg = cold()->tot_gmilli;
          frag = tg > 0 ? (double)stranded / (double)tg : 0.0;
        }
        if (jv == 4) {
          RowAcc acc = load_acc();
          acc.add(4, frag, jv);
          store_acc(acc);
        }
        if (trace_hash) hsh = mix_event(hsh, ((uint64_t)(uint32_t)rank << 2) | 2, (uint64_t)t);
      } else {
        int gmask = 0, ok = 1;
        if (pod.ngpu > 0) {
          int myok = 1;
          const int mymask = pick_gpus<1>(nr, 0, pod.gmilli, pod.ngpu, first_fit_alloc, myok);
          const int packed = row_read(mymask | (myok << 8), 0, best_node);
          gmask = packed & 0xFF;
          ok = packed >> 8;
        }
        if (!ok) { exc = EXC_ALLOC; reply(DUO_ABORT, 0, k); break; }
        const uint64_t dt = (uint64_t)(t + pod.dur);
        if (t + pod.dur < 0 || dt > time_max) { exc = EXC_UNSUPPORTED; reply(DUO_ABORT, 0, k); break; }
        // answer first: H's push runs while S commits
        reply(DUO_PLACED, (dt << tshift) | ((uint64_t)rank << lb) | ((uint64_t)gmask << (2 + nb)) |
                              ((uint64_t)best_node << 2) | kDelete, k);
        if (jv == best_node) {
          nr.cpu_left[0] -= pod.cpu;
          nr.mem_left[0] -= pod.mem;
          nr.gpu_left[0] -= pod.ngpu;
#pragma unroll
          for (int g = 0; g < kGmax; ++g)
            if ((gmask >> g) & 1) nr.g_add(0, g, -pod.gmilli);
          store_nr(nr);
        }
        used_cpu += pod.cpu; used_mem += pod.mem; used_gcnt += pod.ngpu;
        used_gml += pod.gmilli * __popc(gmask);
        if (kind == kRetry && pod.ngpu > 0 && jv == (pod.cls & 15)) wcnt[pod.cls >> 4] -= 1;
        if (trace_hash)
          hsh = mix_event(hsh, ((uint64_t)(uint32_t)rank << 2), ((uint64_t)t << 8) ^ (uint64_t)best_node);
      }
      mark(3);
    }
    // evaluator hook (host-precomputed snapshot schedule), as in replay_rows
    ++processed;
    if (processed >= next_fire) {
      const FKS_CONST DevWorkload* Ws = cold();
      const double r0 = Ws->tot_cpu > 0 ? (double)used_cpu / (double)Ws->tot_cpu : 0.0;
      const double r1 = Ws->tot_mem > 0 ? (double)used_mem / (double)Ws->tot_mem : 0.0;
      const double r2 = Ws->tot_gcnt > 0 ? (double)used_gcnt / (double)Ws->tot_gcnt : 0.0;
      const double r3 = Ws->tot_gmilli > 0 ? (double)used_gml / (double)Ws->tot_gmilli : 0.0;
      if (jv < 4) {
        RowAcc acc = load_acc();
        acc.add(0, r0, jv); acc.add(1, r1, jv); acc.add(2, r2, jv); acc.add(3, r3, jv);
        store_acc(acc);
      }
      ++ksnap;
      if (ksnap < Ws->n_fire) {
        next_fire = (int32_t)*global_ptr(&Ws->snap_fire[ksnap]);
      } else {
        if (ksnap > Ws->n_fire) thr += Ws->snapshot_interval;
        int32_t c = processed + 1;
        while ((double)c / (double)N < thr) ++c;
        next_fire = c;
      }
    }
    mark(5);
    ++k;
  }
  flush(1);
  // wait for H to finish (it may still be pushing / scanning), then take its counters
  {
    uint32_t spins = 0;
    while (!duo_ld(&box->term)) {
      __builtin_amdgcn_s_sleep(FKS_DUO_SLEEP);
      if (++spins > kDuoSpinCap) { exc = exc != EXC_NONE ? exc : EXC_TIMEOUT; break; }
    }
  }
  if (exc == EXC_NONE && box->h_exc != EXC_NONE) {
    exc = box->h_exc;
    --processed;   // H aborted on this event (repush time overflow) before it counted
  }
  const int n_repush = box->n_repush, n_dropped = box->n_dropped;

  // ---------------- result (replay_rows' write-back, fused evaluator)
  const RowAcc acc = load_acc();
  const int64_t n_snap = row_read(acc.count, 0, 0);
  const int64_t n_frag = row_read(acc.count, 0, 4);
  const int inexact = row_ballot(jv < 5 && acc.inexact != 0, 0) != 0;
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
    o->n_repush = n_repush;
    o->max_nodes = 0;
    o->hash = hsh;
    o->exc = exc;
    o->inexact = inexact;
  }
  if (table) {
    double av = 0.0;
    if (jv < 5 && acc.count > 0)
      av = fixed_div_round_dev((i128)(((u128)acc.hi << 64) | acc.lo), (uint64_t)acc.count);
    const uint64_t ab = (uint64_t)__double_as_longlong(av);
    double avg[5];
#pragma unroll
    for (int q = 0; q < 5; ++q)
      avg[q] = __longlong_as_double((long long)(((uint64_t)(uint32_t)row_read((int)(ab >> 32), 0, q) << 32) |
                                                (uint32_t)row_read((int)(uint32_t)ab, 0, q)));
    double score = 0.0;
    if (exc == EXC_NONE && n_snap > 0 && n_dropped == 0) {
      const double overall = (avg[0] + avg[1] + avg[2] + avg[3]) / 4.0;
      const double pen = avg[4] < 0.1 ? avg[4] : 0.1;
      double sc = overall - pen;
      sc = sc < 1.0 ? sc : 1.0;
      score = sc > 0.0 ? sc : 0.0;
    }
    const bool ok = exc == EXC_NONE;
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
      case 12: v = (double)(hsh >> 11); break;
      default: break;
    }
    if (!ok && jv != 10) v = 0.0;
    if (jv < 13) table[(size_t)p * 13 + jv] = v;
  }
}

}  // namespace fksd

// k_native_service (the resident program service built on replay_duo):
// replay_kernels.hip, where its kernel arguments are defined.
