// k_replay_builtin_duo: the 256-node (NPASS 4) builtin-family replay split
// over TWO waves of one workgroup -- replay_one's event loop with its heap and
// its nodes on different waves.
//
// On 256-node clusters one event of the one-wave kernel runs the CPython
// heappop (5.4k cycles: four 5-level subtree gathers, the last from HBM) and
// the scoring of the four node slots per lane (5.3k) back to back
// (profiles/r3_config5_wave_phase_split.json), although the sift of the
// heap's last entry and the scoring of the popped pod are independent.  Here,
// with the handshake of replay_duo.hip.h (DuoBox: LDS ring of popped keys,
// S -> H verdicts),
//   * wave H owns the heap (WaveHeapT: LDS top + HBM slice, deletion bitmap):
//     it pops, publishes the key, sifts; deletions need nothing back, so H runs
//     ahead through them; for a creation it waits for S's verdict and pushes
//     the placement's deletion entry or -- computing the repush time itself
//     (first deletion in array order, or the earliest) -- the re-queued pod;
//   * wave S owns the node registers (NodeRegs<4>), the waiting-class
//     histogram, the utilisation totals and the exact accumulators, and runs
//     the scorer, the argmax, the GPU pick and the snapshot schedule.
// Event order, heap operations and arithmetic are replay_one's (bit-identical
// results; tests/test_gpu_engine.py compares the two kernels row for row).
// Not covered: the invariant check (it reads heap and nodes together; the
// host keeps replay_one for check_invariants runs).
#pragma once

#include "replay.hip.h"
#include "replay_duo.hip.h"

namespace fksd {

__host__ __device__ inline size_t wave_duo_box_bytes() { return (sizeof(DuoBox) + 15) & ~size_t(15); }

template <int NPASS, class Scorer, bool FLAT>
__device__ void replay_wave_duo(const DevWorkload& W, const DevWorkload* Wcold, Scorer& scorer,
                                FKS_GLOBAL uint64_t* hbuf, FKS_LDS uint64_t* htop, int T, FKS_LDS uint32_t* delmap,
                                FKS_LDS DuoBox* box, DevResult* out) {
  const int lane = lane_id();
  const int wave = (int)(threadIdx.x >> 6);   // 0: H (heap), 1: S (nodes, scorer, evaluator)
  const int lb = W.low_bits, nb = W.node_bits, rb = W.rank_bits;
  const int tshift = rb + lb;
  const uint64_t time_max = (W.time_bits >= 63) ? ~0ull : ((1ull << W.time_bits) - 1);
  const int N = W.n_pods;
  auto cold = [&]() {
    const DevWorkload* g = reinterpret_cast<const DevWorkload*>(uniu64(reinterpret_cast<uint64_t>(Wcold)));
    asm volatile("" : "+s"(g));
    return const_ptr(g);
  };

  if (wave == 0) {
    // ================= H: the heap
    WaveHeapT<FLAT> heap;
    heap.h = hbuf;
    heap.top = htop;
    heap.bind();
    heap.T = T;
    heap.delmap = delmap;
    heap.M = W.delmap_slots;
    heap.lb = lb;
    heap.lane = lane;
    for (int i = lane; i < N; i += kWave) heap.st(i, W.heap0[i]);
    for (int i = lane; i < (W.delmap_slots >> 5); i += kWave) heap.delmap[i] = 0u;
    if (lane == 0) {
      box->item = 0; box->head = 0; box->tail = 0; box->rseq = 0; box->code = DUO_NONE; box->term = 0;
      box->sabort = 0;
      box->h_exc = EXC_NONE; box->n_repush = 0; box->n_dropped = 0;
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    const bool earliest = cold()->repush_earliest != 0;
    int n = N, n_repush = 0, n_dropped = 0;
    int32_t hexc = EXC_NONE;
    uint32_t k = 0, tail_seen = 0;
    auto publish = [&](uint64_t key) -> bool {
      uint32_t spins = 0;
      while (k - tail_seen >= (uint32_t)kDuoRing) {
        tail_seen = duo_ld(&box->tail);
        if (k - tail_seen < (uint32_t)kDuoRing) break;
        __builtin_amdgcn_s_sleep(FKS_DUO_SLEEP);
        if (++spins > kDuoSpinCap) { hexc = EXC_TIMEOUT; return false; }
      }
      if (lane == 0) box->ev[k % kDuoRing] = key;
      if (lane == 0) duo_st(&box->head, k + 1);
      return true;
    };
    bool published = false;   // event k already published (the previous push's forecast)
    uint64_t top = 0;
    while (n > 0) {
      {   // lane-derived predicates recomputed per event (replay_one)
        int ol = lane;
        asm volatile("" : "+v"(ol));
        heap.lane = ol;
      }
      if (!published) {
        top = uniu64(heap.ld_u(0));
        if (!publish(top)) break;
      }
      published = false;
      const uint64_t last = uniu64(heap.ld_u(n - 1));
      --n;
      if (n > 0) heap.pop_reinsert(n, last);
      if ((int)(top & 3) != kDelete) {
        uint32_t spins = 0;
        while (duo_ld(&box->rseq) != k + 1) {
          __builtin_amdgcn_s_sleep(FKS_DUO_SLEEP);
          if (++spins > kDuoSpinCap) { hexc = EXC_TIMEOUT; break; }
        }
        if (hexc != EXC_NONE) break;
        const int code = box->code;
        if (code == DUO_ABORT) break;   // S holds the exception
        uint64_t item = box->item;
        if (code == DUO_FAIL) {
          item = 0;
          const int rank = (int)((top >> lb) & ((1ull << rb) - 1));
          int64_t anchor = -1;
          if (!earliest) {
            const int f = heap.first_deletion(n);
            if (f >= 0) anchor = (int64_t)(uniu64(heap.ld(f)) >> tshift);
          } else {
            uint64_t mn = ~0ull;
            for (int base = 0; base < n; base += kWave) {
              const int i = base + lane;
              uint64_t tv = ~0ull;
              if (i < n) { const uint64_t kk = heap.ld(i); if ((kk & 3) == kDelete) tv = kk >> tshift; }
              tv = ~wave_max_u64(~tv);
              mn = tv < mn ? tv : mn;
            }
            anchor = mn == ~0ull ? -1 : (int64_t)mn;
          }
          if (anchor >= 0) {
            const uint64_t nt = (uint64_t)(anchor + 1);
            if (nt > time_max) { hexc = EXC_UNSUPPORTED; break; }
            item = (nt << tshift) | ((uint64_t)rank << lb) | kRetry;
            ++n_repush;
          } else {
            ++n_dropped;
          }
        }
        if (item != 0) {
          // the next pop returns min(root, item) ((time, rank) keys are
          // unique): publish it before the push, S starts on it meanwhile
          const uint64_t root = n > 0 ? uniu64(heap.ld_u(0)) : ~0ull;
          const uint64_t next = item < root ? item : root;
          ++k;
          if (!publish(next)) break;
          published = true;
          top = next;
          heap.push(n, item);
          ++n;
          continue;
        }
      }
      ++k;
    }
    if (lane == 0) {
      box->h_exc = hexc;
      box->n_repush = n_repush;
      box->n_dropped = n_dropped;
      duo_st(&box->term, 1u);
    }
    return;
  }

  // ================= S: nodes, scorer, evaluator
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
  constexpr int KP = 4;  // waiting histogram: class k -> lane k%64, slot k/64
  int32_t wcnt[KP];
#pragma unroll
  for (int q = 0; q < KP; ++q) wcnt[q] = 0;
  int64_t used_cpu = W.used_cpu0, used_mem = W.used_mem0, used_gcnt = W.used_gcnt0, used_gml = W.used_gmilli0;
  LaneAcc acc;   // 0-3: utilisation snapshots, 4: fragmentation
  acc.init();
  int64_t processed = 0;
  int ksnap = 0;
  const int n_fire = W.n_fire;
  int64_t next_fire = n_fire > 0 ? W.snap_fire[0] : INT64_MAX;
  double thr = W.thr_after_fire;
  uint64_t hsh = 0xcbf29ce484222325ull;
  int32_t exc = EXC_NONE;
  __syncthreads();
  auto reply = [&](int code, uint64_t item, uint32_t kk) {
    if (lane == 0) {
      box->item = item;
      box->code = code;
      duo_st(&box->rseq, kk + 1);
    }
  };
  uint32_t k = 0;
  for (;;) {
    const FKS_CONST DevWorkload* Wc = cold();
    {
      const int4* c = reinterpret_cast<const int4*>(uniu64(reinterpret_cast<uint64_t>(nr.cst)));
      asm volatile("" : "+s"(c));
      nr.cst = c;
    }
    uint32_t spins = 0;
    bool have = false;
    for (;;) {
      if (duo_ld(&box->head) > k) { have = true; break; }
      if (duo_ld(&box->term)) { have = duo_ld(&box->head) > k; break; }
      __builtin_amdgcn_s_sleep(FKS_DUO_SLEEP);
      if (++spins > kDuoSpinCap) { exc = EXC_TIMEOUT; break; }
    }
    if (!have) break;
    const uint64_t top = uniu64(box->ev[k % kDuoRing]);
    if (lane == 0) duo_st(&box->tail, k + 1);
    const int rank = (int)((top >> lb) & ((1ull << rb) - 1));
    const int4 precv = load_vgpr(&W.pod[rank]);
    const int kind = (int)(top & 3);
    const int64_t t = (int64_t)(top >> tshift);
    PodView pod;
    const int pw = uni(precv.w);
    pod.cpu = uni(precv.x); pod.mem = uni(precv.y); pod.dur = uni(precv.z);
    pod.gmilli = pw & 0xFFFF; pod.ngpu = (pw >> 16) & 0xFF; pod.cls = (pw >> 24) & 0xFF;
    pod.ctime = t; pod.rank = rank;
    pod.cm = W.pod_cm[rank];

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
    } else {
      // score all nodes, argmax (first node wins ties), as replay_one
      uint64_t lbest = 0;
      int lst = 0;
#pragma unroll
      for (int ps = 0; ps < NPASS; ++ps) {
        const bool valid = (ps * kWave + lane) < W.n_nodes;
        int lexc = EXC_NONE;
        const uint64_t s = valid ? (uint64_t)scorer.template score<NPASS>(ps, nr, pod, lexc) : 0;
        if (valid && lexc != EXC_NONE && (lst >> 8) == 0) lst |= (lexc << 8) | (ps << 2);
        if (s > lbest) { lbest = s; lst = (lst & ~3) | ps; }
      }
      if (ballot((lst >> 8) != 0)) {
#pragma unroll
        for (int ps = 0; ps < NPASS; ++ps) {
          const uint64_t b = ballot((lst >> 8) != 0 && ((lst >> 2) & 3) == ps);
          if (b) { exc = readlane(lst >> 8, first_lane(b)); break; }
        }
        reply(DUO_ABORT, 0, k);
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

      if (best_node < 0) {
        // failed placement: S keeps the metrics, H computes the repush
        reply(DUO_FAIL, 0, k);
        if (kind == kFresh && pod.ngpu > 0) {
#pragma unroll
          for (int q = 0; q < KP; ++q)
            if (q * kWave + lane == pod.cls) wcnt[q] += 1;
        }
        double frag = 0.0;
        int mcls = -1;
#pragma unroll
        for (int q = 0; q < KP; ++q) {
          const uint64_t b = ballot(wcnt[q] > 0);
          if (mcls < 0 && b) mcls = q * kWave + first_lane(b);
        }
        if (mcls >= 0) {
          const int mv = const_ptr(Wc->class_value)[mcls];
          int64_t stranded = 0;
#pragma unroll
          for (int ps = 0; ps < NPASS; ++ps)
#pragma unroll
            for (int j = 0; j < kGmax; ++j) {
              const int l = nr.g(ps, j);
              if (j < nr.ngp(ps) && 0 < l && l < mv) stranded += l;
            }
          stranded = wave_sum_i64(stranded);
          const int64_t tg = Wc->tot_gmilli;
          frag = tg > 0 ? (double)stranded / (double)tg : 0.0;
        }
        acc.add(4, frag);
        if (W.trace_hash) hsh = mix_event(hsh, ((uint64_t)(uint32_t)rank << 2) | 2, (uint64_t)t);
      } else {
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
        if (!ok) { exc = EXC_ALLOC; reply(DUO_ABORT, 0, k); break; }
        const uint64_t dt = (uint64_t)(t + pod.dur);
        if (t + pod.dur < 0 || dt > time_max) { exc = EXC_UNSUPPORTED; reply(DUO_ABORT, 0, k); break; }
        // answer first: H's push runs while S commits
        reply(DUO_PLACED, (dt << tshift) | ((uint64_t)rank << lb) | ((uint64_t)gmask << (2 + nb)) |
                              ((uint64_t)best_node << 2) | kDelete, k);
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
          for (int q = 0; q < KP; ++q)
            if (q * kWave + lane == pod.cls) wcnt[q] -= 1;
        }
        if (W.trace_hash) hsh = mix_event(hsh, ((uint64_t)(uint32_t)rank << 2), ((uint64_t)t << 8) ^ (uint64_t)best_node);
      }
    }

    // evaluator hook (snapshot schedule precomputed on the host), as replay_one
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
    ++k;
  }
  // H may still be pushing / scanning: wait for it, then take its counters
  {
    uint32_t spins = 0;
    while (!duo_ld(&box->term)) {
      __builtin_amdgcn_s_sleep(FKS_DUO_SLEEP);
      if (++spins > kDuoSpinCap) { exc = exc != EXC_NONE ? exc : EXC_TIMEOUT; break; }
    }
  }
  if (exc == EXC_NONE && box->h_exc != EXC_NONE) {
    exc = box->h_exc;
    --processed;   // H stopped on this event (repush time overflow) before replay_one would count it
  }
  const int64_t n_repush = box->n_repush, n_dropped = box->n_dropped;

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
