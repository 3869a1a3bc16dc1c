// Native CPU replay engine: the exact oracle for every device result.
//
// Serial, straightforward C++ implementation of the reference's event loop
// (reference simulator/main.py:50-148, event_simulator.py:19-59,
// evaluator.py:55-164) under the rules of SURVEY.md §2.4:
//   * CPython-heapq-identical heap on (time, pod_rank) keys (the array layout
//     is observable through the repush rule);
//   * first-DELETION-in-heap-array-order repush, drop when none pending;
//   * strict-> argmax over nodes in cluster order, best-fit GPU pick;
//   * snapshot thresholds accumulated in IEEE double, fixed-point exact means.
// The scorer is a template parameter so built-in families inline; the
// bytecode interpreter plugs in through the same interface.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <map>
#include <vector>

#include "fks/exact_mean.hpp"
#include "fks/types.hpp"

namespace fks {

// A Python number as seen by the placement loop (int or float).
struct Num {
  bool is_float = false;
  int64_t i = 0;
  double f = 0.0;
  static Num I(int64_t v) { Num n; n.i = v; return n; }
  static Num F(double v) { Num n; n.is_float = true; n.f = v; return n; }
};

// Exact Python comparison  a > b  for int/float mixes (ints are compared
// exactly, not by conversion to double).
inline bool py_gt(const Num& a, const Num& b) {
  if (!a.is_float && !b.is_float) return a.i > b.i;
  if (a.is_float && b.is_float) return a.f > b.f;
  if (a.is_float) {  // float > int
    double x = a.f; int64_t y = b.i;
    if (std::isnan(x)) return false;
    if (std::isinf(x)) return x > 0;
    double fy = (double)y;
    if (x != fy) return x > fy;          // differ already as doubles -> order agrees
    // x == (double)y: compare exactly via the integer part of x
    if (x >= 9.2233720368547758e18) return true;
    if (x < -9.2233720368547758e18) return false;
    int64_t xi = (int64_t)x;             // x is integral here (|x| >= 2^53 or exact)
    return xi > y;
  }
  // int > float  ==  float < int
  double x = b.f; int64_t y = a.i;
  if (std::isnan(x)) return false;
  if (std::isinf(x)) return x < 0;
  double fy = (double)y;
  if (fy != x) return fy > x;
  if (x >= 9.2233720368547758e18) return false;
  if (x < -9.2233720368547758e18) return true;
  int64_t xi = (int64_t)x;
  return y > xi;
}

// Mutable per-replay cluster state.
struct ClusterState {
  std::vector<int64_t> cpu_left, mem_left;
  std::vector<int32_t> gpu_left;
  std::vector<int32_t> gmilli_left;
  void reset(const Workload& w) {
    cpu_left = w.cpu_left0; mem_left = w.mem_left0;
    gpu_left = w.gpu_left0; gmilli_left = w.gmilli_left0;
  }
};

// What a scorer sees for one (pod, node) pair.
struct ScoreCtx {
  const Workload& w;
  const ClusterState& s;
  int32_t pod;
  int64_t pod_ctime;  // current (possibly re-queued) creation time
};

// Outcome of a scorer call: a Python number or an exception code.
struct ScoreOut {
  Num v;
  int32_t exc = EXC_NONE;
};

struct HeapItem {
  int64_t time;
  int32_t rank;
  int32_t pod;
  int32_t kind;  // 0 creation, 1 deletion
};

inline bool heap_lt(const HeapItem& a, const HeapItem& b) {
  return a.time < b.time || (a.time == b.time && a.rank < b.rank);
}

// CPython Modules/_heapqmodule.c algorithms, verbatim in structure.
inline void heap_siftdown(std::vector<HeapItem>& h, size_t startpos, size_t pos) {
  HeapItem item = h[pos];
  while (pos > startpos) {
    size_t parent = (pos - 1) >> 1;
    if (heap_lt(item, h[parent])) { h[pos] = h[parent]; pos = parent; continue; }
    break;
  }
  h[pos] = item;
}

inline void heap_siftup(std::vector<HeapItem>& h, size_t pos) {
  const size_t end = h.size(), start = pos;
  HeapItem item = h[pos];
  size_t child = 2 * pos + 1;
  while (child < end) {
    size_t right = child + 1;
    if (right < end && !heap_lt(h[child], h[right])) child = right;
    h[pos] = h[child];
    pos = child;
    child = 2 * pos + 1;
  }
  h[pos] = item;
  heap_siftdown(h, start, pos);
}

inline void heap_push(std::vector<HeapItem>& h, const HeapItem& it) {
  h.push_back(it);
  heap_siftdown(h, 0, h.size() - 1);
}

inline HeapItem heap_pop(std::vector<HeapItem>& h) {
  HeapItem last = h.back();
  h.pop_back();
  if (!h.empty()) {
    HeapItem ret = h[0];
    h[0] = last;
    heap_siftup(h, 0);
    return ret;
  }
  return last;
}

inline void heapify(std::vector<HeapItem>& h) {
  for (size_t i = h.size() / 2; i-- > 0;) heap_siftup(h, i);
}

// Feasibility prologue of the reference template / FF / BF policies.
inline bool feasible(const ScoreCtx& c, int n) {
  const Workload& w = c.w;
  const int p = c.pod;
  if (w.pcpu[p] > c.s.cpu_left[n] || w.pmem[p] > c.s.mem_left[n] || w.pngpu[p] > c.s.gpu_left[n])
    return false;
  if (w.pngpu[p] > 0) {
    int avail = 0;
    for (int g = w.gpu_start[n]; g < w.gpu_start[n + 1]; ++g) avail += c.s.gmilli_left[g] >= w.pgmilli[p];
    if (avail < w.pngpu[p]) return false;
  }
  return true;
}

// Resource-accounting invariants (reference `_validate_cluster_invariants`,
// simulator/main.py:201-272): every node's and GPU's remaining capacity is in
// [0, total] and equals total minus what the pods with a pending DELETION
// event (placed, not yet finished) hold.
inline bool invariants_hold(const Workload& w, const ClusterState& st, const std::vector<HeapItem>& heap,
                            const std::vector<int32_t>& assigned, const std::vector<int32_t>& assigned_gpus,
                            const std::vector<int32_t>& gpu_off) {
  const int N = w.n_nodes;
  std::vector<int64_t> ucpu(N, 0), umem(N, 0), ugpu(N, 0), ugm(w.n_gpus, 0);
  for (const HeapItem& it : heap) {
    if (it.kind != 1) continue;
    const int p = it.pod, n = assigned[p];
    if (n < 0 || n >= N) return false;
    ucpu[n] += w.pcpu[p]; umem[n] += w.pmem[p]; ugpu[n] += w.pngpu[p];
    for (int k = gpu_off[p]; k < gpu_off[p + 1]; ++k) ugm[w.gpu_start[n] + assigned_gpus[k]] += w.pgmilli[p];
  }
  for (int n = 0; n < N; ++n) {
    if (st.cpu_left[n] < 0 || st.cpu_left[n] > w.cpu_total[n] || ucpu[n] + st.cpu_left[n] != w.cpu_total[n]) return false;
    if (st.mem_left[n] < 0 || st.mem_left[n] > w.mem_total[n] || umem[n] + st.mem_left[n] != w.mem_total[n]) return false;
    if (st.gpu_left[n] < 0 || st.gpu_left[n] > w.ngpus[n] || ugpu[n] + st.gpu_left[n] != w.ngpus[n]) return false;
  }
  for (int g = 0; g < w.n_gpus; ++g)
    if (st.gmilli_left[g] < 0 || st.gmilli_left[g] > w.gmilli_total[g] ||
        ugm[g] + st.gmilli_left[g] != w.gmilli_total[g])
      return false;
  return true;
}

template <class Scorer>
SimResult simulate(const Workload& w, Scorer& scorer, const SimOptions& opt) {
  SimResult res;
  ClusterState st;
  st.reset(w);
  const int N = w.n_nodes, P = w.n_pods;

  // --- totals (evaluator constructor) and incremental used counters
  int64_t tot_cpu = 0, tot_mem = 0, tot_gcnt = 0, tot_gmilli = 0;
  int64_t used_cpu = 0, used_mem = 0, used_gcnt = 0, used_gmilli = 0;
  for (int n = 0; n < N; ++n) {
    tot_cpu += w.cpu_total[n]; tot_mem += w.mem_total[n]; tot_gcnt += w.ngpus[n];
    used_cpu += w.cpu_total[n] - st.cpu_left[n];
    used_mem += w.mem_total[n] - st.mem_left[n];
    used_gcnt += w.ngpus[n] - st.gpu_left[n];
  }
  for (int g = 0; g < w.n_gpus; ++g) {
    tot_gmilli += w.gmilli_total[g];
    used_gmilli += w.gmilli_total[g] - st.gmilli_left[g];
  }
  auto ratio = [](int64_t a, int64_t b) { return b > 0 ? (double)a / (double)b : 0.0; };

  // --- heap of initial creations, in trace order, then heapify
  std::vector<HeapItem> heap(P);
  std::vector<int64_t> ctime(w.pctime);
  for (int p = 0; p < P; ++p) heap[p] = HeapItem{w.pctime[p], w.prank[p], p, 0};
  heapify(heap);

  std::vector<int32_t> assigned(P, -1);
  std::vector<int32_t> gpu_off(P + 1, 0);
  for (int p = 0; p < P; ++p) gpu_off[p + 1] = gpu_off[p] + std::max(0, w.pngpu[p]);
  std::vector<int32_t> assigned_gpus(gpu_off[P], -1);
  std::vector<uint8_t> waiting(P, 0);
  std::map<int32_t, int32_t> waiting_gmilli;  // multiset of gpu_milli of waiting GPU pods
  int64_t waiting_count = 0;

  FixedAcc acc_cpu, acc_mem, acc_gcnt, acc_gmilli, acc_frag;
  const int64_t total_events = P;
  int64_t processed = 0;
  double threshold = opt.snapshot_interval;
  uint64_t hsh = 0xcbf29ce484222325ull;
  std::vector<int32_t> fits;
  fits.reserve(64);

  while (!heap.empty()) {
    HeapItem ev = heap_pop(heap);
    const int p = ev.pod;
    if (ev.kind == 1) {
      // ---- deletion
      const int n = assigned[p];
      st.cpu_left[n] += w.pcpu[p]; used_cpu -= w.pcpu[p];
      st.mem_left[n] += w.pmem[p]; used_mem -= w.pmem[p];
      st.gpu_left[n] += w.pngpu[p]; used_gcnt -= w.pngpu[p];
      for (int k = gpu_off[p]; k < gpu_off[p + 1]; ++k) {
        st.gmilli_left[w.gpu_start[n] + assigned_gpus[k]] += w.pgmilli[p];
        used_gmilli -= w.pgmilli[p];
      }
      hsh = mix_event(hsh, ((uint64_t)(uint32_t)w.prank[p] << 2) | 1, (uint64_t)ev.time);
    } else {
      // ---- creation: argmax over nodes in cluster order
      ScoreCtx ctx{w, st, p, ev.time};
      Num best = Num::I(0);
      int best_node = -1;
      for (int n = 0; n < N; ++n) {
        ScoreOut o = scorer(ctx, n);
        if (o.exc != EXC_NONE) { res.exc = o.exc; return res; }
        Num s = o.v;
        if (opt.truncate) {
          // int(max(0, s))
          if (s.is_float) {
            double x = s.f;
            if (!(x > 0.0)) { s = Num::I(0); }
            else if (std::isinf(x)) { res.exc = EXC_OVERFLOW; return res; }
            else if (x >= 9.2233720368547758e18) { res.exc = EXC_UNSUPPORTED; return res; }
            else s = Num::I((int64_t)x);
          } else if (s.i < 0) {
            s = Num::I(0);
          }
        }
        if (py_gt(s, best)) { best = s; best_node = n; }
      }
      if (opt.record_states) {
        res.states.push_back(p);
        res.states.push_back(best_node);
        res.states.insert(res.states.end(), st.cpu_left.begin(), st.cpu_left.end());
        res.states.insert(res.states.end(), st.mem_left.begin(), st.mem_left.end());
        res.states.insert(res.states.end(), st.gpu_left.begin(), st.gpu_left.end());
        res.states.insert(res.states.end(), st.gmilli_left.begin(), st.gmilli_left.end());
      }
      if (best_node < 0) {
        // ---- failed placement
        if (!waiting[p]) {
          waiting[p] = 1; ++waiting_count;
          if (w.pngpu[p] > 0) waiting_gmilli[w.pgmilli[p]]++;
        }
        // fragmentation sample (waiting set is non-empty here)
        double frag = 0.0;
        if (!waiting_gmilli.empty()) {
          const int32_t m = waiting_gmilli.begin()->first;
          int64_t stranded = 0;
          for (int g = 0; g < w.n_gpus; ++g) {
            int32_t left = st.gmilli_left[g];
            if (0 < left && left < m) stranded += left;
          }
          frag = ratio(stranded, tot_gmilli);
        }
        acc_frag.add(frag);
        if (opt.record_values) res.frag_values.push_back(frag);
        // repush anchored on a pending deletion
        int64_t anchor = 0;
        bool found = false;
        if (opt.repush == REPUSH_FIRST) {
          for (const HeapItem& it : heap)
            if (it.kind == 1) { anchor = it.time; found = true; break; }
        } else {
          for (const HeapItem& it : heap)
            if (it.kind == 1 && (!found || it.time < anchor)) { anchor = it.time; found = true; }
        }
        if (found) {
          ctime[p] = anchor + 1;
          heap_push(heap, HeapItem{anchor + 1, w.prank[p], p, 0});
          ++res.n_repush;
        } else {
          ++res.n_dropped;
        }
        hsh = mix_event(hsh, ((uint64_t)(uint32_t)w.prank[p] << 2) | 2, (uint64_t)ev.time);
      } else {
        // ---- commit
        const int n = best_node;
        st.cpu_left[n] -= w.pcpu[p]; used_cpu += w.pcpu[p];
        st.mem_left[n] -= w.pmem[p]; used_mem += w.pmem[p];
        st.gpu_left[n] -= w.pngpu[p]; used_gcnt += w.pngpu[p];
        const int need = w.pngpu[p];
        if (need > 0) {
          fits.clear();
          const int g0 = w.gpu_start[n], ng = w.ngpus[n];
          for (int j = 0; j < ng; ++j)
            if (st.gmilli_left[g0 + j] >= w.pgmilli[p]) fits.push_back(j);
          if ((int)fits.size() < need) { res.exc = EXC_ALLOC; return res; }
          if (opt.gpu_alloc == ALLOC_BEST_FIT)
            std::stable_sort(fits.begin(), fits.end(), [&](int a, int b) {
              return st.gmilli_left[g0 + a] < st.gmilli_left[g0 + b];
            });
          for (int k = 0; k < need; ++k) {
            assigned_gpus[gpu_off[p] + k] = fits[k];
            st.gmilli_left[g0 + fits[k]] -= w.pgmilli[p];
            used_gmilli += w.pgmilli[p];
          }
        }
        assigned[p] = n;
        if (waiting[p]) {
          waiting[p] = 0; --waiting_count;
          if (w.pngpu[p] > 0) {
            auto it = waiting_gmilli.find(w.pgmilli[p]);
            if (--(it->second) == 0) waiting_gmilli.erase(it);
          }
        }
        heap_push(heap, HeapItem{ev.time + w.pdur[p], w.prank[p], p, 1});
        hsh = mix_event(hsh, ((uint64_t)(uint32_t)w.prank[p] << 2), ((uint64_t)ev.time << 8) ^ (uint64_t)n);
      }
    }
    // ---- evaluator hook
    ++processed;
    double progress = total_events > 0 ? (double)processed / (double)total_events : 0.0;
    if (progress >= threshold) {
      double r0 = ratio(used_cpu, tot_cpu), r1 = ratio(used_mem, tot_mem);
      double r2 = ratio(used_gcnt, tot_gcnt), r3 = ratio(used_gmilli, tot_gmilli);
      acc_cpu.add(r0); acc_mem.add(r1); acc_gcnt.add(r2); acc_gmilli.add(r3);
      if (opt.record_values) {
        res.snap_values.push_back(r0); res.snap_values.push_back(r1);
        res.snap_values.push_back(r2); res.snap_values.push_back(r3);
      }
      threshold += opt.snapshot_interval;
    }
    // max_nodes (active nodes) -- O(N), informational only
    int active = 0;
    for (int n = 0; n < N; ++n)
      active += (st.cpu_left[n] < w.cpu_total[n] || st.mem_left[n] < w.mem_total[n] ||
                 st.gpu_left[n] < w.ngpus[n]);
    if (active > res.max_nodes) res.max_nodes = active;
    if (opt.check_invariants > 0 && processed % opt.check_invariants == 0 &&
        !invariants_hold(w, st, heap, assigned, assigned_gpus, gpu_off)) {
      res.exc = EXC_INVARIANT;
      return res;
    }
  }
  if (opt.check_invariants > 0 && !invariants_hold(w, st, heap, assigned, assigned_gpus, gpu_off)) {
    res.exc = EXC_INVARIANT;
    return res;
  }

  res.n_events = processed;
  res.n_snapshots = acc_cpu.count;
  res.n_frag_events = acc_frag.count;
  res.trace_hash = hsh;
  for (int p = 0; p < P; ++p) res.n_unplaced += assigned[p] < 0;
  res.inexact = acc_cpu.inexact || acc_mem.inexact || acc_gcnt.inexact || acc_gmilli.inexact ||
                acc_frag.inexact;
  res.avg_cpu = fixed_mean(acc_cpu);
  res.avg_mem = fixed_mean(acc_mem);
  res.avg_gpu_count = fixed_mean(acc_gcnt);
  res.avg_gpu_milli = fixed_mean(acc_gmilli);
  res.frag = acc_frag.count ? fixed_mean(acc_frag) : 0.0;
  if (res.n_snapshots == 0) {
    res.score = 0.0;
  } else if (res.n_unplaced > 0) {
    res.score = 0.0;
  } else {
    double overall = (res.avg_cpu + res.avg_mem + res.avg_gpu_count + res.avg_gpu_milli) / 4.0;
    double pen = std::min(0.1, res.frag);
    double s = overall - pen;
    res.score = std::max(0.0, std::min(1.0, s));
  }
  if (opt.record_placements) res.placement = assigned;
  return res;
}

}  // namespace fks
