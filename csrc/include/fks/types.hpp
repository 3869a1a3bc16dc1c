// Shared plain-data types of the native engines (host side).
//
// The workload is a structure of arrays (see
// funsearch_kubernetes_simulator_amd/core/arrays.py for the field contract);
// results are one fixed-size record per evaluated policy.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace fks {

// Exception classes a policy replay can end with.  They mirror the Python
// exception a reference replay would raise; any of them means score 0 in
// evaluate_policy_standalone and None in _evaluate_policy_full
// (reference funsearch/funsearch_integration.py:63-64, 457-459).
enum ExcCode : int32_t {
  EXC_NONE = 0,
  EXC_ZERO_DIVISION = 1,   // ZeroDivisionError
  EXC_VALUE = 2,           // ValueError: int(nan), math domain error, empty max()
  EXC_OVERFLOW = 3,        // OverflowError: int(inf), math range error
  EXC_TYPE = 4,            // TypeError: complex / None in arithmetic
  EXC_INDEX = 5,           // IndexError: node.gpus[i] out of range
  EXC_ALLOC = 6,           // ValueError from the GPU allocator (not enough GPUs)
  EXC_NAME = 7,            // NameError / UnboundLocalError
  EXC_UNSUPPORTED = 100,   // semantics outside the native subset (bigint, ...): re-run exactly on host
  EXC_BUDGET = 101,        // instruction budget exhausted (runaway program)
  EXC_INVARIANT = 102,     // resource accounting invariant violated (debug check)
  EXC_TIMEOUT = 103,       // engine-internal timeout (two-wave kernel spin cap): re-run on the next engine
  EXC_EVENTS = 104,        // the replay passed the caller's event budget (a resource limit): not scored
};

enum RepushMode : int32_t { REPUSH_FIRST = 0, REPUSH_EARLIEST = 1 };
enum GpuAlloc : int32_t { ALLOC_BEST_FIT = 0, ALLOC_FIRST_FIT = 1 };

struct Workload {
  int32_t n_nodes = 0, n_gpus = 0, n_pods = 0;
  // nodes
  std::vector<int64_t> cpu_total, cpu_left0, mem_total, mem_left0;
  std::vector<int32_t> gpu_left0, ngpus, gpu_start;
  // gpus
  std::vector<int32_t> gmilli_total, gmilli_left0;
  std::vector<int64_t> gmem_total, gmem_left0;
  // pods
  std::vector<int64_t> pcpu, pmem, pctime, pdur;
  std::vector<int32_t> pngpu, pgmilli, prank;
};

struct SimOptions {
  int32_t repush = REPUSH_FIRST;
  int32_t gpu_alloc = ALLOC_BEST_FIT;
  double snapshot_interval = 0.05;
  bool truncate = true;          // FunSearchScheduler: int(max(0, score))
  int64_t budget = 0;            // VM instruction budget per priority evaluation (0 = unlimited)
  bool record_values = false;    // keep snapshot / frag values (exact fallback, tests)
  bool record_placements = false;
  int64_t check_invariants = 0;  // verify resource accounting every K events and at the end (0 = off)
  bool record_states = false;    // per creation event: pod + node/GPU state + decision (screening data)
};

struct SimResult {
  int32_t exc = EXC_NONE;
  double score = 0.0;
  double avg_cpu = 0, avg_mem = 0, avg_gpu_count = 0, avg_gpu_milli = 0, frag = 0;
  int64_t n_snapshots = 0, n_frag_events = 0, n_events = 0, n_unplaced = 0;
  int64_t max_nodes = 0, n_repush = 0, n_dropped = 0;
  int64_t vm_insns = 0;              // bytecode instructions executed (VM scorers)
  bool inexact = false;
  uint64_t trace_hash = 0;
  std::vector<double> snap_values;   // 4 per snapshot (record_values)
  std::vector<double> frag_values;   // record_values
  std::vector<int32_t> placement;    // node per pod (-1 never placed; record_placements)
  // record_states: per creation event, [pod, chosen node (-1 failed), cpu_left[N],
  // mem_left[N], gpu_left[N], gmilli_left[G]]
  std::vector<int32_t> states;
};

// FNV-1a style mixing of the event stream; identical on host and device so a
// divergence between engines can be localised without storing full traces.
inline uint64_t mix_event(uint64_t h, uint64_t a, uint64_t b) {
  h ^= a + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
  h *= 0x100000001B3ull;
  h ^= b + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
  h *= 0x100000001B3ull;
  return h;
}

}  // namespace fks
