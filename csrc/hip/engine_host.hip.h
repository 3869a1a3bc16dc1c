// DeviceEngine: host object owning one workload resident on one MI355X.
//
// Uploads the SoA workload once (pods relabelled by id rank, initial heap
// pre-heapified on the host, snapshot schedule precomputed), then evaluates
// policy batches: one k_replay workgroup (one wave) per policy followed by
// k_eval_reduce.  Two heap placements:
//   * LDS heap  -- the whole event heap in LDS (2 policies per CU on the
//                  8,152-pod trace; lowest latency per event);
//   * HBM heap  -- each policy's heap in its own slice of an HBM buffer, only
//                  the deletion bitmap (and VM registers) in LDS, so 16
//                  policy waves share a CU and hide each other's latency;
//                  also the only placement for traces beyond ~19k pods.
// `heap_mode` = "auto" picks HBM for batches large enough to fill the chip.
//
// Batches run in *slots*: each slot owns a HIP stream, its device buffers and
// pinned host staging.  `evaluate_*` is a synchronous round trip on slot 0;
// `submit_*` / `ready` / `wait` let independent islands keep several batches
// in flight on separate streams, so one island's long-replay stragglers do
// not idle the CUs the other islands could use.
#pragma once

#include <hip/hip_runtime.h>
#include <pybind11/numpy.h>
#include <rocprofiler-sdk-roctx/roctx.h>
#include <pybind11/pybind11.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

namespace fks_host {

namespace py = pybind11;
using namespace fksd;

#define HIP_OK(expr)                                                                    \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess)                                                               \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e) +     \
                               " at " #expr);                                           \
  } while (0)

template <class T>
T* dev_upload(const py::array& a, hipStream_t s, std::vector<void*>& owned) {
  py::buffer_info bi = a.request();
  const size_t bytes = (size_t)bi.size * bi.itemsize;
  void* d = nullptr;
  HIP_OK(hipMalloc(&d, bytes ? bytes : 16));
  if (bytes) HIP_OK(hipMemcpyAsync(d, bi.ptr, bytes, hipMemcpyHostToDevice, s));
  owned.push_back(d);
  return reinterpret_cast<T*>(d);
}

template <class T>
T* dev_upload_vec(const std::vector<T>& v, std::vector<void*>& owned) {
  void* d = nullptr;
  HIP_OK(hipMalloc(&d, v.empty() ? 16 : v.size() * sizeof(T)));
  if (!v.empty()) HIP_OK(hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  owned.push_back(d);
  return reinterpret_cast<T*>(d);
}

// z = RN(1/d) if div_by_recip(n, d, z) equals the IEEE quotient n / d, bit for
// bit, for every integer n in [0, hi]; 0.0 otherwise.  Verified per distinct
// divisor (cache), so the device's reciprocal division is exact on exactly
// the numerators the replay can form.
inline double fks_recip_verified(int64_t d, int64_t hi, std::vector<std::pair<std::pair<int64_t, int64_t>, double>>& cache) {
  for (const auto& c : cache)
    if (c.first.first == d && c.first.second >= hi) return c.second;
  double z = 0.0;
  if (d >= 1 && hi >= 0 && hi < (int64_t(1) << 31)) {
    const double dd = (double)d, zz = 1.0 / dd;
    bool ok = true;
    for (int64_t n = 0; n <= hi && ok; ++n) {
      const double x = (double)n, q = x / dd, f = div_by_recip(x, dd, zz);
      ok = std::memcmp(&q, &f, sizeof(double)) == 0;
    }
    if (ok) z = zz;
  }
  cache.push_back({{d, hi}, z});
  return z;
}

// hipFree / hipHostFree wait for the whole device.  While a persistent kernel
// runs (the program service) such a wait lasts until the kernel leaves, so
// frees are parked here instead and done when no persistent grid is left.
// The queue is process-wide (a hipFree waits for every engine's grid), so
// deferral is a count of running grids, changed under the lock: one engine's
// stop does not free while another engine's grid still runs.
struct FreeQueue {
  std::mutex mu;
  int defer = 0;   // persistent grids running in this process
  std::vector<std::pair<void*, bool>> parked;   // (pointer, pinned host memory)
  void free(void* p, bool host) {
    if (!p) return;
    {
      std::lock_guard<std::mutex> g(mu);
      if (defer > 0) { parked.push_back({p, host}); return; }
    }
    if (host) (void)hipHostFree(p);
    else (void)hipFree(p);
  }
  void begin_defer() {
    std::lock_guard<std::mutex> g(mu);
    ++defer;
  }
  size_t end_defer() {   // one grid left; free what was parked once none runs
    std::vector<std::pair<void*, bool>> items;
    {
      std::lock_guard<std::mutex> g(mu);
      if (defer > 0) --defer;
      if (defer == 0) items.swap(parked);
    }
    for (auto& it : items) {
      if (it.second) (void)hipHostFree(it.first);
      else (void)hipFree(it.first);
    }
    return items.size();
  }
};
inline FreeQueue& free_queue() {
  static FreeQueue q;
  return q;
}

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  void reserve(size_t bytes) {
    if (bytes <= cap) return;
    // geometric growth: hipFree waits for the whole device (every slot), so
    // regrowing per batch would serialise the slots' streams
    bytes = std::max(bytes, cap + cap / 2);
    free_queue().free(p, false);
    HIP_OK(hipMalloc(&p, bytes));
    cap = bytes;
  }
  void release() {
    free_queue().free(p, false);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const { return reinterpret_cast<T*>(p); }
};

// Pinned, device-mapped host memory.  Batch inputs (family ids, weights) are
// read by the kernels straight from here and the result table is written
// straight back (zero-copy): no copy kernels queue behind the replay waves
// that already fill the CUs.
struct HostBuf {
  void* p = nullptr;   // host address
  void* d = nullptr;   // device address of the same pages
  size_t cap = 0;
  void reserve(size_t bytes, bool coherent = false) {
    if (bytes <= cap) return;
    // geometric growth, as DevBuf: batch sizes vary (native constant blocks)
    bytes = std::max(bytes, cap + cap / 2);
    free_queue().free(p, true);
    // coherent (fine-grained): read and written while a kernel runs (the program service)
    HIP_OK(hipHostMalloc(&p, bytes, hipHostMallocMapped | (coherent ? hipHostMallocCoherent : 0)));
    HIP_OK(hipHostGetDevicePointer(&d, p, 0));
    cap = bytes;
  }
  void release() {
    free_queue().free(p, true);
    p = d = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const { return reinterpret_cast<T*>(p); }
  template <class T>
  T* dev() const { return reinterpret_cast<T*>(d); }
};

struct Slot {
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  DevBuf res, tab, fam, w, code, meta, kpay, ktag, gheap, prof, wc, queue, kc;
  HostBuf h_in, h_tab, h_wc;
  bool fused_table = false;   // the launch wrote h_tab itself (row kernels)
  int P = 0;
  int fam_spec = -1;    // family shared by the whole staged batch, or -1
  uint32_t qbase = 0;   // row-kernel queue counter value at the next launch
  bool busy = false;
  roctx_range_id_t range = 0;   // roctx range spanning submit -> wait (rocprofv3 --marker-trace)
  void release() {
    for (DevBuf* b : {&res, &tab, &fam, &w, &code, &meta, &kpay, &ktag, &gheap, &prof, &wc, &queue, &kc}) b->release();
    h_in.release();
    h_tab.release();
    h_wc.release();
    if (done) (void)hipEventDestroy(done);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

class DeviceEngine {
 public:
  DeviceEngine(py::dict d, int device, int n_slots = 4) : device_(device) {
    HIP_OK(hipSetDevice(device_));
    if (n_slots < 1 || n_slots > 64) throw std::invalid_argument("n_slots must be in [1, 64]");
    slots_.resize(n_slots);
    for (auto& s : slots_) {
      s = std::make_unique<Slot>();
      HIP_OK(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
      HIP_OK(hipEventCreateWithFlags(&s->done, hipEventDisableTiming));
      // the persistent-queue counter, zeroed now, before any replay occupies the
      // CUs (launches then offset their claims; nothing is re-zeroed later)
      s->queue.reserve(64);
      zero_queue(*s);
      s->qbase = 0;
    }
    hipStream_t st = slots_[0]->stream;
    auto geti = [&](const char* k) { return d[k].cast<int64_t>(); };
    auto arr = [&](const char* k) { return d[k].cast<py::array>(); };
    std::memset(&W_, 0, sizeof(W_));
    W_.n_nodes = (int32_t)geti("n_nodes");
    W_.n_pods = (int32_t)geti("n_pods");
    W_.n_classes = (int32_t)geti("n_classes");
    npass_ = (int)geti("npass");
    if (!(npass_ == 1 || npass_ == 2 || npass_ == 4)) throw std::invalid_argument("npass must be 1, 2 or 4");
    W_.cpu_total = dev_upload<int32_t>(arr("cpu_total"), st, owned_);
    W_.cpu_left0 = dev_upload<int32_t>(arr("cpu_left"), st, owned_);
    W_.mem_total = dev_upload<int32_t>(arr("mem_total"), st, owned_);
    W_.mem_left0 = dev_upload<int32_t>(arr("mem_left"), st, owned_);
    W_.gpu_left0 = dev_upload<int32_t>(arr("gpu_left"), st, owned_);
    W_.ngpus = dev_upload<int32_t>(arr("ngpus"), st, owned_);
    W_.gml_total = dev_upload<int32_t>(arr("gml_total"), st, owned_);
    W_.gml_left0 = dev_upload<int32_t>(arr("gml_left"), st, owned_);
    W_.gmem_total = dev_upload<int64_t>(arr("gmem_total"), st, owned_);
    W_.pod = dev_upload<int4>(arr("pod"), st, owned_);
    W_.pod_ctime = dev_upload<int32_t>(arr("pod_ctime"), st, owned_);
    W_.heap0 = dev_upload<uint64_t>(arr("heap0"), st, owned_);
    {
      // row-kernel image of the initial heap: slot i at address i + 1
      py::array_t<uint64_t, py::array::c_style | py::array::forcecast> h0(arr("heap0"));
      const int np = (int)geti("n_pods");
      py::array_t<uint64_t> shifted((py::ssize_t)row_heap_entries(np));
      uint64_t* sp = shifted.mutable_data();
      std::memset(sp, 0, sizeof(uint64_t) * (size_t)row_heap_entries(np));
      std::memcpy(sp + 1, h0.data(), sizeof(uint64_t) * (size_t)std::min<py::ssize_t>(np, h0.size()));
      W_.heap0p = dev_upload<uint64_t>(shifted, st, owned_);
      HIP_OK(hipStreamSynchronize(st));   // `shifted` dies with this scope
    }
    {
      // {cpu_total, mem_total, ngpus, GPU-milli total} per node slot (NodeRegs::c4, 256-node kernels)
      py::array_t<int32_t, py::array::c_style | py::array::forcecast> ct(arr("cpu_total")), mt(arr("mem_total")),
          ng(arr("ngpus")), gt(arr("gml_total"));
      const py::ssize_t np = ct.size();
      std::vector<int32_t> c4((size_t)np * 4);
      for (py::ssize_t i = 0; i < np; ++i) {
        c4[4 * i] = ct.data()[i];
        c4[4 * i + 1] = mt.data()[i];
        c4[4 * i + 2] = ng.data()[i];
        c4[4 * i + 3] = gt.data()[i * kGmax];
      }
      W_.node_c4 = reinterpret_cast<const int4*>(dev_upload_vec(c4, owned_));
    }
    W_.class_value = dev_upload<int32_t>(arr("class_value"), st, owned_);
    W_.snap_fire = dev_upload<int64_t>(arr("snap_fire"), st, owned_);
    W_.n_fire = (int32_t)arr("snap_fire").size();
    W_.thr_after_fire = d["thr_after_fire"].cast<double>();
    W_.tot_cpu = geti("tot_cpu"); W_.tot_mem = geti("tot_mem");
    W_.tot_gcnt = geti("tot_gcnt"); W_.tot_gmilli = geti("tot_gmilli");
    W_.used_cpu0 = geti("used_cpu"); W_.used_mem0 = geti("used_mem");
    W_.used_gcnt0 = geti("used_gcnt"); W_.used_gmilli0 = geti("used_gmilli");
    W_.rank_bits = (int32_t)geti("rank_bits"); W_.node_bits = (int32_t)geti("node_bits");
    W_.low_bits = (int32_t)geti("low_bits"); W_.time_bits = (int32_t)geti("time_bits");
    W_.snapshot_interval = 0.05;
    W_.trace_hash = 1;
    prepare_recips(d);
    HIP_OK(hipStreamSynchronize(st));
    hipDeviceProp_t prop;
    HIP_OK(hipGetDeviceProperties(&prop, device_));
    num_cus_ = prop.multiProcessorCount;
    // the native kernels call JIT code through function pointers (dynamic
    // stack): a baseline function's spill slots and a runtime call's save area
    // (csrc/jit) sit on that per-lane stack, next to the runtime library's frames
    {
      size_t st = 0;
      size_t want = kJitStackBytes;
      if (const char* e = std::getenv("FKS_JIT_STACK_BYTES")) want = (size_t)std::atoll(e);
      if (hipDeviceGetLimit(&st, hipLimitStackSize) == hipSuccess && st < want)
        (void)hipDeviceSetLimit(hipLimitStackSize, want);
      if (hipDeviceGetLimit(&st, hipLimitStackSize) == hipSuccess) stack_bytes_ = st;
      (void)hipGetLastError();
    }
    arch_ = prop.gcnArchName;
    heap_bytes_ = (size_t)lds_heap_entries(W_.n_pods) * sizeof(uint64_t);
    delmap_bytes_ = (size_t)lds_delmap_words(W_.n_pods) * 4;
    W_.delmap_slots = lds_delmap_words(W_.n_pods) * 32;   // full bitmap unless a launch narrows it
    lds_heap_ok_ = heap_bytes_ + delmap_bytes_ <= kMaxLds;
    rows_ok_ = npass_ == 1 && W_.n_nodes <= kRow && W_.n_classes <= kRow * kRowClassSlots &&
               W_.n_pods <= kRowMaxHeap && W_.tot_cpu < (int64_t(1) << 31) && W_.tot_mem < (int64_t(1) << 31) &&
               W_.tot_gcnt < (int64_t(1) << 31) && W_.tot_gmilli < (int64_t(1) << 31) &&   // int32 row totals
               max_class_pods_ < (1 << 16) &&    // 16-bit waiting-class counters
               max_gpu_milli_ < (1 << 16);       // 16-bit GPU milli halves (NodeRegs<1, true>)
    set_attrs();
  }

  ~DeviceEngine() {
    (void)hipSetDevice(device_);
    if (svc_.running) {   // the resident grid drains before anything it reads is freed
      __atomic_store_n(svc_.ctl.as<uint32_t>() + 1, 1u, __ATOMIC_RELEASE);
      (void)hipStreamSynchronize(svc_.stream);
      svc_.running = false;
      free_queue().end_defer();
    }
    svc_.release();
    for (auto& s : slots_) {
      if (s->stream) (void)hipStreamSynchronize(s->stream);
      s->release();
    }
    for (void* p : owned_) (void)hipFree(p);
  }

  void set_options(py::dict o) {
    if (o.contains("repush")) W_.repush_earliest = o["repush"].cast<std::string>() == "earliest";
    if (o.contains("gpu_alloc")) W_.first_fit_alloc = o["gpu_alloc"].cast<std::string>() == "first_fit";
    if (o.contains("snapshot_interval")) W_.snapshot_interval = o["snapshot_interval"].cast<double>();
    if (o.contains("budget")) budget_ = o["budget"].cast<int64_t>();
    // two-wave program replays (batch launches and the service): a replay past
    // this many events ends with EXC_EVENTS (0: no limit; checked every 1,024)
    if (o.contains("max_events")) {
      const int64_t me = o["max_events"].cast<int64_t>();
      if (me < 0 || me > 0xFFFFFFFFll) throw std::invalid_argument("max_events must be in [0, 2^32)");
      max_events_ = (uint32_t)me;
    }
    if (o.contains("heap_top")) heap_top_opt_ = o["heap_top"].cast<int>();   // -1: auto
    if (o.contains("partial_delmap")) partial_delmap_off_ = !o["partial_delmap"].cast<bool>();   // A/B
    if (o.contains("trace_hash")) W_.trace_hash = o["trace_hash"].cast<bool>() ? 1 : 0;
    if (o.contains("check_invariants")) {
      const int64_t k = o["check_invariants"].cast<int64_t>();
      W_.check_every = (int32_t)std::max<int64_t>(0, std::min<int64_t>(k, INT32_MAX));
      W_.inv_words = W_.check_every > 0 ? inv_words_for(npass_) : 0;
    }
    if (o.contains("row_kernel")) {
      const std::string m = o["row_kernel"].cast<std::string>();
      if (m != "auto" && m != "on" && m != "off") throw std::invalid_argument("row_kernel: auto | on | off");
      if (m == "on" && !rows_ok_) throw std::invalid_argument("row kernel needs <= 16 nodes, <= 64 gpu_milli classes");
      row_mode_ = m;
    }
    if (o.contains("native_duo")) native_duo_ = o["native_duo"].cast<bool>();
    // 256-node clusters: heap wave + scoring wave per builtin policy (replay_wave_duo.hip.h)
    if (o.contains("wave_duo")) wave_duo_ = o["wave_duo"].cast<bool>();
    // programs the caller keeps in flight on the device at once (all slots): the
    // two-wave kernel sizes its LDS heap top so that many stay resident
    if (o.contains("native_inflight")) native_inflight_ = std::max(0, o["native_inflight"].cast<int>());
    if (o.contains("native_duo_top")) native_duo_top_ = o["native_duo_top"].cast<int>();   // -1: auto
    if (o.contains("native_rows")) {
      const int r = o["native_rows"].cast<int>();
      if (r < 0 || r > kRowsPerWave) throw std::invalid_argument("native_rows must be in [0, 4]");
      native_rows_opt_ = r;
    }
    if (o.contains("row_heap_top")) row_top_opt_ = o["row_heap_top"].cast<int>();   // -1: auto
    if (o.contains("row_composite_waves")) {
      const int w = o["row_composite_waves"].cast<int>();
      if (w != 4 && w != 5) throw std::invalid_argument("row_composite_waves must be 4 or 5");
      comp_waves_ = w;
    }
    if (o.contains("row_flat")) row_flat_ = o["row_flat"].cast<bool>();
    // occupancy experiments: at least this much LDS per row-kernel wave (fewer resident waves)
    if (o.contains("row_min_lds")) row_min_lds_ = (size_t)std::max<int64_t>(0, o["row_min_lds"].cast<int64_t>());
    if (o.contains("row_wave_share")) {
      const double f = o["row_wave_share"].cast<double>();
      if (!(f > 0.0 && f <= 4.0)) throw std::invalid_argument("row_wave_share must be in (0, 4]");
      row_share_ = f;
    }
    if (o.contains("heap_mode")) {
      const std::string m = o["heap_mode"].cast<std::string>();
      if (m != "auto" && m != "lds" && m != "hbm") throw std::invalid_argument("heap_mode: auto | lds | hbm");
      if (m == "lds" && !lds_heap_ok_) throw std::invalid_argument("trace too long for the LDS heap");
      heap_mode_ = m;
    }
  }

  // ---- synchronous round trips (slot 0) -------------------------------------------------
  py::array_t<double> evaluate_builtin(py::array_t<int32_t, py::array::c_style | py::array::forcecast> fam,
                                       py::array_t<double, py::array::c_style | py::array::forcecast> weights) {
    submit_builtin(0, fam, weights);
    return wait(0);
  }

  py::array_t<double> evaluate_programs(py::bytes blob, py::array_t<int32_t> offsets, py::array_t<int32_t> lengths,
                                        py::array_t<int64_t> kpay, py::array_t<int32_t> koff,
                                        py::array_t<uint8_t> ktag, int nregs) {
    submit_programs(0, blob, offsets, lengths, kpay, koff, ktag, nregs);
    return wait(0);
  }

  // ---- asynchronous slots ----------------------------------------------------------------
  void submit_builtin(int slot, py::array_t<int32_t, py::array::c_style | py::array::forcecast> fam,
                      py::array_t<double, py::array::c_style | py::array::forcecast> weights) {
    Slot& s = idle_slot(slot);
    const int P = (int)fam.size();
    if (weights.ndim() != 2 || weights.shape(0) != P || weights.shape(1) != kWeights)
      throw std::invalid_argument("weights must be [P, 16] float64");
    if (P < 1) throw std::invalid_argument("empty batch");
    HIP_OK(hipSetDevice(device_));
    s.range = roctxRangeStartA("fks.batch.builtin");
    stage_builtin(s, fam.data(), weights.data(), P);
    {
      py::gil_scoped_release rel;
      launch_builtin(s);
      finish(s);
    }
  }

  void submit_programs(int slot, py::bytes blob, py::array_t<int32_t> offsets, py::array_t<int32_t> lengths,
                       py::array_t<int64_t> kpay, py::array_t<int32_t> koff, py::array_t<uint8_t> ktag, int nregs) {
    Slot& s = idle_slot(slot);
    const int P = (int)offsets.size();
    if (P < 1) throw std::invalid_argument("empty batch");
    HIP_OK(hipSetDevice(device_));
    s.range = roctxRangeStartA("fks.batch.vm");
    stage_programs(s, blob, offsets, lengths, kpay, koff, ktag, nregs);
    {
      py::gil_scoped_release rel;
      launch_vm(s, nregs);
      finish(s);
    }
  }

  // Natively compiled programs (policy/native_codegen.py + ops/jit.py): fn[p]
  // is the device address of policy p's scorer inside a loaded JIT module,
  // kc the concatenated constant blocks, koff[p] where policy p's starts.
  void submit_native(int slot, py::array_t<uint64_t, py::array::c_style | py::array::forcecast> fn,
                     py::array_t<int64_t, py::array::c_style | py::array::forcecast> kc,
                     py::array_t<int32_t, py::array::c_style | py::array::forcecast> koff) {
    submit_native_impl(slot, fn, kc, koff, false);
  }

  // native programs on the s_memtime-profiled row kernel: (result table, [waves, 16]: phase cycles, kind mix)
  py::tuple profile_native(py::array_t<uint64_t, py::array::c_style | py::array::forcecast> fn,
                           py::array_t<int64_t, py::array::c_style | py::array::forcecast> kc,
                           py::array_t<int32_t, py::array::c_style | py::array::forcecast> koff) {
    if (!use_rows((int)fn.size())) throw std::invalid_argument("native profiling runs on the row kernel (<= 16 nodes)");
    submit_native_impl(0, fn, kc, koff, true);
    Slot& s = *slots_[0];
    const int waves = last_native_waves_;
    py::array_t<uint64_t> prof({(py::ssize_t)waves, (py::ssize_t)kRowProfWords});
    HIP_OK(hipMemcpyAsync(prof.mutable_data(), s.prof.p, (size_t)waves * 8 * kRowProfWords, hipMemcpyDeviceToHost,
                          s.stream));
    py::array_t<double> tab = wait(0);
    HIP_OK(hipStreamSynchronize(s.stream));
    return py::make_tuple(tab, prof);
  }

  void submit_native_impl(int slot, py::array_t<uint64_t, py::array::c_style | py::array::forcecast> fn,
                          py::array_t<int64_t, py::array::c_style | py::array::forcecast> kc,
                          py::array_t<int32_t, py::array::c_style | py::array::forcecast> koff, bool profiled) {
    Slot& s = idle_slot(slot);
    const int P = (int)fn.size();
    if (P < 1) throw std::invalid_argument("empty batch");
    if ((int)koff.size() != P) throw std::invalid_argument("koff must have one entry per policy");
    for (int i = 0; i < P; ++i) {
      if (fn.at(i) == 0) throw std::invalid_argument("null program pointer");
      if (koff.at(i) < 0 || koff.at(i) >= (int64_t)kc.size()) throw std::invalid_argument("koff out of range");
    }
    HIP_OK(hipSetDevice(device_));
    s.range = roctxRangeStartA("fks.batch.native");
    HIP_OK(hipStreamSynchronize(s.stream));   // the previous batch no longer reads the staging
    ensure_batch(s, P);
    s.fam_spec = -1;
    const size_t fb = (size_t)P * 8, ob = (size_t)P * 4, kb = (size_t)kc.size() * 8;
    // fn | koff | kc, all read by the kernel straight from pinned host memory
    // (once per policy: kc is staged into LDS when the policy starts).  No copy
    // is queued: GPU_MAX_HW_QUEUES is 4, so a copy on this slot's stream could
    // share a hardware queue with another slot and wait for its whole batch.
    const size_t kco = (fb + ob + 63) & ~size_t(63);
    s.h_in.reserve(kco + kb + (size_t)kKcLds * 8 + 64);   // the kernels read kKcLds entries from every block start
    std::memcpy(s.h_in.as<char>(), fn.data(), fb);
    std::memcpy(s.h_in.as<char>() + fb, koff.data(), ob);
    std::memcpy(s.h_in.as<char>() + kco, kc.data(), kb);
    std::memset(s.h_in.as<char>() + kco + kb, 0, (size_t)kKcLds * 8);
    const int64_t* kc_dev = reinterpret_cast<const int64_t*>(s.h_in.dev<char>() + kco);
    s.h_wc.reserve(sizeof(DevWorkload));
    {
      py::gil_scoped_release rel;
      if (use_rows(P)) {
        launch_rows_native(s, P, fb, kc_dev, profiled);
        finish(s);
        return;
      }
      const bool g = use_gheap_native(P);
      // kKcLds / 64 VM-register rows of LDS hold the policy's constant block
      const DevWorkload Wl = launch_workload(g, kKcLds / kWave, false);
      const size_t lds = lds_bytes(g, Wl.heap_top, kKcLds / kWave);
      if (lds > kMaxLds) throw std::invalid_argument("replay layout exceeds the 160 KiB LDS");
      uint64_t* gh = g ? gheap_for(s, P) : nullptr;
      const fksk::NativeArgs a{Wl, upload_workload(s, Wl), s.h_in.dev<const uint64_t>(), kc_dev,
                               reinterpret_cast<const int32_t*>(s.h_in.dev<char>() + fb), s.res.as<DevResult>(), gh};
      if (npass_ == 1) HIP_OK(fksk::launch_native_np1(g, P, lds, s.stream, a));
      else if (npass_ == 2) HIP_OK(fksk::launch_native_np2(g, P, lds, s.stream, a));
      else HIP_OK(fksk::launch_native_np4(g, P, lds, s.stream, a));
      finish(s);
    }
  }

  py::array_t<double> evaluate_native(py::array_t<uint64_t, py::array::c_style | py::array::forcecast> fn,
                                      py::array_t<int64_t, py::array::c_style | py::array::forcecast> kc,
                                      py::array_t<int32_t, py::array::c_style | py::array::forcecast> koff) {
    submit_native(0, fn, kc, koff);
    return wait(0);
  }

  // device addresses of the native programs' runtime library
  py::array_t<uint64_t> native_rt_table() {
    HIP_OK(hipSetDevice(device_));
    Slot& s = *slots_[0];
    uint64_t* d = nullptr;
    HIP_OK(hipMalloc(&d, 4 * 8));
    HIP_OK(fksk::native_rt_table(d, s.stream));
    py::array_t<uint64_t> out(4);
    HIP_OK(hipMemcpyAsync(out.mutable_data(), d, 4 * 8, hipMemcpyDeviceToHost, s.stream));
    HIP_OK(hipStreamSynchronize(s.stream));
    (void)hipFree(d);
    return out;
  }

  // ---- resident program service (replay_kernels.hip k_native_service) ----------------
  // A grid of resident two-wave workgroups replays programs the host queues:
  // a workgroup whose replay ends claims the next program at once, so no
  // program waits for another's replay.  Programs are numbered in submission
  // order (the claim order); each gets a data slot (fn, koff, constant block,
  // result row, done flag) from a free list, so a straggler -- a replay of
  // millions of events -- holds its slot and nothing else.  The index queue
  // (`qslot`, `nq` entries) maps index -> slot; the device marks an index
  // `started` once it has read its entry, and the host reuses an entry only
  // after that.  Host memory (coherent, mapped): published / stop, qslot,
  // started, the per-slot arrays; `claimed` and the mirrors live in HBM.
  struct Service {
    hipStream_t stream = nullptr;
    DevBuf claimed, res, gheap;
    HostBuf ctl, qslot, started, done, fn, koff, kc, tab, cost;
    std::vector<uint8_t> busy;        // slot holds a program not collected yet
    std::vector<uint32_t> held;       // index of the program in each slot
    std::vector<uint32_t> free_slots;
    uint32_t nslots = 0, nq = 0, published = 0;
    int blocks = 0, T = 0;
    size_t lds = 0;
    bool running = false;
    int64_t launches = 0;
    uint32_t idle_polls = 1u << 24;   // ~57 s of s_sleep(127) polls with nothing published
    void release() {
      for (DevBuf* b : {&claimed, &res, &gheap}) b->release();
      for (HostBuf* b : {&ctl, &qslot, &started, &done, &fn, &koff, &kc, &tab, &cost}) b->release();
      if (stream) (void)hipStreamDestroy(stream);
      stream = nullptr;
    }
    uint32_t ld(const HostBuf& b, uint32_t i) const { return __atomic_load_n(b.as<uint32_t>() + i, __ATOMIC_ACQUIRE); }
  };
  Service svc_;

  void service_launch(uint32_t first_claim) {
    Service& v = svc_;
    __atomic_store_n(v.ctl.as<uint32_t>() + 1, 0u, __ATOMIC_RELEASE);   // stop = 0
    __atomic_store_n(v.ctl.as<uint32_t>() + 2, 0u, __ATOMIC_RELEASE);   // abort = 0
    // claim counter, HBM mirror of `published` (a lower bound: every index below
    // it is published) and of `stop` (replay_kernels.hip service_claim)
    uint32_t init[96] = {};
    init[0] = first_claim;
    init[32] = first_claim;
    HIP_OK(hipMemcpyAsync(v.claimed.p, init, sizeof(init), hipMemcpyHostToDevice, v.stream));
    HIP_OK(hipStreamSynchronize(v.stream));
    DevWorkload Wl = W_;
    Wl.heap_top = v.T;
    const fksk::BuiltinArgs a{Wl, nullptr, nullptr, nullptr, nullptr, v.res.as<DevResult>(), v.gheap.as<uint64_t>(),
                              nullptr, v.tab.dev<double>()};
    const RowNativeArgs nat{v.fn.dev<const uint64_t>(), v.kc.dev<const int64_t>(), v.koff.dev<const int32_t>(),
                            v.ctl.dev<const uint32_t>() + 2, max_events_};
    // `idle_polls` polls with nothing published: the grid drains (a lost host)
    const ServiceCtl c{v.claimed.as<uint32_t>(), v.ctl.dev<const uint32_t>(), v.ctl.dev<const uint32_t>() + 1,
                       v.done.dev<uint32_t>(), v.qslot.dev<const uint32_t>(), v.started.dev<uint32_t>(), v.nq,
                       v.idle_polls, v.cost.dev<uint64_t>()};
    HIP_OK(fksk::launch_native_service(v.blocks, v.lds, v.stream, fksk::ServiceArgs{a, nat, c}));
    v.running = true;
    ++v.launches;
  }

  // start the resident grid: `share` of the two-wave kernel's resident capacity
  // (the rest of the chip stays free for other kernels: JIT module loads, other
  // slots' launches), `slots` programs queued or running at most
  py::dict service_start(int slots, double share, int64_t idle_polls) {
    HIP_OK(hipSetDevice(device_));
    Service& v = svc_;
    if (v.running) throw std::runtime_error("the program service is already running");
    if (!rows_ok_) throw std::invalid_argument("the program service needs the row-kernel layout (<= 16 nodes)");
    if (slots < 64 || slots > (1 << 22)) throw std::invalid_argument("slots must be in [64, 2^22]");
    if (idle_polls < 64 || idle_polls > (1ll << 30)) throw std::invalid_argument("idle_polls must be in [64, 2^30]");
    v.idle_polls = (uint32_t)idle_polls;
    if (!v.stream) HIP_OK(hipStreamCreateWithFlags(&v.stream, hipStreamNonBlocking));
    v.T = duo_top(1 << 30);   // the heap top that keeps the register-limited count of workgroups per CU
    v.lds = duo_lds_bytes(W_.n_pods, v.T);
    if (v.lds + 64 > kMaxLds) throw std::invalid_argument("service layout exceeds the 160 KiB LDS");
    const int per_cu = std::max(1, fksk::native_service_blocks_per_cu(v.lds));
    v.blocks = std::max(1, (int)(share * per_cu * num_cus_));
    v.nslots = (uint32_t)slots;
    v.nq = 2 * (uint32_t)slots;
    const size_t S = v.nslots, Q = v.nq;
    v.claimed.reserve(4 * 96);
    v.res.reserve(sizeof(DevResult) * S);
    v.gheap.reserve((size_t)row_heap_entries(W_.n_pods) * 8 * (size_t)v.blocks);
    v.ctl.reserve(64, true);
    v.qslot.reserve(4 * Q, true);
    v.started.reserve(4 * Q, true);
    v.done.reserve(4 * S, true);
    v.fn.reserve(8 * S, true);
    v.koff.reserve(4 * S, true);
    v.kc.reserve(8 * (size_t)kKcLds * (S + 1), true);
    v.tab.reserve(8 * 13 * S, true);
    v.cost.reserve(8 * S, true);
    std::memset(v.ctl.p, 0, 64);
    std::memset(v.qslot.p, 0, 4 * Q);
    std::memset(v.started.p, 0, 4 * Q);
    std::memset(v.done.p, 0, 4 * S);
    std::memset(v.cost.p, 0, 8 * S);
    std::memset(v.kc.p, 0, 8 * (size_t)kKcLds * (S + 1));
    for (uint32_t i = 0; i < v.nslots; ++i) v.koff.as<int32_t>()[i] = (int32_t)(i * (uint32_t)kKcLds);
    v.busy.assign(S, 0);
    v.held.assign(S, 0);
    v.free_slots.resize(S);
    for (uint32_t i = 0; i < v.nslots; ++i) v.free_slots[i] = v.nslots - 1 - i;
    v.published = 0;
    free_queue().begin_defer();   // (before the launch; the grid's own buffers are sized above)
    service_launch(0);
    py::dict d;
    d["blocks"] = v.blocks; d["per_cu"] = per_cu; d["heap_top"] = v.T; d["lds"] = (int64_t)v.lds;
    d["slots"] = slots; d["queue"] = (int64_t)v.nq;
    return d;
  }

  // queue programs (fn / kc / koff as for submit_native): (index of the first
  // -- they get consecutive ones --, their data slots), or (-1, []) when there
  // is no room (too many programs not collected, or the oldest index-queue
  // entry not yet started)
  py::tuple service_submit(py::array_t<uint64_t, py::array::c_style | py::array::forcecast> fn,
                           py::array_t<int64_t, py::array::c_style | py::array::forcecast> kc,
                           py::array_t<int32_t, py::array::c_style | py::array::forcecast> koff) {
    Service& v = svc_;
    if (!v.running) throw std::runtime_error("the program service is not running");
    const int P = (int)fn.size();
    if (P < 1 || (int)koff.size() != P) throw std::invalid_argument("fn / koff sizes");
    const int64_t nk = (int64_t)kc.size();
    for (int i = 0; i < P; ++i) {
      if (fn.at(i) == 0) throw std::invalid_argument("null program pointer");
      if (koff.at(i) < 0 || koff.at(i) >= nk) throw std::invalid_argument("koff out of range");
    }
    auto refuse = [] { return py::make_tuple((int64_t)-1, py::array_t<int32_t>(0)); };
    if (v.free_slots.size() < (size_t)P || (uint32_t)P > v.nq) return refuse();
    for (int i = 0; i < P; ++i) {   // the entries this submission reuses: their last index must have started
      const uint32_t idx = v.published + (uint32_t)i;
      if (idx >= v.nq && v.ld(v.started, idx % v.nq) != idx - v.nq + 1u) return refuse();
    }
    const uint32_t first = v.published;
    py::array_t<int32_t> slots(P);
    for (int i = 0; i < P; ++i) {
      const uint32_t idx = first + (uint32_t)i;
      const uint32_t slot = v.free_slots.back();
      v.free_slots.pop_back();
      const int64_t a = koff.at(i);
      const int64_t b = (i + 1 < P && koff.at(i + 1) > a) ? koff.at(i + 1) : nk;
      const int64_t len = std::min<int64_t>(b - a, kKcLds);
      int64_t* dst = v.kc.as<int64_t>() + (size_t)slot * kKcLds;
      std::memcpy(dst, kc.data() + a, (size_t)len * 8);
      if (len < kKcLds) std::memset(dst + len, 0, (size_t)(kKcLds - len) * 8);
      v.fn.as<uint64_t>()[slot] = fn.at(i);
      __atomic_store_n(v.done.as<uint32_t>() + slot, 0u, __ATOMIC_RELAXED);
      __atomic_store_n(v.qslot.as<uint32_t>() + idx % v.nq, slot, __ATOMIC_RELAXED);
      v.busy[slot] = 1;
      v.held[slot] = idx;
      slots.mutable_data()[i] = (int32_t)slot;
    }
    v.published = first + (uint32_t)P;
    __atomic_store_n(v.ctl.as<uint32_t>(), v.published, __ATOMIC_RELEASE);   // after every slot's data
    return py::make_tuple((int64_t)first, slots);
  }

  // if the grid drained (nothing published for ~1 min) while programs wait,
  // launch it again from the first index no workgroup started
  void service_revive() {
    Service& v = svc_;
    if (!v.running) return;
    const hipError_t e = hipStreamQuery(v.stream);
    if (e == hipErrorNotReady) return;   // still resident
    HIP_OK(e);                           // a faulted grid is an error, not "still running"
    uint32_t lo = v.published > v.nq ? v.published - v.nq : 0;
    while (lo != v.published && v.ld(v.started, lo % v.nq) == lo + 1u) ++lo;
    if (lo != v.published) service_launch(lo);
  }

  // every program finished since the last call, over all submissions:
  // (indexes, rows, device cycles of each replay), their slots freed -- one
  // scan of the data slots instead of one call per submission (the steady
  // loop keeps dozens in flight)
  py::tuple service_poll() {
    Service& v = svc_;
    std::vector<uint32_t> hit;
    for (uint32_t slot = 0; slot < v.nslots; ++slot)
      if (v.busy[slot] && v.ld(v.done, slot) == v.held[slot] + 1u) hit.push_back(slot);
    py::array_t<int64_t> idx((py::ssize_t)hit.size());
    py::array_t<double> rows({(py::ssize_t)hit.size(), (py::ssize_t)13});
    py::array_t<int64_t> cyc((py::ssize_t)hit.size());
    double* r = rows.mutable_data();
    for (size_t k = 0; k < hit.size(); ++k) {
      const uint32_t slot = hit[k];
      idx.mutable_data()[k] = (int64_t)v.held[slot];
      std::memcpy(r + k * 13, v.tab.as<double>() + (size_t)slot * 13, 13 * sizeof(double));
      cyc.mutable_data()[k] = (int64_t)__atomic_load_n(v.cost.as<uint64_t>() + slot, __ATOMIC_RELAXED);
      v.busy[slot] = 0;
      v.free_slots.push_back(slot);
    }
    if (hit.empty() && v.free_slots.size() < v.nslots) service_revive();
    return py::make_tuple(idx, rows, cyc);
  }

  // end every replay in flight within ~1k events (rows come back EXC_TIMEOUT):
  // a run that stops does not wait for a straggler's millions of events
  void service_abort() {
    if (svc_.running) __atomic_store_n(svc_.ctl.as<uint32_t>() + 2, 1u, __ATOMIC_RELEASE);
  }

  // tell the grid to leave once nothing published is left, and wait for it
  void service_stop() {
    Service& v = svc_;
    if (!v.running) return;
    __atomic_store_n(v.ctl.as<uint32_t>() + 1, 1u, __ATOMIC_RELEASE);
    {
      py::gil_scoped_release rel;
      HIP_OK(hipStreamSynchronize(v.stream));
    }
    v.running = false;
    free_queue().end_defer();
  }

  py::dict service_info() {
    py::dict d;
    d["running"] = svc_.running; d["blocks"] = svc_.blocks; d["slots"] = (int64_t)svc_.nslots;
    d["queue"] = (int64_t)svc_.nq; d["published"] = (int64_t)svc_.published; d["launches"] = svc_.launches;
    d["idle_polls"] = (int64_t)svc_.idle_polls;
    d["heap_top"] = svc_.T;
    d["unconsumed"] = (int64_t)(svc_.nslots - svc_.free_slots.size());
    return d;
  }

  bool ready(int slot) {
    Slot& s = slot_at(slot);
    if (!s.busy) return true;
    const hipError_t e = hipEventQuery(s.done);
    if (e == hipErrorNotReady) return false;
    HIP_OK(e);
    return true;
  }

  py::array_t<double> wait(int slot) {
    Slot& s = slot_at(slot);
    if (!s.busy) throw std::invalid_argument("slot has no batch in flight");
    {
      py::gil_scoped_release rel;
      HIP_OK(hipEventSynchronize(s.done));
    }
    s.busy = false;
    if (s.range) roctxRangeStop(s.range);
    s.range = 0;
    py::array_t<double> out({(py::ssize_t)s.P, (py::ssize_t)13});
    std::memcpy(out.mutable_data(), s.h_tab.p, sizeof(double) * 13 * (size_t)s.P);
    return out;
  }

  // Stage a builtin batch once, then time repeated launches (no H2D/D2H): tools/.
  void stage_builtin_only(py::array_t<int32_t, py::array::c_style | py::array::forcecast> fam,
                          py::array_t<double, py::array::c_style | py::array::forcecast> weights) {
    Slot& s = idle_slot(0);
    HIP_OK(hipSetDevice(device_));
    stage_builtin(s, fam.data(), weights.data(), (int)fam.size());
    HIP_OK(hipStreamSynchronize(s.stream));
  }
  void launch_builtin_async() {
    py::gil_scoped_release rel;
    launch_builtin(*slots_[0]);
  }
  void synchronize() {
    for (auto& s : slots_) HIP_OK(hipStreamSynchronize(s->stream));
  }

  py::tuple profile(py::object fam_or_none, py::object weights_or_none, py::object programs_or_none) {
    const bool c5 = npass_ == 4 && programs_or_none.is_none();
    if (npass_ != 1 && !c5) throw std::invalid_argument("profiling supports <= 64 nodes, or the composite family on 256");
    HIP_OK(hipSetDevice(device_));
    Slot& s = idle_slot(0);
    bool is_vm = !programs_or_none.is_none();
    int nregs = 0;
    if (is_vm) {
      py::tuple t = programs_or_none.cast<py::tuple>();
      nregs = t[6].cast<int>();
      stage_programs(s, t[0].cast<py::bytes>(), t[1].cast<py::array_t<int32_t>>(), t[2].cast<py::array_t<int32_t>>(),
                     t[3].cast<py::array_t<int64_t>>(), t[4].cast<py::array_t<int32_t>>(),
                     t[5].cast<py::array_t<uint8_t>>(), nregs);
    } else {
      auto fam = fam_or_none.cast<py::array_t<int32_t, py::array::c_style | py::array::forcecast>>();
      auto w = weights_or_none.cast<py::array_t<double, py::array::c_style | py::array::forcecast>>();
      stage_builtin(s, fam.data(), w.data(), (int)fam.size());
    }
    const int P = s.P;
    s.prof.reserve((size_t)P * 64);
    const bool g = use_gheap(P);
    const DevWorkload Wl = launch_workload(g, is_vm ? nregs : 0, is_vm);
    const size_t lds = lds_bytes(g, Wl.heap_top, is_vm ? nregs : 0);
    uint64_t* gh = g ? gheap_for(s, P) : nullptr;
    const DevWorkload* wc = upload_workload(s, Wl);
    if (is_vm) {
      const fksk::VmArgs a{Wl, wc, table(s), s.res.as<DevResult>(), budget_, nregs, gh, s.prof.as<uint64_t>()};
      HIP_OK(fksk::launch_vm_prof(g, P, lds, s.stream, a));
    } else {
      const size_t wb = (size_t)P * kWeights * 8;
      const fksk::BuiltinArgs a{Wl, wc, reinterpret_cast<const int32_t*>(s.h_in.dev<char>() + wb),
                                s.h_in.dev<double>(), s.w.as<double>(), s.res.as<DevResult>(), gh,
                                s.prof.as<uint64_t>()};
      if (c5) {
        // the production composite instance only (fast reciprocal path, HBM heap)
        if (s.fam_spec != FAM_COMPOSITE_LINEAR || !g)
          throw std::invalid_argument("256-node profiling: composite batch with verified reciprocals and an HBM heap");
        HIP_OK(fksk::launch_c5_prof(P, lds, s.stream, a));
      } else {
        HIP_OK(fksk::launch_builtin_prof(g, P, lds, s.stream, a));
      }
    }
    finish(s);
    py::array_t<uint64_t> prof({(py::ssize_t)P, (py::ssize_t)8});
    HIP_OK(hipMemcpyAsync(prof.mutable_data(), s.prof.p, (size_t)P * 64, hipMemcpyDeviceToHost, s.stream));
    py::array_t<double> tab = wait(0);
    HIP_OK(hipStreamSynchronize(s.stream));
    return py::make_tuple(tab, prof);
  }

  // row kernel, s_memtime build: (result table, per wave [waves, 16]: phase cycles [0, 8), wave-steps by kind set [9, 16))
  py::tuple profile_rows(py::array_t<int32_t, py::array::c_style | py::array::forcecast> fam,
                         py::array_t<double, py::array::c_style | py::array::forcecast> weights) {
    if (!rows_ok_) throw std::invalid_argument("row kernel needs <= 16 nodes");
    HIP_OK(hipSetDevice(device_));
    Slot& s = idle_slot(0);
    stage_builtin(s, fam.data(), weights.data(), (int)fam.size());
    const int waves = launch_rows(s, true);
    finish(s);
    py::array_t<uint64_t> prof({(py::ssize_t)waves, (py::ssize_t)kRowProfWords});
    HIP_OK(hipMemcpyAsync(prof.mutable_data(), s.prof.p, (size_t)waves * 8 * kRowProfWords, hipMemcpyDeviceToHost,
                          s.stream));
    py::array_t<double> tab = wait(0);
    HIP_OK(hipStreamSynchronize(s.stream));
    return py::make_tuple(tab, prof);
  }

  py::dict info() const {
    py::dict d;
    d["device"] = device_; d["arch"] = arch_; d["num_cus"] = num_cus_;
    d["heap_bytes_per_policy"] = (int64_t)heap_bytes_;
    d["lds_heap_ok"] = lds_heap_ok_;
    d["npass"] = npass_;
    d["heap_mode"] = heap_mode_;
    d["n_slots"] = (int)slots_.size();
    d["heap_top_hbm"] = heap_top_for(0, false);
    d["row_kernel_ok"] = rows_ok_;
    d["row_kernel"] = row_mode_;
    d["row_heap_top"] = row_top();
    d["row_waves_per_cu"] = row_layout(FAM_COMPOSITE_LINEAR).second;
    d["row_wave_share"] = row_share_;
    d["fast_div"] = (int)W_.fast_div;
    d["cap_recips"] = W_.cap_recip[1] != 0.0;
    d["frag_recip"] = W_.z_tg != 0.0;
    d["row_composite_waves"] = comp_waves_;
    d["stack_bytes"] = (int64_t)stack_bytes_;
    d["row_flat"] = row_flat_;
    d["native_rows_last"] = last_native_rows_;
    d["native_waves_last"] = last_native_waves_;
    d["native_duo_top_last"] = last_duo_top_;
    d["native_duo_per_cu_last"] = last_duo_per_cu_;   // resident programs per CU at that heap top
    d["native_duo_reg_cap"] = fksk::native_duo_blocks_per_cu(0);   // register-limited programs per CU
    d["native_inflight"] = native_inflight_;
    d["max_events"] = (int64_t)max_events_;
    d["wave_duo"] = wave_duo_;
    d["wave_duo_heap_top"] = npass_ >= 4 ? heap_top_for(0, false, true) : 0;
    size_t mfree = 0, mtotal = 0;   // (a host-side query: no device synchronisation)
    if (hipMemGetInfo(&mfree, &mtotal) == hipSuccess) {
      d["mem_used_mb"] = (int64_t)((mtotal - mfree) >> 20);
      d["mem_total_mb"] = (int64_t)(mtotal >> 20);
    }
    return d;
  }

  bool would_use_hbm(int P) const { return use_gheap(P); }
  bool would_use_rows(int P) const { return use_rows(P); }
  int n_slots() const { return (int)slots_.size(); }

 private:
  static constexpr size_t kMaxLds = 160 * 1024;
  static constexpr int kWeightWords = kWeights;   // LDS copy of a builtin policy's weights
  static constexpr size_t kPoliciesPerCu = 16;   // HBM-heap builtin kernels: 4 waves per SIMD
  static constexpr size_t kVmPoliciesPerCu = 8;  // HBM-heap VM kernels: 2 waves per SIMD

  // Reciprocals for the row kernel's composite scorer.  A node's cpu_left
  // stays in [0, cpu_total] (likewise mem) when it starts there and no pod
  // asks for a negative amount (placements need pod <= left, deletions give
  // back what their placement took), so max(total, 1) is verified on
  // numerators [0, total]; max(ngpus, 1) on idle-GPU counts [0, 8]; 1000 on
  // best-fit GPU remainders [0, 2^21) (gpu milli < 2^20 by construction).
  // Any failure clears fast_div and every division runs as a division.
  void prepare_recips(py::dict d) {
    auto i32 = [&](const char* k) {
      return py::array_t<int32_t, py::array::c_style | py::array::forcecast>(d[k].cast<py::array>());
    };
    const auto ct = i32("cpu_total"), cl = i32("cpu_left"), mt = i32("mem_total"), ml = i32("mem_left"), ng = i32("ngpus");
    const auto pod = i32("pod");
    const int nn = (int)ct.size(), np = W_.n_pods;
    std::vector<std::pair<std::pair<int64_t, int64_t>, double>> cache;
    bool ok = true;
    std::vector<double> rec((size_t)nn * 3, 0.0), cm((size_t)std::max(np, 1), 0.0);
    std::vector<int32_t> per_class(256, 0);
    for (int r = 0; r < np; ++r) {
      const int32_t c = pod.data()[4 * r], m = pod.data()[4 * r + 1];
      ok = ok && c >= 0 && m >= 0;
      cm[r] = (double)c / (double)(m > 1 ? m : 1);
      const uint32_t pw = (uint32_t)pod.data()[4 * r + 3];
      if ((pw >> 16) & 0xFF) ++per_class[pw >> 24];
    }
    max_class_pods_ = *std::max_element(per_class.begin(), per_class.end());
    {   // row kernels pack two GPUs' milli left per register (16-bit halves)
      const auto gt = i32("gml_total");
      max_gpu_milli_ = gt.size() ? *std::max_element(gt.data(), gt.data() + gt.size()) : 0;
    }
    for (int n = 0; n < nn; ++n) {
      const int32_t a = ct.data()[n], b = mt.data()[n];
      ok = ok && 0 <= cl.data()[n] && cl.data()[n] <= a && 0 <= ml.data()[n] && ml.data()[n] <= b;
      if (!ok) break;
      rec[3 * n + 0] = fks_recip_verified(a > 1 ? a : 1, a, cache);
      rec[3 * n + 1] = fks_recip_verified(b > 1 ? b : 1, b, cache);
      rec[3 * n + 2] = fks_recip_verified(ng.data()[n] > 1 ? ng.data()[n] : 1, kGmax, cache);
      ok = rec[3 * n] != 0.0 && rec[3 * n + 1] != 0.0 && rec[3 * n + 2] != 0.0;
    }
    const double z1000 = fks_recip_verified(1000, (int64_t(1) << 21) - 1, cache);
    W_.fast_div = ok && z1000 != 0.0 ? 1 : 0;
    // GPU capacity divisors max(k * G, 1), k = 0..8, when every GPU node's
    // per-GPU milli total is one G: numerators cap - free_m lie in
    // [-8G, 8G] and RN is odd, so [0, 8G] is checked
    {
      const auto gt = i32("gml_total");
      int32_t G = -1;
      bool uni = true;
      for (int n = 0; n < std::min<int>(nn, W_.n_nodes); ++n)
        if (ng.data()[n] > 0) {
          const int32_t g0 = gt.data()[(size_t)n * kGmax];
          if (G < 0) G = g0;
          uni = uni && g0 == G;
        }
      W_.cap_milli = uni && G > 0 && G < (1 << 20) ? G : 0;
      for (int k = 0; k <= kGmax; ++k) {
        const int64_t dv = std::max<int64_t>(1, (int64_t)k * W_.cap_milli);
        W_.cap_recip[k] = W_.cap_milli > 0 ? fks_recip_verified(dv, 8 * (int64_t)W_.cap_milli, cache) : 0.0;
      }
      for (int k = 0; k <= kGmax; ++k)
        if (W_.cap_recip[k] == 0.0)
          for (int j = 0; j <= kGmax; ++j) W_.cap_recip[j] = 0.0;   // all or none
    }
    // fragmentation divisor: stranded milli in [0, tot_gmilli]
    W_.tot_gmilli_d = (double)W_.tot_gmilli;
    W_.z_tg = W_.tot_gmilli > 0 && W_.tot_gmilli <= (int64_t(1) << 24)
                  ? fks_recip_verified(W_.tot_gmilli, W_.tot_gmilli, cache) : 0.0;
    W_.z1000 = z1000;
    W_.node_recip = dev_upload_vec(rec, owned_);
    W_.pod_cm = dev_upload_vec(cm, owned_);
  }

  Slot& slot_at(int i) {
    if (i < 0 || i >= (int)slots_.size()) throw std::out_of_range("slot index");
    return *slots_[i];
  }
  Slot& idle_slot(int i) {
    Slot& s = slot_at(i);
    if (s.busy) throw std::runtime_error("slot busy: wait() for its batch first");
    return s;
  }

  void set_attrs() {
    const int mx = (int)kMaxLds;
    HIP_OK(fksk::set_builtin_attrs_np1(mx)); HIP_OK(fksk::set_builtin_attrs_np2(mx));
    HIP_OK(fksk::set_builtin_attrs_np4(mx));
    HIP_OK(fksk::set_vm_attrs_np1(mx)); HIP_OK(fksk::set_vm_attrs_np2(mx)); HIP_OK(fksk::set_vm_attrs_np4(mx));
    HIP_OK(fksk::set_prof_attrs(mx));
    HIP_OK(fksk::set_rows_attrs(mx));
    HIP_OK(fksk::set_native_attrs_np1(mx)); HIP_OK(fksk::set_native_attrs_np2(mx));
    HIP_OK(fksk::set_native_attrs_np4(mx));
    HIP_OK(fksk::set_native_rows_attrs(mx));
    HIP_OK(fksk::set_native_duo_attrs(mx));
    HIP_OK(fksk::set_native_service_attrs(mx));
  }

  // 4-policies-per-wave row kernel: clusters of <= 16 nodes, exact repush
  // rule, no invariant checking (those stay on the wave kernel)
  bool use_rows(int P) const {
    (void)P;
    if (!rows_ok_ || row_mode_ == "off") return false;
    if (row_mode_ == "on") return true;
    return heap_mode_ != "lds" && W_.check_every == 0 && !W_.repush_earliest;
  }

  // Heap slots each row keeps in LDS (2^k - 1) for a family's kernel: the
  // largest top among those that keep the most waves resident per CU (the
  // kernel's register use and the LDS layout both bound residency), or the
  // `row_heap_top` option.  Returns {T, resident waves per CU}.
  std::pair<int, int> row_layout(int fam) const {
    const int entries = row_heap_entries(W_.n_pods);
    if (row_top_opt_ > 0) {
      int T = 1;
      while (2 * T + 1 <= row_top_opt_ && T < entries) T = 2 * T + 1;
      return {T, std::max(1, row_waves(fam, T))};
    }
    const int key = fam + 1;
    if (key >= 0 && key < (int)row_layout_cache_.size() && row_layout_cache_[key].first > 0)
      return row_layout_cache_[key];
    std::pair<int, int> best{1, 0};
    for (int T = 63; T < entries && rows_lds_bytes(W_.n_pods, T) <= kMaxLds; T = 2 * T + 1) {
      // residency as measured: the occupancy query is optimistic about LDS
      // (allocation granules); count 2 KiB granules as well
      const int w = row_waves(fam, T);
      if (w >= best.second && w > 0) best = {T, w};
    }
    if (best.second == 0) best = {1, std::max(1, row_waves(fam, 1))};
    if (key >= 0 && key < (int)row_layout_cache_.size()) row_layout_cache_[key] = best;
    return best;
  }
  int row_top() const { return row_layout(comp_waves_ == 5 ? kRowCompositeW5 : FAM_COMPOSITE_LINEAR).first; }

  // resident row-kernel waves per CU at heap top T: the occupancy query
  // (registers, LDS) is optimistic about LDS allocation granules, so LDS is
  // also counted in 2 KiB granules (what the measured residency follows)
  int row_waves(int fam, int T) const {
    const size_t lds = rows_lds_bytes(W_.n_pods, T);
    return std::min<int>(fksk::rows_waves_per_cu(fam, lds), (int)(kMaxLds / ((lds + 2047) & ~size_t(2047))));
  }

  // native-program kernels allocate 128 VGPRs (the JIT register floor): 2
  // waves per SIMD with the HBM heap, so the LDS heap (2 per CU) wins only for
  // batches that fit it
  bool use_gheap_native(int P) const {
    if (lds_bytes(false, 0, kKcLds / kWave) > kMaxLds) return true;   // LDS heap + constant block
    return use_gheap(P);
  }

  bool use_gheap(int P) const {
    if (!lds_heap_ok_ || lds_bytes(false, 0, 0) > kMaxLds) return true;
    if (heap_mode_ == "hbm") return true;
    if (heap_mode_ == "lds") return false;
    // auto: the HBM heap wins once the batch exceeds what the LDS heap can
    // keep resident (2 policies per CU)
    return P > 2 * num_cus_;
  }

  // Heap slots the wave kernels' LDS deletion bitmap covers.  256-node
  // clusters (NPASS 4) keep only the first kPartialDelmap slots' bits with an
  // HBM heap: the first DELETION in heap-array order sits near the root
  // (deletion times are close, creation times spread over the trace), and
  // WaveHeapT::first_deletion reads the keys beyond; the full bitmap of a
  // 65,536-pod trace (8 KiB) would take most of a 16-policies-per-CU LDS share.
  static constexpr int kPartialDelmap = 4096;
  int delmap_slots(bool g) const {
    const int full = lds_delmap_words(W_.n_pods) * 32;
    return (g && npass_ >= 4 && !partial_delmap_off_) ? std::min(full, kPartialDelmap) : full;
  }
  size_t lds_bytes(bool g, int top, int nregs) const {
    const size_t vregs = (size_t)nregs * 64 * 8;
    const size_t inv = (size_t)(W_.inv_words + kWeightWords) * 8;
    const size_t dm = (size_t)delmap_slots(g) / 8;
    return inv + (g ? dm + (size_t)top * 8 + vregs : heap_bytes_ + delmap_bytes_ + vregs);
  }

  // HBM-heap launches keep the top 2^L - 1 heap slots in LDS, as many levels as
  // fit a 16-policies-per-CU share of the 160 KiB (or the `heap_top` option).
  int heap_top_for(int nregs, bool vm, bool duo = false) const {
    const int entries = (int)(heap_bytes_ / 8);
    if (heap_top_opt_ >= 0) return std::min(heap_top_opt_, entries);
    // (NPASS 4: FKS_NP4_WAVES waves/SIMD, or FKS_NP4_DUO_WAVES two-wave policies; NPASS 2: 3)
    const size_t per_cu = duo ? 2 * FKS_NP4_DUO_WAVES
                              : vm ? kVmPoliciesPerCu : (npass_ >= 4 ? 4 * FKS_NP4_WAVES : npass_ == 2 ? 12 : kPoliciesPerCu);
    const size_t budget = kMaxLds / per_cu;
    const size_t fixed = (size_t)delmap_slots(true) / 8 + (size_t)nregs * 64 * 8 + (size_t)(W_.inv_words + kWeightWords) * 8 +
                         (duo ? fksd::wave_duo_box_bytes() : 0);
    int T = 0;
    while (T < entries && fixed + (size_t)(2 * T + 1) * 8 <= budget) T = 2 * T + 1;
    return std::min(T, entries);
  }

  DevWorkload launch_workload(bool g, int nregs, bool vm, bool duo = false) const {
    DevWorkload Wl = W_;
    Wl.heap_top = g ? heap_top_for(nregs, vm, duo) : 0;
    Wl.delmap_slots = delmap_slots(g);
    return Wl;
  }

  uint64_t* gheap_for(Slot& s, int P) {
    s.gheap.reserve(heap_bytes_ * (size_t)P);
    return s.gheap.as<uint64_t>();
  }

  DevProgramTable table(const Slot& s) const {
    return DevProgramTable{s.code.as<const uint64_t>(), s.meta.as<const int32_t>(), s.kpay.as<const int64_t>(),
                           s.ktag.as<const uint8_t>()};
  }

  void ensure_batch(Slot& s, int P) {
    s.res.reserve(sizeof(DevResult) * (size_t)P);
    s.h_tab.reserve(sizeof(double) * 13 * (size_t)P);
    s.w.reserve(sizeof(double) * kWeights * (size_t)P);
    s.P = P;
  }

  // numpy -> pinned staging -> device (async on the slot's stream)
  void stage_builtin(Slot& s, const int32_t* fam, const double* weights, int P) {
    HIP_OK(hipStreamSynchronize(s.stream));   // the previous batch no longer reads the staging
    ensure_batch(s, P);
    s.fam_spec = P > 0 ? fam[0] : -1;
    for (int i = 1; i < P && s.fam_spec >= 0; ++i)
      if (fam[i] != s.fam_spec) s.fam_spec = -1;
    // the composite instance of the row kernel (composite_row) needs finite
    // weights and verified reciprocals; any other batch of that family runs
    // the mixed-family instance
    if (s.fam_spec == FAM_COMPOSITE_LINEAR && !W_.fast_div) s.fam_spec = -1;
    if (s.fam_spec == FAM_COMPOSITE_LINEAR)
      for (size_t i = 0; i < (size_t)P * kWeights; ++i)
        if (!std::isfinite(weights[i])) { s.fam_spec = -1; break; }
    const size_t fb = (size_t)P * 4, wb = (size_t)P * kWeights * 8;
    s.h_in.reserve(fb + wb + 16);
    char* h = s.h_in.as<char>();
    std::memcpy(h, weights, wb);   // read by the kernel prologue through the mapping
    std::memcpy(h + wb, fam, fb);
  }

  void stage_programs(Slot& s, py::bytes blob, py::array_t<int32_t> offsets, py::array_t<int32_t> lengths,
                      py::array_t<int64_t> kpay, py::array_t<int32_t> koff, py::array_t<uint8_t> ktag, int nregs) {
    const int P = (int)offsets.size();
    if (nregs < 1 || nregs > 64) throw std::invalid_argument("nregs must be in [1, 64]");
    HIP_OK(hipStreamSynchronize(s.stream));
    ensure_batch(s, P);
    s.fam_spec = -1;
    const std::string code = blob;
    std::vector<int32_t> meta((size_t)P * 3);
    for (int i = 0; i < P; ++i) {
      meta[3 * i] = offsets.at(i);
      meta[3 * i + 1] = lengths.at(i);
      meta[3 * i + 2] = koff.at(i);
    }
    const size_t cb = code.size(), mb = meta.size() * 4, kb = (size_t)kpay.size() * 8, tb = (size_t)ktag.size();
    s.code.reserve(cb + 16);
    s.meta.reserve(mb + 16);
    s.kpay.reserve(kb + 16);
    s.ktag.reserve(tb + 16);
    s.h_in.reserve(cb + mb + kb + tb + 64);
    char* h = s.h_in.as<char>();
    size_t o = 0;
    auto put = [&](DevBuf& d, const void* src, size_t n) {
      std::memcpy(h + o, src, n);
      HIP_OK(hipMemcpyAsync(d.p, h + o, n, hipMemcpyHostToDevice, s.stream));
      o += (n + 15) & ~size_t(15);
    };
    put(s.code, code.data(), cb);
    put(s.meta, meta.data(), mb);
    put(s.kpay, kpay.data(), kb);
    put(s.ktag, ktag.data(), tb);
  }

  void launch_builtin(Slot& s) {
    const int P = s.P;
    if (use_rows(P)) {
      launch_rows(s, false);
      return;
    }
    const bool g = use_gheap(P);
    // the two-wave kernel: 256-node clusters, HBM heap, no invariant check (it
    // reads heap and node state together, which live on different waves there)
    const bool duo = g && npass_ == 4 && wave_duo_ && W_.check_every == 0;
    const DevWorkload Wl = launch_workload(g, 0, false, duo);
    const size_t lds = lds_bytes(g, Wl.heap_top, 0) + (duo ? fksd::wave_duo_box_bytes() : 0);
    if (lds > kMaxLds) throw std::invalid_argument("replay layout exceeds the 160 KiB LDS");
    uint64_t* gh = g ? gheap_for(s, P) : nullptr;
    const size_t wb = (size_t)P * kWeights * 8;
    const fksk::BuiltinArgs a{Wl, upload_workload(s, Wl), reinterpret_cast<const int32_t*>(s.h_in.dev<char>() + wb),
                              s.h_in.dev<double>(), s.w.as<double>(), s.res.as<DevResult>(), gh, nullptr};
    if (duo) HIP_OK(fksk::launch_builtin_duo_np4(s.fam_spec, P, lds, s.stream, a));
    else if (npass_ == 1) HIP_OK(fksk::launch_builtin_np1(g, s.fam_spec, P, lds, s.stream, a));
    else if (npass_ == 2) HIP_OK(fksk::launch_builtin_np2(g, s.fam_spec, P, lds, s.stream, a));
    else HIP_OK(fksk::launch_builtin_np4(g, s.fam_spec, P, lds, s.stream, a));
  }

  // row kernel launch (optionally the phase-profiled build); returns the wave count
  int launch_rows(Slot& s, bool profiled) {
    const int P = s.P;
    DevWorkload Wl = W_;
    const int kf = s.fam_spec != FAM_COMPOSITE_LINEAR ? s.fam_spec
                   : comp_waves_ == 5                  ? kRowCompositeW5
                   : !row_flat_                        ? kRowCompositeSplit
                                                       : s.fam_spec;
    const std::pair<int, int> lay = row_layout(kf);
    Wl.heap_top = lay.first;
    const size_t lds = std::max(rows_lds_bytes(W_.n_pods, Wl.heap_top) + (profiled ? kRowProfBytes : 0), row_min_lds_);
    if (lds > kMaxLds) throw std::invalid_argument("row kernel layout exceeds the 160 KiB LDS");
    // persistent waves: at most `row_wave_share` of what stays resident on the
    // chip, each row draining the policy queue.  A wave holds its slot until
    // its last row is done, so fewer waves (more policies per row) shrink the
    // idle tail of every launch; concurrent launches of other slots (islands)
    // fill the rest of the chip.
    const int cap = std::max(1, (int)(row_share_ * lay.second * num_cus_));
    const int waves = std::max(1, std::min((P + kRowsPerWave - 1) / kRowsPerWave, cap));
    s.gheap.reserve((size_t)row_heap_entries(W_.n_pods) * 8 * (size_t)waves * kRowsPerWave);
    if (profiled) s.prof.reserve((size_t)waves * 8 * kRowProfWords);
    const size_t wb = (size_t)P * kWeights * 8;
    const fksk::BuiltinArgs a{Wl, upload_workload(s, Wl), reinterpret_cast<const int32_t*>(s.h_in.dev<char>() + wb),
                              s.h_in.dev<double>(), s.w.as<double>(), s.res.as<DevResult>(), s.gheap.as<uint64_t>(),
                              profiled ? s.prof.as<uint64_t>() : nullptr, s.h_tab.dev<double>()};
    s.fused_table = true;
    if (profiled) HIP_OK(fksk::launch_builtin_rows_prof(kf, P, waves, s.queue.as<uint32_t>(), s.qbase, lds, s.stream, a));
    else HIP_OK(fksk::launch_builtin_rows(kf, P, waves, s.queue.as<uint32_t>(), s.qbase, lds, s.stream, a));
    s.qbase += (uint32_t)P + (uint32_t)waves * kRowsPerWave;   // every row makes one final, empty claim
    return waves;
  }

  // Native programs on the row kernel.  LLM-sized batches (up to two waves per
  // CU) run one program per wave with the whole heap in LDS -- the replay is
  // latency-bound there, and a lone row has no other row's divergence in its
  // event loop; larger batches pack four programs per wave.
  // Heap top of the two-wave kernel: the largest 2^k - 1 (at most the whole
  // heap) with which `want` programs stay resident at once -- the whole heap in
  // LDS (two programs per CU on the OpenB trace) for LLM-sized batches, a
  // shallower LDS top over the HBM slice when the caller keeps thousands of
  // programs in flight (up to the register limit: 128 VGPRs, 8 per CU).
  int duo_top(int want) const {
    const int entries = row_heap_entries(W_.n_pods);
    if (native_duo_top_ >= 0) {
      int T = 1;
      while (T < entries - 1 && 2 * T + 1 <= native_duo_top_) T = 2 * T + 1;
      return T;
    }
    const int reg_cap = std::max(1, fksk::native_duo_blocks_per_cu(0));
    const int need = std::min(reg_cap, std::max(1, (want + num_cus_ - 1) / std::max(1, num_cus_)));
    auto per_cu = [&](int T) {
      const size_t lds = duo_lds_bytes(W_.n_pods, T);
      if (lds > kMaxLds) return 0;
      return std::max(0, fksk::native_duo_blocks_per_cu(lds));
    };
    int T = 63;
    while (T < entries - 1 && per_cu(2 * T + 1) >= std::max(2, need)) T = 2 * T + 1;
    return T;
  }

  void launch_rows_native(Slot& s, int P, size_t fn_bytes, const int64_t* kc_dev, bool profiled = false) {
    // the two-wave kernel for every batch (its heap top follows the programs in
    // flight); four programs per wave only on request (native_rows = 4)
    const int ra = native_rows_opt_ > 0 ? native_rows_opt_ : (native_duo_ || P <= 2 * num_cus_ ? 1 : kRowsPerWave);
    DevWorkload Wl = W_;
    const int entries = row_heap_entries(W_.n_pods);
    if (ra == 1 && native_duo_) {
      // two waves per program (heap wave + scoring wave, replay_duo.hip.h)
      const int T = duo_top(std::max(P, native_inflight_));
      Wl.heap_top = T;
      last_duo_top_ = T;
      last_duo_per_cu_ = fksk::native_duo_blocks_per_cu(duo_lds_bytes(W_.n_pods, T));
      const size_t lds = duo_lds_bytes(W_.n_pods, T);
      if (lds > kMaxLds) throw std::invalid_argument("native duo layout exceeds the 160 KiB LDS");
      s.gheap.reserve((size_t)entries * 8 * (size_t)P);
      if (profiled) s.prof.reserve((size_t)P * 128);
      const fksk::BuiltinArgs a{Wl, upload_workload(s, Wl), nullptr, nullptr, nullptr, s.res.as<DevResult>(),
                                s.gheap.as<uint64_t>(), profiled ? s.prof.as<uint64_t>() : nullptr,
                                s.h_tab.dev<double>()};
      s.fused_table = true;
      const RowNativeArgs nat{s.h_in.dev<const uint64_t>(), kc_dev,
                              reinterpret_cast<const int32_t*>(s.h_in.dev<char>() + fn_bytes), nullptr, max_events_};
      if (std::getenv("FKS_DEBUG_LAUNCH"))
        std::fprintf(stderr, "[fks] native duo: P=%d T=%d lds=%zu per_cu=%d stream=%p\n", P, T, lds,
                     last_duo_per_cu_, (void*)s.stream);
      HIP_OK(fksk::launch_native_duo(P, lds, s.stream, a, nat));
      last_native_rows_ = 0;   // 0: the two-wave kernel
      last_native_waves_ = 2 * P;
      return;
    }
    // largest heap top (2^k - 1 slots, at most the whole heap) that keeps two waves per CU
    int T = 1;
    while (T < entries - 1 && rows_lds_bytes(W_.n_pods, 2 * T + 1, ra, true) <= kMaxLds / 2) T = 2 * T + 1;
    Wl.heap_top = T;
    const size_t lds = rows_lds_bytes(W_.n_pods, T, ra, true) + (profiled ? kRowProfBytes : 0);
    if (lds > kMaxLds) throw std::invalid_argument("native row kernel layout exceeds the 160 KiB LDS");
    const int per_cu = std::max(1, std::min(fksk::native_rows_waves_per_cu(lds), (int)(kMaxLds / ((lds + 2047) & ~size_t(2047)))));
    const int cap = std::max(1, (int)(row_share_ * per_cu * num_cus_));
    const int waves = std::max(1, std::min((P + ra - 1) / ra, cap));
    s.gheap.reserve((size_t)entries * 8 * (size_t)waves * kRowsPerWave);
    if (profiled) s.prof.reserve((size_t)waves * 8 * kRowProfWords);
    const fksk::BuiltinArgs a{Wl, upload_workload(s, Wl), nullptr, nullptr, nullptr, s.res.as<DevResult>(),
                              s.gheap.as<uint64_t>(), profiled ? s.prof.as<uint64_t>() : nullptr, s.h_tab.dev<double>()};
    s.fused_table = true;
    const RowNativeArgs nat{s.h_in.dev<const uint64_t>(), kc_dev,
                            reinterpret_cast<const int32_t*>(s.h_in.dev<char>() + fn_bytes)};
    if (std::getenv("FKS_DEBUG_LAUNCH"))
      std::fprintf(stderr, "[fks] native rows: P=%d rows=%d waves=%d T=%d lds=%zu qbase=%u stream=%p\n", P, ra, waves, T,
                   lds, s.qbase, (void*)s.stream);
    HIP_OK(fksk::launch_native_rows(P, waves, ra, s.queue.as<uint32_t>(), s.qbase, lds, s.stream, a, nat));
    s.qbase += (uint32_t)P + (uint32_t)waves * (uint32_t)ra;   // every active row makes one final, empty claim
    last_native_rows_ = ra;
    last_native_waves_ = waves;
  }

  void launch_vm(Slot& s, int nregs) {
    const int P = s.P;
    const bool g = use_gheap(P);
    const DevWorkload Wl = launch_workload(g, nregs, true);
    const size_t lds = lds_bytes(g, Wl.heap_top, nregs);
    if (lds > kMaxLds) throw std::invalid_argument("heap + VM registers exceed the 160 KiB LDS");
    uint64_t* gh = g ? gheap_for(s, P) : nullptr;
    const fksk::VmArgs a{Wl, upload_workload(s, Wl), table(s), s.res.as<DevResult>(), budget_, nregs, gh, nullptr};
    if (npass_ == 1) HIP_OK(fksk::launch_vm_np1(g, P, lds, s.stream, a));
    else if (npass_ == 2) HIP_OK(fksk::launch_vm_np2(g, P, lds, s.stream, a));
    else HIP_OK(fksk::launch_vm_np4(g, P, lds, s.stream, a));
  }

  // the persistent-queue counter starts at zero once per slot: a copy-engine
  // transfer, not a fill kernel (a fill kernel would wait for a CU slot behind
  // the other slots' persistent waves -- hundreds of ms in a profile)
  static void zero_queue(Slot& s) {
    static const uint64_t zeros[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    HIP_OK(hipMemcpyAsync(s.queue.p, zeros, 64, hipMemcpyHostToDevice, s.stream));
    HIP_OK(hipStreamSynchronize(s.stream));
  }

  // The kernels read their cold workload fields from their own kernarg
  // segment (replay_kernels.hip kernarg_workload), so a launch copies nothing
  // to the device.  A per-slot HBM copy used to be sent with hipMemcpyAsync,
  // which the runtime runs as a copy kernel: on a slot's first launch it had
  // to wait for a CU slot behind the other slots' persistent replay waves
  // (0.9-1.1 s per slot at config-5 shape, profiles/r3_config5_copy_trace.txt).
  static const DevWorkload* upload_workload(Slot&, const DevWorkload&) { return nullptr; }

  // k_eval_reduce, result table -> pinned host, completion event
  void finish(Slot& s) {
    const int P = s.P;
    // row kernels write the result table themselves (evaluator fused into the
    // write-back); the wave kernels leave it to k_eval_reduce
    if (!s.fused_table)
      hipLaunchKernelGGL(k_eval_reduce, dim3((P + 63) / 64), dim3(64), 0, s.stream, s.res.as<DevResult>(),
                         s.h_tab.dev<double>(), P);   // zero-copy into the pinned result table
    s.fused_table = false;
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(s.done, s.stream));
    s.busy = true;
  }

  int device_ = 0;
  std::vector<std::unique_ptr<Slot>> slots_;
  DevWorkload W_;
  int npass_ = 1;
  size_t heap_bytes_ = 0, delmap_bytes_ = 0;
  bool lds_heap_ok_ = true;
  bool rows_ok_ = false;
  std::string row_mode_ = "auto";
  int row_top_opt_ = -1;
  double row_share_ = 1.0;
  bool native_duo_ = true;     // two-wave kernel for one-program-per-wave batches
  int native_rows_opt_ = 0;    // rows per wave for native programs (0: auto)
  int native_inflight_ = 0;    // programs kept in flight across slots (two-wave heap-top sizing)
  int native_duo_top_ = -1;    // forced two-wave heap top (-1: auto)
  int last_duo_top_ = 0, last_duo_per_cu_ = 0;
  int last_native_rows_ = 0, last_native_waves_ = 0;
  size_t row_min_lds_ = 0;
  int32_t max_class_pods_ = 0;   // most GPU pods of one gpu_milli class (row kernel: < 2^16)
  int32_t max_gpu_milli_ = 0;    // largest per-GPU milli total (row kernel: < 2^16)
  static constexpr size_t kJitStackBytes = 2048;   // per-lane stack of the native kernels
  size_t stack_bytes_ = 0;
  bool row_flat_ = true;  // composite row kernel: flat heap accesses (false: exec-masked ds / global)
  int comp_waves_ = 5;   // composite row kernel: 4 or 5 waves per SIMD (row_composite_waves)
  mutable std::vector<std::pair<int, int>> row_layout_cache_ = std::vector<std::pair<int, int>>(8, {0, 0});
  int num_cus_ = 0;
  std::string arch_;
  std::string heap_mode_ = "auto";
  int64_t budget_ = 0;
  uint32_t max_events_ = 0;
  int heap_top_opt_ = -1;
  bool partial_delmap_off_ = false;
  bool wave_duo_ = false;   // NPASS-4 builtin launches on the two-wave kernel (`wave_duo`)
  std::vector<void*> owned_;
};

}  // namespace fks_host
