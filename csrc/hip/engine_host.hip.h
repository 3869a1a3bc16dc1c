// DeviceEngine: host object owning one workload resident on one MI355X.
//
// Uploads the SoA workload once (pods relabelled by id rank, initial heap
// pre-heapified on the host, snapshot schedule precomputed), then evaluates
// policy batches on its own HIP stream: one k_replay workgroup (one wave) per
// policy followed by k_eval_reduce.  Two heap placements:
//   * LDS heap  -- the whole event heap in LDS (2 policies per CU on the
//                  8,152-pod trace; lowest latency per event);
//   * HBM heap  -- each policy's heap in its own slice of an HBM buffer, only
//                  the deletion bitmap (and VM registers) in LDS, so 12+
//                  policy waves share a CU and hide each other's latency;
//                  also the only placement for traces beyond ~19k pods.
// `heap_mode` = "auto" picks HBM for batches large enough to fill the chip.
#pragma once

#include <hip/hip_runtime.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

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

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  void reserve(size_t bytes) {
    if (bytes <= cap) return;
    if (p) HIP_OK(hipFree(p));
    HIP_OK(hipMalloc(&p, bytes));
    cap = bytes;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const { return reinterpret_cast<T*>(p); }
};

class DeviceEngine {
 public:
  DeviceEngine(py::dict d, int device) : device_(device) {
    HIP_OK(hipSetDevice(device_));
    HIP_OK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    auto geti = [&](const char* k) { return d[k].cast<int64_t>(); };
    auto arr = [&](const char* k) { return d[k].cast<py::array>(); };
    std::memset(&W_, 0, sizeof(W_));
    W_.n_nodes = (int32_t)geti("n_nodes");
    W_.n_pods = (int32_t)geti("n_pods");
    W_.n_classes = (int32_t)geti("n_classes");
    npass_ = (int)geti("npass");
    if (!(npass_ == 1 || npass_ == 2 || npass_ == 4)) throw std::invalid_argument("npass must be 1, 2 or 4");
    W_.cpu_total = dev_upload<int32_t>(arr("cpu_total"), stream_, owned_);
    W_.cpu_left0 = dev_upload<int32_t>(arr("cpu_left"), stream_, owned_);
    W_.mem_total = dev_upload<int32_t>(arr("mem_total"), stream_, owned_);
    W_.mem_left0 = dev_upload<int32_t>(arr("mem_left"), stream_, owned_);
    W_.gpu_left0 = dev_upload<int32_t>(arr("gpu_left"), stream_, owned_);
    W_.ngpus = dev_upload<int32_t>(arr("ngpus"), stream_, owned_);
    W_.gml_total = dev_upload<int32_t>(arr("gml_total"), stream_, owned_);
    W_.gml_left0 = dev_upload<int32_t>(arr("gml_left"), stream_, owned_);
    W_.gmem_total = dev_upload<int64_t>(arr("gmem_total"), stream_, owned_);
    W_.pod = dev_upload<int4>(arr("pod"), stream_, owned_);
    W_.pod_ctime = dev_upload<int32_t>(arr("pod_ctime"), stream_, owned_);
    W_.heap0 = dev_upload<uint64_t>(arr("heap0"), stream_, owned_);
    W_.class_value = dev_upload<int32_t>(arr("class_value"), stream_, owned_);
    W_.snap_fire = dev_upload<int64_t>(arr("snap_fire"), stream_, owned_);
    W_.n_fire = (int32_t)arr("snap_fire").size();
    W_.thr_after_fire = d["thr_after_fire"].cast<double>();
    W_.tot_cpu = geti("tot_cpu"); W_.tot_mem = geti("tot_mem");
    W_.tot_gcnt = geti("tot_gcnt"); W_.tot_gmilli = geti("tot_gmilli");
    W_.used_cpu0 = geti("used_cpu"); W_.used_mem0 = geti("used_mem");
    W_.used_gcnt0 = geti("used_gcnt"); W_.used_gmilli0 = geti("used_gmilli");
    W_.rank_bits = (int32_t)geti("rank_bits"); W_.node_bits = (int32_t)geti("node_bits");
    W_.low_bits = (int32_t)geti("low_bits"); W_.time_bits = (int32_t)geti("time_bits");
    W_.snapshot_interval = 0.05;
    HIP_OK(hipStreamSynchronize(stream_));
    hipDeviceProp_t prop;
    HIP_OK(hipGetDeviceProperties(&prop, device_));
    num_cus_ = prop.multiProcessorCount;
    arch_ = prop.gcnArchName;
    heap_bytes_ = (size_t)lds_heap_entries(W_.n_pods) * sizeof(uint64_t);
    delmap_bytes_ = (size_t)lds_delmap_words(W_.n_pods) * 4;
    lds_heap_ok_ = heap_bytes_ + delmap_bytes_ <= kMaxLds;
    set_attrs();
  }

  ~DeviceEngine() {
    (void)hipSetDevice(device_);
    for (void* p : owned_) (void)hipFree(p);
    for (DevBuf* b : {&res_, &tab_, &fam_, &w_, &code_, &meta_, &kpay_, &ktag_, &gheap_, &prof_}) b->release();
    (void)hipStreamDestroy(stream_);
  }

  void set_options(py::dict o) {
    if (o.contains("repush")) W_.repush_earliest = o["repush"].cast<std::string>() == "earliest";
    if (o.contains("gpu_alloc")) W_.first_fit_alloc = o["gpu_alloc"].cast<std::string>() == "first_fit";
    if (o.contains("snapshot_interval")) W_.snapshot_interval = o["snapshot_interval"].cast<double>();
    if (o.contains("budget")) budget_ = o["budget"].cast<int64_t>();
    if (o.contains("heap_mode")) {
      const std::string m = o["heap_mode"].cast<std::string>();
      if (m != "auto" && m != "lds" && m != "hbm") throw std::invalid_argument("heap_mode: auto | lds | hbm");
      if (m == "lds" && !lds_heap_ok_) throw std::invalid_argument("trace too long for the LDS heap");
      heap_mode_ = m;
    }
  }

  py::array_t<double> evaluate_builtin(py::array_t<int32_t, py::array::c_style | py::array::forcecast> fam,
                                       py::array_t<double, py::array::c_style | py::array::forcecast> weights) {
    const int P = (int)fam.size();
    stage_builtin(fam, weights);
    {
      py::gil_scoped_release rel;
      launch_builtin(P);
    }
    return collect(P);
  }

  py::array_t<double> evaluate_programs(py::bytes blob, py::array_t<int32_t> offsets, py::array_t<int32_t> lengths,
                                        py::array_t<int64_t> kpay, py::array_t<int32_t> koff,
                                        py::array_t<uint8_t> ktag, int nregs) {
    const int P = (int)offsets.size();
    stage_programs(blob, offsets, lengths, kpay, koff, ktag, nregs);
    {
      py::gil_scoped_release rel;
      launch_vm(P, nregs);
    }
    return collect(P);
  }

  // Stage a builtin batch once, then time repeated launches (no H2D/D2H).
  void stage_builtin(py::array_t<int32_t, py::array::c_style | py::array::forcecast> fam,
                     py::array_t<double, py::array::c_style | py::array::forcecast> weights) {
    const int P = (int)fam.size();
    if (weights.ndim() != 2 || weights.shape(0) != P || weights.shape(1) != kWeights)
      throw std::invalid_argument("weights must be [P, 16] float64");
    HIP_OK(hipSetDevice(device_));
    ensure_batch(P);
    fam_spec_ = P > 0 ? fam.at(0) : -1;
    for (int i = 1; i < P && fam_spec_ >= 0; ++i)
      if (fam.at(i) != fam_spec_) fam_spec_ = -1;
    HIP_OK(hipMemcpyAsync(fam_.p, fam.data(), (size_t)P * 4, hipMemcpyHostToDevice, stream_));
    HIP_OK(hipMemcpyAsync(w_.p, weights.data(), (size_t)P * kWeights * 8, hipMemcpyHostToDevice, stream_));
    HIP_OK(hipStreamSynchronize(stream_));
  }
  void launch_builtin_async(int P) { launch_builtin(P); }
  void synchronize() { HIP_OK(hipStreamSynchronize(stream_)); }
  py::array_t<double> collect_table(int P) { return collect(P); }

  py::tuple profile(py::object fam_or_none, py::object weights_or_none, py::object programs_or_none) {
    if (npass_ != 1) throw std::invalid_argument("profiling supports <= 64 nodes");
    HIP_OK(hipSetDevice(device_));
    int P;
    bool is_vm = !programs_or_none.is_none();
    int nregs = 0;
    if (is_vm) {
      py::tuple t = programs_or_none.cast<py::tuple>();
      auto offsets = t[1].cast<py::array_t<int32_t>>();
      P = (int)offsets.size();
      nregs = t[6].cast<int>();
      stage_programs(t[0].cast<py::bytes>(), offsets, t[2].cast<py::array_t<int32_t>>(),
                     t[3].cast<py::array_t<int64_t>>(), t[4].cast<py::array_t<int32_t>>(),
                     t[5].cast<py::array_t<uint8_t>>(), nregs);
    } else {
      auto fam = fam_or_none.cast<py::array_t<int32_t, py::array::c_style | py::array::forcecast>>();
      P = (int)fam.size();
      stage_builtin(fam, weights_or_none.cast<py::array_t<double, py::array::c_style | py::array::forcecast>>());
    }
    prof_.reserve((size_t)P * 64);
    const bool g = use_gheap(P);
    const size_t lds = lds_bytes(g, is_vm ? nregs : 0);
    uint64_t* gh = g ? gheap_for(P) : nullptr;
    if (is_vm) {
      const fksk::VmArgs a{W_, table(), res_.as<DevResult>(), budget_, gh, prof_.as<uint64_t>()};
      HIP_OK(fksk::launch_vm_prof(g, P, lds, stream_, a));
    } else {
      const fksk::BuiltinArgs a{W_, fam_.as<int32_t>(), w_.as<double>(), res_.as<DevResult>(), gh,
                                prof_.as<uint64_t>()};
      HIP_OK(fksk::launch_builtin_prof(g, P, lds, stream_, a));
    }
    reduce(P);
    py::array_t<uint64_t> prof({(py::ssize_t)P, (py::ssize_t)8});
    HIP_OK(hipMemcpyAsync(prof.mutable_data(), prof_.p, (size_t)P * 64, hipMemcpyDeviceToHost, stream_));
    py::array_t<double> tab = collect(P);
    return py::make_tuple(tab, prof);
  }

  py::dict info() const {
    py::dict d;
    d["device"] = device_; d["arch"] = arch_; d["num_cus"] = num_cus_;
    d["heap_bytes_per_policy"] = (int64_t)heap_bytes_;
    d["lds_heap_ok"] = lds_heap_ok_;
    d["npass"] = npass_;
    d["heap_mode"] = heap_mode_;
    return d;
  }

  bool would_use_hbm(int P) const { return use_gheap(P); }

 private:
  static constexpr size_t kMaxLds = 160 * 1024;

  void set_attrs() {
    const int mx = (int)kMaxLds;
    HIP_OK(fksk::set_builtin_attrs_np1(mx)); HIP_OK(fksk::set_builtin_attrs_np2(mx));
    HIP_OK(fksk::set_builtin_attrs_np4(mx));
    HIP_OK(fksk::set_vm_attrs_np1(mx)); HIP_OK(fksk::set_vm_attrs_np2(mx)); HIP_OK(fksk::set_vm_attrs_np4(mx));
    HIP_OK(fksk::set_prof_attrs(mx));
  }

  bool use_gheap(int P) const {
    if (!lds_heap_ok_) return true;
    if (heap_mode_ == "hbm") return true;
    if (heap_mode_ == "lds") return false;
    // auto: the HBM heap wins once the batch exceeds what the LDS heap can
    // keep resident (2 policies per CU)
    return P > 2 * num_cus_;
  }

  size_t lds_bytes(bool g, int nregs) const {
    const size_t vregs = (size_t)nregs * 64 * 8;
    return g ? delmap_bytes_ + vregs : heap_bytes_ + delmap_bytes_ + vregs;
  }

  uint64_t* gheap_for(int P) {
    gheap_.reserve(heap_bytes_ * (size_t)P);
    return gheap_.as<uint64_t>();
  }

  DevProgramTable table() const {
    return DevProgramTable{code_.as<const uint64_t>(), meta_.as<const int32_t>(), kpay_.as<const int64_t>(),
                           ktag_.as<const uint8_t>()};
  }

  void ensure_batch(int P) {
    res_.reserve(sizeof(DevResult) * (size_t)P);
    tab_.reserve(sizeof(double) * 13 * (size_t)P);
    fam_.reserve(sizeof(int32_t) * (size_t)P);
    w_.reserve(sizeof(double) * kWeights * (size_t)P);
  }

  void stage_programs(py::bytes blob, py::array_t<int32_t> offsets, py::array_t<int32_t> lengths,
                      py::array_t<int64_t> kpay, py::array_t<int32_t> koff, py::array_t<uint8_t> ktag, int nregs) {
    const int P = (int)offsets.size();
    if (nregs < 1 || nregs > 64) throw std::invalid_argument("nregs must be in [1, 64]");
    HIP_OK(hipSetDevice(device_));
    ensure_batch(P);
    std::string code = blob;
    code_.reserve(code.size() + 16);
    meta_.reserve((size_t)P * 12 + 16);
    kpay_.reserve((size_t)kpay.size() * 8 + 16);
    ktag_.reserve((size_t)ktag.size() + 16);
    std::vector<int32_t> meta((size_t)P * 3);
    for (int i = 0; i < P; ++i) {
      meta[3 * i] = offsets.at(i);
      meta[3 * i + 1] = lengths.at(i);
      meta[3 * i + 2] = koff.at(i);
    }
    HIP_OK(hipMemcpyAsync(code_.p, code.data(), code.size(), hipMemcpyHostToDevice, stream_));
    HIP_OK(hipMemcpyAsync(meta_.p, meta.data(), meta.size() * 4, hipMemcpyHostToDevice, stream_));
    HIP_OK(hipMemcpyAsync(kpay_.p, kpay.data(), (size_t)kpay.size() * 8, hipMemcpyHostToDevice, stream_));
    HIP_OK(hipMemcpyAsync(ktag_.p, ktag.data(), (size_t)ktag.size(), hipMemcpyHostToDevice, stream_));
    HIP_OK(hipStreamSynchronize(stream_));
  }

  void launch_builtin(int P) {
    const bool g = use_gheap(P);
    const size_t lds = lds_bytes(g, 0);
    uint64_t* gh = g ? gheap_for(P) : nullptr;
    const fksk::BuiltinArgs a{W_, fam_.as<int32_t>(), w_.as<double>(), res_.as<DevResult>(), gh, nullptr};
    if (npass_ == 1) HIP_OK(fksk::launch_builtin_np1(g, fam_spec_, P, lds, stream_, a));
    else if (npass_ == 2) HIP_OK(fksk::launch_builtin_np2(g, fam_spec_, P, lds, stream_, a));
    else HIP_OK(fksk::launch_builtin_np4(g, fam_spec_, P, lds, stream_, a));
    reduce(P);
  }

  void launch_vm(int P, int nregs) {
    const bool g = use_gheap(P);
    const size_t lds = lds_bytes(g, nregs);
    if (lds > kMaxLds) throw std::invalid_argument("heap + VM registers exceed the 160 KiB LDS");
    uint64_t* gh = g ? gheap_for(P) : nullptr;
    const fksk::VmArgs a{W_, table(), res_.as<DevResult>(), budget_, gh, nullptr};
    if (npass_ == 1) HIP_OK(fksk::launch_vm_np1(g, P, lds, stream_, a));
    else if (npass_ == 2) HIP_OK(fksk::launch_vm_np2(g, P, lds, stream_, a));
    else HIP_OK(fksk::launch_vm_np4(g, P, lds, stream_, a));
    reduce(P);
  }

  void reduce(int P) {
    hipLaunchKernelGGL(k_eval_reduce, dim3((P + 63) / 64), dim3(64), 0, stream_, res_.as<DevResult>(),
                       tab_.as<double>(), P);
    HIP_OK(hipGetLastError());
  }

  py::array_t<double> collect(int P) {
    py::array_t<double> out({(py::ssize_t)P, (py::ssize_t)13});
    {
      py::gil_scoped_release rel;
      HIP_OK(hipMemcpyAsync(out.mutable_data(), tab_.p, sizeof(double) * 13 * (size_t)P, hipMemcpyDeviceToHost,
                            stream_));
      HIP_OK(hipStreamSynchronize(stream_));
    }
    return out;
  }

  int device_ = 0;
  hipStream_t stream_ = nullptr;
  DevWorkload W_;
  int npass_ = 1;
  int fam_spec_ = -1;   // family shared by the whole staged batch, or -1
  size_t heap_bytes_ = 0, delmap_bytes_ = 0;
  bool lds_heap_ok_ = true;
  int num_cus_ = 0;
  std::string arch_;
  std::string heap_mode_ = "auto";
  int64_t budget_ = 0;
  std::vector<void*> owned_;
  DevBuf res_, tab_, fam_, w_, code_, meta_, kpay_, ktag_, gheap_, prof_;
};

}  // namespace fks_host
