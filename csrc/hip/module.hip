// _fks_hip: pybind11 host side of the MI355X replay engine.
//
// DeviceEngine uploads one workload (SoA, already relabelled by pod rank and
// with the initial heap pre-heapified on the host) to HBM once, then
// evaluates batches of candidate policies: one k_replay workgroup per policy
// (LDS-resident heap), followed by k_eval_reduce, on the engine's own HIP
// stream.  Results come back as a float64 [P, 13] table with the same
// columns as the CPU oracle's batch API.
#include <hip/hip_runtime.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "replay.hip.h"
#include "scorers.hip.h"
#include "vm_dev.hip.h"

namespace py = pybind11;
using namespace fksd;

#define HIP_OK(expr)                                                                    \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess)                                                               \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e) +     \
                               " at " #expr);                                           \
  } while (0)

namespace {

template <int NPASS>
__global__ __launch_bounds__(64) void k_replay_builtin(DevWorkload W, const int32_t* __restrict__ fam,
                                                       const double* __restrict__ weights, DevResult* out,
                                                       int p0) {
  extern __shared__ uint64_t heap[];
  const int p = p0 + blockIdx.x;
  BuiltinScorerDev sc;
  sc.family = fam[p];
#pragma unroll
  for (int k = 0; k < kWeights; ++k) sc.w[k] = weights[(size_t)p * kWeights + k];
  replay_one<NPASS>(W, sc, heap, out + p);
}

template <int NPASS>
__global__ __launch_bounds__(64) void k_replay_vm(DevWorkload W, DevProgramTable T, DevResult* out, int p0,
                                                  int64_t budget) {
  extern __shared__ uint64_t heap[];
  const int p = p0 + blockIdx.x;
  VmScorerDev sc;
  sc.init(T, p, W, budget);
  replay_one<NPASS>(W, sc, heap, out + p);
}

// Phase-profiled variants (s_memtime per phase; diagnostics only, NPASS = 1).
__global__ __launch_bounds__(64) void k_replay_builtin_prof(DevWorkload W, const int32_t* __restrict__ fam,
                                                            const double* __restrict__ weights, DevResult* out,
                                                            uint64_t* prof) {
  extern __shared__ uint64_t heap[];
  const int p = blockIdx.x;
  BuiltinScorerDev sc;
  sc.family = fam[p];
#pragma unroll
  for (int k = 0; k < kWeights; ++k) sc.w[k] = weights[(size_t)p * kWeights + k];
  replay_one<1, BuiltinScorerDev, PhaseProf>(W, sc, heap, out + p, prof + (size_t)p * 8);
}

__global__ __launch_bounds__(64) void k_replay_vm_prof(DevWorkload W, DevProgramTable T, DevResult* out,
                                                       int64_t budget, uint64_t* prof) {
  extern __shared__ uint64_t heap[];
  const int p = blockIdx.x;
  VmScorerDev sc;
  sc.init(T, p, W, budget);
  replay_one<1, VmScorerDev, PhaseProf>(W, sc, heap, out + p, prof + (size_t)p * 8);
}

// ---- primitive self-tests (one wave) ----------------------------------------------
// out[0] = wave max, out[1] = wave sum, out[2..65] = pair-swapped values,
// out[66..129] = row_shr:1 of the low 32 bits
__global__ __launch_bounds__(64) void k_test_wave_ops(const uint64_t* in, uint64_t* out) {
  const int lane = lane_id();
  const uint64_t v = in[lane];
  const uint64_t m = wave_max_u64(v);
  const int64_t s = wave_sum_i64((int64_t)v);
  const uint64_t sw = swap_pairs64(v);
  const int sh = __builtin_amdgcn_update_dpp(-1, (int)(uint32_t)v, 0x111, 0xF, 0xF, false);
  if (lane == 0) { out[0] = m; out[1] = (uint64_t)s; }
  out[2 + lane] = sw;
  out[66 + lane] = (uint64_t)(int64_t)sh;
}

// Run a sequence of heap operations (op >= 0: push key op; op < 0: pop) on the
// wave-parallel LDS heap; returns the final array (size in out_n).
__global__ __launch_bounds__(64) void k_test_heap(const uint64_t* init, int n0, const int64_t* ops, int nops,
                                                   int lb, uint64_t* out, int* out_n, uint64_t* popped) {
  extern __shared__ uint64_t lds[];
  const int lane = lane_id();
  WaveHeap hp;
  hp.h = lds;
  hp.delmap = reinterpret_cast<uint32_t*>(lds + 4096);
  hp.lb = lb;
  for (int i = lane; i < n0; i += 64) lds[i] = init[i];
  for (int i = lane; i < 256; i += 64) hp.delmap[i] = 0;
  __syncthreads();
  int n = n0, np = 0;
  for (int k = 0; k < nops; ++k) {
    const int64_t op = ops[k];
    if (op >= 0) { hp.push(n, (uint64_t)op); ++n; }
    else if (n > 0) {
      const uint64_t top = uniu64(lds[0]);
      const uint64_t last = uniu64(lds[n - 1]);
      --n;
      if (n > 0) hp.pop_reinsert(n, last);
      if (lane == 0) popped[np] = top;
      ++np;
    }
  }
  __syncthreads();
  for (int i = lane; i < n; i += 64) out[i] = lds[i];
  if (lane == 0) *out_n = n;
}

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

class DeviceEngine {
 public:
  DeviceEngine(py::dict d, int device) : device_(device) {
    HIP_OK(hipSetDevice(device_));
    HIP_OK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    auto geti = [&](const char* k) { return d[k].cast<int64_t>(); };
    std::memset(&W_, 0, sizeof(W_));
    W_.n_nodes = (int32_t)geti("n_nodes");
    W_.n_pods = (int32_t)geti("n_pods");
    W_.n_classes = (int32_t)geti("n_classes");
    npass_ = (int)geti("npass");
    if (!(npass_ == 1 || npass_ == 2 || npass_ == 4)) throw std::invalid_argument("npass must be 1, 2 or 4");
    auto arr = [&](const char* k) { return d[k].cast<py::array>(); };
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
    lds_bytes_ = (size_t)lds_heap_entries(W_.n_pods) * sizeof(uint64_t) + (size_t)lds_delmap_words(W_.n_pods) * 4;
    hipDeviceProp_t prop;
    HIP_OK(hipGetDeviceProperties(&prop, device_));
    num_cus_ = prop.multiProcessorCount;
    arch_ = prop.gcnArchName;
    max_lds_ = prop.sharedMemPerBlock;
    if (lds_bytes_ > (size_t)160 * 1024)
      throw std::invalid_argument("trace too long for the LDS-resident heap (needs the HBM heap variant)");
    set_lds_attr(reinterpret_cast<const void*>(&k_replay_builtin<1>), lds_bytes_);
    set_lds_attr(reinterpret_cast<const void*>(&k_replay_builtin<2>), lds_bytes_);
    set_lds_attr(reinterpret_cast<const void*>(&k_replay_builtin<4>), lds_bytes_);
    // VM launches add the virtual register file behind the (64-aligned) heap
    heap_pad_bytes_ = (size_t)lds_vreg_offset(W_.n_pods) * sizeof(uint64_t);
    const size_t vm_max = (size_t)160 * 1024;
    set_lds_attr(reinterpret_cast<const void*>(&k_replay_vm<1>), vm_max);
    set_lds_attr(reinterpret_cast<const void*>(&k_replay_vm<2>), vm_max);
    set_lds_attr(reinterpret_cast<const void*>(&k_replay_vm<4>), vm_max);
  }

  ~DeviceEngine() {
    (void)hipSetDevice(device_);
    for (void* p : owned_) (void)hipFree(p);
    free_batch();
    for (void* p : {d_code_, d_poff_, d_kpay_, d_ktag_}) if (p) (void)hipFree(p);
    (void)hipStreamDestroy(stream_);
  }

  void set_options(py::dict o) {
    if (o.contains("repush")) W_.repush_earliest = o["repush"].cast<std::string>() == "earliest";
    if (o.contains("gpu_alloc")) W_.first_fit_alloc = o["gpu_alloc"].cast<std::string>() == "first_fit";
    if (o.contains("snapshot_interval")) W_.snapshot_interval = o["snapshot_interval"].cast<double>();
    if (o.contains("budget")) budget_ = o["budget"].cast<int64_t>();
  }

  py::array_t<double> evaluate_builtin(py::array_t<int32_t, py::array::c_style | py::array::forcecast> fam,
                                       py::array_t<double, py::array::c_style | py::array::forcecast> weights) {
    const int P = (int)fam.size();
    if (weights.ndim() != 2 || weights.shape(0) != P || weights.shape(1) != kWeights)
      throw std::invalid_argument("weights must be [P, 16] float64");
    HIP_OK(hipSetDevice(device_));
    ensure_batch(P);
    HIP_OK(hipMemcpyAsync(d_fam_, fam.data(), (size_t)P * 4, hipMemcpyHostToDevice, stream_));
    HIP_OK(hipMemcpyAsync(d_w_, weights.data(), (size_t)P * kWeights * 8, hipMemcpyHostToDevice, stream_));
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
    if (nregs < 1 || nregs > 64) throw std::invalid_argument("nregs must be in [1, 64]");
    const size_t lds = heap_pad_bytes_ + (size_t)nregs * 64 * sizeof(uint64_t);
    if (lds > (size_t)160 * 1024) throw std::invalid_argument("heap + VM registers exceed the 160 KiB LDS");
    HIP_OK(hipSetDevice(device_));
    ensure_batch(P);
    std::string code = blob;
    upload_programs(code, offsets, lengths, kpay, koff, ktag);
    {
      py::gil_scoped_release rel;
      launch_vm(P, lds);
    }
    return collect(P);
  }

  // Per-policy phase cycle counts (s_memtime) of a builtin or program batch.
  py::tuple profile(py::object fam_or_none, py::object weights_or_none, py::object programs_or_none) {
    if (npass_ != 1) throw std::invalid_argument("profiling supports <= 64 nodes");
    HIP_OK(hipSetDevice(device_));
    int P;
    uint64_t* d_prof = nullptr;
    if (!programs_or_none.is_none()) {
      py::tuple t = programs_or_none.cast<py::tuple>();
      auto offsets = t[1].cast<py::array_t<int32_t>>();
      P = (int)offsets.size();
      int nregs = t[6].cast<int>();
      ensure_batch(P);
      std::string code = t[0].cast<py::bytes>();
      upload_programs(code, offsets, t[2].cast<py::array_t<int32_t>>(), t[3].cast<py::array_t<int64_t>>(),
                      t[4].cast<py::array_t<int32_t>>(), t[5].cast<py::array_t<uint8_t>>());
      HIP_OK(hipMalloc(&d_prof, (size_t)P * 8 * 8));
      DevProgramTable T{reinterpret_cast<const uint64_t*>(d_code_), reinterpret_cast<const int32_t*>(d_poff_),
                        reinterpret_cast<const int64_t*>(d_kpay_), reinterpret_cast<const uint8_t*>(d_ktag_)};
      const size_t lds = heap_pad_bytes_ + (size_t)nregs * 64 * 8;
      set_lds_attr(reinterpret_cast<const void*>(&k_replay_vm_prof), (size_t)160 * 1024);
      hipLaunchKernelGGL(k_replay_vm_prof, dim3(P), dim3(64), lds, stream_, W_, T, d_res_, budget_, d_prof);
    } else {
      auto fam = fam_or_none.cast<py::array_t<int32_t, py::array::c_style | py::array::forcecast>>();
      auto weights = weights_or_none.cast<py::array_t<double, py::array::c_style | py::array::forcecast>>();
      P = (int)fam.size();
      ensure_batch(P);
      HIP_OK(hipMemcpyAsync(d_fam_, fam.data(), (size_t)P * 4, hipMemcpyHostToDevice, stream_));
      HIP_OK(hipMemcpyAsync(d_w_, weights.data(), (size_t)P * kWeights * 8, hipMemcpyHostToDevice, stream_));
      HIP_OK(hipMalloc(&d_prof, (size_t)P * 8 * 8));
      set_lds_attr(reinterpret_cast<const void*>(&k_replay_builtin_prof), lds_bytes_);
      hipLaunchKernelGGL(k_replay_builtin_prof, dim3(P), dim3(64), lds_bytes_, stream_, W_, d_fam_, d_w_, d_res_,
                         d_prof);
    }
    HIP_OK(hipGetLastError());
    hipLaunchKernelGGL(k_eval_reduce, dim3((P + 63) / 64), dim3(64), 0, stream_, d_res_, d_tab_, P);
    py::array_t<uint64_t> prof({(py::ssize_t)P, (py::ssize_t)8});
    HIP_OK(hipMemcpyAsync(prof.mutable_data(), d_prof, (size_t)P * 64, hipMemcpyDeviceToHost, stream_));
    py::array_t<double> tab = collect(P);
    HIP_OK(hipFree(d_prof));
    return py::make_tuple(tab, prof);
  }

  // Launch only (no host sync / copy-back): for timing loops and graph capture.
  void launch_builtin_async(int P) { launch_builtin(P); }
  void synchronize() { HIP_OK(hipStreamSynchronize(stream_)); }

  py::dict info() const {
    py::dict d;
    d["device"] = device_; d["arch"] = arch_; d["num_cus"] = num_cus_;
    d["lds_bytes_per_policy"] = (int64_t)lds_bytes_; d["npass"] = npass_;
    d["max_lds_per_block"] = (int64_t)max_lds_;
    return d;
  }

 private:
  void set_lds_attr(const void* fn, size_t bytes) {
    HIP_OK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
  }

  void free_batch() {
    if (d_res_) (void)hipFree(d_res_);
    if (d_tab_) (void)hipFree(d_tab_);
    if (d_fam_) (void)hipFree(d_fam_);
    if (d_w_) (void)hipFree(d_w_);
    d_res_ = nullptr; d_tab_ = nullptr; d_fam_ = nullptr; d_w_ = nullptr;
    cap_ = 0;
  }

  void ensure_batch(int P) {
    if (P <= cap_) return;
    free_batch();
    cap_ = P;
    HIP_OK(hipMalloc(&d_res_, sizeof(DevResult) * (size_t)P));
    HIP_OK(hipMalloc(&d_tab_, sizeof(double) * 13 * (size_t)P));
    HIP_OK(hipMalloc(&d_fam_, sizeof(int32_t) * (size_t)P));
    HIP_OK(hipMalloc(&d_w_, sizeof(double) * kWeights * (size_t)P));
  }

  void launch_builtin(int P) {
    dim3 grid(P), block(64);
    switch (npass_) {
      case 1: hipLaunchKernelGGL(k_replay_builtin<1>, grid, block, lds_bytes_, stream_, W_, d_fam_, d_w_, d_res_, 0); break;
      case 2: hipLaunchKernelGGL(k_replay_builtin<2>, grid, block, lds_bytes_, stream_, W_, d_fam_, d_w_, d_res_, 0); break;
      default: hipLaunchKernelGGL(k_replay_builtin<4>, grid, block, lds_bytes_, stream_, W_, d_fam_, d_w_, d_res_, 0); break;
    }
    HIP_OK(hipGetLastError());
    hipLaunchKernelGGL(k_eval_reduce, dim3((P + 63) / 64), dim3(64), 0, stream_, d_res_, d_tab_, P);
    HIP_OK(hipGetLastError());
  }

  void upload_programs(const std::string& code, py::array_t<int32_t> offsets, py::array_t<int32_t> lengths,
                       py::array_t<int64_t> kpay, py::array_t<int32_t> koff, py::array_t<uint8_t> ktag) {
    const int P = (int)offsets.size();
    auto realloc = [&](void** p, size_t& cap, size_t bytes) {
      if (bytes <= cap) return;
      if (*p) HIP_OK(hipFree(*p));
      HIP_OK(hipMalloc(p, bytes));
      cap = bytes;
    };
    realloc(&d_code_, code_cap_, code.size() + 16);
    realloc(&d_poff_, poff_cap_, (size_t)P * 4 * 3 + 16);
    realloc(&d_kpay_, kpay_cap_, (size_t)kpay.size() * 8 + 16);
    realloc(&d_ktag_, ktag_cap_, (size_t)ktag.size() + 16);
    HIP_OK(hipMemcpyAsync(d_code_, code.data(), code.size(), hipMemcpyHostToDevice, stream_));
    std::vector<int32_t> meta((size_t)P * 3);
    for (int i = 0; i < P; ++i) {
      meta[3 * i] = offsets.at(i);
      meta[3 * i + 1] = lengths.at(i);
      meta[3 * i + 2] = koff.at(i);
    }
    HIP_OK(hipMemcpyAsync(d_poff_, meta.data(), meta.size() * 4, hipMemcpyHostToDevice, stream_));
    HIP_OK(hipMemcpyAsync(d_kpay_, kpay.data(), (size_t)kpay.size() * 8, hipMemcpyHostToDevice, stream_));
    HIP_OK(hipMemcpyAsync(d_ktag_, ktag.data(), (size_t)ktag.size(), hipMemcpyHostToDevice, stream_));
    // host copies stay alive until the stream syncs in collect()
    HIP_OK(hipStreamSynchronize(stream_));
  }

  void launch_vm(int P, size_t lds) {
    DevProgramTable T;
    T.code = reinterpret_cast<const uint64_t*>(d_code_);
    T.meta = reinterpret_cast<const int32_t*>(d_poff_);
    T.kpay = reinterpret_cast<const int64_t*>(d_kpay_);
    T.ktag = reinterpret_cast<const uint8_t*>(d_ktag_);
    dim3 grid(P), block(64);
    switch (npass_) {
      case 1: hipLaunchKernelGGL(k_replay_vm<1>, grid, block, lds, stream_, W_, T, d_res_, 0, budget_); break;
      case 2: hipLaunchKernelGGL(k_replay_vm<2>, grid, block, lds, stream_, W_, T, d_res_, 0, budget_); break;
      default: hipLaunchKernelGGL(k_replay_vm<4>, grid, block, lds, stream_, W_, T, d_res_, 0, budget_); break;
    }
    HIP_OK(hipGetLastError());
    hipLaunchKernelGGL(k_eval_reduce, dim3((P + 63) / 64), dim3(64), 0, stream_, d_res_, d_tab_, P);
    HIP_OK(hipGetLastError());
  }

  py::array_t<double> collect(int P) {
    py::array_t<double> out({(py::ssize_t)P, (py::ssize_t)13});
    {
      py::gil_scoped_release rel;
      HIP_OK(hipMemcpyAsync(out.mutable_data(), d_tab_, sizeof(double) * 13 * (size_t)P, hipMemcpyDeviceToHost, stream_));
      HIP_OK(hipStreamSynchronize(stream_));
    }
    return out;
  }

  int device_ = 0;
  hipStream_t stream_ = nullptr;
  DevWorkload W_;
  int npass_ = 1;
  size_t lds_bytes_ = 0;
  size_t heap_pad_bytes_ = 0;
  int num_cus_ = 0;
  size_t max_lds_ = 0;
  std::string arch_;
  int64_t budget_ = 0;
  std::vector<void*> owned_;
  int cap_ = 0;
  DevResult* d_res_ = nullptr;
  double* d_tab_ = nullptr;
  int32_t* d_fam_ = nullptr;
  double* d_w_ = nullptr;
  void* d_code_ = nullptr; size_t code_cap_ = 0;
  void* d_poff_ = nullptr; size_t poff_cap_ = 0;
  void* d_kpay_ = nullptr; size_t kpay_cap_ = 0;
  void* d_ktag_ = nullptr; size_t ktag_cap_ = 0;
};

py::array_t<uint64_t> test_wave_ops(py::array_t<uint64_t, py::array::c_style | py::array::forcecast> vals) {
  if (vals.size() != 64) throw std::invalid_argument("need 64 values");
  uint64_t *din = nullptr, *dout = nullptr;
  HIP_OK(hipMalloc(&din, 64 * 8));
  HIP_OK(hipMalloc(&dout, 130 * 8));
  HIP_OK(hipMemcpy(din, vals.data(), 64 * 8, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_test_wave_ops, dim3(1), dim3(64), 0, 0, din, dout);
  HIP_OK(hipGetLastError());
  py::array_t<uint64_t> out(130);
  HIP_OK(hipMemcpy(out.mutable_data(), dout, 130 * 8, hipMemcpyDeviceToHost));
  (void)hipFree(din);
  (void)hipFree(dout);
  return out;
}

py::tuple test_heap(py::array_t<uint64_t, py::array::c_style | py::array::forcecast> init,
                    py::array_t<int64_t, py::array::c_style | py::array::forcecast> ops, int lb) {
  const int n0 = (int)init.size(), nops = (int)ops.size();
  if (n0 + nops > 4096) throw std::invalid_argument("test heap too large");
  uint64_t *di, *dout, *dpop;
  int64_t* dops;
  int* dn;
  HIP_OK(hipMalloc(&di, (n0 + 1) * 8));
  HIP_OK(hipMalloc(&dops, (nops + 1) * 8));
  HIP_OK(hipMalloc(&dout, 4096 * 8));
  HIP_OK(hipMalloc(&dpop, (nops + 1) * 8));
  HIP_OK(hipMalloc(&dn, 4));
  if (n0) HIP_OK(hipMemcpy(di, init.data(), n0 * 8, hipMemcpyHostToDevice));
  if (nops) HIP_OK(hipMemcpy(dops, ops.data(), nops * 8, hipMemcpyHostToDevice));
  const size_t lds = 4096 * 8 + 1024;
  HIP_OK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_test_heap), hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)lds));
  hipLaunchKernelGGL(k_test_heap, dim3(1), dim3(64), lds, 0, di, n0, dops, nops, lb, dout, dn, dpop);
  HIP_OK(hipGetLastError());
  int n = 0;
  HIP_OK(hipMemcpy(&n, dn, 4, hipMemcpyDeviceToHost));
  py::array_t<uint64_t> out(n), popped(nops);
  if (n) HIP_OK(hipMemcpy(out.mutable_data(), dout, (size_t)n * 8, hipMemcpyDeviceToHost));
  if (nops) HIP_OK(hipMemcpy(popped.mutable_data(), dpop, (size_t)nops * 8, hipMemcpyDeviceToHost));
  for (void* p : {(void*)di, (void*)dops, (void*)dout, (void*)dpop, (void*)dn}) (void)hipFree(p);
  return py::make_tuple(out, popped);
}

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

}  // namespace

PYBIND11_MODULE(_fks_hip, m) {
  m.doc() = "MI355X replay kernels of funsearch_kubernetes_simulator_amd";
  m.def("device_count", &device_count);
  m.def("test_wave_ops", &test_wave_ops);
  m.def("test_heap", &test_heap);
  py::class_<DeviceEngine>(m, "DeviceEngine")
      .def(py::init<py::dict, int>(), py::arg("workload"), py::arg("device") = 0)
      .def("set_options", &DeviceEngine::set_options)
      .def("evaluate_builtin", &DeviceEngine::evaluate_builtin)
      .def("evaluate_programs", &DeviceEngine::evaluate_programs)
      .def("profile", &DeviceEngine::profile)
      .def("launch_builtin_async", &DeviceEngine::launch_builtin_async)
      .def("synchronize", &DeviceEngine::synchronize)
      .def("info", &DeviceEngine::info);
  m.attr("WEIGHTS_PER_POLICY") = kWeights;
  // host builds of the device math, for differential tests against glibc
  m.def("dd_pow", [](double x, double y) { double o = 0; int s = fksd::dd_pow(x, y, o); return py::make_tuple(s, o); });
  m.def("dd_exp", [](double x) { double o = 0; int s = fksd::dd_exp_d(x, o); return py::make_tuple(s, o); });
  m.def("dd_log", [](double x) { double o = 0; int s = fksd::dd_log_d(x, o); return py::make_tuple(s, o); });
  m.def("dd_pow_batch", [](py::array_t<double, py::array::c_style | py::array::forcecast> x,
                           py::array_t<double, py::array::c_style | py::array::forcecast> y) {
    const py::ssize_t n = x.size();
    py::array_t<double> out(n);
    py::array_t<int32_t> st(n);
    for (py::ssize_t i = 0; i < n; ++i) {
      double o = 0;
      st.mutable_data()[i] = fksd::dd_pow(x.data()[i], y.data()[i], o);
      out.mutable_data()[i] = o;
    }
    return py::make_tuple(st, out);
  });
}
