// pybind11 bindings of the native CPU oracle engine (_fks_cpu).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <cstring>
#include <pybind11/stl.h>

#include <atomic>
#include <thread>

#include "builtin_scorers.hpp"
#include "engine.hpp"
#include "parallel.hpp"
#include "seqmatch.hpp"
#include "trace_io.hpp"
#include "vm_cpu.hpp"
#include "../jit/gcn_api.hpp"

namespace py = pybind11;
using namespace fks;

namespace {

template <class T>
std::vector<T> vec(const py::dict& d, const char* key) {
  auto a = py::array_t<T, py::array::c_style | py::array::forcecast>(d[key]);
  return std::vector<T>(a.data(), a.data() + a.size());
}

Workload make_workload(const py::dict& d) {
  Workload w;
  w.cpu_total = vec<int64_t>(d, "node_cpu_total");
  w.cpu_left0 = vec<int64_t>(d, "node_cpu_left");
  w.mem_total = vec<int64_t>(d, "node_mem_total");
  w.mem_left0 = vec<int64_t>(d, "node_mem_left");
  w.gpu_left0 = vec<int32_t>(d, "node_gpu_left");
  w.ngpus = vec<int32_t>(d, "node_ngpus");
  w.gpu_start = vec<int32_t>(d, "gpu_start");
  w.gmilli_total = vec<int32_t>(d, "gpu_milli_total");
  w.gmilli_left0 = vec<int32_t>(d, "gpu_milli_left");
  w.gmem_total = vec<int64_t>(d, "gpu_mem_total");
  w.gmem_left0 = vec<int64_t>(d, "gpu_mem_left");
  w.pcpu = vec<int64_t>(d, "pod_cpu");
  w.pmem = vec<int64_t>(d, "pod_mem");
  w.pngpu = vec<int32_t>(d, "pod_ngpu");
  w.pgmilli = vec<int32_t>(d, "pod_gmilli");
  w.pctime = vec<int64_t>(d, "pod_ctime");
  w.pdur = vec<int64_t>(d, "pod_dur");
  w.prank = vec<int32_t>(d, "pod_rank");
  w.n_nodes = (int32_t)w.cpu_total.size();
  w.n_gpus = (int32_t)w.gmilli_total.size();
  w.n_pods = (int32_t)w.pcpu.size();
  if ((int)w.gpu_start.size() != w.n_nodes + 1) throw std::invalid_argument("gpu_start must have n_nodes+1 entries");
  return w;
}

SimOptions make_options(const py::dict& o) {
  SimOptions s;
  if (o.contains("repush")) s.repush = o["repush"].cast<std::string>() == "earliest" ? REPUSH_EARLIEST : REPUSH_FIRST;
  if (o.contains("gpu_alloc")) s.gpu_alloc = o["gpu_alloc"].cast<std::string>() == "first_fit" ? ALLOC_FIRST_FIT : ALLOC_BEST_FIT;
  if (o.contains("snapshot_interval")) s.snapshot_interval = o["snapshot_interval"].cast<double>();
  if (o.contains("truncate")) s.truncate = o["truncate"].cast<bool>();
  if (o.contains("budget")) s.budget = o["budget"].cast<int64_t>();
  if (o.contains("record_values")) s.record_values = o["record_values"].cast<bool>();
  if (o.contains("record_placements")) s.record_placements = o["record_placements"].cast<bool>();
  if (o.contains("check_invariants")) s.check_invariants = o["check_invariants"].cast<int64_t>();
  if (o.contains("record_states")) s.record_states = o["record_states"].cast<bool>();
  return s;
}

py::dict to_dict(const SimResult& r) {
  py::dict d;
  d["exc"] = r.exc; d["score"] = r.score; d["vm_insns"] = r.vm_insns;
  d["avg_cpu"] = r.avg_cpu; d["avg_mem"] = r.avg_mem;
  d["avg_gpu_count"] = r.avg_gpu_count; d["avg_gpu_milli"] = r.avg_gpu_milli; d["frag"] = r.frag;
  d["n_snapshots"] = r.n_snapshots; d["n_frag_events"] = r.n_frag_events; d["n_events"] = r.n_events;
  d["n_unplaced"] = r.n_unplaced; d["max_nodes"] = r.max_nodes; d["n_repush"] = r.n_repush;
  d["n_dropped"] = r.n_dropped; d["inexact"] = r.inexact; d["trace_hash"] = r.trace_hash;
  if (!r.snap_values.empty()) d["snap_values"] = r.snap_values;
  if (!r.frag_values.empty()) d["frag_values"] = r.frag_values;
  if (!r.placement.empty()) d["placement"] = r.placement;
  if (!r.states.empty()) {
    py::array_t<int32_t> a((py::ssize_t)r.states.size());
    std::memcpy(a.mutable_data(), r.states.data(), r.states.size() * 4);
    d["states"] = a;
  }
  return d;
}

// Result table columns for batch calls (float64 [P, 13]).
constexpr int kCols = 13;
void fill_row(double* row, const SimResult& r) {
  row[0] = r.score; row[1] = r.avg_cpu; row[2] = r.avg_mem; row[3] = r.avg_gpu_count;
  row[4] = r.avg_gpu_milli; row[5] = r.frag; row[6] = (double)r.n_snapshots;
  row[7] = (double)r.n_frag_events; row[8] = (double)r.n_events; row[9] = (double)r.n_unplaced;
  row[10] = (double)r.exc; row[11] = r.inexact ? 1.0 : 0.0; row[12] = (double)(r.trace_hash >> 11);
}


// Scorer calling a natively compiled program (policy/native_codegen.py built
// for the host with g++, ops/jit.py compile_host_module): same ABI as the
// device path (csrc/hip/jit_abi.h ProgFn), one call per node.
typedef int64_t (*HostProgFn)(int32_t, int32_t, int32_t, int32_t, int32_t, int32_t, int32_t, int32_t, int32_t, int32_t,
                              int32_t, int32_t, int32_t, int32_t, int32_t, int32_t, int32_t, int32_t, int32_t, int32_t,
                              int32_t, const int64_t*, int32_t, int32_t, int32_t, int64_t, int32_t,
                              const int64_t*);
struct NativeHostScorer {
  HostProgFn fn;
  const int64_t* kc;
  const std::vector<int64_t>* gmem8;   // [node][8]
  int32_t exc = EXC_NONE;
  ScoreOut operator()(const ScoreCtx& c, int n) {
    ScoreOut o;
    const Workload& w = c.w;
    const int g0 = w.gpu_start[n], ng = w.gpu_start[n + 1] - g0;
    if (ng > 8) { o.exc = EXC_UNSUPPORTED; return o; }
    int32_t gl[8] = {0}, gt[8] = {0};
    for (int j = 0; j < ng; ++j) { gl[j] = c.s.gmilli_left[g0 + j]; gt[j] = w.gmilli_total[g0 + j]; }
    const int64_t r = fn((int32_t)c.s.cpu_left[n], (int32_t)w.cpu_total[n], (int32_t)c.s.mem_left[n],
                         (int32_t)w.mem_total[n],
                         (int32_t)(((uint32_t)c.s.gpu_left[n] & 0xFFFFu) | ((uint32_t)w.ngpus[n] << 16)), gl[0], gl[1], gl[2], gl[3], gl[4],
                         gl[5], gl[6], gl[7], gt[0], gt[1], gt[2], gt[3], gt[4], gt[5], gt[6], gt[7],
                         gmem8->data() + (size_t)n * 8, (int32_t)w.pcpu[c.pod], (int32_t)w.pmem[c.pod],
                         w.pgmilli[c.pod] | (w.pngpu[c.pod] << 16), c.pod_ctime, (int32_t)w.pdur[c.pod], kc);
    if (r < 0) { o.exc = (int32_t)(-r); exc = o.exc; return o; }
    o.v = Num::I(r);
    return o;
  }
};

}  // namespace

template <class T>
py::array_t<T> np_of(const std::vector<T>& v) {
  py::array_t<T> a((py::ssize_t)v.size());
  if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(T));
  return a;
}

namespace fks {

// One-shot evaluation for compiler unit tests: a single node.
static pybind11::object vm_score_once(const Program& prog, const pybind11::dict& pod, const pybind11::dict& node,
                                      const std::vector<int64_t>& gl, const std::vector<int64_t>& gt,
                                      const std::vector<int64_t>& gm) {
  namespace py = pybind11;
  VmCore vm(prog, 1000000);
  vm.resize(1);
  std::vector<int32_t> gl32(gl.begin(), gl.end()), gt32(gt.begin(), gt.end());
  int64_t cpu_left = node["cpu_milli_left"].cast<int64_t>(), cpu_total = node["cpu_milli_total"].cast<int64_t>();
  int64_t mem_left = node["memory_mib_left"].cast<int64_t>(), mem_total = node["memory_mib_total"].cast<int64_t>();
  int32_t gpu_left = node["gpu_left"].cast<int32_t>();
  int32_t ngpus = (int32_t)gl.size();
  int32_t gstart[2] = {0, ngpus};
  VmCore::World W;
  W.pod[PF_CPU] = pod["cpu_milli"].cast<int64_t>(); W.pod[PF_MEM] = pod["memory_mib"].cast<int64_t>();
  W.pod[PF_NGPU] = pod["num_gpu"].cast<int64_t>(); W.pod[PF_GMILLI] = pod["gpu_milli"].cast<int64_t>();
  W.pod[PF_CTIME] = pod["creation_time"].cast<int64_t>(); W.pod[PF_DUR] = pod["duration_time"].cast<int64_t>();
  W.cpu_left = &cpu_left; W.cpu_total = &cpu_total; W.mem_left = &mem_left; W.mem_total = &mem_total;
  W.gpu_left = &gpu_left; W.ngpus = &ngpus; W.gpu_start = gstart;
  W.gmilli_left = gl32.data(); W.gmilli_total = gt32.data(); W.gmem_left = gm.data(); W.gmem_total = gm.data();
  bool ok = vm.run(W);
  if (!ok) return py::make_tuple("exc", vm.exc);
  if (!vm.has_result[0]) return py::make_tuple("none", 0);
  const PyNum& v = vm.result[0];
  if (v.fl) return py::make_tuple("float", v.f);
  return py::make_tuple("int", v.i);
}

}  // namespace fks

#ifndef FKS_SOURCE_HASH
#define FKS_SOURCE_HASH ""
#endif
// provenance marker, found by ops/build.py without importing the module
extern "C" __attribute__((used, visibility("default"))) const char fks_source_mark[] = "FKS_SOURCE_HASH=" FKS_SOURCE_HASH;

PYBIND11_MODULE(_fks_cpu, m) {
  m.attr("SOURCE_HASH") = FKS_SOURCE_HASH;
  m.def("load_pod_csv", [](const std::string& path) {
    fks::PodColumns p;
    try {
      p = fks::load_pods(path);
    } catch (const fks::MissingColumn& e) {
      throw py::key_error(e.what());
    }
    py::dict d;
    d["name"] = p.name; d["gpu_spec"] = p.gpu_spec;
    d["cpu"] = np_of(p.cpu); d["mem"] = np_of(p.mem); d["ngpu"] = np_of(p.ngpu); d["gmilli"] = np_of(p.gmilli);
    d["ctime"] = np_of(p.ctime); d["dur"] = np_of(p.dur);
    return d;
  }, py::arg("path"));
  m.def("load_node_csv", [](const std::string& path, const std::unordered_map<std::string, int64_t>& mem_map) {
    fks::NodeColumns n;
    try {
      n = fks::load_nodes(path, mem_map);
    } catch (const fks::MissingColumn& e) {
      throw py::key_error(e.what());
    }
    py::dict d;
    d["sn"] = n.sn;
    d["cpu"] = np_of(n.cpu); d["mem"] = np_of(n.mem); d["gpu_count"] = np_of(n.gpu_count);
    d["ngpus"] = np_of(n.ngpus); d["gpu_mem"] = np_of(n.gpu_mem);
    return d;
  }, py::arg("path"), py::arg("gpu_mem_mapping"));
  m.doc() = "Native CPU oracle engine of funsearch_kubernetes_simulator_amd";
  py::class_<Workload>(m, "Workload")
      .def(py::init(&make_workload))
      .def_readonly("n_nodes", &Workload::n_nodes)
      .def_readonly("n_gpus", &Workload::n_gpus)
      .def_readonly("n_pods", &Workload::n_pods);

  m.def("simulate_builtin", [](const Workload& w, int family, std::vector<double> weights, py::dict opts) {
    BuiltinScorer sc; sc.family = family;
    for (size_t i = 0; i < weights.size() && i < 16; ++i) sc.w[i] = weights[i];
    SimOptions o = make_options(opts);
    SimResult r;
    { py::gil_scoped_release rel; r = simulate(w, sc, o); }
    return to_dict(r);
  }, py::arg("workload"), py::arg("family"), py::arg("weights") = std::vector<double>{}, py::arg("options") = py::dict());

  m.def("simulate_builtin_batch", [](const Workload& w, int family,
                                     py::array_t<double, py::array::c_style | py::array::forcecast> weights,
                                     py::dict opts, int threads) {
    const int64_t P = weights.shape(0), K = weights.ndim() > 1 ? weights.shape(1) : 0;
    SimOptions o = make_options(opts);
    py::array_t<double> out({P, (int64_t)kCols});
    double* op = out.mutable_data();
    const double* wp = weights.data();
    {
      py::gil_scoped_release rel;
      parallel_for(P, threads, [&](int64_t i) {
        BuiltinScorer sc; sc.family = family;
        for (int64_t k = 0; k < K && k < 16; ++k) sc.w[k] = wp[i * K + k];
        SimResult r = simulate(w, sc, o);
        fill_row(op + i * kCols, r);
      });
    }
    return out;
  }, py::arg("workload"), py::arg("family"), py::arg("weights"), py::arg("options") = py::dict(), py::arg("threads") = 1);

  m.def("simulate_program", [](const Workload& w, py::bytes code, std::vector<double> fconst,
                               std::vector<int64_t> iconst, std::vector<uint8_t> ctag, py::dict opts) {
    Program prog = make_program(std::string(code), fconst, iconst, ctag);
    SimOptions o = make_options(opts);
    SimResult r;
    {
      py::gil_scoped_release rel;
      VmScorer sc(prog, o.budget);
      r = simulate(w, sc, o);
      if (r.exc == EXC_NONE && sc.exc) r.exc = sc.exc;
      r.vm_insns = sc.insns;
    }
    return to_dict(r);
  }, py::arg("workload"), py::arg("code"), py::arg("fconst"), py::arg("iconst"), py::arg("ctag"), py::arg("options") = py::dict());

  m.def("simulate_program_batch", [](const Workload& w, std::vector<py::bytes> codes,
                                     std::vector<std::vector<double>> fconsts,
                                     std::vector<std::vector<int64_t>> iconsts,
                                     std::vector<std::vector<uint8_t>> ctags, py::dict opts, int threads) {
    const int64_t P = (int64_t)codes.size();
    std::vector<Program> progs;
    for (int64_t i = 0; i < P; ++i) progs.push_back(make_program(std::string(codes[i]), fconsts[i], iconsts[i], ctags[i]));
    SimOptions o = make_options(opts);
    py::array_t<double> out({P, (int64_t)kCols});
    double* op = out.mutable_data();
    {
      py::gil_scoped_release rel;
      parallel_for(P, threads, [&](int64_t i) {
        VmScorer sc(progs[i], o.budget);
        SimResult r = simulate(w, sc, o);
        if (r.exc == EXC_NONE && sc.exc) r.exc = sc.exc;
        fill_row(op + i * kCols, r);
      });
    }
    return out;
  }, py::arg("workload"), py::arg("codes"), py::arg("fconsts"), py::arg("iconsts"), py::arg("ctags"),
     py::arg("options") = py::dict(), py::arg("threads") = 1);

  m.def("simulate_native_batch", [](const Workload& w, std::vector<uint64_t> fns,
                                    py::array_t<int64_t, py::array::c_style | py::array::forcecast> kc,
                                    py::array_t<int32_t, py::array::c_style | py::array::forcecast> koff,
                                    py::dict opts, int threads) {
    const int64_t P = (int64_t)fns.size();
    if ((int64_t)koff.size() != P) throw std::invalid_argument("koff must have one entry per program");
    for (int n = 0; n < w.n_nodes; ++n) {
      const int64_t vals[4] = {w.cpu_total[n], w.cpu_left0[n], w.mem_total[n], w.mem_left0[n]};
      for (int64_t v : vals)
        if (v > INT32_MAX || v < -(int64_t)INT32_MAX) throw std::invalid_argument("node resources outside int32");
    }
    for (int i = 0; i < w.n_pods; ++i)
      if (w.pgmilli[i] >= (1 << 16) || w.pngpu[i] >= (1 << 8) || w.pcpu[i] > INT32_MAX || w.pmem[i] > INT32_MAX ||
          w.pdur[i] > INT32_MAX)
        throw std::invalid_argument("pod request outside the native ABI's packing");
    std::vector<int64_t> gmem8((size_t)w.n_nodes * 8, 0);
    for (int n = 0; n < w.n_nodes; ++n)
      for (int j = 0; j < std::min(8, w.gpu_start[n + 1] - w.gpu_start[n]); ++j)
        gmem8[(size_t)n * 8 + j] = w.gmem_total[w.gpu_start[n] + j];
    SimOptions o = make_options(opts);
    py::array_t<double> out({P, (int64_t)kCols});
    double* op = out.mutable_data();
    const int64_t* kp = kc.data();
    const int32_t* ko = koff.data();
    {
      py::gil_scoped_release rel;
      parallel_for(P, threads, [&](int64_t i) {
        NativeHostScorer sc{reinterpret_cast<HostProgFn>(fns[i]), kp + ko[i], &gmem8};
        SimResult r = simulate(w, sc, o);
        if (r.exc == EXC_NONE && sc.exc) r.exc = sc.exc;
        fill_row(op + i * kCols, r);
      });
    }
    return out;
  }, py::arg("workload"), py::arg("fns"), py::arg("kc"), py::arg("koff"), py::arg("options") = py::dict(),
     py::arg("threads") = 1);

  m.def("score_program_once", [](py::bytes code, std::vector<double> fconst, std::vector<int64_t> iconst,
                                 std::vector<uint8_t> ctag, py::dict pod, py::dict node, std::vector<int64_t> gpu_left,
                                 std::vector<int64_t> gpu_total, std::vector<int64_t> gpu_mem) {
    // Single (pod, node) evaluation of a program; used by compiler unit tests.
    Program prog = make_program(std::string(code), fconst, iconst, ctag);
    return vm_score_once(prog, pod, node, gpu_left, gpu_total, gpu_mem);
  });

  m.def("seq_ratio", [](const std::u32string& a, const std::u32string& b) {
    // difflib.SequenceMatcher(None, a, b).ratio(), exactly
    return SeqMatcher(a, b).ratio();
  });
  m.def("similar_at_least", [](const std::u32string& a, const std::u32string& b, double threshold) {
    // difflib.SequenceMatcher(None, a, b).ratio() >= threshold
    return SeqMatcher(a, b).at_least(threshold);
  });
  m.def("similar_to_any", [](const std::u32string& a, const std::vector<std::u32string>& bs, double threshold,
                             int threads) {
    // the index of some b with difflib ratio(a, b) >= threshold, or -1: the
    // similarity gate of one child against a population, off the GIL (the
    // steady search's stager and collection threads keep running) and over
    // `threads` host threads (a 4 kB pair is ~0.1-1 ms; an island holds ~20)
    py::gil_scoped_release rel;
    const size_t n = bs.size();
    const size_t T = std::min<size_t>(n, (size_t)std::max(1, threads));
    if (T <= 1) {
      for (size_t i = 0; i < n; ++i)
        if (SeqMatcher(a, bs[i]).at_least(threshold)) return (int64_t)i;
      return (int64_t)-1;
    }
    std::atomic<size_t> next{0};
    std::atomic<int64_t> found{-1};
    auto work = [&] {
      for (size_t i; found.load(std::memory_order_relaxed) < 0 && (i = next.fetch_add(1)) < n;)
        if (SeqMatcher(a, bs[i]).at_least(threshold)) found.store((int64_t)i);
    };
    std::vector<std::thread> pool;
    for (size_t t = 1; t < T; ++t) pool.emplace_back(work);
    work();
    for (auto& th : pool) th.join();
    return found.load();
  }, py::arg("a"), py::arg("bs"), py::arg("threshold"), py::arg("threads") = 1);
  m.def("exact_mean", [](std::vector<double> xs) {
    FixedAcc a; for (double x : xs) a.add(x);
    return py::make_tuple(fixed_mean(a), a.inexact);
  });

  // ---- baseline program JIT (csrc/jit): bytecode -> gfx950 machine code
  m.def("gcn_compile", [](py::bytes code, py::array_t<uint8_t, py::array::c_style | py::array::forcecast> ctag,
                          py::array_t<uint8_t, py::array::c_style | py::array::forcecast> is_lit,
                          py::array_t<int64_t, py::array::c_style | py::array::forcecast> iconst,
                          py::array_t<double, py::array::c_style | py::array::forcecast> fconst) {
    const std::string c = code;
    gcnapi::ProgramDesc p;
    p.code = reinterpret_cast<const uint8_t*>(c.data());
    p.code_bytes = c.size();
    p.ctag = ctag.data(); p.is_lit = is_lit.data(); p.iconst = iconst.data(); p.fconst = fconst.data();
    p.n_const = (size_t)ctag.size();
    if ((size_t)is_lit.size() != p.n_const || (size_t)iconst.size() != p.n_const || (size_t)fconst.size() != p.n_const)
      throw std::invalid_argument("constant arrays differ in length");
    gcnapi::Result r;
    {
      py::gil_scoped_release rel;
      r = gcnapi::compile(p);
    }
    py::dict out;
    out["ok"] = r.ok;
    out["reason"] = r.reason;
    out["elided"] = r.elided;
    out["words"] = np_of(r.words);
    out["relocs"] = np_of(r.relocs);
    out["n_insns"] = r.n_insns; out["vgprs"] = r.vgprs; out["sgprs"] = r.sgprs; out["calls"] = r.calls;
    out["vregs"] = r.vregs; out["tagged"] = r.tagged; out["mir"] = r.mir; out["spills"] = r.spills; out["unrolled"] = r.unrolled;
    return out;
  }, py::arg("code"), py::arg("ctag"), py::arg("is_lit"), py::arg("iconst"), py::arg("fconst"));
  // A batch of programs on `threads` host threads (the generator is
  // re-entrant): one dict per program, as gcn_compile.  The steady-state
  // search and the novel-program bench compile hundreds of new shapes at once.
  m.def("gcn_compile_many", [](py::list progs, int threads) {
    struct Owned {
      std::string code;
      std::vector<uint8_t> ctag, is_lit;
      std::vector<int64_t> iconst;
      std::vector<double> fconst;
      int elide_lo = 0, elide_hi = 0;
    };
    const size_t n = progs.size();
    std::vector<Owned> own(n);
    for (size_t i = 0; i < n; ++i) {
      py::tuple t = progs[i].cast<py::tuple>();
      if (t.size() != 5 && t.size() != 7)
        throw std::invalid_argument("program tuple: (code, ctag, is_lit, iconst, fconst[, elide_lo, elide_hi])");
      if (t.size() == 7) {
        own[i].elide_lo = t[5].cast<int>();
        own[i].elide_hi = t[6].cast<int>();
      }
      own[i].code = t[0].cast<std::string>();
      auto ct = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>(t[1]);
      auto il = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>(t[2]);
      auto ic = py::array_t<int64_t, py::array::c_style | py::array::forcecast>(t[3]);
      auto fc = py::array_t<double, py::array::c_style | py::array::forcecast>(t[4]);
      if (il.size() != ct.size() || ic.size() != ct.size() || fc.size() != ct.size())
        throw std::invalid_argument("constant arrays differ in length");
      own[i].ctag.assign(ct.data(), ct.data() + ct.size());
      own[i].is_lit.assign(il.data(), il.data() + il.size());
      own[i].iconst.assign(ic.data(), ic.data() + ic.size());
      own[i].fconst.assign(fc.data(), fc.data() + fc.size());
    }
    std::vector<gcnapi::Result> res(n);
    {
      py::gil_scoped_release rel;
      std::atomic<size_t> next{0};
      auto work = [&]() {
        for (size_t i = next++; i < n; i = next++) {
          gcnapi::ProgramDesc p;
          p.code = reinterpret_cast<const uint8_t*>(own[i].code.data());
          p.code_bytes = own[i].code.size();
          p.ctag = own[i].ctag.data(); p.is_lit = own[i].is_lit.data();
          p.iconst = own[i].iconst.data(); p.fconst = own[i].fconst.data();
          p.n_const = own[i].ctag.size();
          p.elide_lo = own[i].elide_lo;
          p.elide_hi = own[i].elide_hi;
          res[i] = gcnapi::compile(p);
        }
      };
      const int nt = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::max(1, threads), n));
      std::vector<std::thread> pool;
      for (int t = 1; t < nt; ++t) pool.emplace_back(work);
      work();
      for (auto& th : pool) th.join();
    }
    py::list out;
    for (const auto& r : res) {
      py::dict d;
      d["ok"] = r.ok;
      d["reason"] = r.reason;
      d["elided"] = r.elided;
      d["words"] = np_of(r.words);
      d["relocs"] = np_of(r.relocs);
      d["n_insns"] = r.n_insns; d["vgprs"] = r.vgprs; d["sgprs"] = r.sgprs; d["calls"] = r.calls;
      d["vregs"] = r.vregs; d["tagged"] = r.tagged; d["mir"] = r.mir; d["spills"] = r.spills; d["unrolled"] = r.unrolled;
      out.append(d);
    }
    return out;
  }, py::arg("programs"), py::arg("threads") = 1);
  // Link a batch into a code-object skeleton: program i at arena offset
  // offsets[i] (align-byte aligned), its runtime-table references relocated
  // (PC-relative: lo / hi literal words at byte pc of the s_getpc), and the
  // runtime table's initial value written into the image, so loading needs no
  // device-side fix-up.  Returns (image, offsets) or raises if the arena is
  // too small.
  m.def("gcn_link", [](py::bytes skel, int64_t arena_off, int64_t arena_vaddr, int64_t capacity, int64_t rt_vaddr,
                       int64_t rt_off, py::array_t<uint64_t, py::array::c_style | py::array::forcecast> rt_vals,
                       py::list words, py::list relocs, int64_t align) {
    std::string img = skel;
    const size_t n = words.size();
    if (relocs.size() != n) throw std::invalid_argument("one relocation array per program");
    if (align <= 0 || (align & (align - 1))) throw std::invalid_argument("align must be a power of two");
    py::array_t<int64_t> offs((py::ssize_t)n);
    int64_t pos = 0;
    for (size_t i = 0; i < n; ++i) {
      auto w = py::array_t<uint32_t, py::array::c_style | py::array::forcecast>(words[i]);
      auto r = py::array_t<uint32_t, py::array::c_style | py::array::forcecast>(relocs[i]);
      const int64_t bytes = (int64_t)w.size() * 4;
      if (pos + bytes > capacity) throw std::length_error("batch exceeds the skeleton arena");
      if (arena_off + pos + bytes > (int64_t)img.size()) throw std::length_error("arena outside the image");
      std::vector<uint32_t> code(w.data(), w.data() + w.size());
      if (r.size() % 3) throw std::invalid_argument("relocations come in triples");
      for (py::ssize_t k = 0; k + 2 < r.size(); k += 3) {
        const uint32_t lo = r.data()[k], hi = r.data()[k + 1], pc = r.data()[k + 2];
        if (lo >= code.size() || hi >= code.size()) throw std::out_of_range("relocation outside the program");
        const int64_t d = rt_vaddr - (arena_vaddr + pos + (int64_t)pc);
        code[lo] = (uint32_t)((uint64_t)d & 0xFFFFFFFFull);
        code[hi] = (uint32_t)(((uint64_t)d >> 32) & 0xFFFFFFFFull);
      }
      std::memcpy(&img[(size_t)(arena_off + pos)], code.data(), (size_t)bytes);
      offs.mutable_data()[i] = pos;
      pos += (bytes + align - 1) / align * align;
    }
    if (rt_off >= 0) {
      if (rt_off + rt_vals.size() * 8 > (py::ssize_t)img.size()) throw std::length_error("runtime table outside the image");
      std::memcpy(&img[(size_t)rt_off], rt_vals.data(), (size_t)rt_vals.size() * 8);
    }
    return py::make_tuple(py::bytes(img), offs);
  }, py::arg("skeleton"), py::arg("arena_off"), py::arg("arena_vaddr"), py::arg("capacity"), py::arg("rt_vaddr"),
     py::arg("rt_off"), py::arg("rt_vals"), py::arg("words"), py::arg("relocs"), py::arg("align") = 256);
  // test hook: at most `pairs` VGPR pairs for virtual registers (0: no cap),
  // which sends ordinary programs down the spill path
  m.def("gcn_set_pair_cap", [](int pairs) { fks::gcnapi::set_pair_cap(pairs); });
  // unrolling of node.gpus loops: max expanded body (bytecode insns); 0 = off; returns the previous cap
  m.def("gcn_set_unroll_cap", [](int cap) { return fks::gcnapi::set_unroll_cap(cap); });
  m.def("gcn_listing", [](py::bytes code, std::vector<uint8_t> ctag, std::vector<uint8_t> is_lit,
                          std::vector<int64_t> iconst, std::vector<double> fconst, int elide_lo, int elide_hi) {
    const std::string c = code;
    gcnapi::ProgramDesc p;
    p.code = reinterpret_cast<const uint8_t*>(c.data());
    p.code_bytes = c.size();
    p.ctag = ctag.data(); p.is_lit = is_lit.data(); p.iconst = iconst.data(); p.fconst = fconst.data();
    p.n_const = ctag.size();
    p.elide_lo = elide_lo;
    p.elide_hi = elide_hi;
    return gcnapi::listing(p);
  }, py::arg("code"), py::arg("ctag"), py::arg("is_lit"), py::arg("iconst"), py::arg("fconst"),
     py::arg("elide_lo") = 0, py::arg("elide_hi") = 0);
  m.def("gcn_emu_event", [](py::bytes code, std::vector<uint8_t> ctag, std::vector<uint8_t> is_lit,
                            std::vector<int64_t> iconst, std::vector<double> fconst, std::vector<int64_t> kc,
                            std::vector<int64_t> node, std::vector<int32_t> gl, std::vector<int32_t> gt,
                            std::vector<int64_t> gmem, std::vector<int64_t> pod, int elide_lo, int elide_hi) {
    const std::string c = code;
    gcnapi::ProgramDesc p;
    p.code = reinterpret_cast<const uint8_t*>(c.data());
    p.code_bytes = c.size();
    p.ctag = ctag.data(); p.is_lit = is_lit.data(); p.iconst = iconst.data(); p.fconst = fconst.data();
    p.n_const = ctag.size();
    p.elide_lo = elide_lo;
    p.elide_hi = elide_hi;
    return gcnapi::emu_event(p, kc, node, gl, gt, gmem, pod);
  }, py::arg("code"), py::arg("ctag"), py::arg("is_lit"), py::arg("iconst"), py::arg("fconst"), py::arg("kc"),
     py::arg("node"), py::arg("gl"), py::arg("gt"), py::arg("gmem"), py::arg("pod"), py::arg("elide_lo") = 0,
     py::arg("elide_hi") = 0);
  m.def("gcn_emu_profile", [](bool on) { gcnapi::emu_profile(on); });
  m.def("gcn_emu_profile_counts", []() {
    py::dict d;
    for (const auto& kv : gcnapi::emu_profile_counts()) d[py::str(kv.first)] = kv.second;
    return d;
  });
  m.def("gcn_emu_batch", [](const Workload& w, std::vector<py::bytes> codes, std::vector<std::vector<uint8_t>> ctags,
                            std::vector<std::vector<uint8_t>> lits, std::vector<std::vector<int64_t>> iconsts,
                            std::vector<std::vector<double>> fconsts, std::vector<std::vector<int64_t>> kcs,
                            py::dict opts, int threads, std::vector<std::pair<int, int>> elide) {
    const size_t P = codes.size();
    std::vector<std::string> cs(P);
    std::vector<gcnapi::ProgramDesc> ps(P);
    for (size_t i = 0; i < P; ++i) {
      cs[i] = codes[i];
      ps[i].code = reinterpret_cast<const uint8_t*>(cs[i].data());
      ps[i].code_bytes = cs[i].size();
      ps[i].ctag = ctags[i].data(); ps[i].is_lit = lits[i].data(); ps[i].iconst = iconsts[i].data();
      ps[i].fconst = fconsts[i].data(); ps[i].n_const = ctags[i].size();
      if (i < elide.size()) { ps[i].elide_lo = elide[i].first; ps[i].elide_hi = elide[i].second; }
    }
    SimOptions o = make_options(opts);
    std::vector<SimResult> rs;
    {
      py::gil_scoped_release rel;
      rs = gcnapi::emu_simulate_batch(w, ps, kcs, o, threads);
    }
    py::array_t<double> out({(int64_t)P, (int64_t)kCols});
    for (size_t i = 0; i < P; ++i) fill_row(out.mutable_data() + i * kCols, rs[i]);
    return out;
  }, py::arg("w"), py::arg("codes"), py::arg("ctags"), py::arg("lits"), py::arg("iconsts"), py::arg("fconsts"),
     py::arg("kcs"), py::arg("opts"), py::arg("threads"), py::arg("elide") = std::vector<std::pair<int, int>>{});
  m.attr("RESULT_COLUMNS") = py::make_tuple("score", "avg_cpu", "avg_mem", "avg_gpu_count", "avg_gpu_milli",
                                            "frag", "n_snapshots", "n_frag_events", "n_events", "n_unplaced",
                                            "exc", "inexact", "trace_hash_hi");
}
