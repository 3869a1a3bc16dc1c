// Standalone native self-test of the C++ engine, built with host sanitizers
// (tools/sanitize_cpu.sh: -fsanitize=address,undefined).  Loads the default
// OpenB trace with the native CSV reader, replays first-fit, best-fit and a
// random-linear policy with the invariant checker on, and compares the
// first-fit / best-fit scores with the reference's published values
// (BASELINE.md).  Optionally replays compiled policy programs through the CPU
// bytecode VM: argv[2] names a directory of `<name>.code` (raw Insn array) +
// `<name>.consts` (one "tag payload" line per constant; float payloads are the IEEE bits)
// pairs written by tools/sanitize_cpu.py, which compares the printed scores
// with the regular (unsanitized) extension.  Finally the same policies run as
// one batch on argv[3] threads (default 4) over the shared workload and must
// reproduce the serial results (the ThreadSanitizer build checks the batch
// path for races).  Exit status 0 = all exact.
#include <algorithm>
#include <dirent.h>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>

#include "builtin_scorers.hpp"
#include "engine.hpp"
#include "parallel.hpp"
#include "trace_io.hpp"
#include "vm_cpu.hpp"

using namespace fks;

static std::unordered_map<std::string, int64_t> read_mem_mapping(const std::string& path) {
  std::ifstream in(path);
  std::stringstream ss;
  ss << in.rdbuf();
  const std::string s = ss.str();
  std::unordered_map<std::string, int64_t> m;
  size_t i = 0;
  while ((i = s.find('"', i)) != std::string::npos) {
    const size_t j = s.find('"', i + 1);
    if (j == std::string::npos) break;
    const std::string key = s.substr(i + 1, j - i - 1);
    size_t k = s.find(':', j);
    if (k == std::string::npos) break;
    ++k;
    while (k < s.size() && (s[k] == ' ' || s[k] == '\n')) ++k;
    m[key] = std::strtoll(s.c_str() + k, nullptr, 10);
    i = s.find_first_of(",}", k);
  }
  return m;
}

static Workload build(const std::string& dir) {
  const auto mem = read_mem_mapping(dir + "/gpu_mem_mapping.json");
  const NodeColumns n = load_nodes(dir + "/csv/gpu_models_filtered.csv", mem);
  const PodColumns p = load_pods(dir + "/csv/openb_pod_list_default.csv");
  Workload w;
  w.n_nodes = (int32_t)n.sn.size();
  w.cpu_total = n.cpu; w.cpu_left0 = n.cpu;
  w.mem_total = n.mem; w.mem_left0 = n.mem;
  w.gpu_left0 = n.gpu_count; w.ngpus = n.ngpus;
  w.gpu_start.assign(w.n_nodes + 1, 0);
  for (int i = 0; i < w.n_nodes; ++i) {
    w.gpu_start[i + 1] = w.gpu_start[i] + n.ngpus[i];
    for (int g = 0; g < n.ngpus[i]; ++g) {
      w.gmilli_total.push_back(1000); w.gmilli_left0.push_back(1000);
      w.gmem_total.push_back(n.gpu_mem[i]); w.gmem_left0.push_back(n.gpu_mem[i]);
    }
  }
  w.n_gpus = (int32_t)w.gmilli_total.size();
  w.n_pods = (int32_t)p.name.size();
  w.pcpu = p.cpu; w.pmem = p.mem; w.pngpu = p.ngpu; w.pgmilli = p.gmilli; w.pctime = p.ctime; w.pdur = p.dur;
  // dense rank of the pod ids in string order (the heap tie-break key)
  std::vector<std::string> ids = p.name;
  std::sort(ids.begin(), ids.end());
  ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
  for (const auto& s : p.name)
    w.prank.push_back((int32_t)(std::lower_bound(ids.begin(), ids.end(), s) - ids.begin()));
  return w;
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "data/traces";
  const Workload w = build(dir);
  SimOptions o;
  o.check_invariants = 97;
  const double golden[2] = {0.42920557012850735, 0.44654782731316534};
  int bad = 0;
  for (int fam = 0; fam < 3; ++fam) {
    BuiltinScorer sc;
    sc.family = fam;
    if (fam == FAM_RANDOM_LINEAR) { sc.w[0] = 2500.0; sc.w[1] = 0.003; sc.w[2] = 0.0002; sc.w[3] = 300.0; }
    const SimResult r = simulate(w, sc, o);
    std::printf("family %d: exc %d score %.17g events %lld snapshots %lld\n", fam, r.exc, r.score,
                (long long)r.n_events, (long long)r.n_snapshots);
    if (r.exc != EXC_NONE) ++bad;
    if (fam < 2 && r.score != golden[fam]) ++bad;
  }
  std::vector<std::string> pnames;
  std::vector<Program> progs;
  if (argc > 2) {
    const std::string pdir = argv[2];
    if (DIR* d = opendir(pdir.c_str())) {
      while (dirent* e = readdir(d)) {
        const std::string f = e->d_name;
        if (f.size() > 5 && f.compare(f.size() - 5, 5, ".code") == 0) pnames.push_back(f.substr(0, f.size() - 5));
      }
      closedir(d);
    }
    std::sort(pnames.begin(), pnames.end());
    for (const auto& nm : pnames) {
      std::ifstream cf(pdir + "/" + nm + ".code", std::ios::binary);
      const std::string code((std::istreambuf_iterator<char>(cf)), std::istreambuf_iterator<char>());
      std::ifstream kf(pdir + "/" + nm + ".consts");
      std::vector<double> fk; std::vector<int64_t> ik; std::vector<uint8_t> tk;
      long long tag, iv;   // float constants carry their IEEE-754 bits
      while (kf >> tag >> iv) {
        double fv; std::memcpy(&fv, &iv, 8);
        tk.push_back((uint8_t)tag); ik.push_back(iv); fk.push_back(fv);
      }
      progs.push_back(make_program(code, fk, ik, tk));
    }
  }
  SimOptions po = o;
  po.budget = 1 << 22;
  auto run_prog = [&](size_t i) {
    VmScorer sc(progs[i], po.budget);
    SimResult r = simulate(w, sc, po);
    if (r.exc == EXC_NONE && sc.exc) r.exc = sc.exc;
    r.vm_insns = sc.insns;
    return r;
  };
  std::vector<SimResult> serial;
  for (size_t i = 0; i < progs.size(); ++i) {
    serial.push_back(run_prog(i));
    std::printf("program %s: exc %d score %.17g insns %lld\n", pnames[i].c_str(), serial[i].exc, serial[i].score,
                (long long)serial[i].vm_insns);
  }
  // threaded batch: builtin random-linear weights + every program, shared inputs
  const int threads = argc > 3 ? std::atoi(argv[3]) : 4;
  constexpr int kLinear = 8;
  const int64_t total = kLinear + (int64_t)progs.size();
  std::vector<SimResult> batch(total);
  auto linear = [&](int64_t i) {
    BuiltinScorer sc;
    sc.family = FAM_RANDOM_LINEAR;
    for (int k = 0; k < 4; ++k) sc.w[k] = 1.0 + 0.37 * (double)((i * 7 + k * 3) % 11);
    return simulate(w, sc, o);
  };
  parallel_for(total, threads, [&](int64_t i) { batch[i] = i < kLinear ? linear(i) : run_prog(i - kLinear); });
  int diff = 0;
  for (int64_t i = 0; i < total; ++i) {
    const SimResult ref = i < kLinear ? linear(i) : serial[i - kLinear];
    if (ref.exc != batch[i].exc || ref.score != batch[i].score || ref.trace_hash != batch[i].trace_hash) ++diff;
  }
  std::printf("threaded batch: %lld policies on %d threads, %d differ from serial\n", (long long)total, threads, diff);
  bad += diff;
  std::printf("%s\n", bad ? "SELFTEST FAILED" : "selftest ok");
  return bad ? 1 : 0;
}
