// Baseline program JIT: API of the code generator (gcn_codegen.hpp) and the
// emulator-backed replays used to validate it on the CPU.  Compiled into the
// _fks_cpu extension (ops/build.py) as its own translation unit, because the
// runtime-library host build it emulates (pyops_dev.h under FKS_HOST_JIT)
// defines HIP-style attribute macros.
#include <chrono>
#include <cstdlib>
#include <mutex>
#include <cstring>
#include <sstream>
#include <string>
#include <vector>

#include "../cpu/engine.hpp"
#include "../cpu/parallel.hpp"
#include "gcn_api.hpp"

#define FKS_HOST_JIT 1
#include "gcn_codegen.hpp"
#include "gcn_emu.hpp"

namespace fks {
namespace gcnapi {

namespace {

gcn::ProgIn make_in(const ProgramDesc& p) {
  if (p.code_bytes % 8 != 0) throw gcn::CodegenError("bytecode length is not a multiple of 8");
  gcn::ProgIn in;
  in.code = reinterpret_cast<const Insn*>(p.code);
  in.n = (int)(p.code_bytes / 8);
  in.ctag = p.ctag;
  in.is_lit = p.is_lit;
  in.iconst = p.iconst;
  in.fconst = p.fconst;
  in.n_const = (int)p.n_const;
  in.elide_lo = p.elide_lo;
  in.elide_hi = p.elide_hi;
  return in;
}

const char* reg_name(uint16_t c, char* buf) {
  using namespace gcn;
  if (c == NONE) return "-";
  if (c >= 256) { std::snprintf(buf, 16, "v%d", c - 256); return buf; }
  if (c == VCC) return "vcc";
  if (c == EXEC) return "exec";
  if (c == LIT) return "lit";
  if (c >= 128 && c <= 208) {
    std::snprintf(buf, 16, "#%d", c <= 192 ? c - 128 : 192 - c);
    return buf;
  }
  if (c >= 240 && c <= 247) {
    static const char* f[] = {"0.5", "-0.5", "1.0", "-1.0", "2.0", "-2.0", "4.0", "-4.0"};
    return f[c - 240];
  }
  std::snprintf(buf, 16, "s%d", c);
  return buf;
}

}  // namespace

// Code for one program: with its feasibility prologue compiled out (when the
// caller asks) and its node.gpus loops unrolled, else without either, in that
// order of preference (a program the first form does not fit -- registers,
// SGPR frames -- usually fits the next); *elided: the prologue is out.
gcn::Func generate(gcn::ProgIn in, gcn::GenStats* st, bool* elided) {
  const bool can_elide = in.elide_lo < in.elide_hi;
  std::string first_error;
  for (int attempt = 0; attempt < 4; ++attempt) {
    const bool elide = attempt < 2, unroll = attempt % 2 == 0;
    if (elide && !can_elide) continue;
    gcn::ProgIn q = in;
    if (!elide) q.elide_lo = q.elide_hi = 0;   // the whole program (valid for any caller)
    q.no_unroll = !unroll;
    try {
      if (st) *st = gcn::GenStats{};
      gcn::Codegen cg(q);
      gcn::Func f = cg.run(st);
      if (elided) *elided = elide;
      return f;
    } catch (const gcn::CodegenError& e) {
      if (first_error.empty()) first_error = e.what();
    }
  }
  throw gcn::CodegenError(first_error);
}

Result compile(const ProgramDesc& p) {
  Result r;
  try {
    gcn::ProgIn in = make_in(p);
    gcn::GenStats st;
    bool elided = false;
    gcn::Func f = generate(in, &st, &elided);
    r.elided = elided;
    gcn::Code code = gcn::assemble(f);
    r.words = std::move(code.words);
    for (const gcn::Reloc& rl : code.relocs) {
      r.relocs.push_back(rl.lo_word);
      r.relocs.push_back(rl.hi_word);
      r.relocs.push_back(rl.pc_off);
    }
    r.n_insns = code.n_insns;
    r.vgprs = st.vgprs_used;
    r.sgprs = st.sgprs_used;
    r.calls = st.calls;
    r.vregs = st.vregs;
    r.tagged = st.tagged;
    r.spills = st.spills;
    r.unrolled = st.unrolled;
    r.mir = (int)f.mi.size();
    r.ok = true;
  } catch (const std::exception& e) {
    r.ok = false;
    r.reason = e.what();
  }
  return r;
}

void set_pair_cap(int pairs) { gcn::pair_cap() = pairs < 0 ? 0 : pairs; }

int set_unroll_cap(int cap) {
  const int old = gcn::unroll_cap();
  gcn::unroll_cap() = cap < 0 ? 0 : cap;
  return old;
}

std::string listing(const ProgramDesc& p) {
  std::ostringstream os;
  try {
    gcn::ProgIn in = make_in(p);
    gcn::Func f = generate(in, nullptr, nullptr);
    char b0[16], b1[16], b2[16], b3[16], b4[16];
    int last_bc = -1;
    for (const gcn::MI& m : f.mi) {
      if (m.bc != last_bc) {
        last_bc = m.bc;
        os << "    ; bc " << (int)m.bc << "\n";
      }
      if (m.op == gcn::LABEL) { os << "L" << m.imm << ":\n"; continue; }
      os << "  " << gcn::info(m.op).name << " d=" << reg_name(m.d, b0) << " sd=" << reg_name(m.sd, b1)
         << " s0=" << reg_name(m.s0, b2) << " s1=" << reg_name(m.s1, b3) << " s2=" << reg_name(m.s2, b4);
      if (m.s0 == gcn::LIT || m.s1 == gcn::LIT || m.s2 == gcn::LIT) os << " lit=0x" << std::hex << m.lit << std::dec;
      if (m.imm) os << " imm=" << m.imm;
      if (m.neg) os << " neg=" << (int)m.neg;
      if (m.abs) os << " abs=" << (int)m.abs;
      os << "\n";
    }
  } catch (const std::exception& e) {
    os << "error: " << e.what() << "\n";
  }
  return os.str();
}

namespace {

constexpr uint64_t kRetMagic = 0xFEEDFACE00C0FFEEull;

// Scorer: on the first node of every creation event, one emulated wave scores
// all nodes (lanes = nodes), exactly as the replay kernel calls the program.
struct EmuScorer {
  const gcn::Func* f;
  const std::vector<int64_t>* kc;
  const std::vector<int64_t>* gmem8;
  gcn::Emu* emu;
  std::vector<int64_t> res;
  int32_t exc = EXC_NONE;
  bool feas_only = false;   // called for feasible nodes only (code without its prologue), others score 0
  uint64_t poison_seq = 0;
  bool traced = false;

  ScoreOut operator()(const ScoreCtx& c, int n) {
    if (n == 0) run_event(c);
    ScoreOut o;
    const int64_t r = res[(size_t)n];
    if (r < 0) { o.exc = (int32_t)(-r); exc = o.exc; return o; }
    o.v = Num::I(r);
    return o;
  }

  void run_event(const ScoreCtx& c) {
    const Workload& w = c.w;
    const int N = w.n_nodes;
    if (N > 64) throw std::runtime_error("emulated replays need <= 64 nodes");
    gcn::Emu& E = *emu;
    // registers the caller does not pass hold garbage (the first 120 VGPRs:
    // everything the generator may allocate)
    // (FKS_EMU_POISON=1: a different value per register, lane and call -- a
    // read of a register the caller did not pass then shows as a result that
    // changes with the seed)
    static const bool vary = std::getenv("FKS_EMU_POISON") != nullptr;
    uint64_t z = vary ? 0x9E3779B97F4A7C15ull * (uint64_t)(++poison_seq) : 0;
    auto next = [&](uint32_t dflt) {
      if (!vary) return dflt;
      z += 0x9E3779B97F4A7C15ull;
      uint64_t x = z;
      x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
      x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
      return (uint32_t)(x ^ (x >> 31));
    };
    for (int g = 0; g < 256; ++g)
      for (int l = 0; l < 64; ++l) E.vg[g][l] = (g < 120 && l < N) || vary ? next(0xBADC0DE5u) : E.vg[g][l];
    for (auto& x : E.sg) x = next(0x5CA1AB1Eu);
    for (int l = 0; l < N; ++l) {
      const int g0 = w.gpu_start[(size_t)l], ng = w.gpu_start[(size_t)l + 1] - g0;
      E.vg[0][l] = (uint32_t)(int32_t)c.s.cpu_left[(size_t)l];
      E.vg[1][l] = (uint32_t)(int32_t)w.cpu_total[(size_t)l];
      E.vg[2][l] = (uint32_t)(int32_t)c.s.mem_left[(size_t)l];
      E.vg[3][l] = (uint32_t)(int32_t)w.mem_total[(size_t)l];
      E.vg[4][l] = ((uint32_t)c.s.gpu_left[(size_t)l] & 0xFFFFu) | ((uint32_t)w.ngpus[(size_t)l] << 16);
      for (int j = 0; j < 8; ++j) {
        E.vg[5 + j][l] = j < ng ? (uint32_t)c.s.gmilli_left[(size_t)(g0 + j)] : 0u;
        E.vg[13 + j][l] = j < ng ? (uint32_t)w.gmilli_total[(size_t)(g0 + j)] : 0u;
      }
      const uint64_t gp = (uint64_t)(uintptr_t)(gmem8->data() + (size_t)l * 8);
      E.vg[21][l] = (uint32_t)gp;
      E.vg[22][l] = (uint32_t)(gp >> 32);
      E.vg[23][l] = (uint32_t)(int32_t)w.pcpu[(size_t)c.pod];
      E.vg[24][l] = (uint32_t)(int32_t)w.pmem[(size_t)c.pod];
      E.vg[25][l] = (uint32_t)(w.pgmilli[(size_t)c.pod] | (w.pngpu[(size_t)c.pod] << 16));
      E.vg[26][l] = (uint32_t)(uint64_t)c.pod_ctime;
      E.vg[27][l] = (uint32_t)((uint64_t)c.pod_ctime >> 32);
      E.vg[28][l] = (uint32_t)(int32_t)w.pdur[(size_t)c.pod];
      E.vg[29][l] = 0;   // kc at LDS offset 0
    }
    E.sg[32] = 0;
    E.wr64s(30, kRetMagic);
    uint64_t lanes = N == 64 ? ~0ull : ((1ull << N) - 1);
    if (feas_only) {   // as the kernels' feasible() (scorers.hip.h)
      const int32_t pc = w.pcpu[(size_t)c.pod], pm = w.pmem[(size_t)c.pod];
      const int32_t pg = w.pngpu[(size_t)c.pod], gm = w.pgmilli[(size_t)c.pod];
      for (int l = 0; l < N; ++l) {
        bool ok = pc <= c.s.cpu_left[(size_t)l] && pm <= c.s.mem_left[(size_t)l] && pg <= c.s.gpu_left[(size_t)l];
        if (ok && pg > 0) {
          const int g0 = w.gpu_start[(size_t)l], ng = std::min(8, w.gpu_start[(size_t)l + 1] - g0);
          int avail = 0;
          for (int j = 0; j < ng; ++j) avail += c.s.gmilli_left[(size_t)(g0 + j)] >= gm;
          ok = avail >= pg;
        }
        if (!ok) lanes &= ~(1ull << l);
      }
    }
    res.assign((size_t)N, 0);
    if (lanes == 0) return;
    E.set_exec(lanes);
    E.scc = false;
    E.run(*f, kRetMagic);
    for (int l = 0; l < N; ++l)
      if (lanes >> l & 1) res[(size_t)l] = (int64_t)((uint64_t)E.vg[0][l] | (uint64_t)E.vg[1][l] << 32);
    if (std::getenv("FKS_EMU_TRACE_EXC") && !traced)
      for (int l = 0; l < N; ++l)
        if ((lanes >> l & 1) && res[(size_t)l] < 0) {
          traced = true;
          std::fprintf(stderr, "exc %lld lane %d pod %d ctime %lld: node cpu %d/%d mem %d/%d gpu_left %d ngpu %d gl", (long long)-res[(size_t)l], l, c.pod,
                       (long long)c.pod_ctime, (int)c.s.cpu_left[(size_t)l], (int)w.cpu_total[(size_t)l],
                       (int)c.s.mem_left[(size_t)l], (int)w.mem_total[(size_t)l], (int)c.s.gpu_left[(size_t)l],
                       (int)w.ngpus[(size_t)l]);
          for (int j = 0; j < 8; ++j) std::fprintf(stderr, " %u/%u", E.vg[5 + j][l], E.vg[13 + j][l]);
          std::fprintf(stderr, " pod cpu %d mem %d gm %d ng %d dur %d\n", (int)w.pcpu[(size_t)c.pod], (int)w.pmem[(size_t)c.pod],
                       (int)w.pgmilli[(size_t)c.pod], (int)w.pngpu[(size_t)c.pod], (int)w.pdur[(size_t)c.pod]);
          std::fprintf(stderr, "LANES %llx", (unsigned long long)lanes);
          for (int q = 0; q < N; ++q) {
            std::fprintf(stderr, " |%d,%d,%d,%d,%d,%d", (int)c.s.cpu_left[(size_t)q], (int)w.cpu_total[(size_t)q],
                         (int)c.s.mem_left[(size_t)q], (int)w.mem_total[(size_t)q], (int)c.s.gpu_left[(size_t)q],
                         (int)w.ngpus[(size_t)q]);
            const int g0 = w.gpu_start[(size_t)q], ng = w.gpu_start[(size_t)q + 1] - g0;
            for (int j = 0; j < 8; ++j) std::fprintf(stderr, ",%d", j < ng ? (int)c.s.gmilli_left[(size_t)(g0 + j)] : 0);
            for (int j = 0; j < 8; ++j) std::fprintf(stderr, ",%d", j < ng ? (int)w.gmilli_total[(size_t)(g0 + j)] : 0);
          }
          std::fprintf(stderr, "\n");
          break;
        }
  }
};

}  // namespace

namespace {
std::mutex g_prof_mu;
std::vector<int64_t> g_prof, g_prof_bc;
bool g_prof_on = false;
}  // namespace

void emu_profile(bool on) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  g_prof.assign((size_t)gcn::NUM_OPC, 0);
  g_prof_bc.assign(256, 0);
  g_prof_on = on;
}

std::vector<std::pair<std::string, int64_t>> emu_profile_counts() {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  std::vector<std::pair<std::string, int64_t>> out;
  for (size_t i = 0; i < g_prof.size(); ++i)
    if (g_prof[i]) out.emplace_back(gcn::info((gcn::Opc)i).name, g_prof[i]);
  for (size_t i = 0; i < g_prof_bc.size(); ++i)
    if (g_prof_bc[i]) out.emplace_back("bc:" + std::to_string(i), g_prof_bc[i]);
  return out;
}

std::vector<SimResult> emu_simulate_batch(const Workload& w, const std::vector<ProgramDesc>& progs,
                                          const std::vector<std::vector<int64_t>>& kc, const SimOptions& o,
                                          int threads) {
  const int64_t P = (int64_t)progs.size();
  std::vector<gcn::Func> funcs((size_t)P);
  std::vector<char> elided((size_t)P, 0);
  for (int64_t i = 0; i < P; ++i) {
    bool el = false;
    funcs[(size_t)i] = generate(make_in(progs[(size_t)i]), nullptr, &el);   // as compile()
    elided[(size_t)i] = el;
  }
  std::vector<int64_t> gmem8((size_t)w.n_nodes * 8, 0);
  for (int n = 0; n < w.n_nodes; ++n)
    for (int j = 0; j < std::min(8, w.gpu_start[(size_t)n + 1] - w.gpu_start[(size_t)n]); ++j)
      gmem8[(size_t)n * 8 + (size_t)j] = w.gmem_total[(size_t)(w.gpu_start[(size_t)n] + j)];
  std::vector<SimResult> out((size_t)P);
  std::vector<std::string> errs((size_t)P);
  parallel_for(P, threads, [&](int64_t i) {
    try {
      auto emu = std::make_unique<gcn::Emu>();
      std::vector<int64_t> hist, hist_bc;
      if (g_prof_on) {
        hist.assign((size_t)gcn::NUM_OPC, 0);
        hist_bc.assign(256, 0);
        emu->hist = hist.data();
        emu->hist_bc = hist_bc.data();
      }
      const std::vector<int64_t>& k = kc[(size_t)i];
      emu->lds.resize(k.size() * 8 + 64, 0);
      std::memcpy(emu->lds.data(), k.data(), k.size() * 8);
      EmuScorer sc{&funcs[(size_t)i], &k, &gmem8, emu.get(), {}, EXC_NONE, elided[(size_t)i] != 0};
      SimResult r = simulate(w, sc, o);
      if (r.exc == EXC_NONE && sc.exc) r.exc = sc.exc;
      out[(size_t)i] = std::move(r);
      if (!hist.empty()) {
        std::lock_guard<std::mutex> lk(g_prof_mu);
        for (size_t j = 0; j < hist.size() && j < g_prof.size(); ++j) g_prof[j] += hist[j];
        for (size_t j = 0; j < hist_bc.size() && j < g_prof_bc.size(); ++j) g_prof_bc[j] += hist_bc[j];
      }
    } catch (const std::exception& e) {
      errs[(size_t)i] = e.what();
    }
  });
  for (int64_t i = 0; i < P; ++i)
    if (!errs[(size_t)i].empty())
      throw std::runtime_error("emulated replay of program " + std::to_string(i) + ": " + errs[(size_t)i]);
  return out;
}

std::vector<int64_t> emu_event(const ProgramDesc& p, const std::vector<int64_t>& kc,
                               const std::vector<int64_t>& node, const std::vector<int32_t>& gl,
                               const std::vector<int32_t>& gt, const std::vector<int64_t>& gmem,
                               const std::vector<int64_t>& pod) {
  const int N = (int)(node.size() / 6);
  if (N < 1 || N > 64 || gl.size() != (size_t)N * 8 || gt.size() != (size_t)N * 8 || gmem.size() != (size_t)N * 8 ||
      (pod.size() != 6 && pod.size() != (size_t)N * 6))
    throw std::invalid_argument("emu_event: bad shapes");
  const bool per_lane_pod = pod.size() != 6;   // one pod per lane: several programs' rows in one call
  gcn::Func f = generate(make_in(p), nullptr, nullptr);
  auto E = std::make_unique<gcn::Emu>();
  E->lds.resize(kc.size() * 8 + 64, 0);
  std::memcpy(E->lds.data(), kc.data(), kc.size() * 8);
  for (auto& row : E->vg)
    for (auto& x : row) x = 0xBADC0DE5u;
  for (auto& x : E->sg) x = 0x5CA1AB1Eu;
  for (int l = 0; l < N; ++l) {
    const int64_t* nd = node.data() + (size_t)l * 6;
    E->vg[0][l] = (uint32_t)nd[0]; E->vg[1][l] = (uint32_t)nd[1];
    E->vg[2][l] = (uint32_t)nd[2]; E->vg[3][l] = (uint32_t)nd[3];
    E->vg[4][l] = ((uint32_t)nd[4] & 0xFFFFu) | ((uint32_t)nd[5] << 16);
    for (int j = 0; j < 8; ++j) {
      E->vg[5 + j][l] = (uint32_t)gl[(size_t)l * 8 + (size_t)j];
      E->vg[13 + j][l] = (uint32_t)gt[(size_t)l * 8 + (size_t)j];
    }
    const uint64_t gp = (uint64_t)(uintptr_t)(gmem.data() + (size_t)l * 8);
    E->vg[21][l] = (uint32_t)gp; E->vg[22][l] = (uint32_t)(gp >> 32);
    const int64_t* pd = pod.data() + (per_lane_pod ? (size_t)l * 6 : 0);
    E->vg[23][l] = (uint32_t)pd[0]; E->vg[24][l] = (uint32_t)pd[1];
    E->vg[25][l] = (uint32_t)(pd[3] | (pd[2] << 16));
    E->vg[26][l] = (uint32_t)(uint64_t)pd[4]; E->vg[27][l] = (uint32_t)((uint64_t)pd[4] >> 32);
    E->vg[28][l] = (uint32_t)pd[5];
    E->vg[29][l] = 0;
  }
  E->sg[32] = 0;
  E->wr64s(30, kRetMagic);
  E->set_exec(N == 64 ? ~0ull : ((1ull << N) - 1));
  E->run(f, kRetMagic);
  std::vector<int64_t> out((size_t)N);
  for (int l = 0; l < N; ++l) out[(size_t)l] = (int64_t)((uint64_t)E->vg[0][l] | (uint64_t)E->vg[1][l] << 32);
  return out;
}

}  // namespace gcnapi
}  // namespace fks
