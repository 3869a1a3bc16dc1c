// Interface of the baseline program JIT (gcn_jit.cpp) for the _fks_cpu
// extension: a plain C++ API, so module.cpp never sees the device-math
// headers' host macros.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "fks/types.hpp"

namespace fks {
namespace gcnapi {

struct ProgramDesc {
  const uint8_t* code = nullptr;    // bytecode (8-byte instructions)
  size_t code_bytes = 0;
  const uint8_t* ctag = nullptr;    // per constant: 0 int, 1 float
  const uint8_t* is_lit = nullptr;  // per constant: read from the kc block at run time
  const int64_t* iconst = nullptr;
  const double* fconst = nullptr;
  size_t n_const = 0;
  int elide_lo = 0, elide_hi = 0;   // bytecode range of a kernel-checked feasibility prologue (0, 0: none)
};

struct Result {
  bool ok = false;
  std::string reason;
  std::vector<uint32_t> words;      // machine code (position independent except relocs)
  std::vector<uint32_t> relocs;     // triples: lo literal word, hi literal word, byte offset of the PC
  int n_insns = 0, vgprs = 0, sgprs = 0, calls = 0, vregs = 0, tagged = 0, mir = 0, spills = 0, unrolled = 0;
  bool elided = false;              // compiled without the prologue (ProgramDesc elide range)
};

// bytecode -> gfx950 machine code (never throws: failures come back as !ok + reason)
Result compile(const ProgramDesc& p);

// Test hook: cap the VGPR pairs for virtual registers (0: none) -> forces spills.
void set_pair_cap(int pairs);
int set_unroll_cap(int cap);

// Human-readable listing of the generated machine-instruction stream (debugging).
std::string listing(const ProgramDesc& p);

// Full replays with each program's generated code run on the wave64 emulator
// as the scorer (CPU validation of the generator); kc[i] is program i's
// constant block [budget, constants...].
// Dynamic instruction counts of emulated replays (emu_simulate_batch) per
// opcode name, collected while enabled (enabling resets them).
void emu_profile(bool on);
std::vector<std::pair<std::string, int64_t>> emu_profile_counts();

std::vector<SimResult> emu_simulate_batch(const Workload& w, const std::vector<ProgramDesc>& progs,
                                          const std::vector<std::vector<int64_t>>& kc, const SimOptions& o,
                                          int threads);

// One emulated call: lanes = nodes (N <= 64).  node: per lane [cpu_left,
// cpu_total, mem_left, mem_total, gpu_left, ngpus]; gl / gt / gmem: [N][8];
// pod: [cpu, mem, ngpu, gmilli, ctime, dur].  Returns per lane the program's
// int(max(0, score)) or -exception code.
std::vector<int64_t> emu_event(const ProgramDesc& p, const std::vector<int64_t>& kc,
                               const std::vector<int64_t>& node, const std::vector<int32_t>& gl,
                               const std::vector<int32_t>& gt, const std::vector<int64_t>& gmem,
                               const std::vector<int64_t>& pod);

}  // namespace gcnapi
}  // namespace fks
