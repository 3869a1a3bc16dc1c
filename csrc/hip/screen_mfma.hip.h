// k_score_linear_mfma: behavioural screening of linear-family candidates on
// recorded cluster states, on the matrix cores (the
// shared-operand case: every candidate is scored on the SAME recorded states,
// so the per-state node-feature block is a real GEMM operand).
//
//   scores[s] = X[s] (16 nodes x 20 feature slots) . W^T (20 x P candidates)
//
// One v_mfma_f32_16x16x4_f32 tile is one state's 16 nodes x 16 candidates;
// K = 20 feature slots = five k-steps.  Each wave owns 16 candidates: their weight
// fragments (the B operand, one f32 per lane per k-step) stay in registers for
// the whole launch while the wave streams every recorded state's A fragments
// (1.25 KB per state, coalesced: the host lays X out as [state][k-step][lane]).
// Per state the wave turns the tile into each candidate's decision: the
// family's own rule in f32 -- score max(1, trunc(v)) for feasible nodes, first
// maximum wins, 255 when no node is feasible (slot 19 carries 0 for a
// feasible node and -1e30 otherwise, with weight 1) -- and folds it into a
// 64-bit FNV-1a signature per candidate.  Candidates with equal signatures
// place every recorded pod alike: the search replays one of them exactly.
//
// This is a screen, not a score: f32 products can differ from the replay's f64
// arithmetic at near-ties, and the exact replay stays the only fitness.
//
// Fragment maps (gfx950, f32 16x16x4): A lane l = A[row l&15][k l>>4],
// B lane l = B[k l>>4][col l&15], D reg i of lane l = D[row 4(l>>4)+i][col l&15].
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fks_screen {

constexpr int kScreenSteps = 5;       // k-steps of 4: K = 20 slots (<= 19 family features + the feasibility bias)
constexpr int kScreenNodes = 16;      // M: nodes per state (clusters of <= 16 nodes)
constexpr int kScreenCands = 16;      // N: candidates per wave tile
constexpr int kScreenWaves = 4;       // waves per workgroup

typedef float f32x4 __attribute__((ext_vector_type(4)));

// X: [S][5][64] (k-step t, lane l: X[s][node l&15][feature 4t + (l>>4)])
// W: [tiles][5][64] (k-step t, lane l: W[16 tile + (l&15)][feature 4t + (l>>4)])
// dec: [P][S] uint8 node index or 255 (none feasible), may be null;
// sig: [P][C] the signature of each chunk of `spc` states (blockIdx.y = chunk):
// a launch of few candidate tiles splits the states over more waves, so the
// SIMDs hold enough waves to cover the MFMA chain's latency (the host folds
// the chunk signatures in order)
__global__ __launch_bounds__(64 * kScreenWaves) void k_score_linear_mfma(const float* __restrict__ X,
                                                                      const float* __restrict__ W, int S, int tiles,
                                                                      uint8_t* __restrict__ dec,
                                                                      uint64_t* __restrict__ sig, int P, int spc) {
  const int lane = threadIdx.x & 63;
  const int tile = blockIdx.x * kScreenWaves + (threadIdx.x >> 6);
  const int C = gridDim.y, chunk = blockIdx.y;
  const int s0 = chunk * spc, s1 = min(S, s0 + spc);
  if (tile >= tiles) return;   // whole waves only: no MFMA runs with a partial wave
  const float* wt = W + (size_t)tile * kScreenSteps * 64;
  float b[kScreenSteps];
#pragma unroll
  for (int t = 0; t < kScreenSteps; ++t) b[t] = wt[64 * t + lane];
  const int col = lane & 15;
  const int rbase = (lane >> 4) * 4;
  const int cand = tile * kScreenCands + col;
  uint64_t h = 0xcbf29ce484222325ull;
  for (int s = s0; s < s1; ++s) {
    const float* xs = X + (size_t)s * kScreenSteps * 64;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < kScreenSteps; ++t) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xs[64 * t + lane], b[t], acc, 0, 0, 0);
    // this lane's four nodes (rows rbase..rbase+3) for candidate `col`
    float best = -1.f;   // below every feasible score (>= 1)
    int brow = 255;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float v = acc[i];
      const float sc = v < -1e29f ? -2.f : fmaxf(1.f, truncf(v));   // the family's max(1, int(score))
      if (sc > best) { best = sc; brow = rbase + i; }                 // strict: the first maximum
    }
    // the other three row groups of the same column: lanes l ^ 16, l ^ 32
#pragma unroll
    for (int m = 16; m <= 32; m <<= 1) {
      const float ob = __shfl_xor(best, m, 64);
      const int orow = __shfl_xor(brow, m, 64);
      if (ob > best || (ob == best && orow < brow)) { best = ob; brow = orow; }
    }
    const uint32_t d = best >= 1.f ? (uint32_t)brow : 255u;
    if (dec != nullptr && lane < 16 && cand < P) dec[(size_t)cand * S + s] = (uint8_t)d;
    h = (h ^ (uint64_t)(d + 1)) * 0x100000001b3ull;
  }
  if (lane < 16 && cand < P) sig[(size_t)cand * C + chunk] = h;
}

}  // namespace fks_screen
