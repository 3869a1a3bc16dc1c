// k_screen_linear: MFMA surrogate screening of linear policy candidates.
//
// The exact replay is block-diagonal (every candidate walks its own cluster
// state), so matrix cores only pay where states are SHARED: score P weight
// vectors on S recorded (pod, cluster-state) pairs from a reference replay,
//     Y[s*Np + n, p] = sum_k X[s*Np + n, k] * W[k, p]        (MFMA, fp32)
// then, per (state, candidate), take the argmax node (first node wins ties,
// the reference's strict `>` scan; a best value <= 0 means "no placement")
// and accumulate the reward of that decision, R[s*Np + n] (or Rfail[s]).
// fit[p] = sum_s reward is a cheap fitness surrogate that pre-filters
// candidates before exact replay (ops/screening.py).
//
// Layout: one wave = 32 candidates x one state at a time; the B operand
// (32 candidates' weights, K/2 k-steps) stays in VGPRs for the whole launch.
// v_mfma_f32_32x32x2_f32: A[i][k] from lane i + 32k, B[k][j] from lane j + 32k,
// D[i][j] in lane j + 32*((i/4)%2), register 4*(i/8) + i%4.  Np is a multiple
// of 32 (padding rows carry the infeasible bias); K = KP <= 18, even.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kMaxKSteps = 9;    // KP <= 18 (ops/screening.py: 16 features + bias + pad)

// kTiles candidate tiles (32 candidates each) per wave: every X fragment a
// wave loads feeds kTiles MFMA chains, so the X stream from L2 / MALL is read
// Ppad / (32 kTiles) times instead of Ppad / 32 times.
constexpr int kTiles = 4;

__global__ __launch_bounds__(256) void k_screen_linear(const float* __restrict__ X, const float* __restrict__ Wt,
                                                       const float* __restrict__ R, const float* __restrict__ Rfail,
                                                       int S, int Np, int KP, int Ppad, int states_per_wave,
                                                       float* __restrict__ fit) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int p0 = blockIdx.y * 32 * kTiles;
  const int col = lane & 31, half = lane >> 5;
  const int ksteps = KP >> 1;
  // B fragments: lane holds W[2t + half][p0 + 32 b + col] (zero columns past Ppad)
  float b[kTiles][kMaxKSteps];
#pragma unroll
  for (int tb = 0; tb < kTiles; ++tb) {
    const int pc = p0 + 32 * tb + col;
#pragma unroll
    for (int t = 0; t < kMaxKSteps; ++t)
      b[tb][t] = (t < ksteps && pc < Ppad) ? Wt[(size_t)(2 * t + half) * Ppad + pc] : 0.0f;
  }

  float acc_fit[kTiles];
#pragma unroll
  for (int tb = 0; tb < kTiles; ++tb) acc_fit[tb] = 0.0f;
  const int s_begin = (blockIdx.x * (blockDim.x >> 6) + wave) * states_per_wave;
  const int s_end = min(S, s_begin + states_per_wave);
  for (int s = s_begin; s < s_end; ++s) {
    float best_v[kTiles];
    int best_row[kTiles];
#pragma unroll
    for (int tb = 0; tb < kTiles; ++tb) { best_v[tb] = -INFINITY; best_row[tb] = 0x7fffffff; }
    for (int rt = 0; rt < Np; rt += 32) {
      const float* xt = X + ((size_t)s * Np + rt + col) * KP + half;
      float a[kMaxKSteps];
#pragma unroll
      for (int t = 0; t < kMaxKSteps; ++t) a[t] = t < ksteps ? xt[2 * t] : 0.0f;
#pragma unroll
      for (int tb = 0; tb < kTiles; ++tb) {
        floatx16 d = {0};
#pragma unroll
        for (int t = 0; t < kMaxKSteps; ++t)
          if (t < ksteps) d = __builtin_amdgcn_mfma_f32_32x32x2f32(a[t], b[tb][t], d, 0, 0, 0);
        // this lane's 16 rows of the tile, ascending: 8*(r/4) + 4*half + r%4
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = rt + 8 * (r >> 2) + 4 * half + (r & 3);
          const float v = d[r];
          if (v > best_v[tb]) { best_v[tb] = v; best_row[tb] = row; }   // ascending rows: first max kept
        }
      }
    }
#pragma unroll
    for (int tb = 0; tb < kTiles; ++tb) {
      // combine with the other half-wave (same candidate column)
      float bv = best_v[tb];
      int br = best_row[tb];
      const float ov = __shfl_xor(bv, 32, 64);
      const int orow = __shfl_xor(br, 32, 64);
      if (ov > bv || (ov == bv && orow < br)) { bv = ov; br = orow; }
      acc_fit[tb] += bv > 0.0f ? R[(size_t)s * Np + br] : Rfail[s];
    }
  }
  if (half == 0 && s_begin < S) {
#pragma unroll
    for (int tb = 0; tb < kTiles; ++tb)
      if (p0 + 32 * tb + col < Ppad) atomicAdd(&fit[p0 + 32 * tb + col], acc_fit[tb]);
  }
}

// Probe of the MFMA output layout (tests): D = A * B for A[i][k] = i + 100k, B[k][j] = j + 1000k.
__global__ __launch_bounds__(64) void k_mfma_probe(float* out) {
  const int lane = threadIdx.x;
  const int col = lane & 31, half = lane >> 5;
  floatx16 d = {0};
  const float a = (float)(col + 100 * half), b = (float)(col + 1000 * half);
  d = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, d, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 16; ++r) out[lane * 16 + r] = d[r];
}

}  // namespace

namespace fksk {

hipError_t launch_screen_linear(const float* X, const float* Wt, const float* R, const float* Rfail, int S, int Np,
                                int KP, int Ppad, float* fit, hipStream_t stream) {
  if (Np % 32 != 0 || KP % 2 != 0 || KP > 2 * kMaxKSteps || Ppad % 32 != 0) return hipErrorInvalidValue;
  const int waves = 4, spw = 8;
  const int gx = (S + waves * spw - 1) / (waves * spw);
  hipLaunchKernelGGL(k_screen_linear, dim3(gx, (Ppad + 32 * kTiles - 1) / (32 * kTiles)), dim3(64 * waves), 0, stream,
                     X, Wt, R, Rfail, S, Np, KP, Ppad, spw, fit);
  return hipGetLastError();
}

hipError_t launch_mfma_probe(float* out, hipStream_t stream) {
  hipLaunchKernelGGL(k_mfma_probe, dim3(1), dim3(64), 0, stream, out);
  return hipGetLastError();
}

}  // namespace fksk
