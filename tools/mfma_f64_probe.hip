// FP64 matrix cores vs FP64 vector FMA on gfx950 -- the measurement behind the
// "exact FP64-MFMA scorer" decision (docs/ARCHITECTURE.md, Considered and not built).
//
//   k_mfma:  every wave issues ITER x 4 independent v_mfma_f64_16x16x4_f64
//            (16*16*4 = 1,024 FMA each, accumulators in registers)
//   k_valu:  every wave issues ITER x 8 independent v_fma_f64 chains (64 FMA
//            per instruction)
// Both launched to fill the chip (and at one wave per SIMD); TFLOP/s from hip
// events.  Then the numerics question an exact scorer faces: a 16-term
// feature x weight sum computed by four chained MFMAs (K = 4 each) against the
// scorers' left-to-right `s = s + w * f` (every product and every sum rounded,
// scorers.hip.h composite_row): how many of the results differ in the last bits.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/mfma_f64_probe.hip -o tools/scratch/mfma_f64_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

typedef double v4d __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(64) void k_mfma(const double* in, double* out, int iter) {
  const int lane = threadIdx.x;
  double a = in[lane], b = in[64 + lane];
  v4d c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  for (int i = 0; i < iter; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
  }
  const v4d s = c0 + c1 + c2 + c3;
  out[(size_t)blockIdx.x * 64 + lane] = s.x + s.y + s.z + s.w;
}

__global__ __launch_bounds__(64) void k_valu(const double* in, double* out, int iter) {
  const int lane = threadIdx.x;
  const double a = in[lane], b = in[64 + lane];
  double c[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) c[k] = in[k];
  for (int i = 0; i < iter; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = __builtin_fma(a, b, c[k]);
  }
  double s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += c[k];
  out[(size_t)blockIdx.x * 64 + lane] = s;
}

// 16 nodes x 16 features (f) times one weight vector (w), per wave (one wave
// per 4 independent problems would be the row kernel's shape; one problem per
// wave is enough for the numerics).  MFMA 16x16x4 f64 operands: A (16x4) lane l
// holds A[l % 16][l / 16]; B (4x16) lane l holds B[l / 16][l % 16].  B = the
// weight column replicated over the 16 output columns, so every output element
// is some node's sum; the host identifies the row each (lane, element) holds
// (measured: element i of lane l is row 4 * i + l / 16,
// profiles/r5_mfma_f64_probe.txt).
__global__ __launch_bounds__(64) void k_dot(const double* f, const double* w, double* mf, double* seq, int nprob) {
  const int lane = threadIdx.x;
  const int p = blockIdx.x;
  if (p >= nprob) return;
  const double* F = f + (size_t)p * 256;   // [node][feature]
  const double* W = w + (size_t)p * 16;
  v4d c = {0, 0, 0, 0};
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
    const double a = F[(lane % 16) * 16 + kb * 4 + lane / 16];
    const double b = W[kb * 4 + lane / 16];
    c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  // every output element: B's columns are all the weight vector, so each holds
  // one node's sum; the host identifies which (the f64 output layout)
  for (int i = 0; i < 4; ++i) mf[(size_t)p * 256 + lane * 4 + i] = c[i];
  if (lane < 16) {
    double s = 0.0;
    for (int k = 0; k < 16; ++k) {
      const double prod = W[k] * F[lane * 16 + k];   // -ffp-contract=off: rounded product, rounded sum
      s = s + prod;
    }
    seq[(size_t)p * 16 + lane] = s;
  }
}

int main(int argc, char** argv) {
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int iter = argc > 1 ? std::atoi(argv[1]) : 20000;
  std::vector<double> hin(128);
  for (int i = 0; i < 128; ++i) hin[i] = 1.0 + 1e-9 * i;
  double *din, *dout;
  CHECK(hipMalloc(&din, 128 * sizeof(double)));
  CHECK(hipMalloc(&dout, (size_t)cus * 16 * 64 * sizeof(double)));
  CHECK(hipMemcpy(din, hin.data(), 128 * sizeof(double), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::printf("{\"cus\": %d, \"iter\": %d}\n", cus, iter);
  for (int wps : {1, 2, 4}) {   // waves per SIMD
    const int blocks = cus * 4 * wps;
    for (int kind = 0; kind < 2; ++kind) {
      for (int rep = 0; rep < 2; ++rep) {   // first launch warms up
        CHECK(hipEventRecord(e0));
        if (kind == 0) hipLaunchKernelGGL(k_mfma, dim3(blocks), dim3(64), 0, 0, din, dout, iter);
        else hipLaunchKernelGGL(k_valu, dim3(blocks), dim3(64), 0, 0, din, dout, iter);
        CHECK(hipGetLastError());
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (rep == 0) continue;
        const double fma = kind == 0 ? (double)blocks * iter * 4 * 1024 : (double)blocks * iter * 8 * 64;
        std::printf("{\"kernel\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"tflops\": %.2f}\n",
                    kind == 0 ? "v_mfma_f64_16x16x4_f64" : "v_fma_f64", wps, ms, 2.0 * fma / (ms * 1e-3) / 1e12);
      }
    }
  }
  // numerics: MFMA sums vs the scorers' rounded left-to-right order
  const int nprob = 4096;
  std::mt19937_64 rng(7);
  std::uniform_real_distribution<double> uf(0.0, 1.0), uw(-1000.0, 1000.0);
  std::vector<double> hf((size_t)nprob * 256), hw((size_t)nprob * 16);
  for (auto& x : hf) x = uf(rng);
  for (auto& x : hw) x = uw(rng);
  double *df, *dw, *dmf, *dseq;
  CHECK(hipMalloc(&df, hf.size() * 8));
  CHECK(hipMalloc(&dw, hw.size() * 8));
  CHECK(hipMalloc(&dmf, (size_t)nprob * 256 * 8));
  CHECK(hipMalloc(&dseq, (size_t)nprob * 16 * 8));
  CHECK(hipMemcpy(df, hf.data(), hf.size() * 8, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dw, hw.data(), hw.size() * 8, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_dot, dim3(nprob), dim3(64), 0, 0, df, dw, dmf, dseq, nprob);
  CHECK(hipGetLastError());
  std::vector<double> mf((size_t)nprob * 256), sq((size_t)nprob * 16);
  CHECK(hipMemcpy(mf.data(), dmf, mf.size() * 8, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(sq.data(), dseq, sq.size() * 8, hipMemcpyDeviceToHost));
  // output layout: the node (row) each (lane, element) holds, from problem 0
  // (nearest sequential sum); then every node's MFMA sum read through it
  int node_of[256];
  for (int e = 0; e < 256; ++e) {
    int best = 0;
    for (int r = 1; r < 16; ++r)
      if (std::fabs(mf[e] - sq[r]) < std::fabs(mf[e] - sq[best])) best = r;
    node_of[e] = best;
  }
  int first_e[16];
  for (int r = 0; r < 16; ++r) first_e[r] = -1;
  for (int e = 0; e < 256; ++e)
    if (first_e[node_of[e]] < 0) first_e[node_of[e]] = e;
  std::printf("{\"layout\": \"lane 0..3 elements -> rows %d %d %d %d, lane 16 -> %d, lane 1 -> %d\"}\n", node_of[0], node_of[1],
              node_of[2], node_of[3], node_of[64], node_of[4]);
  std::vector<double> mfn((size_t)nprob * 16);
  for (int p = 0; p < nprob; ++p)
    for (int r = 0; r < 16; ++r) mfn[(size_t)p * 16 + r] = first_e[r] >= 0 ? mf[(size_t)p * 256 + first_e[r]] : NAN;
  size_t differ = 0, trunc_differ = 0, argmax_differ = 0;
  double max_rel = 0.0;
  for (size_t i = 0; i < mfn.size(); ++i) {
    if (mfn[i] != sq[i]) ++differ;
    if (std::trunc(mfn[i]) != std::trunc(sq[i])) ++trunc_differ;
    if (sq[i] != 0.0) max_rel = std::fmax(max_rel, std::fabs(mfn[i] - sq[i]) / std::fabs(sq[i]));
  }
  for (int p = 0; p < nprob; ++p) {
    int am = 0, as = 0;
    for (int j = 1; j < 16; ++j) {
      if (mfn[(size_t)p * 16 + j] > mfn[(size_t)p * 16 + am]) am = j;
      if (sq[(size_t)p * 16 + j] > sq[(size_t)p * 16 + as]) as = j;
    }
    argmax_differ += am != as;
  }
  std::printf("{\"numerics\": \"16-term feature x weight sums, MFMA (4 x K=4) vs rounded left-to-right\", \"sums\": %zu, "
              "\"bitwise_differ\": %zu, \"trunc_differ\": %zu, \"argmax_differ\": %zu, \"max_rel_err\": %.3e}\n",
              mfn.size(), differ, trunc_differ, argmax_differ, max_rel);
  return 0;
}
