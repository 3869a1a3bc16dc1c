// Built-in policy families on the device (twins of csrc/cpu/builtin_scorers.hpp,
// op-for-op, so the replays are bit-identical; compiled with
// -ffp-contract=off: Python never fuses a multiply into an add).
#pragma once

#include "replay.hip.h"

namespace fksd {

enum BuiltinFamily : int32_t {
  FAM_FIRST_FIT = 0, FAM_BEST_FIT = 1, FAM_RANDOM_LINEAR = 2, FAM_FEATURE_LINEAR = 3, FAM_COMPOSITE_LINEAR = 4
};
constexpr int kFeatureCount = 12;
constexpr int kCompositeCount = 16;
constexpr int kWeights = 16;

// int(max(0, s)) of a float score produced by `max(1, int(score))`-style code
__device__ __forceinline__ int64_t trunc_score(double s, int& exc) {
  if (isnan(s)) { exc = EXC_VALUE; return 0; }
  if (isinf(s)) { exc = EXC_OVERFLOW; return 0; }
  if (fabs(s) >= 9.2233720368547758e18) { exc = EXC_UNSUPPORTED; return 0; }
  const int64_t v = (int64_t)s;
  return v > 1 ? v : 1;
}

// trunc_score as a double: |s| < 2^63, so trunc(s) is exactly the int64 the
// integer path produces and doubles order like those integers (row kernel:
// no f64 -> i64 conversion, 64-bit max as v_max_f64)
__device__ __forceinline__ double trunc_score_f(double s, int& exc) {
  if (!(fabs(s) < 9.2233720368547758e18)) {   // NaN, infinity or beyond int64: one compare on the common path
    exc = isnan(s) ? EXC_VALUE : isinf(s) ? EXC_OVERFLOW : EXC_UNSUPPORTED;
    return 0.0;
  }
  const double v = trunc(s);
  return v > 1.0 ? v : 1.0;
}

template <int NPASS, bool GP>
__device__ __forceinline__ bool feasible(int ps, const NodeRegs<NPASS, GP>& nr, const PodView& pod) {
  if (pod.cpu > nr.cpu_left[ps] || pod.mem > nr.mem_left[ps] || pod.ngpu > nr.gpu_left[ps]) return false;
  if (pod.ngpu > 0) {
    int avail = 0;
#pragma unroll
    for (int j = 0; j < kGmax; ++j) avail += (j < nr.ngp(ps) && nr.g(ps, j) >= pod.gmilli);
    if (avail < pod.ngpu) return false;
  }
  return true;
}

// Number of weights a family reads (the rest are never loaded).
__host__ __device__ constexpr int family_weights(int fam) {
  return fam == FAM_RANDOM_LINEAR ? 4 : fam == FAM_FEATURE_LINEAR ? kFeatureCount
       : fam == FAM_COMPOSITE_LINEAR ? kCompositeCount : fam < 0 ? kWeights : 0;
}

// FAM >= 0: the family is a compile-time constant (one kernel instance per
// family, so a launch only carries the registers of its own scorer);
// FAM = -1: mixed-family batches dispatch on the per-policy id.
template <int FAM = -1>
struct BuiltinScorerDev {
  int32_t family;
  const double* wp;   // this policy's kWeights weights (device copy, HBM)
  // composite instance (FAM fixed): DevWorkload::node_recip ([node][3]) and
  // cap_recip, for the reciprocal divisions of composite_fast
  const double* zp = nullptr;
  const double* capz = nullptr;

  __device__ void load(int32_t fam_id, const double* p) {
    family = FAM >= 0 ? FAM : fam_id;
    wp = p;
  }

  template <int NPASS, bool GP>
  __device__ int64_t score(int ps, const NodeRegs<NPASS, GP>& nr, const PodView& pod, int& exc) const {
    if (!feasible<NPASS>(ps, nr, pod)) return 0;
    // weights are re-read (scalar-cache hits) at every call rather than held in
    // SGPRs across the event loop: the opaque pointer stops the compiler from
    // hoisting the loads and spilling 8-32 SGPRs per event
    const double* qg = reinterpret_cast<const double*>(uniu64(reinterpret_cast<uint64_t>(wp)));
    asm volatile("" : "+s"(qg));
    const FKS_CONST double* q = const_ptr(qg);   // scalar loads
    double w[kWeights];
#pragma unroll
    for (int k = 0; k < kWeights; ++k) w[k] = k < family_weights(FAM) ? q[k] : 0.0;
    if constexpr (FAM == FAM_COMPOSITE_LINEAR) {
      // the composite instance: the host runs it only on finite weights with
      // verified reciprocals (engine_host stage_builtin).  The truncated score
      // (>= 0) is returned as its double's bit pattern: non-negative doubles
      // order like their bits, so the wave argmax (u64) is unchanged and no
      // f64 -> i64 conversion is needed.
      const double* z = zp + (size_t)(ps * kWave + lane_id()) * 3;
      const double zcap = pod.ngpu > 0 ? capz[nr.gpu_left[ps]] : 0.0;
      return (int64_t)__double_as_longlong(
          trunc_score_f(composite_fast<NPASS>(ps, nr, pod, (const double*)w, z, zcap), exc));
    }
    return score_weights<NPASS>(family, (const double*)w, ps, nr, pod, exc);
  }

  // The family formulas on an already-loaded weight vector (shared with the
  // 4-policies-per-wave row kernel, replay_rows.hip.h, whose weights come
  // from LDS).  The caller has checked feasibility.
  template <int NPASS, class WP, bool GP>
  __device__ static int64_t score_weights(int family, WP w, int ps, const NodeRegs<NPASS, GP>& nr,
                                          const PodView& pod, int& exc) {
    switch (FAM >= 0 ? FAM : family) {
      case FAM_FIRST_FIT:
        return 1000;
      case FAM_BEST_FIT: {
        const int64_t rc = (int64_t)nr.cpu_left[ps] - pod.cpu;
        const int64_t rm = (int64_t)nr.mem_left[ps] - pod.mem;
        const int64_t rg = (int64_t)nr.gpu_left[ps] - pod.ngpu;
        if (nr.ctot(ps) == 0 || nr.mtot(ps) == 0) { exc = EXC_ZERO_DIVISION; return 0; }
        const double nc = (double)rc / (double)nr.ctot(ps);
        const double nm = (double)rm / (double)nr.mtot(ps);
        const int gd = nr.ngp(ps) > 1 ? nr.ngp(ps) : 1;
        const double ng = (double)rg / (double)gd;
        const double t = nc * 0.33 + nm * 0.33;
        const double nrm = t + ng * 0.34;
        const double x = (1.0 - nrm) * 10000.0;
        return trunc_score(x, exc);
      }
      case FAM_RANDOM_LINEAR: {
        double s = w[0] + (double)nr.cpu_left[ps] * w[1];
        s = s + (double)nr.mem_left[ps] * w[2];
        if (pod.ngpu > 0 && nr.gpu_left[ps] > 0) s = s + (double)nr.gpu_left[ps] * w[3];
        return trunc_score(s, exc);
      }
      case FAM_FEATURE_LINEAR: {
        double f[kFeatureCount];
        features<NPASS>(ps, nr, pod, f);
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < kFeatureCount; ++k)
          if (w[k] != 0.0) s = s + w[k] * f[k];
        return trunc_score(s, exc);
      }
      case FAM_COMPOSITE_LINEAR:
            return trunc_score(composite<NPASS>(ps, nr, pod, w), exc);
    }
    exc = EXC_UNSUPPORTED;
    return 0;
  }

  // twin of fks::BuiltinScorer::composite_vector (csrc/cpu/builtin_scorers.hpp):
  // the weighted terms are accumulated as they are produced (same order and
  // rounding as `score += w_k * (f_k)`), so no 16-double feature vector is
  // held live across the node loop.
  template <int NPASS, class WP, bool GP>
  __device__ static double composite(int ps, const NodeRegs<NPASS, GP>& nr, const PodView& pod, WP w) {
    const int ng = nr.ngp(ps);
    const bool gpod = pod.ngpu > 0;
    // 32-bit temporaries: GPU milli totals < 2^20 (prepare_device_workload),
    // so sums over <= 8 GPUs cannot overflow; differences widen where formed
    const int32_t ct = nr.ctot(ps), mt = nr.mtot(ps);
    const int32_t cl = nr.cpu_left[ps], ml = nr.mem_left[ps];
    const double cpu_u = (double)((int64_t)ct - cl) / (double)(ct > 1 ? ct : 1);
    const double mem_u = (double)((int64_t)mt - ml) / (double)(mt > 1 ? mt : 1);
    int32_t free_m = 0, idle = 0, gmax = 0, gmin = 0, best = -1;
#pragma unroll
    for (int j = 0; j < kGmax; ++j) {
      if (j < ng) {
        const int32_t l = nr.g(ps, j);
        free_m += l;
        idle += (l == nr.gt(ps, j));
        gmax = (j == 0 || l > gmax) ? l : gmax;
        gmin = (j == 0 || l < gmin) ? l : gmin;
        if (gpod && l >= pod.gmilli && (best < 0 || l - pod.gmilli < best)) best = l - pod.gmilli;
      }
    }
    double gpu_u = 0.0;
    if (gpod) {
      const int64_t cap = (int64_t)nr.gpu_left[ps] * nr.gt(ps, 0);
      gpu_u = (double)(cap - free_m) / (double)(cap > 1 ? cap : 1);   // cap is int64
    }
    double s = 0.0;
    auto acc = [&](int k, double f) { if (w[k] != 0.0) s = s + w[k] * f; };
    acc(0, 1.0);
    acc(1, cpu_u < 0.7 ? 1.0 - cpu_u : 0.0);
    acc(2, cpu_u >= 0.7 ? 1.0 - cpu_u : 0.0);
    acc(3, mem_u < 0.7 ? 1.0 - mem_u : 0.0);
    acc(4, mem_u >= 0.7 ? 1.0 - mem_u : 0.0);
    acc(5, gpod ? (gpu_u < 0.7 ? 1.0 - gpu_u : 0.0) : 0.0);
    acc(6, gpod ? (gpu_u >= 0.7 ? 1.0 - gpu_u : 0.0) : 0.0);
    {
      // free_m >= 0, d >= 1: Python's floor modulo is the unsigned remainder
      const uint32_t d = pod.gmilli > 1 ? (uint32_t)pod.gmilli : 1u;
      acc(7, gpod ? (double)((uint32_t)free_m % d) : 0.0);
    }
    const double a = (double)cl / (double)(ml > 1 ? ml : 1);
    const double b = (double)pod.cpu / (double)(pod.mem > 1 ? pod.mem : 1);
    acc(8, fabs(a - b));
    acc(9, (cl > (int64_t)pod.cpu * 2 && ml > (int64_t)pod.mem * 2) ? 1.0 : 0.0);
    acc(10, gpod ? (double)(gmax - gmin) : 0.0);
    acc(11, (ct > 10000 && mt > 64) ? 1.0 : 0.0);
    acc(12, (cpu_u > 0.9 || mem_u > 0.9) ? 1.0 : 0.0);
    acc(13, best < 0 ? 0.0 : (double)best / 1000.0);
    acc(14, (double)idle / (double)(ng > 1 ? ng : 1));
    acc(15, (!gpod && ng > 0) ? 1.0 : 0.0);
    return s;
  }

  // composite() on the wave kernel for finite weights, bit for bit: no `w != 0`
  // tests, one member per threshold pair, 0/1 indicators add the weight (see
  // composite_row), the host's pod quotient, the verified 1/1000 (the literal
  // 0.001 is RN(1/1000); the host's fast_div check covers [0, 2^21)) and the
  // host-verified node / GPU-capacity reciprocals, read per node pass from the
  // workload's tables (no registers held across passes).
  template <int NPASS, class WP, bool GP>
  __device__ static double composite_fast(int ps, const NodeRegs<NPASS, GP>& nr, const PodView& pod, WP w,
                                          const double* z, double zcap) {
    const int ng = nr.ngp(ps);
    const bool gpod = pod.ngpu > 0;
    const int32_t ct = nr.ctot(ps), mt = nr.mtot(ps);
    const int32_t cl = nr.cpu_left[ps], ml = nr.mem_left[ps];
    // the host's verified reciprocals (DeviceEngine::prepare_recips): numerators in [0, total]
    const double cpu_u = div_by_recip((double)(ct - cl), (double)(ct > 1 ? ct : 1), z[0]);
    const double mem_u = div_by_recip((double)(mt - ml), (double)(mt > 1 ? mt : 1), z[1]);
    int32_t free_m = 0, idle = 0, gmax = 0, gmin = 0, best = -1;
#pragma unroll
    for (int j = 0; j < kGmax; ++j) {
      if (j < ng) {
        const int32_t l = nr.g(ps, j);
        free_m += l;
        idle += (l == nr.gt(ps, j));
        gmax = (j == 0 || l > gmax) ? l : gmax;
        gmin = (j == 0 || l < gmin) ? l : gmin;
        if (gpod && l >= pod.gmilli && (best < 0 || l - pod.gmilli < best)) best = l - pod.gmilli;
      }
    }
    double s = 0.0 + w[0];
    s = s + (cpu_u < 0.7 ? w[1] : w[2]) * (1.0 - cpu_u);
    s = s + (mem_u < 0.7 ? w[3] : w[4]) * (1.0 - mem_u);
    if (gpod) {
      const int64_t cap = (int64_t)nr.gpu_left[ps] * nr.gt(ps, 0);
      const double nu = (double)(cap - free_m), du = (double)(cap > 1 ? cap : 1);
      const double gpu_u = zcap != 0.0 ? div_by_recip(nu, du, zcap) : nu / du;
      s = s + (gpu_u < 0.7 ? w[5] : w[6]) * (1.0 - gpu_u);
      const uint32_t d = pod.gmilli > 1 ? (uint32_t)pod.gmilli : 1u;
      s = s + w[7] * (double)((uint32_t)free_m % d);
    }
    const double a = (double)cl / (double)(ml > 1 ? ml : 1);
    s = s + w[8] * fabs(a - pod.cm);
    if (cl > (int64_t)pod.cpu * 2 && ml > (int64_t)pod.mem * 2) s = s + w[9];
    if (gpod) s = s + w[10] * (double)(gmax - gmin);
    if (ct > 10000 && mt > 64) s = s + w[11];
    if (cpu_u > 0.9 || mem_u > 0.9) s = s + w[12];
    if (best >= 0) s = s + w[13] * div_by_recip((double)best, 1000.0, 0.001);
    s = s + w[14] * div_by_recip((double)idle, (double)(ng > 1 ? ng : 1), z[2]);
    if (!gpod && ng > 0) s = s + w[15];
    return s;
  }

  // composite() on the row kernel, bit for bit, with less f64 work:
  //  * the divisions by max(cpu_total, 1), max(mem_total, 1), max(ngpus, 1)
  //    and 1000 run as div_by_recip on host-verified reciprocals (rz, see
  //    DeviceEngine::prepare_recips); pod.cpu / max(pod.mem, 1) is the host's
  //    per-pod quotient (rz.pcm);
  //  * no `w != 0` tests: every feature is finite and the sum starts at +0.0
  //    and can never become -0.0, so a zero weight adds +-0 and changes
  //    nothing;
  //  * each complementary threshold pair (f1/f2, f3/f4, f5/f6) adds only its
  //    nonzero member, and 0/1 indicators add the weight itself: the other
  //    member's w * 0.0 is +-0 -- which needs every weight finite (inf * 0 is
  //    NaN), so the caller passes here only policies whose weights all are.
  struct RowRecip {
    double zc, zm, zg, z1000, pcm;
    double zcap;         // RN(1 / max(gpu_left * gmilli_total, 1)) when fast_cap, else 0
    double dc, dm, dg;   // max(cpu_total, 1), max(mem_total, 1), max(ngpus, 1) as doubles
  };
  template <class WP, bool GP>
  __device__ static double composite_row(const NodeRegs<1, GP>& nr, const PodView& pod, WP w, const RowRecip& rz) {
    const int ng = nr.ngpus[0];
    const bool gpod = pod.ngpu > 0;
    const int32_t ct = nr.cpu_total[0], mt = nr.mem_total[0];
    const int32_t cl = nr.cpu_left[0], ml = nr.mem_left[0];
    // numerators in [0, total]: the host's invariant check behind rz
    const double cpu_u = div_by_recip((double)(ct - cl), rz.dc, rz.zc);
    const double mem_u = div_by_recip((double)(mt - ml), rz.dm, rz.zm);
    int32_t free_m = 0, idle = 0, gmax = 0, gmin = 0, best = -1;
#pragma unroll
    for (int j = 0; j < kGmax; ++j) {
      if (j < ng) {
        const int32_t l = nr.g(0, j);
        free_m += l;
        idle += (l == nr.gmt1[0]);
        gmax = (j == 0 || l > gmax) ? l : gmax;
        gmin = (j == 0 || l < gmin) ? l : gmin;
        if (gpod && l >= pod.gmilli && (best < 0 || l - pod.gmilli < best)) best = l - pod.gmilli;
      }
    }
    double s = 0.0 + w[0];
    s = s + (cpu_u < 0.7 ? w[1] : w[2]) * (1.0 - cpu_u);
    s = s + (mem_u < 0.7 ? w[3] : w[4]) * (1.0 - mem_u);
    if (gpod) {
      const int64_t cap = (int64_t)nr.gpu_left[0] * nr.gt(0, 0);
      const double nu = (double)(cap - free_m), du = (double)(cap > 1 ? cap : 1);
      // zcap: verified for |numerator| <= 8 x the cluster's one per-GPU milli total
      const double gpu_u = rz.zcap != 0.0 ? div_by_recip(nu, du, rz.zcap) : nu / du;
      s = s + (gpu_u < 0.7 ? w[5] : w[6]) * (1.0 - gpu_u);
      const uint32_t d = pod.gmilli > 1 ? (uint32_t)pod.gmilli : 1u;
      s = s + w[7] * (double)((uint32_t)free_m % d);
    }
    const double a = (double)cl / (double)(ml > 1 ? ml : 1);
    s = s + w[8] * fabs(a - rz.pcm);
    if (cl > (int64_t)pod.cpu * 2 && ml > (int64_t)pod.mem * 2) s = s + w[9];
    if (gpod) s = s + w[10] * (double)(gmax - gmin);
    if (ct > 10000 && mt > 64) s = s + w[11];
    if (cpu_u > 0.9 || mem_u > 0.9) s = s + w[12];
    if (best >= 0) s = s + w[13] * div_by_recip((double)best, 1000.0, rz.z1000);
    s = s + w[14] * div_by_recip((double)idle, rz.dg, rz.zg);
    if (!gpod && ng > 0) s = s + w[15];
    return s;
  }

  template <int NPASS, bool GP>
  __device__ static void features(int ps, const NodeRegs<NPASS, GP>& nr, const PodView& pod, double* f) {
    const int ng = nr.ngp(ps);
    const int64_t cpu_tot = nr.ctot(ps) > 1 ? nr.ctot(ps) : 1;
    const int64_t mem_tot = nr.mtot(ps) > 1 ? nr.mtot(ps) : 1;
    const int ngd = ng > 1 ? ng : 1;
    f[0] = 1.0;
    const double rc = (double)((int64_t)nr.cpu_left[ps] - pod.cpu) / (double)cpu_tot;
    const double rm = (double)((int64_t)nr.mem_left[ps] - pod.mem) / (double)mem_tot;
    f[1] = rc;
    f[2] = rm;
    f[3] = (double)((int64_t)nr.gpu_left[ps] - pod.ngpu) / (double)ngd;
    f[4] = fabs(rc - rm);
    int32_t free_m = 0, idle = 0, part = 0, best = -1;
#pragma unroll
    for (int j = 0; j < kGmax; ++j) {
      if (j < ng) {
        const int32_t l = nr.g(ps, j);
        free_m += l;
        idle += (l == nr.gt(ps, j));
        part += (0 < l && l < nr.gt(ps, j));
        if (pod.ngpu > 0 && l >= pod.gmilli && (best < 0 || l - pod.gmilli < best)) best = l - pod.gmilli;
      }
    }
    f[5] = (double)free_m / 1000.0;
    {
      const uint32_t d = pod.gmilli > 1 ? (uint32_t)pod.gmilli : 1u;
      f[6] = (double)((uint32_t)free_m % d) / 1000.0;
    }
    f[7] = (double)idle / (double)ngd;
    f[8] = (double)part / (double)ngd;
    f[9] = (pod.ngpu == 0 && ng > 0) ? 1.0 : 0.0;
    f[10] = best < 0 ? 0.0 : (double)best / 1000.0;
    f[11] = (double)nr.ctot(ps) / 100000.0;
  }
};

}  // namespace fksd
