// Built-in policy families of the native engines.
//
// Each is the exact native twin of a policy *program* (the text the Python
// API exposes, see funsearch_kubernetes_simulator_amd/models/families.py):
// the same IEEE operations in the same order, so a built-in replay and a
// replay of its program text (object engine or bytecode VM) agree bit-for-bit.
#pragma once

#include "engine.hpp"

namespace fks {

enum BuiltinFamily : int32_t {
  FAM_FIRST_FIT = 0,   // reference _create_first_fit_policy
  FAM_BEST_FIT = 1,    // reference _create_best_fit_policy
  FAM_RANDOM_LINEAR = 2,  // reference _create_random_policy (base, cpu, mem, gpu factors)
  FAM_FEATURE_LINEAR = 3, // generalised linear feature family (models/families.py)
  FAM_COMPOSITE_LINEAR = 4, // champion-containing 16-term basis (models/families.py)
};

constexpr int kFeatureCount = 12;
constexpr int kCompositeCount = 16;

struct BuiltinScorer {
  int32_t family = FAM_FIRST_FIT;
  double w[16] = {0};

  ScoreOut operator()(const ScoreCtx& c, int n) const {
    ScoreOut o;
    if (!feasible(c, n)) { o.v = Num::I(0); return o; }
    const Workload& W = c.w;
    const ClusterState& S = c.s;
    const int p = c.pod;
    switch (family) {
      case FAM_FIRST_FIT:
        o.v = Num::I(1000);
        return o;
      case FAM_BEST_FIT: {
        const int64_t rc = S.cpu_left[n] - W.pcpu[p];
        const int64_t rm = S.mem_left[n] - W.pmem[p];
        const int64_t rg = (int64_t)S.gpu_left[n] - W.pngpu[p];
        if (W.cpu_total[n] == 0 || W.mem_total[n] == 0) { o.exc = EXC_ZERO_DIVISION; return o; }
        const double nc = (double)rc / (double)W.cpu_total[n];
        const double nm = (double)rm / (double)W.mem_total[n];
        const double ng = (double)rg / (double)std::max<int32_t>(W.ngpus[n], 1);
        const double t = nc * 0.33 + nm * 0.33;
        const double nr = t + ng * 0.34;
        const double x = (1.0 - nr) * 10000.0;
        // int(x) then max(1, .)
        if (std::isnan(x)) { o.exc = EXC_VALUE; return o; }
        if (std::isinf(x)) { o.exc = EXC_OVERFLOW; return o; }
        const int64_t s = (int64_t)x;
        o.v = Num::I(std::max<int64_t>(1, s));
        return o;
      }
      case FAM_RANDOM_LINEAR: {
        // score = base + cpu_left * cf + mem_left * mf
        double s = w[0] + (double)S.cpu_left[n] * w[1];
        s = s + (double)S.mem_left[n] * w[2];
        if (W.pngpu[p] > 0 && S.gpu_left[n] > 0) s = s + (double)S.gpu_left[n] * w[3];
        if (std::isnan(s)) { o.exc = EXC_VALUE; return o; }
        if (std::isinf(s)) { o.exc = EXC_OVERFLOW; return o; }
        if (std::fabs(s) >= 9.2233720368547758e18) { o.exc = EXC_UNSUPPORTED; return o; }
        o.v = Num::I(std::max<int64_t>(1, (int64_t)s));
        return o;
      }
      case FAM_FEATURE_LINEAR: {
        double f[kFeatureCount];
        feature_vector(c, n, f);
        double s = 0.0;
        for (int k = 0; k < kFeatureCount; ++k)
          if (w[k] != 0.0) s = s + w[k] * f[k];
        if (std::isnan(s)) { o.exc = EXC_VALUE; return o; }
        if (std::isinf(s)) { o.exc = EXC_OVERFLOW; return o; }
        if (std::fabs(s) >= 9.2233720368547758e18) { o.exc = EXC_UNSUPPORTED; return o; }
        o.v = Num::I(std::max<int64_t>(1, (int64_t)s));
        return o;
      }
      case FAM_COMPOSITE_LINEAR: {
        double f[kCompositeCount];
        composite_vector(c, n, f);
        double s = 0.0;
        for (int k = 0; k < kCompositeCount; ++k)
          if (w[k] != 0.0) s = s + w[k] * f[k];
        if (std::isnan(s)) { o.exc = EXC_VALUE; return o; }
        if (std::isinf(s)) { o.exc = EXC_OVERFLOW; return o; }
        if (std::fabs(s) >= 9.2233720368547758e18) { o.exc = EXC_UNSUPPORTED; return o; }
        o.v = Num::I(std::max<int64_t>(1, (int64_t)s));
        return o;
      }
    }
    o.exc = EXC_UNSUPPORTED;
    return o;
  }

  // Composite family (models/families.py COMPOSITE_FEATURES), Python
  // int/float rules, feasible (pod, node) only.
  static void composite_vector(const ScoreCtx& c, int n, double* f) {
    const Workload& W = c.w;
    const ClusterState& S = c.s;
    const int p = c.pod;
    const int g0 = W.gpu_start[n], ng = W.ngpus[n];
    const bool gpod = W.pngpu[p] > 0;
    const double cpu_u = (double)(W.cpu_total[n] - S.cpu_left[n]) / (double)std::max<int64_t>(1, W.cpu_total[n]);
    const double mem_u = (double)(W.mem_total[n] - S.mem_left[n]) / (double)std::max<int64_t>(1, W.mem_total[n]);
    int64_t free_m = 0, idle = 0, gmax = 0, gmin = 0, best = -1;
    for (int j = 0; j < ng; ++j) {
      const int64_t l = S.gmilli_left[g0 + j];
      free_m += l;
      idle += (l == W.gmilli_total[g0 + j]);
      gmax = j == 0 ? l : std::max(gmax, l);
      gmin = j == 0 ? l : std::min(gmin, l);
      if (gpod && l >= W.pgmilli[p] && (best < 0 || l - W.pgmilli[p] < best)) best = l - W.pgmilli[p];
    }
    double gpu_u = 0.0;
    if (gpod) {
      const int64_t cap = (int64_t)S.gpu_left[n] * W.gmilli_total[g0];
      gpu_u = (double)(cap - free_m) / (double)std::max<int64_t>(1, cap);
    }
    f[0] = 1.0;
    f[1] = cpu_u < 0.7 ? 1.0 - cpu_u : 0.0;
    f[2] = cpu_u >= 0.7 ? 1.0 - cpu_u : 0.0;
    f[3] = mem_u < 0.7 ? 1.0 - mem_u : 0.0;
    f[4] = mem_u >= 0.7 ? 1.0 - mem_u : 0.0;
    f[5] = gpod ? (gpu_u < 0.7 ? 1.0 - gpu_u : 0.0) : 0.0;
    f[6] = gpod ? (gpu_u >= 0.7 ? 1.0 - gpu_u : 0.0) : 0.0;
    if (gpod) {
      const int64_t d = std::max<int64_t>(1, W.pgmilli[p]);
      int64_t m = free_m % d;
      if (m != 0 && ((m < 0) != (d < 0))) m += d;
      f[7] = (double)m;
    } else {
      f[7] = 0.0;
    }
    const double a = (double)S.cpu_left[n] / (double)std::max<int64_t>(1, S.mem_left[n]);
    const double b = (double)W.pcpu[p] / (double)std::max<int64_t>(1, W.pmem[p]);
    f[8] = std::fabs(a - b);
    f[9] = (S.cpu_left[n] > W.pcpu[p] * 2 && S.mem_left[n] > W.pmem[p] * 2) ? 1.0 : 0.0;
    f[10] = gpod ? (double)(gmax - gmin) : 0.0;
    f[11] = (W.cpu_total[n] > 10000 && W.mem_total[n] > 64) ? 1.0 : 0.0;
    f[12] = (cpu_u > 0.9 || mem_u > 0.9) ? 1.0 : 0.0;
    f[13] = best < 0 ? 0.0 : (double)best / 1000.0;
    f[14] = (double)idle / (double)std::max(1, ng);
    f[15] = (W.pngpu[p] == 0 && ng > 0) ? 1.0 : 0.0;
  }

  // Feature vector of the generalised linear family.  Each entry is the
  // value of one Python expression (models/families.py FEATURES), evaluated
  // with Python's int/float rules.  Only called on feasible (pod, node).
  static void feature_vector(const ScoreCtx& c, int n, double* f) {
    const Workload& W = c.w;
    const ClusterState& S = c.s;
    const int p = c.pod;
    const int g0 = W.gpu_start[n], ng = W.ngpus[n];
    const int64_t cpu_tot = std::max<int64_t>(1, W.cpu_total[n]);
    const int64_t mem_tot = std::max<int64_t>(1, W.mem_total[n]);
    // f0: 1
    f[0] = 1.0;
    // f1: (node.cpu_milli_left - pod.cpu_milli) / max(1, node.cpu_milli_total)
    const double rc = (double)(S.cpu_left[n] - W.pcpu[p]) / (double)cpu_tot;
    f[1] = rc;
    // f2: (node.memory_mib_left - pod.memory_mib) / max(1, node.memory_mib_total)
    const double rm = (double)(S.mem_left[n] - W.pmem[p]) / (double)mem_tot;
    f[2] = rm;
    // f3: (node.gpu_left - pod.num_gpu) / max(1, len(node.gpus))
    f[3] = (double)((int64_t)S.gpu_left[n] - W.pngpu[p]) / (double)std::max(1, ng);
    // f4: abs(f1 - f2)
    f[4] = std::fabs(rc - rm);
    // f5: sum(g.gpu_milli_left for g in node.gpus) / 1000
    int64_t free_m = 0, idle = 0, part = 0;
    for (int j = 0; j < ng; ++j) {
      const int32_t l = S.gmilli_left[g0 + j];
      free_m += l;
      idle += (l == W.gmilli_total[g0 + j]);
      part += (0 < l && l < W.gmilli_total[g0 + j]);
    }
    f[5] = (double)free_m / 1000.0;
    // f6: sum(g.gpu_milli_left ...) % max(1, pod.gpu_milli) / 1000   (python int %)
    {
      const int64_t d = std::max<int64_t>(1, W.pgmilli[p]);
      int64_t m = free_m % d;
      if (m != 0 && ((m < 0) != (d < 0))) m += d;
      f[6] = (double)m / 1000.0;
    }
    // f7: idle GPU count / max(1, len(node.gpus))
    f[7] = (double)idle / (double)std::max(1, ng);
    // f8: partially used GPU count / max(1, len(node.gpus))
    f[8] = (double)part / (double)std::max(1, ng);
    // f9: 1 if (pod.num_gpu == 0 and len(node.gpus) > 0) else 0  (CPU pod on GPU node)
    f[9] = (W.pngpu[p] == 0 && ng > 0) ? 1.0 : 0.0;
    // f10: best-fit slack of the tightest fitting GPU / 1000 (0 for CPU pods)
    {
      int64_t best = -1;
      if (W.pngpu[p] > 0)
        for (int j = 0; j < ng; ++j) {
          const int32_t l = S.gmilli_left[g0 + j];
          if (l >= W.pgmilli[p] && (best < 0 || l - W.pgmilli[p] < best)) best = l - W.pgmilli[p];
        }
      f[10] = best < 0 ? 0.0 : (double)best / 1000.0;
    }
    // f11: node.cpu_milli_total / 100000
    f[11] = (double)W.cpu_total[n] / 100000.0;
  }
};

}  // namespace fks
