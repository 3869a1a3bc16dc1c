// Host check of the device's correctly rounded exp / log / pow (csrc/hip/dd_math.h)
// against glibc, which CPython calls for `**`, math.exp and math.log.  The
// device code is __host__ __device__, so this is the same arithmetic the
// kernels run.  A result the device accepts (status 0) must equal glibc's
// bit for bit; near-midpoint cases may defer (status 2) to the host engines.
//
//   g++ -O2 -std=c++17 -DFKS_HOST_JIT -ffp-contract=off -I csrc/hip dd_math_check.cpp
//   ./a.out N SEED   ->  one line per function: calls mismatches defers overflow ns/call
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "dd_math.h"

namespace {
struct Tally { long calls = 0, bad = 0, defer = 0, ovf = 0; double ns = 0; };

void report(const char* name, const Tally& t) {
  std::printf("%s calls=%ld mismatches=%ld defers=%ld overflow=%ld ns_per_call=%.1f\n", name, t.calls, t.bad, t.defer,
              t.ovf, t.calls ? t.ns / t.calls : 0.0);
}
bool same(double a, double b) { return std::memcmp(&a, &b, sizeof a) == 0; }
}  // namespace

int main(int argc, char** argv) {
  const long n = argc > 1 ? std::atol(argv[1]) : 100000;
  std::mt19937_64 rng(argc > 2 ? std::atoll(argv[2]) : 1);
  std::uniform_real_distribution<double> u(0.0, 1.0);
  // exponents programs use (fractional powers, small integers, reciprocals) and random ones
  const double common[] = {0.5, 1.5, 2.0, 2.5, 3.0, 0.6, 0.7, 0.8, 0.3, 0.25, 1.2, 4.0, -1.0, -0.5, -2.0, 0.1, 1.0 / 3.0};
  std::vector<double> xs(n), ys(n), outs(n);
  std::vector<int> st(n);
  for (long i = 0; i < n; ++i) {
    const double r = u(rng);
    xs[i] = r < 0.5 ? std::exp(-7.0 + 14.0 * u(rng)) : std::exp(-30.0 + 60.0 * u(rng));   // positive, wide range
    if (i % 4 == 0) xs[i] = std::floor(xs[i] * 1000.0) / 1000.0 + 0.001;                       // decimal-ish
    ys[i] = (i % 3 == 0) ? common[i % (sizeof common / sizeof common[0])] : -6.0 + 12.0 * u(rng);
  }
  Tally tp, te, tl;
  auto t0 = std::chrono::steady_clock::now();
  std::vector<int> all_st;
  std::vector<double> all_out;
  auto keep = [&]() {
    all_st.insert(all_st.end(), st.begin(), st.end());
    all_out.insert(all_out.end(), outs.begin(), outs.end());
  };
  for (long i = 0; i < n; ++i) st[i] = fksd::dd_pow(xs[i], ys[i], outs[i]);
  keep();
  tp.ns = std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count();
  for (long i = 0; i < n; ++i) {
    if (xs[i] == 1.0) continue;
    ++tp.calls;
    const double ref = std::pow(xs[i], ys[i]);
    if (st[i] == 2) ++tp.defer;
    else if (st[i] == 1) { ++tp.ovf; if (!std::isinf(ref)) ++tp.bad; }
    else if (!same(outs[i], ref)) {
      ++tp.bad;
      if (tp.bad <= 5) std::printf("pow mismatch x=%.17g y=%.17g dev=%.17g glibc=%.17g\n", xs[i], ys[i], outs[i], ref);
    }
  }
  for (long i = 0; i < n; ++i) xs[i] = -700.0 + 1400.0 * u(rng) * ((i % 2) ? 1.0 : 0.02);
  t0 = std::chrono::steady_clock::now();
  for (long i = 0; i < n; ++i) st[i] = fksd::dd_exp_d(xs[i], outs[i]);
  keep();
  te.ns = std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count();
  for (long i = 0; i < n; ++i) {
    ++te.calls;
    const double ref = std::exp(xs[i]);
    if (st[i] == 2) ++te.defer;
    else if (st[i] == 1) { ++te.ovf; if (!std::isinf(ref)) ++te.bad; }
    else if (!same(outs[i], ref)) {
      ++te.bad;
      if (te.bad <= 5) std::printf("exp mismatch x=%.17g dev=%.17g glibc=%.17g\n", xs[i], outs[i], ref);
    }
  }
  for (long i = 0; i < n; ++i) xs[i] = std::exp(-700.0 + 1400.0 * u(rng));
  t0 = std::chrono::steady_clock::now();
  for (long i = 0; i < n; ++i) st[i] = fksd::dd_log_d(xs[i], outs[i]);
  keep();
  tl.ns = std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count();
  for (long i = 0; i < n; ++i) {
    ++tl.calls;
    const double ref = std::log(xs[i]);
    if (st[i] == 2) ++tl.defer;
    else if (!same(outs[i], ref)) {
      ++tl.bad;
      if (tl.bad <= 5) std::printf("log mismatch x=%.17g dev=%.17g glibc=%.17g\n", xs[i], outs[i], ref);
    }
  }
  if (argc > 3) {   // optional: dump every status / result (A/B of two builds)
    if (FILE* f = std::fopen(argv[3], "wb")) {
      std::fwrite(all_st.data(), sizeof(int), all_st.size(), f);
      std::fwrite(all_out.data(), sizeof(double), all_out.size(), f);
      std::fclose(f);
    }
  }
  report("pow", tp);
  report("exp", te);
  report("log", tl);
  return (tp.bad || te.bad || tl.bad) ? 1 : 0;
}
