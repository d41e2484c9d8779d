// Host sanitizer driver for the C++ CPU simulator ("host ASan builds of the C++ CPU
// simulator").  Built with -fsanitize=address,undefined by tests/test_sanitizers.py; links the
// simulator source directly, so no preload is needed.  Checks, for several (n, L):
//   * every <Z_i> lies in [-1, 1];
//   * the adjoint gradients match the exact parameter-shift rule (f(t+pi/2) - f(t-pi/2)) / 2
//     for every input angle and every weight.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

extern "C" int qd_cpu_qsim_fwd(const float* x, const float* w, float* E, int B, int n, int L);
extern "C" int qd_cpu_qsim_bwd(const float* x, const float* w, const float* gE, float* dx, float* dw, int B, int n,
                               int L);

static double objective(std::vector<float>& x, std::vector<float>& w, const std::vector<float>& g, int B, int n,
                        int L) {
  std::vector<float> E(B * n);
  if (qd_cpu_qsim_fwd(x.data(), w.data(), E.data(), B, n, L)) std::abort();
  double s = 0;
  for (int i = 0; i < B * n; ++i) s += double(E[i]) * g[i];
  return s;
}

int main() {
  std::mt19937 rng(1234);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  int failures = 0;
  const int cases[][3] = {{2, 1, 3}, {3, 2, 2}, {4, 3, 5}, {6, 2, 2}, {9, 1, 1}};
  for (const auto& c : cases) {
    const int n = c[0], L = c[1], B = c[2];
    std::vector<float> x(B * n), w(L * n * 2), g(B * n), E(B * n), dx(B * n), dw(L * n * 2);
    for (auto& v : x) v = U(rng);
    for (auto& v : w) v = 3.14159f * U(rng);
    for (auto& v : g) v = U(rng);
    if (qd_cpu_qsim_fwd(x.data(), w.data(), E.data(), B, n, L)) return 2;
    for (float e : E)
      if (!(e >= -1.0001f && e <= 1.0001f)) ++failures;
    if (qd_cpu_qsim_bwd(x.data(), w.data(), g.data(), dx.data(), dw.data(), B, n, L)) return 3;
    const float h = 1.5707963267948966f;
    for (size_t i = 0; i < w.size(); ++i) {
      const float t = w[i];
      w[i] = t + h;
      const double fp = objective(x, w, g, B, n, L);
      w[i] = t - h;
      const double fm = objective(x, w, g, B, n, L);
      w[i] = t;
      if (std::fabs(0.5 * (fp - fm) - dw[i]) > 1e-4 * (1 + std::fabs(dw[i]))) {
        std::printf("dw mismatch n=%d L=%d i=%zu: %g vs %g\n", n, L, i, 0.5 * (fp - fm), dw[i]);
        ++failures;
      }
    }
    for (size_t i = 0; i < x.size(); ++i) {
      const float t = x[i];
      x[i] = t + h;
      const double fp = objective(x, w, g, B, n, L);
      x[i] = t - h;
      const double fm = objective(x, w, g, B, n, L);
      x[i] = t;
      if (std::fabs(0.5 * (fp - fm) - dx[i]) > 1e-4 * (1 + std::fabs(dx[i]))) {
        std::printf("dx mismatch n=%d L=%d i=%zu: %g vs %g\n", n, L, i, 0.5 * (fp - fm), dx[i]);
        ++failures;
      }
    }
  }
  std::printf("qsim_cpu_check: %d failures\n", failures);
  return failures ? 1 : 0;
}
