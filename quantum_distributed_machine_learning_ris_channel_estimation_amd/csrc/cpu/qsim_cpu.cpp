// CPU state-vector simulator (C++17 + OpenMP) for the QSC variational circuit.
//
// Same circuit as csrc/hip/qsim.hip (reference: Estimators_QuantumNAT_onchipQNN.py:125-142)
// but implemented independently and literally, gate by gate, in double precision:
// it is (a) the compute path of the CPU configuration ("4-qubit VQC, CPU state-vector
// sim, batch=32") and (b) the oracle the HIP kernels are tested against.
//
// Wire i <-> bit i of the basis index.  Backward is adjoint differentiation over the
// explicit gate list; per-sample weight gradients are summed in sample order so the
// result is deterministic for any thread count.
#include <cmath>
#include <complex>
#include <cstdint>
#include <cstring>
#include <vector>

#define QD_API extern "C" __attribute__((visibility("default")))

namespace {

using cd = std::complex<double>;

enum GateType { kRY = 0, kRZ = 1, kCNOT = 2 };

struct Gate {
  int type;
  int q;      // target wire
  int c;      // control wire (CNOT)
  int wparam; // index into flattened weights, -1 if none
  int xparam; // index into the sample's input angles, -1 if none
  double angle;
};

std::vector<Gate> build_circuit(const float* xs, const float* w, int n, int L) {
  std::vector<Gate> g;
  g.reserve(n + L * 3 * n);
  for (int i = 0; i < n; ++i) g.push_back({kRY, i, -1, -1, i, (double)xs[i]});
  for (int l = 0; l < L; ++l) {
    for (int i = 0; i < n; ++i) {
      const int p = (l * n + i) * 2;
      g.push_back({kRY, i, -1, p, -1, (double)w[p]});
      g.push_back({kRZ, i, -1, p + 1, -1, (double)w[p + 1]});
    }
    for (int i = 0; i + 1 < n; ++i) g.push_back({kCNOT, i + 1, i, -1, -1, 0.0});
    g.push_back({kCNOT, 0, n - 1, -1, -1, 0.0});
  }
  return g;
}

// Apply gate (or its adjoint) in place.
void apply(std::vector<cd>& s, const Gate& g, bool adjoint) {
  const size_t D = s.size();
  const size_t m = size_t(1) << g.q;
  if (g.type == kCNOT) {
    const size_t cm = size_t(1) << g.c;
    for (size_t k = 0; k < D; ++k)
      if ((k & cm) && !(k & m)) std::swap(s[k], s[k | m]);
    return;
  }
  const double a = adjoint ? -g.angle : g.angle;
  if (g.type == kRY) {
    const double c = std::cos(a / 2), sn = std::sin(a / 2);
    for (size_t k = 0; k < D; ++k) {
      if (k & m) continue;
      const cd a0 = s[k], a1 = s[k | m];
      s[k] = c * a0 - sn * a1;
      s[k | m] = sn * a0 + c * a1;
    }
  } else {  // RZ
    const cd e0 = std::polar(1.0, -a / 2), e1 = std::polar(1.0, a / 2);
    for (size_t k = 0; k < D; ++k) s[k] *= (k & m) ? e1 : e0;
  }
}

// Im <lam| G_gen |psi> where G_gen = Y (RY) or Z (RZ) on wire q.
double gen_im(const std::vector<cd>& lam, const std::vector<cd>& psi, const Gate& g) {
  const size_t D = psi.size();
  const size_t m = size_t(1) << g.q;
  cd acc = 0;
  if (g.type == kRZ) {
    for (size_t k = 0; k < D; ++k) acc += std::conj(lam[k]) * ((k & m) ? -psi[k] : psi[k]);
  } else {  // Y: (Y psi)_k = -i psi_{k^m} if bit 0, +i psi_{k^m} if bit 1
    const cd I(0, 1);
    for (size_t k = 0; k < D; ++k) acc += std::conj(lam[k]) * ((k & m) ? I : -I) * psi[k ^ m];
  }
  return acc.imag();
}

void forward_state(std::vector<cd>& s, const std::vector<Gate>& gates) {
  std::fill(s.begin(), s.end(), cd(0));
  s[0] = 1.0;
  for (const Gate& g : gates) apply(s, g, false);
}

}  // namespace

QD_API int qd_cpu_qsim_fwd(const float* x, const float* w, float* E, int B, int n, int L) {
  if (n < 1 || n > 24) return 1;
  const size_t D = size_t(1) << n;
#pragma omp parallel for schedule(static)
  for (int b = 0; b < B; ++b) {
    std::vector<cd> s(D);
    forward_state(s, build_circuit(x + (size_t)b * n, w, n, L));
    for (int q = 0; q < n; ++q) {
      double e = 0;
      for (size_t k = 0; k < D; ++k) e += std::norm(s[k]) * (((k >> q) & 1) ? -1.0 : 1.0);
      E[(size_t)b * n + q] = (float)e;
    }
  }
  return 0;
}

QD_API int qd_cpu_qsim_bwd(const float* x, const float* w, const float* gE, float* dx, float* dw, int B, int n,
                           int L) {
  if (n < 1 || n > 24) return 1;
  const size_t D = size_t(1) << n;
  const int P = 2 * n * L;
  std::vector<double> per(size_t(B) * P, 0.0);
#pragma omp parallel for schedule(static)
  for (int b = 0; b < B; ++b) {
    const auto gates = build_circuit(x + (size_t)b * n, w, n, L);
    std::vector<cd> psi(D), lam(D);
    forward_state(psi, gates);
    for (size_t k = 0; k < D; ++k) {
      double o = 0;
      for (int q = 0; q < n; ++q) o += (((k >> q) & 1) ? -1.0 : 1.0) * gE[(size_t)b * n + q];
      lam[k] = o * psi[k];
    }
    double* pw = per.data() + (size_t)b * P;
    for (int q = 0; q < n; ++q) dx[(size_t)b * n + q] = 0.f;
    for (int gi = (int)gates.size() - 1; gi >= 0; --gi) {
      const Gate& g = gates[gi];
      if (g.type != kCNOT) {
        const double d = gen_im(lam, psi, g);  // dL/dangle = 2 Re<lam| dG |psi_before> = Im<lam|Gen|psi_after>
        if (g.wparam >= 0) pw[g.wparam] += d;
        if (g.xparam >= 0) dx[(size_t)b * n + g.xparam] += (float)d;
      }
      apply(psi, g, true);
      apply(lam, g, true);
    }
  }
  for (int p = 0; p < P; ++p) {
    double t = 0;
    for (int b = 0; b < B; ++b) t += per[(size_t)b * P + p];
    dw[p] = (float)t;
  }
  return 0;
}
