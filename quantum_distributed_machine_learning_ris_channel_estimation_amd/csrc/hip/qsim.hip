// Batched variational-quantum-circuit simulator for the QSC scenario classifier.
//
// Circuit (reference: Estimators_QuantumNAT_onchipQNN.py:125-142, PennyLane
// default.qubit through TorchLayer at E:144-149):
//   AngleEmbedding(x, rotation="Y")                         RY(x_i) on wire i
//   for l in 0..L-1:  RY(w[l,i,0]), RZ(w[l,i,1]) on every wire i
//                     CNOT(i,i+1) i=0..n-2, then CNOT(n-1,0)
//   return <Z_i> for every wire
//
// MI355X design (not a translation of PennyLane's gate-by-gate tape):
//  * one wave64 owns one sample's state for n >= 6 (R = 2^(n-6) complex amplitudes
//    per lane, register-resident); for n < 6 a wave holds 2^(6-n) samples.
//    Amplitude index k = r | (lane_in_sample << RB): wires 0..RB-1 are register
//    bits (pairs swap inside a lane), wires >= RB are lane bits (pairs via
//    __shfl_xor, ds_bpermute on CDNA).
//  * the embedding + layer-0 rotations collapse to a closed-form product state
//    (RY(x)RY(w) = RY(x+w); a product state needs no gate passes).
//  * the CNOT ring is a GF(2)-linear permutation of basis states: applied as ONE
//    LDS gather per layer (write natural order, read at f^-1(j)) instead of n
//    shuffle rounds.
//  * backward = adjoint differentiation: recompute psi_final, lambda = O psi with
//    O = sum_i gE_i Z_i, then sweep gates in reverse un-computing psi and lambda.
//    Per-sample dx (= layer-0 RY grads) is reduced across the sample's lanes;
//    weight grads are accumulated per lane in LDS over all samples a wave owns and
//    written as one slab row per wave (deterministic, no float atomics); the slab
//    is summed by qsim_reduce_slab (or by the fused optimizer).
#include "common.h"

namespace qd {
namespace qsim {

struct cf {
  float x, y;
};

__device__ __forceinline__ cf cmul(cf a, cf b) { return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }
__device__ __forceinline__ cf cscale(cf a, float s) { return {a.x * s, a.y * s}; }

template <int N>
struct Cfg {
  static constexpr int D = 1 << N;
  static constexpr int RB = N > 6 ? N - 6 : 0;  // register bits
  static constexpr int R = 1 << RB;             // amplitudes per lane
  static constexpr int LB = N - RB;             // lane bits per sample
  static constexpr int LPS = 1 << LB;           // lanes per sample
  static constexpr int SPW = kWave / LPS;       // samples per wave
  static constexpr int SLOTS = kWave * R;       // complex slots per wave (= SPW * D)
};

// f(k): basis-state map of the CNOT ring (CNOT(0,1) first ... CNOT(n-1,0) last).
template <int N>
__device__ __forceinline__ int ring_fwd(int k) {
#pragma unroll
  for (int i = 0; i < N - 1; ++i) k ^= ((k >> i) & 1) << (i + 1);
  k ^= (k >> (N - 1)) & 1;
  return k;
}
// f^-1(k): the same self-inverse CNOTs in reverse order.
template <int N>
__device__ __forceinline__ int ring_inv(int k) {
  k ^= (k >> (N - 1)) & 1;
#pragma unroll
  for (int i = N - 2; i >= 0; --i) k ^= ((k >> i) & 1) << (i + 1);
  return k;
}

// Apply the ring permutation (or its inverse) to a wave's states through LDS.
// `lds` is this wave's SLOTS-entry region; `sbase` = sample-in-wave * D.
template <int N, bool INVERSE>
__device__ __forceinline__ void ring_permute(cf (&a)[Cfg<N>::R], cf* lds, int sbase, int li) {
  using C = Cfg<N>;
#pragma unroll
  for (int r = 0; r < C::R; ++r) lds[sbase + (r | (li << C::RB))] = a[r];
  wave_lds_fence();
#pragma unroll
  for (int r = 0; r < C::R; ++r) {
    const int j = r | (li << C::RB);
    const int src = INVERSE ? ring_fwd<N>(j) : ring_inv<N>(j);
    a[r] = lds[sbase + src];
  }
  wave_lds_fence();
}

// Product state after AngleEmbedding + layer-0 rotations:
// amp_k = prod_i c_i(bit_i(k)), c_i(0) = cos(t/2) e^{-i p/2}, c_i(1) = sin(t/2) e^{+i p/2}.
template <int N>
__device__ __forceinline__ void product_state(cf (&a)[Cfg<N>::R], const float* xs, const float* w, int li) {
  using C = Cfg<N>;
  cf c0[N], c1[N];
#pragma unroll
  for (int q = 0; q < N; ++q) {
    float sh, ch, sp, cp;
    __sincosf(0.5f * (xs[q] + w[2 * q]), &sh, &ch);
    __sincosf(0.5f * w[2 * q + 1], &sp, &cp);
    c0[q] = {ch * cp, -ch * sp};
    c1[q] = {sh * cp, sh * sp};
  }
  cf lp = {1.f, 0.f};
#pragma unroll
  for (int q = C::RB; q < N; ++q) lp = cmul(lp, ((li >> (q - C::RB)) & 1) ? c1[q] : c0[q]);
#pragma unroll
  for (int r = 0; r < C::R; ++r) {
    cf p = lp;
#pragma unroll
    for (int q = 0; q < C::RB; ++q) p = cmul(p, ((r >> q) & 1) ? c1[q] : c0[q]);
    a[r] = p;
  }
}

// psi <- RZ(phi) RY(theta) psi on wire Q.
template <int N, int Q>
__device__ __forceinline__ void apply_rot(cf (&a)[Cfg<N>::R], float theta, float phi, int li) {
  using C = Cfg<N>;
  float s, c, sp, cp;
  __sincosf(0.5f * theta, &s, &c);
  __sincosf(0.5f * phi, &sp, &cp);
  if constexpr (Q < C::RB) {
#pragma unroll
    for (int r = 0; r < C::R; ++r) {
      if ((r >> Q) & 1) continue;
      const int r1 = r | (1 << Q);
      const cf a0 = a[r], a1 = a[r1];
      const cf t0 = {c * a0.x - s * a1.x, c * a0.y - s * a1.y};
      const cf t1 = {s * a0.x + c * a1.x, s * a0.y + c * a1.y};
      a[r] = cmul(t0, cf{cp, -sp});
      a[r1] = cmul(t1, cf{cp, sp});
    }
  } else {
    constexpr int M = 1 << (Q - C::RB);
    const float sg = ((li >> (Q - C::RB)) & 1) ? 1.f : -1.f;
    const cf ph = {cp, sg * sp};
#pragma unroll
    for (int r = 0; r < C::R; ++r) {
      const cf b = {__shfl_xor(a[r].x, M), __shfl_xor(a[r].y, M)};
      const cf t = {c * a[r].x + sg * s * b.x, c * a[r].y + sg * s * b.y};
      a[r] = cmul(ph, t);
    }
  }
}

// Forward pass up to (not including) the measurement; leaves psi_final in `a`.
template <int N>
__device__ __forceinline__ void run_circuit(cf (&a)[Cfg<N>::R], const float* xs, const float* w, int L,
                                            cf* lds, int sbase, int li) {
  product_state<N>(a, xs, w, li);
  ring_permute<N, false>(a, lds, sbase, li);
  for (int l = 1; l < L; ++l) {
    const float* wl = w + 2 * N * l;
    static_for<0, N>([&](auto qc) {
      constexpr int Q = decltype(qc)::value;
      apply_rot<N, Q>(a, wl[2 * Q], wl[2 * Q + 1], li);
    });
    ring_permute<N, false>(a, lds, sbase, li);
  }
}

// Sum over the lanes of one sample (xor butterfly over the LB lane bits).
template <int N>
__device__ __forceinline__ float sample_sum(float v) {
#pragma unroll
  for (int m = 1; m < Cfg<N>::LPS; m <<= 1) v += __shfl_xor(v, m);
  return v;
}

template <int N>
// psave (nullable): every sample's final state, [sample][r][lane-in-sample] (coalesced), for the
// backward to start from instead of re-running the circuit
__global__ void __launch_bounds__(64) qsim_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                      float* __restrict__ E, int B, int L, int wgroup,
                                                      cf* __restrict__ psave) {
  using C = Cfg<N>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  cf* lds = reinterpret_cast<cf*>(smem);
  const int lane = threadIdx.x;
  const int sw = lane >> C::LB;             // sample within wave
  const int li = lane & (C::LPS - 1);       // lane within sample
  const int sbase = sw * C::D;
  for (int base = blockIdx.x * C::SPW; base < B; base += gridDim.x * C::SPW) {
    const int smp = base + sw;
    const int sld = smp < B ? smp : B - 1;
    float xs[N];
#pragma unroll
    for (int q = 0; q < N; ++q) xs[q] = x[sld * N + q];
    const float* ws = w + (wgroup > 0 ? (size_t)(sld / wgroup) * 2 * N * L : 0);
    cf a[C::R];
    run_circuit<N>(a, xs, ws, L, lds, sbase, li);
    if (psave != nullptr && smp < B) {
#pragma unroll
      for (int r = 0; r < C::R; ++r) psave[(size_t)smp * C::D + r * C::LPS + li] = a[r];
    }
    float p[C::R], ptot = 0.f;
#pragma unroll
    for (int r = 0; r < C::R; ++r) {
      p[r] = a[r].x * a[r].x + a[r].y * a[r].y;
      ptot += p[r];
    }
#pragma unroll
    for (int q = 0; q < N; ++q) {
      float v;
      if (q < C::RB) {
        v = 0.f;
#pragma unroll
        for (int r = 0; r < C::R; ++r) v += ((r >> q) & 1) ? -p[r] : p[r];
      } else {
        v = ((li >> (q - C::RB)) & 1) ? -ptot : ptot;
      }
      v = sample_sum<N>(v);
      if (li == 0 && smp < B) E[smp * N + q] = v;
    }
  }
}

// Adjoint backward. gE: dL/dE (B,N).  dx: (B,N).  slab: (gridDim.x, L*N*2) partial dW.
template <int N>
__global__ void __launch_bounds__(64) qsim_bwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                      const float* __restrict__ gE, float* __restrict__ dx,
                                                      float* __restrict__ slab, int B, int L, int wgroup,
                                                      const cf* __restrict__ psave) {
  using C = Cfg<N>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  cf* lds = reinterpret_cast<cf*>(smem);
  float* acc = reinterpret_cast<float*>(smem + sizeof(cf) * C::SLOTS);  // [P][64] per-lane partials
  const int P = 2 * N * L;
  const int lane = threadIdx.x;
  const int sw = lane >> C::LB;
  const int li = lane & (C::LPS - 1);
  const int sbase = sw * C::D;
  for (int p = 0; p < P; ++p) acc[p * kWave + lane] = 0.f;

  for (int base = blockIdx.x * C::SPW; base < B; base += gridDim.x * C::SPW) {
    const int smp = base + sw;
    const bool valid = smp < B;
    const int sld = valid ? smp : B - 1;
    float xs[N], g[N];
#pragma unroll
    for (int q = 0; q < N; ++q) {
      xs[q] = x[sld * N + q];
      g[q] = valid ? gE[sld * N + q] : 0.f;  // padded samples contribute nothing
    }
    const float* ws = w + (wgroup > 0 ? (size_t)(sld / wgroup) * 2 * N * L : 0);
    cf psi[C::R], lam[C::R];
    if (psave != nullptr) {   // the forward's final state (same x, w): no recompute
#pragma unroll
      for (int r = 0; r < C::R; ++r) psi[r] = psave[(size_t)sld * C::D + r * C::LPS + li];
    } else {
      run_circuit<N>(psi, xs, ws, L, lds, sbase, li);
    }
    // lambda = (sum_q g_q Z_q) psi
#pragma unroll
    for (int r = 0; r < C::R; ++r) {
      const int k = r | (li << C::RB);
      float o = 0.f;
#pragma unroll
      for (int q = 0; q < N; ++q) o += ((k >> q) & 1) ? -g[q] : g[q];
      lam[r] = cscale(psi[r], o);
    }
    float dxp[N];
    for (int l = L - 1; l >= 0; --l) {
      ring_permute<N, true>(psi, lds, sbase, li);
      ring_permute<N, true>(lam, lds, sbase, li);
      const float* wl = ws + 2 * N * l;
      float* accl = acc + 2 * N * l * kWave;
      static_for<0, N>([&](auto qc) {
        constexpr int Q = N - 1 - decltype(qc)::value;  // reverse wire order
        const float theta = wl[2 * Q] + (l == 0 ? xs[Q] : 0.f);
        const float phi = wl[2 * Q + 1];
        float s, c, sp, cp;
        __sincosf(0.5f * theta, &s, &c);
        __sincosf(0.5f * phi, &sp, &cp);
        float dphi = 0.f, dth = 0.f;
        if constexpr (Q < C::RB) {
#pragma unroll
          for (int r = 0; r < C::R; ++r) {
            if ((r >> Q) & 1) continue;
            const int r1 = r | (1 << Q);
            // RZ^dagger: dphi = Im <lam| Z |psi>; bit0 *= e^{+i phi/2}, bit1 *= e^{-i phi/2}
            dphi += (lam[r].x * psi[r].y - lam[r].y * psi[r].x) - (lam[r1].x * psi[r1].y - lam[r1].y * psi[r1].x);
            psi[r] = cmul(psi[r], cf{cp, sp});
            lam[r] = cmul(lam[r], cf{cp, sp});
            psi[r1] = cmul(psi[r1], cf{cp, -sp});
            lam[r1] = cmul(lam[r1], cf{cp, -sp});
            // RY^dagger: dtheta = Im <lam| Y |psi> = sum_k sg_k Re(conj(lam_k) psi_partner)
            dth += -(lam[r].x * psi[r1].x + lam[r].y * psi[r1].y) + (lam[r1].x * psi[r].x + lam[r1].y * psi[r].y);
            const cf p0 = psi[r], p1 = psi[r1], l0 = lam[r], l1 = lam[r1];
            psi[r] = {c * p0.x + s * p1.x, c * p0.y + s * p1.y};
            psi[r1] = {c * p1.x - s * p0.x, c * p1.y - s * p0.y};
            lam[r] = {c * l0.x + s * l1.x, c * l0.y + s * l1.y};
            lam[r1] = {c * l1.x - s * l0.x, c * l1.y - s * l0.y};
          }
        } else {
          constexpr int M = 1 << (Q - C::RB);
          const float sg = ((li >> (Q - C::RB)) & 1) ? 1.f : -1.f;
          const cf ph = {cp, -sg * sp};  // conj of the forward phase
#pragma unroll
          for (int r = 0; r < C::R; ++r) {
            dphi += -sg * (lam[r].x * psi[r].y - lam[r].y * psi[r].x);
            psi[r] = cmul(psi[r], ph);
            lam[r] = cmul(lam[r], ph);
            const cf bp = {__shfl_xor(psi[r].x, M), __shfl_xor(psi[r].y, M)};
            const cf bl = {__shfl_xor(lam[r].x, M), __shfl_xor(lam[r].y, M)};
            dth += sg * (lam[r].x * bp.x + lam[r].y * bp.y);
            psi[r] = {c * psi[r].x - sg * s * bp.x, c * psi[r].y - sg * s * bp.y};
            lam[r] = {c * lam[r].x - sg * s * bl.x, c * lam[r].y - sg * s * bl.y};
          }
        }
        accl[(2 * Q) * kWave + lane] += dth;
        accl[(2 * Q + 1) * kWave + lane] += dphi;
        dxp[Q] = dth;
      });
    }
    // dx = dtheta of layer 0 (theta = x + w[0,:,0]); full per-sample reduction.
#pragma unroll
    for (int q = 0; q < N; ++q) {
      const float v = sample_sum<N>(dxp[q]);
      if (li == 0 && valid) dx[smp * N + q] = v;
    }
  }
  wave_lds_fence();
  // Reduce per-lane partials -> one slab row for this wave.
  for (int p = lane; p < P; p += kWave) {
    float t = 0.f;
    for (int j = 0; j < kWave; ++j) t += acc[p * kWave + j];
    slab[(size_t)blockIdx.x * P + p] = t;
  }
}

// dW[p] = beta * dW[p] + sum_rows slab[row][p]   (deterministic order)
__global__ void __launch_bounds__(256) reduce_slab_kernel(const float* __restrict__ slab, float* __restrict__ out,
                                                          int rows, int P, float beta) {
  __shared__ float red[4];
  const int p = blockIdx.x;
  float t = 0.f;
  for (int r = threadIdx.x; r < rows; r += 256) t += slab[(size_t)r * P + p];
  t = block_sum<256>(t, red);
  if (threadIdx.x == 0) out[p] = (beta == 0.f ? 0.f : beta * out[p]) + t;
}

template <int N>
static int launch_fwd(const float* x, const float* w, float* E, int B, int L, int wgroup, int grid, hipStream_t st,
                      cf* psave = nullptr) {
  using C = Cfg<N>;
  const int need = (B + C::SPW - 1) / C::SPW;
  if (grid <= 0 || grid > need) grid = need;
  const size_t sm = sizeof(cf) * C::SLOTS;
  hipLaunchKernelGGL(qsim_fwd_kernel<N>, dim3(grid), dim3(64), sm, st, x, w, E, B, L, wgroup, psave);
  return (int)hipGetLastError();
}

template <int N>
static int launch_bwd(const float* x, const float* w, const float* gE, float* dx, float* slab, int B, int L,
                      int wgroup, int grid, hipStream_t st, const cf* psave = nullptr) {
  using C = Cfg<N>;
  const size_t sm = sizeof(cf) * C::SLOTS + sizeof(float) * 2 * N * L * kWave;
  if (sm > 160 * 1024) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(qsim_bwd_kernel<N>, dim3(grid), dim3(64), sm, st, x, w, gE, dx, slab, B, L, wgroup, psave);
  return (int)hipGetLastError();
}

}  // namespace qsim
}  // namespace qd

using namespace qd::qsim;

#define QD_DISPATCH_N(n, CALL)      \
  switch (n) {                      \
    case 2: return CALL(2);         \
    case 3: return CALL(3);         \
    case 4: return CALL(4);         \
    case 5: return CALL(5);         \
    case 6: return CALL(6);         \
    case 7: return CALL(7);         \
    case 8: return CALL(8);         \
    case 9: return CALL(9);         \
    case 10: return CALL(10);       \
    default: return (int)hipErrorInvalidValue; \
  }

QD_API int qd_qsim_max_qubits() { return 10; }

// Number of slab rows (= waves launched) the backward will use for a batch of B.
QD_API int qd_qsim_bwd_grid(int n, int B) {
  if (n < 2 || n > 10) return -1;
  const int spw = n >= 6 ? 1 : (64 >> n);
  int need = (B + spw - 1) / spw;
  return need < 4096 ? need : 4096;
}

// wgroup > 0: sample b uses weights w[b / wgroup] (per-stream QuantumNAT noise); 0: shared.
QD_API int qd_qsim_fwd(const float* x, const float* w, float* E, int B, int n, int L, int wgroup, void* stream) {
  if (wgroup > 0 && B % wgroup != 0) return (int)hipErrorInvalidValue;   // (G = B / wgroup weight groups, workspace)
  hipStream_t st = (hipStream_t)stream;
#define CALL_F(NN) launch_fwd<NN>(x, w, E, B, L, wgroup, 0, st)
  QD_DISPATCH_N(n, CALL_F)
#undef CALL_F
}

QD_API int qd_qsim_bwd(const float* x, const float* w, const float* gE, float* dx, float* slab, int B, int n, int L,
                       int wgroup, void* stream) {
  if (wgroup > 0 && B % wgroup != 0) return (int)hipErrorInvalidValue;   // (G = B / wgroup weight groups, workspace)
  hipStream_t st = (hipStream_t)stream;
  const int grid = qd_qsim_bwd_grid(n, B);
#define CALL_B(NN) launch_bwd<NN>(x, w, gE, dx, slab, B, L, wgroup, grid, st)
  QD_DISPATCH_N(n, CALL_B)
#undef CALL_B
}

// As qd_qsim_fwd / qd_qsim_bwd, with psave = (B, 2^n) complex64 scratch: the forward keeps each
// sample's final state there and the backward starts from it (no circuit recompute).
QD_API int qd_qsim_fwd_save(const float* x, const float* w, float* E, int B, int n, int L, int wgroup, void* psave,
                            void* stream) {
  if (wgroup > 0 && B % wgroup != 0) return (int)hipErrorInvalidValue;   // (G = B / wgroup weight groups, workspace)
  hipStream_t st = (hipStream_t)stream;
#define CALL_F(NN) launch_fwd<NN>(x, w, E, B, L, wgroup, 0, st, (cf*)psave)
  QD_DISPATCH_N(n, CALL_F)
#undef CALL_F
}

QD_API int qd_qsim_bwd_saved(const float* x, const float* w, const float* gE, float* dx, float* slab, int B, int n,
                             int L, int wgroup, const void* psave, void* stream) {
  if (wgroup > 0 && B % wgroup != 0) return (int)hipErrorInvalidValue;   // (G = B / wgroup weight groups, workspace)
  hipStream_t st = (hipStream_t)stream;
  const int grid = qd_qsim_bwd_grid(n, B);
#define CALL_B(NN) launch_bwd<NN>(x, w, gE, dx, slab, B, L, wgroup, grid, st, (const cf*)psave)
  QD_DISPATCH_N(n, CALL_B)
#undef CALL_B
}

QD_API int qd_reduce_slab(const float* slab, float* out, int rows, int P, float beta, void* stream) {
  hipLaunchKernelGGL(reduce_slab_kernel, dim3(P), dim3(256), 0, (hipStream_t)stream, slab, out, rows, P, beta);
  return (int)hipGetLastError();
}
