// Batched VQC simulator for LARGE qubit counts (n = 11 .. 16): one 256-thread workgroup per sample,
// gate-fused passes.
//
// Same circuit and adjoint method as csrc/hip/qsim.hip (reference E:125-142: RY embedding, L x
// [RY, RZ on every wire, CNOT ring], <Z_i>); that kernel keeps a sample's state in one wave's
// registers, which stops at n = 10.  Here the state (2^n complex fp32: 16 KiB .. 512 KiB) lives in
// LDS when it fits (n <= 12) or in a per-workgroup HBM workspace, and a layer is TWO passes over it
// instead of one pass per gate:
//   low pass   qubits 0 .. TB-1 (TB = min(n, 12)).  The state is cut into 2^(n-TB) tiles of 2^TB
//              contiguous amplitudes (32 KiB); a tile is staged in LDS and the TB rotations are
//              applied three qubits at a time in registers (each thread owns the 8 amplitudes that
//              differ in those 3 bits): 4 LDS round trips per tile, not TB.
//   high pass  qubits TB .. n-1 (HB = n - TB <= 4).  A thread owns a "column" of 2^HB amplitudes
//              (same low bits), applies the HB rotations in registers and stores every amplitude at
//              its CNOT-ring image f(k): the ring permutation costs nothing extra.
// Layer 0 (embedding + first rotations) is a product state written directly at its ring images.
// Forward traffic per layer: ~2 reads + 2 writes of the state (the per-gate version made 17 of
// each at 16 qubits).  Backward (adjoint): recompute psi, then per layer in reverse: the high pass
// gathers psi and lambda from f(k) (inverse ring) and undoes the high rotations, the low pass
// undoes the low ones; lambda = (sum_q g_q Z_q) psi is formed on the fly in the first reverse pass.
// Per-gate gradient partials stay in registers across tiles and are block-reduced once per pass.
#include "common.h"

namespace qd {
namespace qsimbig {

struct cf {
  float x, y;
};
__device__ __forceinline__ cf cmul(cf a, cf b) { return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }

constexpr int NT = 256;   // 4 waves: lets the backward use AGPRs instead of scratch (512-thread groups spilled)
// waves per SIMD the register allocation must allow (launch-bounds hint; the n <= 12 LDS state fits 4 forward /
// 2 backward workgroups per CU)
#ifndef QD_BIG_FWD_WAVES
#define QD_BIG_FWD_WAVES 4
#endif
#ifndef QD_BIG_BWD_WAVES
#define QD_BIG_BWD_WAVES 2
#endif
constexpr int NW = NT / 64;

template <int N>
struct G {
  static constexpr int D = 1 << N;
  static constexpr int TB = N < 12 ? N : 12;   // low (tile) qubits
  static constexpr int HB = N - TB;            // high (column) qubits
  static constexpr int T = 1 << TB;            // tile size (amplitudes)
  static constexpr int NTILE = 1 << HB;
  static constexpr int NGRP = (TB + 2) / 3;    // 3-qubit groups of the low pass
  static constexpr bool LDS_STATE = N <= 12;
};

// LDS carve (bytes): reduction scratch | trig (<= 16 float4) | gE (16) | acc (2nL <= 256) + per-sample
// layer-0 scratch (2n <= 32) | phase table PI (n <= 12: <= 16 complex) | data (tiles, or the whole state
// when n <= 12).
constexpr int O_RED = 0, O_TRIG = 2048, O_G = 2304, O_ACC = 2368, O_TMP = 3392, O_PHI = 3584, O_DATA = 3712;

template <int N>
__device__ __forceinline__ int ring_fwd(int k) {
#pragma unroll
  for (int i = 0; i < N - 1; ++i) k ^= ((k >> i) & 1) << (i + 1);
  k ^= (k >> (N - 1)) & 1;
  return k;
}
template <int N>
__device__ __forceinline__ int ring_inv(int k) {
  k ^= (k >> (N - 1)) & 1;
#pragma unroll
  for (int i = N - 2; i >= 0; --i) k ^= ((k >> i) & 1) << (i + 1);
  return k;
}

// insert NB zero bits at position P into t
template <int P, int NB>
__device__ __forceinline__ int ins_bits(int t) {
  return ((t >> P) << (P + NB)) | (t & ((1 << P) - 1));
}

// Per-qubit trig of one layer, (cos, sin) of theta/2 and (cos, sin) of phi/2, into LDS.
__device__ __forceinline__ void layer_trig(float4* trig, const float* wl, const float* xs, int n) {
  if (threadIdx.x < n) {
    const int q = threadIdx.x;
    float s, c, sp, cp;
    __sincosf(0.5f * (wl[2 * q] + (xs ? xs[q] : 0.f)), &s, &c);
    __sincosf(0.5f * wl[2 * q + 1], &sp, &cp);
    trig[q] = make_float4(c, s, cp, sp);
  }
}

// forward gate RZ(phi) RY(theta) on the pair (a0: bit 0, a1: bit 1)
__device__ __forceinline__ void gate_fwd(cf& a0, cf& a1, float4 t) {
  const cf t0 = {t.x * a0.x - t.y * a1.x, t.x * a0.y - t.y * a1.y};
  const cf t1 = {t.y * a0.x + t.x * a1.x, t.y * a0.y + t.x * a1.y};
  a0 = cmul(t0, cf{t.z, -t.w});
  a1 = cmul(t1, cf{t.z, t.w});
}

// adjoint step: given psi, lambda AFTER the gate, accumulate d(theta), d(phi) and undo the gate
__device__ __forceinline__ void gate_adj(cf& p0, cf& p1, cf& l0, cf& l1, float4 t, float& dth, float& dph) {
  dph += (l0.x * p0.y - l0.y * p0.x) - (l1.x * p1.y - l1.y * p1.x);   // Im <lam| Z |psi>
  p0 = cmul(p0, cf{t.z, t.w});
  l0 = cmul(l0, cf{t.z, t.w});
  p1 = cmul(p1, cf{t.z, -t.w});
  l1 = cmul(l1, cf{t.z, -t.w});
  dth += -(l0.x * p1.x + l0.y * p1.y) + (l1.x * p0.x + l1.y * p0.y); // Im <lam| Y |psi>
  const cf q0 = p0, q1 = p1, m0 = l0, m1 = l1;
  p0 = {t.x * q0.x + t.y * q1.x, t.x * q0.y + t.y * q1.y};
  p1 = {t.x * q1.x - t.y * q0.x, t.x * q1.y - t.y * q0.y};
  l0 = {t.x * m0.x + t.y * m1.x, t.x * m0.y + t.y * m1.y};
  l1 = {t.x * m1.x - t.y * m0.x, t.x * m1.y - t.y * m0.y};
}

// Block-reduce NV per-thread values; dst[off + i] += sum_i (thread i < NV).  red: NW*NV floats.
template <int NV>
__device__ __forceinline__ void block_add(const float (&v)[NV], float* red, float* dst, int off) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const float s = wave_sum(v[i]);
    if (lane == 0) red[w * NV + i] = s;
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NW; ++k) s += red[k * NV + threadIdx.x];
    dst[off + threadIdx.x] += s;
  }
  __syncthreads();
}

// ------------------------------------------------------------------------------- forward passes
// Layer 0 + ring: A[j] = prod_q c_q(bit_q(f^-1(j))), c(0) = cos(t/2)e^{-ip/2}, c(1) = sin(t/2)e^{ip/2}
template <int N>
__device__ void product_pass(cf* A, const float4* trig) {
  for (int j = threadIdx.x; j < G<N>::D; j += NT) {
    const int k = ring_inv<N>(j);
    cf a = {1.f, 0.f};
#pragma unroll
    for (int q = 0; q < N; ++q) {
      const float4 t = trig[q];
      a = cmul(a, ((k >> q) & 1) ? cf{t.y * t.z, t.y * t.w} : cf{t.x * t.z, -t.x * t.w});
    }
    A[j] = a;
  }
  __syncthreads();
}

// Low pass (forward): rotations on qubits 0..TB-1 of every tile of A (in place).
template <int N>
__device__ void low_pass_fwd(cf* A, cf* tile, const float4* trig) {
  using C = G<N>;
  for (int h = 0; h < C::NTILE; ++h) {
    cf* tl = C::LDS_STATE ? A : tile;
    if constexpr (!C::LDS_STATE) {
      const cf* src = A + (size_t)h * C::T;
      for (int i = threadIdx.x; i < C::T; i += NT) tl[i] = src[i];
      __syncthreads();
    }
    static_for<0, C::NGRP>([&](auto gc) {
      constexpr int g0 = 3 * decltype(gc)::value;
      constexpr int NB = (C::TB - g0) < 3 ? (C::TB - g0) : 3;
      constexpr int ACT = C::T >> NB;
      for (int t = threadIdx.x; t < ACT; t += NT) {
        const int base = ins_bits<g0, NB>(t);
        cf a[1 << NB];
#pragma unroll
        for (int j = 0; j < (1 << NB); ++j) a[j] = tl[base | (j << g0)];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          const float4 tg = trig[g0 + b];
#pragma unroll
          for (int j = 0; j < (1 << NB); ++j)
            if (!((j >> b) & 1)) gate_fwd(a[j], a[j | (1 << b)], tg);
        }
#pragma unroll
        for (int j = 0; j < (1 << NB); ++j) tl[base | (j << g0)] = a[j];
      }
      __syncthreads();
    });
    if constexpr (!C::LDS_STATE) {
      cf* dst = A + (size_t)h * C::T;
      for (int i = threadIdx.x; i < C::T; i += NT) dst[i] = tl[i];
      __syncthreads();
    }
  }
}

// High pass (forward): rotations on qubits TB..N-1 column-wise, stored at ring images: B[f(k)].
template <int N>
__device__ void high_pass_fwd(const cf* A, cf* B, const float4* trig) {
  using C = G<N>;
  for (int c = threadIdx.x; c < C::T; c += NT) {
    cf a[C::NTILE];
#pragma unroll
    for (int h = 0; h < C::NTILE; ++h) a[h] = A[c | (h << C::TB)];
#pragma unroll
    for (int b = 0; b < C::HB; ++b) {
      const float4 tg = trig[C::TB + b];
#pragma unroll
      for (int h = 0; h < C::NTILE; ++h)
        if (!((h >> b) & 1)) gate_fwd(a[h], a[h | (1 << b)], tg);
    }
#pragma unroll
    for (int h = 0; h < C::NTILE; ++h) B[ring_fwd<N>(c | (h << C::TB))] = a[h];
  }
  __syncthreads();
}

// LDS-resident states with no high qubits (n <= 12): the high pass is the bare CNOT-ring permutation,
// done IN PLACE through registers (every thread holds its D / NT amplitudes across one barrier), so the
// forward needs one state buffer instead of two and the adjoint two instead of four -- 2x / 4x fewer
// bytes of LDS per workgroup, hence 2x the resident workgroups per CU (round 3).
template <int N>
__device__ void ring_fwd_inplace(cf* A) {
  constexpr int PER = G<N>::D / NT;
  cf a[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) a[i] = A[threadIdx.x + i * NT];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < PER; ++i) A[ring_fwd<N>(threadIdx.x + i * NT)] = a[i];
  __syncthreads();
}

// ---- n <= 12 (LDS-resident, no high qubits): the diagonal-RZ formulation (round 3) -------------------------
// The 2n gates of a layer act on n DIFFERENT wires, so they commute: layer = D . Y with Y = prod_q RY_q (real
// 2x2 rotations of amplitude pairs) and D = prod_q RZ_q = diag_k prod_q e^{+-i phi_q / 2} (+ for bit_q(k) = 1).
// The forward applies Y in the 3-qubit register groups WITHOUT phases and D once per amplitude, inside the
// in-place ring pass -- where thread t holds amplitudes c = t + i * NT (bits 0..7 = t, bits 8.. = i), so
// D(c) = PT(t) * PI(i): one per-thread factor and a PER-entry table.  The adjoint takes every phi_q gradient
// Im<lam|Z_q|psi> at ONE point (after the layer, before the ring: Z_q commutes with the layer's other gates),
// undoes D on psi and lambda there, then every theta_q gradient Im<lam|Y_q|psi> inside the RY-only reverse
// groups (Y_q commutes with every RY of the layer).  Per amplitude and layer: ~60 (forward) and ~140
// (adjoint) vector operations instead of ~110 and ~250 with per-gate RZ phases.

__device__ __forceinline__ cf rz_factor(float4 t, bool one) { return one ? cf{t.z, t.w} : cf{t.z, -t.w}; }

// PI(i) = prod over the qubits 8.. of rz_factor(bit of i) for i < PER (threads < PER; trig must be visible)
template <int N>
__device__ __forceinline__ void phase_table(cf* phi, const float4* trig) {
  constexpr int PER = G<N>::D / NT;
  if (threadIdx.x < PER) {
    cf p = {1.f, 0.f};
#pragma unroll
    for (int b = 0; 8 + b < N; ++b) p = cmul(p, rz_factor(trig[8 + b], (threadIdx.x >> b) & 1));
    phi[threadIdx.x] = p;
  }
}
// PT(t): this thread's factor over qubits 0..7
__device__ __forceinline__ cf phase_thread(const float4* trig) {
  cf p = {1.f, 0.f};
#pragma unroll
  for (int q = 0; q < 8; ++q) p = cmul(p, rz_factor(trig[q], (threadIdx.x >> q) & 1));
  return p;
}

// forward RY on the pair (bit 0: a0, bit 1: a1)
__device__ __forceinline__ void ry_fwd(cf& a0, cf& a1, float c, float s) {
  const cf t0 = {c * a0.x - s * a1.x, c * a0.y - s * a1.y};
  a1 = {s * a0.x + c * a1.x, s * a0.y + c * a1.y};
  a0 = t0;
}
// adjoint RY step: theta gradient Im<lam|Y|psi> of the pair, then RY^-1 on psi and lambda
__device__ __forceinline__ void ry_adj(cf& p0, cf& p1, cf& l0, cf& l1, float c, float s, float& dth) {
  dth += -(l0.x * p1.x + l0.y * p1.y) + (l1.x * p0.x + l1.y * p0.y);
  const cf q0 = p0, m0 = l0;
  p0 = {c * q0.x + s * p1.x, c * q0.y + s * p1.y};
  p1 = {c * p1.x - s * q0.x, c * p1.y - s * q0.y};
  l0 = {c * m0.x + s * l1.x, c * m0.y + s * l1.y};
  l1 = {c * l1.x - s * m0.x, c * l1.y - s * m0.y};
}

// RY of every qubit on the LDS state A, three qubits per register round trip (no phases: see above)
template <int N>
__device__ void low_pass_ry(cf* A, const float4* trig) {
  using C = G<N>;
  static_for<0, C::NGRP>([&](auto gc) {
    constexpr int g0 = 3 * decltype(gc)::value;
    constexpr int NB = (C::TB - g0) < 3 ? (C::TB - g0) : 3;
    constexpr int ACT = C::T >> NB;
    float cs[NB], sn[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      cs[b] = trig[g0 + b].x;
      sn[b] = trig[g0 + b].y;
    }
    for (int t = threadIdx.x; t < ACT; t += NT) {
      const int base = ins_bits<g0, NB>(t);
      cf a[1 << NB];
#pragma unroll
      for (int j = 0; j < (1 << NB); ++j) a[j] = A[base | (j << g0)];
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int j = 0; j < (1 << NB); ++j)
          if (!((j >> b) & 1)) ry_fwd(a[j], a[j | (1 << b)], cs[b], sn[b]);
#pragma unroll
      for (int j = 0; j < (1 << NB); ++j) A[base | (j << g0)] = a[j];
    }
    __syncthreads();
  });
}

// D (the layer's RZ phases), then the CNOT ring, in place: A'[f(c)] = D(c) A[c]
template <int N>
__device__ void ring_phase_fwd(cf* A, const float4* trig, const cf* phi) {
  constexpr int PER = G<N>::D / NT;
  const cf pt = phase_thread(trig);
  cf a[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) a[i] = cmul(A[threadIdx.x + i * NT], cmul(pt, phi[i]));
  __syncthreads();
#pragma unroll
  for (int i = 0; i < PER; ++i) A[ring_fwd<N>(threadIdx.x + i * NT)] = a[i];
  __syncthreads();
}

// Low pass of layer 1 with the layer-0 product state GENERATED per tile (HBM-state builds): the
// product amplitudes are never written to and re-read from HBM.  trig0: layer-0 (embedding) trig.
template <int N>
__device__ void low_pass_fwd_gen(cf* A, cf* tile, const float4* trig, const float4* trig0) {
  using C = G<N>;
  static_assert(!C::LDS_STATE, "HBM-state builds");
  for (int h = 0; h < C::NTILE; ++h) {
    for (int i = threadIdx.x; i < C::T; i += NT) {
      const int k = ring_inv<N>(i | (h << C::TB));
      cf a = {1.f, 0.f};
#pragma unroll
      for (int q = 0; q < N; ++q) {
        const float4 t = trig0[q];
        a = cmul(a, ((k >> q) & 1) ? cf{t.y * t.z, t.y * t.w} : cf{t.x * t.z, -t.x * t.w});
      }
      tile[i] = a;
    }
    __syncthreads();
    static_for<0, C::NGRP>([&](auto gc) {
      constexpr int g0 = 3 * decltype(gc)::value;
      constexpr int NB = (C::TB - g0) < 3 ? (C::TB - g0) : 3;
      constexpr int ACT = C::T >> NB;
      for (int t = threadIdx.x; t < ACT; t += NT) {
        const int base = ins_bits<g0, NB>(t);
        cf a[1 << NB];
#pragma unroll
        for (int j = 0; j < (1 << NB); ++j) a[j] = tile[base | (j << g0)];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          const float4 tg = trig[g0 + b];
#pragma unroll
          for (int j = 0; j < (1 << NB); ++j)
            if (!((j >> b) & 1)) gate_fwd(a[j], a[j | (1 << b)], tg);
        }
#pragma unroll
        for (int j = 0; j < (1 << NB); ++j) tile[base | (j << g0)] = a[j];
      }
      __syncthreads();
    });
    cf* dst = A + (size_t)h * C::T;
    for (int i = threadIdx.x; i < C::T; i += NT) dst[i] = tile[i];
    __syncthreads();
  }
}

// Last high pass with the <Z_q> reduction fused in: part[q] accumulates sum |psi_k|^2 (+-1) at
// the ring images k; the state is stored (for the backward) only when B != null.
template <int N>
__device__ void high_pass_fwd_expect(const cf* A, cf* B, const float4* trig, float (&part)[N]) {
  using C = G<N>;
  for (int c = threadIdx.x; c < C::T; c += NT) {
    cf a[C::NTILE];
#pragma unroll
    for (int h = 0; h < C::NTILE; ++h) a[h] = A[c | (h << C::TB)];
#pragma unroll
    for (int b = 0; b < C::HB; ++b) {
      const float4 tg = trig[C::TB + b];
#pragma unroll
      for (int h = 0; h < C::NTILE; ++h)
        if (!((h >> b) & 1)) gate_fwd(a[h], a[h | (1 << b)], tg);
    }
#pragma unroll
    for (int h = 0; h < C::NTILE; ++h) {
      const int k = ring_fwd<N>(c | (h << C::TB));
      if (B != nullptr) B[k] = a[h];
      const float p = a[h].x * a[h].x + a[h].y * a[h].y;
#pragma unroll
      for (int q = 0; q < N; ++q) part[q] += ((k >> q) & 1) ? -p : p;
    }
  }
  __syncthreads();
}

// Full forward circuit of one sample; returns the buffer holding psi_final (A or B).
// final_out (HBM-state builds, L > 1): the last high pass stores psi_final there instead of B.
template <int N>
__device__ cf* run_circuit(cf* A, cf* B, cf* tile, float4* trig, const float* xs, const float* w, int L,
                           cf* final_out = nullptr) {
  layer_trig(trig, w, xs, N);
  __syncthreads();
  product_pass<N>(A, trig);
  if constexpr (G<N>::HB == 0 && G<N>::LDS_STATE) {   // (one buffer, diagonal RZ: see low_pass_ry)
    cf* phi = reinterpret_cast<cf*>(reinterpret_cast<char*>(trig) - O_TRIG + O_PHI);
    for (int l = 1; l < L; ++l) {
      layer_trig(trig, w + 2 * N * l, nullptr, N);
      __syncthreads();
      phase_table<N>(phi, trig);
      low_pass_ry<N>(A, trig);   // (its barriers publish phi)
      ring_phase_fwd<N>(A, trig, phi);
    }
    return A;
  }
  for (int l = 1; l < L; ++l) {
    layer_trig(trig, w + 2 * N * l, nullptr, N);
    __syncthreads();
    low_pass_fwd<N>(A, tile, trig);
    cf* dst = (final_out != nullptr && l == L - 1) ? final_out : B;
    high_pass_fwd<N>(A, dst, trig);
    if (dst == B) {
      cf* t = A;
      A = B;
      B = t;
    } else {
      A = dst;
    }
  }
  return A;
}

// ------------------------------------------------------------------------------- kernels

template <int N>
// psave (nullable): (B, 2^N) per-sample psi_final, kept for the backward (which then skips its
// forward recompute: ~1/3 of its state traffic at n = 16)
__global__ void __launch_bounds__(NT, G<N>::LDS_STATE ? QD_BIG_FWD_WAVES : 1) qsim_big_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                          float* __restrict__ E, int B, int L, int wgroup,
                                                          cf* __restrict__ ws, cf* __restrict__ psave) {
  using C = G<N>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* red = reinterpret_cast<float*>(smem + O_RED);
  float4* trig = reinterpret_cast<float4*>(smem + O_TRIG);
  float* outv = reinterpret_cast<float*>(smem + O_TMP);
  cf* data = reinterpret_cast<cf*>(smem + O_DATA);
  cf *A, *Bf, *tile;
  if constexpr (C::LDS_STATE) {
    A = data;
    Bf = data + C::D;
    tile = nullptr;
  } else {
    A = ws + (size_t)blockIdx.x * 2 * C::D;
    Bf = A + C::D;
    tile = data;
  }
  for (int s = blockIdx.x; s < B; s += gridDim.x) {
    const float* wsmp = w + (wgroup > 0 ? (size_t)(s / wgroup) * 2 * N * L : 0);
    cf* sv = psave ? psave + (size_t)s * C::D : nullptr;
    float part[N];
#pragma unroll
    for (int q = 0; q < N; ++q) part[q] = 0.f;
    if constexpr (!C::LDS_STATE) {
      if (L >= 2) {
        // HBM-resident state: layer 0 generated inside layer 1's low pass, <Z> reduced inside the
        // last high pass -- 3 state reads + 4 writes (3 without psave) instead of 5 + 5
        float4* trig0 = reinterpret_cast<float4*>(smem + O_ACC);
        layer_trig(trig0, wsmp, x + (size_t)s * N, N);
        cf* Acur = A;
        cf* Bcur = Bf;
        for (int l = 1; l < L; ++l) {
          layer_trig(trig, wsmp + 2 * N * l, nullptr, N);
          __syncthreads();
          if (l == 1) low_pass_fwd_gen<N>(Acur, tile, trig, trig0);
          else low_pass_fwd<N>(Acur, tile, trig);
          if (l == L - 1) {
            high_pass_fwd_expect<N>(Acur, sv, trig, part);
          } else {
            high_pass_fwd<N>(Acur, Bcur, trig);
            cf* t = Acur;
            Acur = Bcur;
            Bcur = t;
          }
        }
        goto reduce;
      }
    }
    {
      cf* psi = run_circuit<N>(A, Bf, tile, trig, x + (size_t)s * N, wsmp, L, C::LDS_STATE ? nullptr : sv);
      if (sv != nullptr && psi != sv) {   // (LDS-resident state, or L == 1)
        for (int k = threadIdx.x; k < C::D; k += NT) sv[k] = psi[k];
      }
      for (int k = threadIdx.x; k < C::D; k += NT) {
        const cf a = psi[k];
        const float p = a.x * a.x + a.y * a.y;
#pragma unroll
        for (int q = 0; q < N; ++q) part[q] += ((k >> q) & 1) ? -p : p;
      }
    }
  reduce:
    if (threadIdx.x < N) outv[threadIdx.x] = 0.f;
    __syncthreads();
    block_add<N>(part, red, outv, 0);
    if (threadIdx.x < N) E[(size_t)s * N + threadIdx.x] = outv[threadIdx.x];
    __syncthreads();
  }
}

// slab: (gridDim.x, 2*N*L) partial weight grads (one row per workgroup); dx: (B, N)
// psave (nullable): psi_final of every sample from qsim_big_fwd_kernel (same x, w); the backward
// starts from it instead of re-running the circuit (the buffer is consumed: it may be overwritten)
template <int N>
__global__ void __launch_bounds__(NT, G<N>::LDS_STATE ? QD_BIG_BWD_WAVES : 1) qsim_big_bwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                          const float* __restrict__ gE, float* __restrict__ dx,
                                                          float* __restrict__ slab, int B, int L, int wgroup,
                                                          cf* __restrict__ ws, cf* __restrict__ psave) {
  using C = G<N>;
  constexpr int HV = C::HB > 0 ? C::HB : 1;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* red = reinterpret_cast<float*>(smem + O_RED);
  float4* trig = reinterpret_cast<float4*>(smem + O_TRIG);
  float* gq = reinterpret_cast<float*>(smem + O_G);
  float* acc = reinterpret_cast<float*>(smem + O_ACC);
  float* tmp = reinterpret_cast<float*>(smem + O_TMP);
  cf* data = reinterpret_cast<cf*>(smem + O_DATA);
  const int P = 2 * N * L;
  cf *b0, *b1, *b2, *b3, *tp = nullptr, *tq = nullptr;
  if constexpr (C::LDS_STATE && C::HB == 0) {   // in-place ring passes: psi in b0, lambda in b2
    b0 = data;
    b2 = data + C::D;
    b1 = b3 = nullptr;
  } else if constexpr (C::LDS_STATE) {
    b0 = data;
    b1 = data + C::D;
    b2 = data + 2 * C::D;
    b3 = data + 3 * C::D;
  } else {
    b0 = ws + (size_t)blockIdx.x * 4 * C::D;
    b1 = b0 + C::D;
    b2 = b0 + 2 * C::D;
    b3 = b0 + 3 * C::D;
    tp = data;
    tq = data + C::T;
  }
  for (int i = threadIdx.x; i < P; i += NT) acc[i] = 0.f;
  for (int s = blockIdx.x; s < B; s += gridDim.x) {
    const float* wsmp = w + (wgroup > 0 ? (size_t)(s / wgroup) * 2 * N * L : 0);
    const float* xs = x + (size_t)s * N;
    if (threadIdx.x < N) gq[threadIdx.x] = gE[(size_t)s * N + threadIdx.x];
    if (threadIdx.x < 2 * N) tmp[threadIdx.x] = 0.f;
    cf* psi;
    cf* psi_o;
    if (psave != nullptr) {
      cf* sv = psave + (size_t)s * C::D;
      if constexpr (C::LDS_STATE) {
        for (int k = threadIdx.x; k < C::D; k += NT) b0[k] = sv[k];
        psi = b0;
        psi_o = b1;
      } else {
        psi = sv;       // read in place; the first reverse pass writes b1 and the ping-pong
        psi_o = b1;     // continues over (sv, b1) -- the saved state is consumed
      }
      __syncthreads();  // (publishes gq / tmp, as run_circuit's barriers do)
    } else {
      psi = run_circuit<N>(b0, b1, tp, trig, xs, wsmp, L);   // its barriers publish gq / tmp
      psi_o = (psi == b0) ? b1 : b0;
    }
    cf* lam = b2;
    cf* lam_o = b3;
    for (int l = L - 1; l >= 0; --l) {
      layer_trig(trig, wsmp + 2 * N * l, l == 0 ? xs : nullptr, N);
      __syncthreads();
      // layer-0 gradients go to the per-sample scratch first (their theta part is also dx)
      float* gdst = (l == 0) ? tmp : acc + 2 * N * l;
      const bool first = (l == L - 1);   // lambda = O psi formed on the fly
      constexpr bool DIAG = C::HB == 0 && C::LDS_STATE;   // (the diagonal-RZ adjoint: phi gradients in dph_l)
      float dph_l[N];
#pragma unroll
      for (int q = 0; q < N; ++q) dph_l[q] = 0.f;
      // ---- high pass (reverse): gather psi/lam at f(k) (inverse ring), undo high rotations
      if constexpr (C::HB == 0 && C::LDS_STATE) {
        // diagonal-RZ adjoint (see low_pass_ry): gather psi / lam at the ring images (the point after the
        // layer), every phi gradient there, undo D on both, store in place; then the RY-only reverse groups
        constexpr int PER = C::D / NT;
        cf* phi = reinterpret_cast<cf*>(smem + O_PHI);
        phase_table<N>(phi, trig);
        __syncthreads();
        const cf pt = phase_thread(trig);
        cf p[PER], m[PER];
        float wsum = 0.f, whi[N > 8 ? N - 8 : 1];
#pragma unroll
        for (int b = 0; 8 + b < N; ++b) whi[b] = 0.f;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
          const int src = ring_fwd<N>(threadIdx.x + i * NT);
          p[i] = psi[src];
          if (first) {
            float o = 0.f;
#pragma unroll
            for (int q = 0; q < N; ++q) o += ((src >> q) & 1) ? -gq[q] : gq[q];
            m[i] = {p[i].x * o, p[i].y * o};
          } else {
            m[i] = lam[src];
          }
          // Im<lam|Z_q|psi> summand (sign + for bit_q = 0): qubits 0..7 are this thread's fixed bits
          const float wv = m[i].x * p[i].y - m[i].y * p[i].x;
          wsum += wv;
#pragma unroll
          for (int b = 0; 8 + b < N; ++b) whi[b] += ((i >> b) & 1) ? -wv : wv;
          const cf dc = cmul(pt, phi[i]);
          const cf dinv = {dc.x, -dc.y};
          p[i] = cmul(p[i], dinv);
          m[i] = cmul(m[i], dinv);
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) dph_l[q] = ((threadIdx.x >> q) & 1) ? -wsum : wsum;
#pragma unroll
        for (int b = 0; 8 + b < N; ++b) dph_l[8 + b] = whi[b];
        __syncthreads();
#pragma unroll
        for (int i = 0; i < PER; ++i) {
          psi[threadIdx.x + i * NT] = p[i];
          lam[threadIdx.x + i * NT] = m[i];
        }
        __syncthreads();
      } else {
        float dth[HV], dph[HV];
#pragma unroll
        for (int b = 0; b < HV; ++b) dth[b] = dph[b] = 0.f;
        for (int c = threadIdx.x; c < C::T; c += NT) {
          cf p[C::NTILE], m[C::NTILE];
#pragma unroll
          for (int h = 0; h < C::NTILE; ++h) {
            const int src = ring_fwd<N>(c | (h << C::TB));
            p[h] = psi[src];
            if (first) {
              float o = 0.f;
#pragma unroll
              for (int q = 0; q < N; ++q) o += ((src >> q) & 1) ? -gq[q] : gq[q];
              m[h] = {p[h].x * o, p[h].y * o};
            } else {
              m[h] = lam[src];
            }
          }
#pragma unroll
          for (int bb = 0; bb < C::HB; ++bb) {
            const int b = C::HB - 1 - bb;   // reverse qubit order
            const float4 tg = trig[C::TB + b];
#pragma unroll
            for (int h = 0; h < C::NTILE; ++h)
              if (!((h >> b) & 1)) gate_adj(p[h], p[h | (1 << b)], m[h], m[h | (1 << b)], tg, dth[b], dph[b]);
          }
#pragma unroll
          for (int h = 0; h < C::NTILE; ++h) {
            psi_o[c | (h << C::TB)] = p[h];
            lam_o[c | (h << C::TB)] = m[h];
          }
        }
        __syncthreads();
        if constexpr (C::HB > 0) {
          float v[2 * HV];
#pragma unroll
          for (int b = 0; b < HV; ++b) {
            v[2 * b] = dth[b];
            v[2 * b + 1] = dph[b];
          }
          block_add<2 * HV>(v, red, gdst, 2 * C::TB);
        }
        cf* t = psi;
        psi = psi_o;
        psi_o = t;
        t = lam;
        lam = lam_o;
        lam_o = t;
      }
      // ---- low pass (reverse): tiles of psi/lam in place, groups and qubits in reverse order
      {
        float dth[C::TB], dph[C::TB];
#pragma unroll
        for (int q = 0; q < C::TB; ++q) dth[q] = dph[q] = 0.f;
        for (int h = 0; h < C::NTILE; ++h) {
          cf* tpp = C::LDS_STATE ? psi : tp;
          cf* tqq = C::LDS_STATE ? lam : tq;
          if constexpr (!C::LDS_STATE) {
            const cf* sp_ = psi + (size_t)h * C::T;
            const cf* sl_ = lam + (size_t)h * C::T;
            for (int i = threadIdx.x; i < C::T; i += NT) {
              tpp[i] = sp_[i];
              tqq[i] = sl_[i];
            }
            __syncthreads();
          }
          static_for<0, C::NGRP>([&](auto gc) {
            constexpr int gi = C::NGRP - 1 - decltype(gc)::value;
            constexpr int g0 = 3 * gi;
            constexpr int NB = (C::TB - g0) < 3 ? (C::TB - g0) : 3;
            constexpr int ACT = C::T >> NB;
            for (int t = threadIdx.x; t < ACT; t += NT) {
              const int base = ins_bits<g0, NB>(t);
              cf p[1 << NB], m[1 << NB];
#pragma unroll
              for (int j = 0; j < (1 << NB); ++j) {
                p[j] = tpp[base | (j << g0)];
                m[j] = tqq[base | (j << g0)];
              }
#pragma unroll
              for (int bb = 0; bb < NB; ++bb) {
                const int b = NB - 1 - bb;
                const float4 tg = trig[g0 + b];
#pragma unroll
                for (int j = 0; j < (1 << NB); ++j)
                  if (!((j >> b) & 1)) {
                    if constexpr (DIAG) ry_adj(p[j], p[j | (1 << b)], m[j], m[j | (1 << b)], tg.x, tg.y, dth[g0 + b]);
                    else gate_adj(p[j], p[j | (1 << b)], m[j], m[j | (1 << b)], tg, dth[g0 + b], dph[g0 + b]);
                  }
              }
#pragma unroll
              for (int j = 0; j < (1 << NB); ++j) {
                tpp[base | (j << g0)] = p[j];
                tqq[base | (j << g0)] = m[j];
              }
            }
            __syncthreads();
          });
          if constexpr (!C::LDS_STATE) {
            if (l > 0) {  // after layer 0 nothing reads the state again
              cf* dp_ = psi + (size_t)h * C::T;
              cf* dl_ = lam + (size_t)h * C::T;
              for (int i = threadIdx.x; i < C::T; i += NT) {
                dp_[i] = tpp[i];
                dl_[i] = tqq[i];
              }
            }
            __syncthreads();
          }
        }
        float v[2 * C::TB];
#pragma unroll
        for (int q = 0; q < C::TB; ++q) {
          v[2 * q] = dth[q];
          if constexpr (DIAG) v[2 * q + 1] = dph_l[q];
          else v[2 * q + 1] = dph[q];
        }
        block_add<2 * C::TB>(v, red, gdst, 0);
      }
    }
    // layer 0: theta grads are this sample's d(angles); fold the scratch into the slab accumulators
    if (threadIdx.x < N) {
      dx[(size_t)s * N + threadIdx.x] = tmp[2 * threadIdx.x];
      acc[2 * threadIdx.x] += tmp[2 * threadIdx.x];
      acc[2 * threadIdx.x + 1] += tmp[2 * threadIdx.x + 1];
    }
    __syncthreads();
  }
  __syncthreads();
  for (int i = threadIdx.x; i < P; i += NT) slab[(size_t)blockIdx.x * P + i] = acc[i];
}

template <int N>
static size_t smem_bytes(bool backward) {
  using C = G<N>;
  if (C::LDS_STATE && C::HB == 0) return O_DATA + (backward ? 2 : 1) * sizeof(cf) * C::D;   // in-place rings
  if (C::LDS_STATE) return O_DATA + (backward ? 4 : 2) * sizeof(cf) * C::D;
  return O_DATA + (backward ? 2 : 1) * sizeof(cf) * C::T;
}

template <int N>
static int launch(bool backward, const float* x, const float* w, const float* gE, float* E_or_dx, float* slab, int B,
                  int L, int wgroup, cf* ws, int grid, hipStream_t st, cf* psave = nullptr) {
  const size_t sm = smem_bytes<N>(backward);
  if (!G<N>::LDS_STATE && ws == nullptr) return (int)hipErrorInvalidValue;
  if (backward) {
    if (hipError_t e = allow_lds(qsim_big_bwd_kernel<N>, sm)) return (int)e;
    hipLaunchKernelGGL(qsim_big_bwd_kernel<N>, dim3(grid), dim3(NT), sm, st, x, w, gE, E_or_dx, slab, B, L, wgroup, ws,
                       psave);
  } else {
    if (hipError_t e = allow_lds(qsim_big_fwd_kernel<N>, sm)) return (int)e;
    hipLaunchKernelGGL(qsim_big_fwd_kernel<N>, dim3(grid), dim3(NT), sm, st, x, w, E_or_dx, B, L, wgroup, ws, psave);
  }
  return (int)hipGetLastError();
}

}  // namespace qsimbig
}  // namespace qd

using namespace qd::qsimbig;

#define QD_BIG_DISPATCH(n, CALL)            \
  switch (n) {                              \
    case 11: return CALL(11);               \
    case 12: return CALL(12);               \
    case 13: return CALL(13);               \
    case 14: return CALL(14);               \
    case 15: return CALL(15);               \
    case 16: return CALL(16);               \
    default: return (int)hipErrorInvalidValue; \
  }

// Workspace (bytes) for a given grid: zero when the state is LDS-resident (n <= 12).
QD_API long long qd_qsim_big_workspace(int n, int grid, int backward) {
  if (n <= 12) return 0;
  return (long long)grid * (backward ? 4 : 2) * (8ll << n);
}

// Workgroups (= slab rows of the backward) for a batch of B: one sample in flight per workgroup.
// The cap trades HBM workspace (2 / 4 states of 2^n complex per workgroup: 1 / 2 MiB at n = 16) for
// occupancy; measured at n = 16, B = 2304: 512 / 1152 / 2304 workgroups -> 28.2 / 31.1 / 28.6 ms per
// flagship step -- not occupancy-bound, so the small workspace stays.
constexpr int kBigGridCap = 512;
QD_API int qd_qsim_big_grid(int B) { return B < kBigGridCap ? B : kBigGridCap; }

// psave (nullable): (B, 2^n) complex64 buffer keeping every sample's psi_final for qd_qsim_big_bwd.
QD_API int qd_qsim_big_fwd(const float* x, const float* w, float* E, int B, int n, int L, int wgroup, void* ws,
                           void* psave, void* stream) {
  if (wgroup > 0 && B % wgroup != 0) return (int)hipErrorInvalidValue;   // (G = B / wgroup weight groups, workspace)
  if (B < 1 || L < 1 || 2 * n * L > 256) return (int)hipErrorInvalidValue;
  // (n <= 12: one 32 KiB state per workgroup, 4 resident per CU -- 768 workgroups, 3 samples each at B = 2304)
  const int grid = n <= 12 ? (B < 768 ? B : 768) : qd_qsim_big_grid(B);
#define CALL_F(NN) \
  launch<NN>(false, x, w, nullptr, E, nullptr, B, L, wgroup, (cf*)ws, grid, (hipStream_t)stream, (cf*)psave)
  QD_BIG_DISPATCH(n, CALL_F)
#undef CALL_F
}

// psave (nullable): the forward's saved psi_final (same x, w); consumed (may be overwritten).
QD_API int qd_qsim_big_bwd(const float* x, const float* w, const float* gE, float* dx, float* slab, int B, int n, int L,
                           int wgroup, void* ws, void* psave, void* stream) {
  if (wgroup > 0 && B % wgroup != 0) return (int)hipErrorInvalidValue;   // (G = B / wgroup weight groups, workspace)
  if (B < 1 || L < 1 || 2 * n * L > 256) return (int)hipErrorInvalidValue;
  const int grid = qd_qsim_big_grid(B);
#define CALL_B(NN) \
  launch<NN>(true, x, w, gE, dx, slab, B, L, wgroup, (cf*)ws, grid, (hipStream_t)stream, (cf*)psave)
  QD_BIG_DISPATCH(n, CALL_B)
#undef CALL_B
}
