// 8-qubit VQC forward with the layer unitaries on the matrix cores (complex MFMA GEMM).
//
// Same circuit as csrc/hip/qsim.hip (reference E:125-142: RY angle embedding, L x [RY, RZ on every
// wire, CNOT ring], <Z_i>).  A layer's rotations are a Kronecker product: with the state as a 16 x 16
// complex matrix X[hi][lo] (amplitude k = hi << 4 | lo; lo = qubits 0..3, hi = qubits 4..7),
//     (R_7 (x) ... (x) R_0) psi   <->   X' = A_hi X A_lo^T,   A_lo = R_3 (x) .. (x) R_0,  A_hi = R_7 (x) .. (x) R_4
// -- two 16 x 16 complex products per sample, i.e. two pairs of mfma_f32_16x16x32 in real form
// ([Xr Xi] times a 32 x 32 real block of A_lo, then a 32 x 32 real block of A_hi times [Yr; Yi]).
// One wave per sample.  The first product's accumulator tile feeds the second as its B operand with
// NO data movement: lane group g of a 16x16 accumulator holds rows 4g..4g+3 of Yr and of Yi, exactly
// the 8 k-slots that lane group needs, in a permuted k order that the A_hi operand is built in.
//
// Precision: MFMA inputs are fp16 split in two, x = hi + lo * 2^-11 (hi = fp16(x), lo = fp16((x - hi)
// 2^11)), and each product is hi.hi + (hi.lo + lo.hi) 2^-11 in fp32 accumulators: ~22 mantissa bits,
// i.e. fp32-grade amplitudes from the fp16 rate (6 MFMAs per product instead of 2).
//
// Per layer l >= 1: the two products, then the CNOT ring as one LDS permutation back into the first
// product's operand layout.  Layer 0 (embedding + first rotations + ring) is the closed-form product
// state, generated straight in that layout.  The last layer reduces <Z_q> and (optionally) stores
// psi_final in the layout qsim.hip's adjoint backward reads (psave[s][r][lane], k = r | lane << 2).
//
// qd_qsim_mfma_prep builds every (group, layer) operand image once per step (fp16 hi / lo, per-lane
// register order); the forward streams them from L2.  In training with QuantumNAT the build rides in the noise
// draw's launch (qd_qsim_mfma_prep_noise replaces qsc.hip's single-block qd_qnoise): no extra launch per step.
//
// Measured (scripts/probe_qsim_mfma.py, 9 groups x 256 samples, 3 layers, MI355X): forward 11.1 us vs
// 12.4 us for the register kernel (qsim.hip); a separate operand build would add a 4 us launch, so in the
// training step the build rides in the QuantumNAT draw's launch and this forward is the flagship's default
// (ops/qsc.py; step 0.4044 / 0.4100 vs 0.4096 / 0.4100 ms with the register forward, profiles/r3_14_*).
// Exact to 3e-6 against the register kernel and the fp64 CPU oracle
// (tests/test_kernels_gpu.py::test_qsim_mfma_forward_matches_register_kernel,
// tests/test_qsc_gpu.py::test_qsc_circuit_forward_on_mfma_matches_register_kernel).
#include <cstdlib>

#include "common.h"

namespace qd {
namespace qmfma {

typedef __attribute__((ext_vector_type(8))) _Float16 h8;
typedef __attribute__((ext_vector_type(4))) float f4;

constexpr int N = 8;
constexpr int D = 256;
constexpr float LO_SCALE = 2048.f, LO_INV = 1.f / 2048.f;
// operand image of one (group, layer): [op][hl][lane][8] halves; op 0/1 = A_lo blocks for Yr / Yi
// (B operands of product 1), op 2/3 = A_hi blocks for Zr / Zi (A operands of product 2)
constexpr int OP_HALVES = 4 * 2 * 64 * 8;

struct cf {
  float x, y;
};
__device__ __forceinline__ cf cmul(cf a, cf b) { return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }

// R = RZ(phi) RY(theta): [[c e^-ip, -s e^-ip], [s e^ip, c e^ip]] (p = phi / 2), gate_fwd's matrix
__device__ __forceinline__ cf rot(float c, float s, float cp, float sp, int a, int b) {
  const float m = (a == b) ? c : (a == 0 ? -s : s);
  return a == 0 ? cf{m * cp, -m * sp} : cf{m * cp, m * sp};
}
// Kronecker product of 4 rotations (qubits q0..q0+3): entry [a][b] (4-bit row / column)
__device__ __forceinline__ cf kron4(const float4* tr, int q0, int a, int b) {
  cf v = {1.f, 0.f};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float4 t = tr[q0 + i];
    v = cmul(v, rot(t.x, t.y, t.z, t.w, (a >> i) & 1, (b >> i) & 1));
  }
  return v;
}

__device__ __forceinline__ void split(float v, _Float16& hi, _Float16& lo) {
  hi = (_Float16)v;
  lo = (_Float16)((v - (float)hi) * LO_SCALE);
}

// QuantumNAT noise draw of qsc.hip's qnoise_kernel, element i of the (G, L, N, 2) noisy-weight tensor (the same
// counter-based hash: the fused prep below writes bit-identical noisy weights)
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ float hash_normal(unsigned long long seed, unsigned long long ctr, unsigned int i) {
  const unsigned long long h = mix64(seed ^ mix64(ctr * 0x100000001b3ull + i));
  const float u1 = ((h >> 40) + 1u) * (1.0f / 16777217.0f);          // (0, 1]
  const float u2 = ((h >> 16) & 0xffffffu) * (1.0f / 16777216.0f);   // [0, 1)
  return sqrtf(-2.f * __logf(u1)) * __cosf(6.283185307179586f * u2);
}

struct Noise {
  const float* w;                 // (L, N, 2) master weights, shared by the G groups
  float* out;                     // (G, L, N, 2) noisy copies (the forward's layer 0 and the adjoint read them)
  float sigma;
  unsigned long long seed;
  unsigned long long* counter;    // draws so far: read by every block, advanced by the last one to finish
  unsigned int* done;             // zero-initialised arrival counter (re-armed by the last block)
};

// grid (G, L), block 64: block (g, l) builds the operand images of layer l >= 1 of weight group g.  w (G, L, N, 2),
// or with nz.out the noisy weights of that layer drawn here first (QuantumNAT: one launch for the draw and the
// images, the draw's counter advanced by the last block).  Blocks with l = 0 only draw.
__global__ void __launch_bounds__(64) prep_kernel(const float* __restrict__ w, _Float16* __restrict__ ops, int L,
                                                  Noise nz) {
  __shared__ float4 tr[N];
  __shared__ float wn[2 * N];
  const int g = blockIdx.x, l = blockIdx.y, lane = threadIdx.x;
  if (nz.out != nullptr) {
    const unsigned long long ctr = *nz.counter;
    if (lane < 2 * N) {
      const int P = L * 2 * N, j = l * 2 * N + lane;
      const float v = nz.w[j] + nz.sigma * hash_normal(nz.seed, ctr, (unsigned int)(g * P + j));
      nz.out[(size_t)g * P + j] = v;
      wn[lane] = v;
    }
    __syncthreads();
    if (lane == 0) {   // every block read *counter above: the last to arrive advances it
      const unsigned int prev = __hip_atomic_fetch_add(nz.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (prev == gridDim.x * gridDim.y - 1) {
        *nz.counter = ctr + 1;
        __hip_atomic_store(nz.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  } else if (lane < 2 * N) {
    wn[lane] = w[((size_t)g * L + l) * 2 * N + lane];
  }
  if (l == 0) return;
  __syncthreads();
  if (lane < N) {
    float s, c, sp, cp;
    __sincosf(0.5f * wn[2 * lane], &s, &c);
    __sincosf(0.5f * wn[2 * lane + 1], &sp, &cp);
    tr[lane] = make_float4(c, s, cp, sp);
  }
  __syncthreads();
  _Float16* img = ops + ((size_t)g * (L - 1) + (l - 1)) * OP_HALVES;
  const int gq = lane >> 4, col = lane & 15;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    // product 1 (Y = X A_lo^T), B operand: k = 8 gq + j over [Xr lo 0..15 | Xi lo 0..15], column c
    const int k = 8 * gq + j;
    const cf a = kron4(tr, 0, col, k & 15);                 // A_lo[c][lo]
    const float byr = k < 16 ? a.x : -a.y;                  // Yr = Xr Ar^T - Xi Ai^T
    const float byi = k < 16 ? a.y : a.x;                   // Yi = Xr Ai^T + Xi Ar^T
    // product 2 (Z = A_hi Y), A operand: row h' = col, permuted k slot 8 gq + j <-> Y row 4 gq + (j & 3),
    // real part for j < 4, imaginary part for j >= 4
    const cf b = kron4(tr, 4, col, 4 * gq + (j & 3));       // A_hi[h'][h]
    const float azr = j < 4 ? b.x : -b.y;                   // Zr = Ahr Yr - Ahi Yi
    const float azi = j < 4 ? b.y : b.x;                    // Zi = Ahi Yr + Ahr Yi
    const float v[4] = {byr, byi, azr, azi};
#pragma unroll
    for (int op = 0; op < 4; ++op) {
      _Float16 hi, lo;
      split(v[op], hi, lo);
      img[((op * 2 + 0) * 64 + lane) * 8 + j] = hi;
      img[((op * 2 + 1) * 64 + lane) * 8 + j] = lo;
    }
  }
}

__device__ __forceinline__ f4 mfma(h8 a, h8 b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); }

// CNOT ring f (closed form, see qsim_stream.hip) and inverse
__device__ __forceinline__ int ring_fwd(int k) {
  int p = k ^ (k << 1);
  p ^= p << 2;
  p ^= p << 4;
  p &= D - 1;
  return (p & ~1) | ((k ^ (p >> (N - 1))) & 1);
}
__device__ __forceinline__ int ring_inv(int j) {
  const int j2 = j ^ ((j >> (N - 1)) & 1);
  return j2 ^ ((j2 << 1) & (D - 1));
}

// x (B, 8) angles, w (G, L, 8, 2) weights (group of sample s = s / wgroup; wgroup 0: one group),
// ops from prep_kernel; E (B, 8); psave (nullable) psi_final as qsim.hip stores it.
// Block: 4 waves; each wave runs SPW samples of one group side by side (independent MFMA chains for
// the scheduler to interleave; the layer operands are loaded once per wave, up front).
template <int SPW>
__global__ void __launch_bounds__(256) fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                  const _Float16* __restrict__ ops, float* __restrict__ E, int B, int L,
                                                  int wgroup, cf* __restrict__ psave) {
  __shared__ float st[4][SPW][2][D];     // per wave and sample: re / im planes for the ring permutation
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int s0 = (blockIdx.x * 4 + wv) * SPW;
  if (s0 >= B) return;                   // (whole wave: no block barrier below)
  const int gq = lane >> 4, row = lane & 15;
  // the wave's samples share one group (SPW divides wgroup: checked by the launcher)
  const int grp = wgroup > 0 ? s0 / wgroup : 0;
  const h8* opv = reinterpret_cast<const h8*>(ops) + (size_t)grp * (L - 1) * 4 * 2 * 64;
  // layer 1's operands now; each layer prefetches the next one's behind its MFMAs
  h8 o[8], on[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) o[q] = opv[q * 64 + lane];
  // layer-0 product state as two 16-entry factor tables per sample (qubits 0..3 / 4..7):
  // psi0[k] = PL[k & 15] * PH[k >> 4]; lane (i, t): sample i, entry t & 15 of PL (t < 16) or PH
  __shared__ cf pt[4][SPW][32];
  if (lane < 32 * SPW && lane < 64) {
    const int i = lane / 32, t = lane % 32;
    const int s = s0 + i < B ? s0 + i : B - 1;
    const float* w0 = w + (size_t)grp * L * 2 * N;
    const int q0 = t < 16 ? 0 : 4, e = t & 15;
    cf a = {1.f, 0.f};
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int q = q0 + b;
      float sn, c, sp, cp;
      __sincosf(0.5f * (x[(size_t)s * N + q] + w0[2 * q]), &sn, &c);
      __sincosf(0.5f * w0[2 * q + 1], &sp, &cp);
      a = cmul(a, ((e >> b) & 1) ? cf{sn * cp, sn * sp} : cf{c * cp, -c * sp});
    }
    pt[wv][i][t] = a;
  }
  if (SPW > 2) {   // (more than 64 table entries: a second round)
    for (int idx = lane + 64; idx < 32 * SPW; idx += 64) {
      const int i = idx / 32, t = idx % 32;
      const int s = s0 + i < B ? s0 + i : B - 1;
      const float* w0 = w + (size_t)grp * L * 2 * N;
      const int q0 = t < 16 ? 0 : 4, e = t & 15;
      cf a = {1.f, 0.f};
      for (int b = 0; b < 4; ++b) {
        const int q = q0 + b;
        float sn, c, sp, cp;
        __sincosf(0.5f * (x[(size_t)s * N + q] + w0[2 * q]), &sn, &c);
        __sincosf(0.5f * w0[2 * q + 1], &sp, &cp);
        a = cmul(a, ((e >> b) & 1) ? cf{sn * cp, sn * sp} : cf{c * cp, -c * sp});
      }
      pt[wv][i][t] = a;
    }
  }
  wave_lds_fence();
  // layer 0 + ring, straight into the X operand layout: lane (row hi, gq) holds
  // re/im (gq >> 1) of X[hi][8 (gq & 1) + j] = psi1[hi << 4 | lo] = psi0[f^-1(.)]
  h8 xh[SPW], xl[SPW];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = ring_inv((row << 4) | (8 * (gq & 1) + j));
#pragma unroll
    for (int i = 0; i < SPW; ++i) {
      const cf a = cmul(pt[wv][i][k & 15], pt[wv][i][16 + (k >> 4)]);
      _Float16 hi, lo;
      split(gq >> 1 ? a.y : a.x, hi, lo);
      xh[i][j] = hi;
      xl[i][j] = lo;
    }
  }
  f4 zr[SPW], zi[SPW];
  const f4 z0 = {0.f, 0.f, 0.f, 0.f};
  for (int l = 1; l < L; ++l) {
    // o: [0/1] A_lo Yr hi/lo, [2/3] A_lo Yi, [4/5] A_hi Zr, [6/7] A_hi Zi
    if (l + 1 < L)
#pragma unroll
      for (int q = 0; q < 8; ++q) on[q] = opv[((size_t)l * 8 + q) * 64 + lane];
    f4 yr[SPW], yrc[SPW], yi[SPW], yic[SPW];
#pragma unroll
    for (int i = 0; i < SPW; ++i) {   // product 1 of every sample, then product 2: independent chains
      yr[i] = mfma(xh[i], o[0], z0);
      yi[i] = mfma(xh[i], o[2], z0);
      yrc[i] = mfma(xh[i], o[1], mfma(xl[i], o[0], z0));
      yic[i] = mfma(xh[i], o[3], mfma(xl[i], o[2], z0));
    }
#pragma unroll
    for (int i = 0; i < SPW; ++i) {
      // Y as product 2's B operand: slots 8 gq + j = (Yr rows 4 gq + j, j < 4; Yi rows 4 gq + j - 4)
      h8 yh, yl;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        _Float16 hi, lo;
        split(yr[i][r] + yrc[i][r] * LO_INV, hi, lo);
        yh[r] = hi;
        yl[r] = lo;
        split(yi[i][r] + yic[i][r] * LO_INV, hi, lo);
        yh[4 + r] = hi;
        yl[4 + r] = lo;
      }
      const f4 zrc = mfma(o[4], yl, mfma(o[5], yh, z0)), zic = mfma(o[6], yl, mfma(o[7], yh, z0));
      zr[i] = mfma(o[4], yh, z0);
      zi[i] = mfma(o[6], yh, z0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        zr[i][r] += zrc[r] * LO_INV;
        zi[i][r] += zic[r] * LO_INV;
      }
    }
    if (l + 1 < L) {
      // the ring: amplitude k = h' << 4 | c moves to f(k); read back in the X operand layout
#pragma unroll
      for (int i = 0; i < SPW; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int j = ring_fwd(((4 * gq + r) << 4) | row);
          st[wv][i][0][j] = zr[i][r];
          st[wv][i][1][j] = zi[i][r];
        }
      wave_lds_fence();
#pragma unroll
      for (int i = 0; i < SPW; ++i) {
        const float* src = st[wv][i][gq >> 1] + (row << 4) + 8 * (gq & 1);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          _Float16 hi, lo;
          split(src[j], hi, lo);
          xh[i][j] = hi;
          xl[i][j] = lo;
        }
      }
      wave_lds_fence();
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = on[q];
    }
  }
  // final ring image j = f(k) of this lane's 4 amplitudes: <Z_q> partials (+ psi_final)
#pragma unroll
  for (int i = 0; i < SPW; ++i) {
    const int s = s0 + i;
    if (s >= B) break;
    float part[N];
#pragma unroll
    for (int q = 0; q < N; ++q) part[q] = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = ring_fwd(((4 * gq + r) << 4) | row);
      const float p = zr[i][r] * zr[i][r] + zi[i][r] * zi[i][r];
#pragma unroll
      for (int q = 0; q < N; ++q) part[q] += ((j >> q) & 1) ? -p : p;
      if (psave) psave[(size_t)s * D + (j & 3) * 64 + (j >> 2)] = cf{zr[i][r], zi[i][r]};
    }
#pragma unroll
    for (int q = 0; q < N; ++q) {
      const float v = wave_sum(part[q]);
      if (lane == q) E[(size_t)s * N + q] = v;
    }
  }
}

}  // namespace qmfma
}  // namespace qd

using namespace qd::qmfma;

// halves of operand image per (group, layer >= 1)
QD_API long long qd_qsim_mfma_ops_halves(int G, int L) { return (long long)G * (L > 1 ? L - 1 : 0) * OP_HALVES; }

// w (G, L, 8, 2) -> ops (qd_qsim_mfma_ops_halves fp16 values)
QD_API int qd_qsim_mfma_prep(const float* w, void* ops, int G, int L, void* stream) {
  if (G < 1 || L < 2) return (int)hipErrorInvalidValue;
  Noise nz{nullptr, nullptr, 0.f, 0ull, nullptr, nullptr};
  // (without noise the layer-0 blocks of the (G, L) grid return at once)
  hipLaunchKernelGGL(prep_kernel, dim3(G, L), dim3(64), 0, (hipStream_t)stream, w, (_Float16*)ops, L, nz);
  return (int)hipGetLastError();
}

// QuantumNAT draw + operand images in ONE launch: out (G, L, 8, 2) = w (L, 8, 2) + sigma N(0, 1) -- bit-identical to
// qd_qnoise with the same seed / counter -- and the images of the noisy layers 1..L-1.  done: zero-initialised
// uint32 (re-armed by the kernel).
QD_API int qd_qsim_mfma_prep_noise(const float* w, float* out, void* ops, int G, int L, float sigma,
                                   unsigned long long seed, unsigned long long* counter, unsigned int* done,
                                   void* stream) {
  if (G < 1 || L < 2 || !w || !out || !counter || !done) return (int)hipErrorInvalidValue;
  Noise nz{w, out, sigma, seed, counter, done};
  hipLaunchKernelGGL(prep_kernel, dim3(G, L), dim3(64), 0, (hipStream_t)stream, out, (_Float16*)ops, L, nz);
  return (int)hipGetLastError();
}

// n = 8 only, 2 <= L <= 8.  psave nullable ((B, 256) complex64, qsim.hip's layout).
// samples per wave: 1 (measured 11.1 / 12.5 / 16.6 us at the flagship shape for 1 / 2 / 4)
QD_API int qd_qsim_mfma_fwd(const float* x, const float* w, const void* ops, float* E, int B, int L, int wgroup,
                            void* psave, void* stream) {
  if (wgroup > 0 && B % wgroup != 0) return (int)hipErrorInvalidValue;   // (G = B / wgroup weight groups, workspace)
  if (B < 1 || L < 2 || L > 8) return (int)hipErrorInvalidValue;
  constexpr int spw = 1;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((B + 4 * spw - 1) / (4 * spw));
  const _Float16* o = (const _Float16*)ops;
#define QM_S(SPW) hipLaunchKernelGGL((fwd_kernel<SPW>), grid, dim3(256), 0, st, x, w, o, E, B, L, wgroup, (cf*)psave);
  QM_S(1)
#undef QM_S
  return (int)hipGetLastError();
}
