// 12-qubit VQC simulator -- forward AND adjoint backward -- with every gate layer on the matrix cores.
//
// Same circuit and outputs as csrc/hip/qsim_big.hip's n = 12 kernels (reference E:125-142: RY angle embedding,
// L x [RY, RZ on every wire, CNOT ring], <Z_i>; adjoint differentiation), which apply the 24 rotations of a
// layer gate by gate on the vector ALUs (qsim_big_bwd_kernel<12> 439 us, fwd 166 us per P256 training step,
// profiles/r4_11_p256_kernel_stats.md).  Here the 4096-amplitude state is a 16 x 16 x 16 complex tensor
// X[c][b][a] (amplitude k = c << 8 | b << 4 | a: a = qubits 0..3, b = 4..7, c = 8..11), and a layer's rotations
// are a Kronecker product A2 (x) A1 (x) A0 of three 16 x 16 complex factors (each the product of 4 qubits'
// R = RZ(phi) RY(theta)), applied as three mode products -- 16 x 16 complex GEMM tiles on
// mfma_f32_16x16x32_f16 in real form:
//     Y = A X_mode      Yr = [Ar | -Ai] [Xr ; Xi],   Yi = [Ai | Ar] [Xr ; Xi]      (K = 32 = 16 re + 16 im)
// The factor is the MFMA A operand (a per-(group, layer, mode) image built once per step by prep_kernel and held
// in registers), the state tile the B operand (read from the LDS-resident state), the 16 x 16 result is written
// back in place: a tile's inputs and outputs are the same 256 amplitudes, so no other wave touches them.  The
// CNOT ring (a GF(2)-linear permutation f of the basis) rides in the last mode's write-back.
//
// Precision: fp16 operands split in two (x = hi + lo 2^-11, qsim_mfma.hip's scheme), products
// hi.hi + (hi.lo + lo.hi) 2^-11 in fp32 accumulators: ~22 mantissa bits, fp32-grade amplitudes.
//
// Adjoint backward (per sample, from the forward's saved final state): lambda = (sum_q g_q Z_q) psi; then per
// layer in reverse: undo the ring on psi and lambda (a permutation), the layer's 24 gate gradients, and (l > 0)
// psi <- U^dagger psi, lambda <- U^dagger lambda (the same mode products with the adjoint factors).  Gradients
// of the rotations of one layer commute with the other qubits' rotations, so they come from the 2 x 2 cross
// densities rho_q[x][y] = sum_(other bits) conj(lambda[..x..]) psi[..y..] of the layer's output states:
//     dphi_q = Im(rho_00 - rho_11),     dtheta_q = Re(e^{i phi} rho_10) - Re(e^{-i phi} rho_01)
// (qsim.hip's per-gate formulas, with RZ's phase folded in).  rho for the 4 qubits of a mode are partial traces
// of C_m[alpha][beta] = sum_o conj(lambda[o, alpha]) psi[o, beta] (o = the other two modes' 256 indices): a
// 16 x 16 x 256 complex contraction, again on the MFMA (K steps of 16 o x {re, im}; the 4 waves take 4 K steps
// each and their partial tiles are summed in a fixed order).
//
// Layout: one 256-thread workgroup per sample (a loop over the batch), the state as fp32 re / im planes in LDS
// (32 KiB per state; the backward holds psi and lambda: 2 workgroups per CU).  Outputs match qsim_big.hip:
// E (B, 12); dx (B, 12); slab (gridDim.x, 2 n L) per-workgroup dW partials in a fixed sample order (summed by
// the caller); psave (B, 2, 4096) fp32 planes, written by the forward, read by the backward.
#include "common.h"

namespace qd {
namespace qm12 {

typedef __attribute__((ext_vector_type(8))) _Float16 h8;
typedef __attribute__((ext_vector_type(4))) float f4;

constexpr int N = 12;
constexpr int D = 1 << N;
constexpr int NT = 256;
constexpr float LO_SCALE = 2048.f, LO_INV = 1.f / 2048.f;
// operand image of one (group, layer >= 1, mode, direction): [form r / i][hi / lo][lane] h8
constexpr int IMG_H8 = 2 * 2 * 64;
// per (group, layer >= 1): 3 modes x {forward, adjoint}
constexpr int LAYER_H8 = 3 * 2 * IMG_H8;

struct cf {
  float x, y;
};
__device__ __forceinline__ cf cmul(cf a, cf b) { return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }

// R = RZ(phi) RY(theta) entry [a][b] from (cos, sin) of theta / 2 and of phi / 2 (qsim_mfma.hip's rot)
__device__ __forceinline__ cf rot(float4 t, int a, int b) {
  const float m = (a == b) ? t.x : (a == 0 ? -t.y : t.y);
  return a == 0 ? cf{m * t.z, -m * t.w} : cf{m * t.z, m * t.w};
}
// (R_{q0+3} (x) .. (x) R_{q0})[a][b], 4-bit row / column
__device__ __forceinline__ cf kron4(const float4* tr, int q0, int a, int b) {
  cf v = {1.f, 0.f};
#pragma unroll
  for (int i = 0; i < 4; ++i) v = cmul(v, rot(tr[q0 + i], (a >> i) & 1, (b >> i) & 1));
  return v;
}
__device__ __forceinline__ void split(float v, _Float16& hi, _Float16& lo) {
  hi = (_Float16)v;
  lo = (_Float16)((v - (float)hi) * LO_SCALE);
}
__device__ __forceinline__ f4 mfma(h8 a, h8 b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); }

// 8 floats -> fp16 hi / lo operands in pairs: hi = the packed round-toward-zero convert of two values, lo = the
// exact residual v - hi (hi converted back) times 2^11, packed the same way -- two values per convert and no
// separate packing step (the per-value split cost 5-6 vector instructions per value).  The residual is taken
// from the converted hi, so values in fp16's subnormal range (adjoint vectors of small loss gradients: 1e-5 and
// below) keep their precision in lo.  (Cutting hi's mantissa in fp32 instead lost 1 % on such values.)
typedef __attribute__((ext_vector_type(4))) unsigned int u4;
__device__ __forceinline__ void split8(const float (&v)[8], h8& hi, h8& lo) {
  u4 H, L;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const auto h = __builtin_amdgcn_cvt_pkrtz(v[2 * p], v[2 * p + 1]);
    H[p] = __builtin_bit_cast(unsigned int, h);
    L[p] = __builtin_bit_cast(unsigned int, __builtin_amdgcn_cvt_pkrtz((v[2 * p] - (float)h[0]) * LO_SCALE,
                                                                      (v[2 * p + 1] - (float)h[1]) * LO_SCALE));
  }
  hi = __builtin_bit_cast(h8, H);
  lo = __builtin_bit_cast(h8, L);
}
// LDS plane address of amplitude k: one float of padding per 16 (a 17-float row; pad()), so the strided operand reads of
// all three modes are at most 2-way bank conflicts (8-way on the unpadded mode-0 reads)
__device__ __forceinline__ int pad(int k) { return k + (k >> 4); }

// CNOT ring CNOT(0,1) .. CNOT(n-2,n-1), CNOT(n-1,0) as a basis map, and its inverse (qsim_big.hip's)
__device__ __forceinline__ int ring_fwd(int k) {
#pragma unroll
  for (int i = 0; i < N - 1; ++i) k ^= ((k >> i) & 1) << (i + 1);
  k ^= (k >> (N - 1)) & 1;
  return k;
}

// state index of mode index `e` (0..15) of mode M with the other two modes' index o (0..255, in k order)
template <int M>
__device__ __forceinline__ int sidx(int o, int e) {
  if constexpr (M == 0) return (o << 4) | e;
  else if constexpr (M == 1) return ((o >> 4) << 8) | (e << 4) | (o & 15);
  else return (e << 8) | o;
}

// grid (G, L - 1), block 64: the operand images of layer l = 1 + blockIdx.y of weight group blockIdx.x.  For
// lane (i, g) = (lane & 15, lane >> 4) and k = 8 g + j: form r = [Ar | -Ai][i][k], form i = [Ai | Ar][i][k] of the
// mode's factor A (direction 0) or of its adjoint A^dagger[i][k'] = conj(A[k'][i]) (direction 1).
template <int NQ>
__global__ void __launch_bounds__(64) prep_kernel(const float* __restrict__ w, h8* __restrict__ img, int L) {
  constexpr int NM = NQ / 4;   // modes
  __shared__ float4 tr[NQ];
  const int g = blockIdx.x, l = 1 + blockIdx.y, lane = threadIdx.x;
  if (lane < NQ) {
    const float* wl = w + ((size_t)g * L + l) * 2 * NQ;
    float s, c, sp, cp;
    __sincosf(0.5f * wl[2 * lane], &s, &c);
    __sincosf(0.5f * wl[2 * lane + 1], &sp, &cp);
    tr[lane] = make_float4(c, s, cp, sp);
  }
  __syncthreads();
  const int i = lane & 15, gq = lane >> 4;
  h8* out = img + ((size_t)g * (L - 1) + (l - 1)) * (NM * 2 * IMG_H8);
#pragma unroll
  for (int m = 0; m < NM; ++m)
#pragma unroll
    for (int dir = 0; dir < 2; ++dir) {
      h8 rh, rl, ih, il;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 8 * gq + j, kk = k & 15;
        cf a = dir == 0 ? kron4(tr, 4 * m, i, kk) : kron4(tr, 4 * m, kk, i);
        if (dir == 1) a.y = -a.y;
        const float vr = k < 16 ? a.x : -a.y;
        const float vi = k < 16 ? a.y : a.x;
        _Float16 h, lo;
        split(vr, h, lo);
        rh[j] = h;
        rl[j] = lo;
        split(vi, h, lo);
        ih[j] = h;
        il[j] = lo;
      }
      h8* o = out + (m * 2 + dir) * IMG_H8;
      o[(0 * 2 + 0) * 64 + lane] = rh;
      o[(0 * 2 + 1) * 64 + lane] = rl;
      o[(1 * 2 + 0) * 64 + lane] = ih;
      o[(1 * 2 + 1) * 64 + lane] = il;
    }
}

// The 4 h8 of one (mode, direction) image for this lane: r hi, r lo, i hi, i lo
struct Op {
  h8 rh, rl, ih, il;
};
__device__ __forceinline__ Op load_op(const h8* img, int lane) {
  return Op{img[lane], img[64 + lane], img[128 + lane], img[192 + lane]};
}

// The B operand of state tile (t, column jj) of mode M: lane (jj, gq) holds slots k = 8 gq + 0..7 = plane gq >> 1
// (re / im) at mode index 8 (gq & 1) + 0..7, other index t * 16 + jj; split into fp16 hi / lo
template <int M>
__device__ __forceinline__ void load_b(const float* pr, const float* pi, int t, int jj, int gq, h8& bh, h8& bl) {
  const float* pl = (gq >> 1) ? pi : pr;
  const int o = t * 16 + jj;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = pl[pad(sidx<M>(o, 8 * (gq & 1) + j))];
  split8(v, bh, bl);
}

// Y = A X along mode M for the 4 tiles of wave wv; RING: written at the CNOT-ring images (after a workgroup
// barrier: the permutation crosses tiles), else in place.
template <int M, bool RING>
__device__ __forceinline__ void mode_apply(float* pr, float* pi, const Op& A, int wv, int lane) {
  const int jj = lane & 15, gq = lane >> 4;
  const f4 z = {0.f, 0.f, 0.f, 0.f};
  f4 yr[RING ? 4 : 1], yi[RING ? 4 : 1];
  // (one tile at a time unless the ring needs all four held: unrolled, the compiler hoisted every tile's loads and
  // the backward spilled)
#pragma unroll RING ? 4 : 1
  for (int tt = 0; tt < 4; ++tt) {
    const int t = wv * 4 + tt;
    const int ts = RING ? tt : 0;
    h8 bh, bl;
    load_b<M>(pr, pi, t, jj, gq, bh, bl);
    const f4 rc = mfma(A.rl, bh, mfma(A.rh, bl, z));
    const f4 ic = mfma(A.il, bh, mfma(A.ih, bl, z));
    yr[ts] = mfma(A.rh, bh, z);
    yi[ts] = mfma(A.ih, bh, z);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      yr[ts][r] += rc[r] * LO_INV;
      yi[ts][r] += ic[r] * LO_INV;
    }
    if constexpr (!RING) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = pad(sidx<M>(t * 16 + jj, 4 * gq + r));
        pr[k] = yr[0][r];
        pi[k] = yi[0][r];
      }
    }
  }
  if constexpr (RING) {
    __syncthreads();
#pragma unroll
    for (int tt = 0; tt < 4; ++tt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = pad(ring_fwd(sidx<M>((wv * 4 + tt) * 16 + jj, 4 * gq + r)));
        pr[k] = yr[tt][r];
        pi[k] = yi[tt][r];
      }
  }
}

// layer-0 product state (embedding + the first rotations), written at its ring images.  tab: 48 complex
// scratch (3 modes x 16 entries).
__device__ __forceinline__ void layer0(float* pr, float* pi, cf* tab, const float* xs, const float* w0, int tid) {
  if (tid < 48) {
    const int m = tid >> 4, e = tid & 15;
    cf a = {1.f, 0.f};
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int q = 4 * m + b;
      float sn, c, sp, cp;
      __sincosf(0.5f * (xs[q] + w0[2 * q]), &sn, &c);
      __sincosf(0.5f * w0[2 * q + 1], &sp, &cp);
      a = cmul(a, ((e >> b) & 1) ? cf{sn * cp, sn * sp} : cf{c * cp, -c * sp});
    }
    tab[tid] = a;
  }
  __syncthreads();
#pragma unroll 4
  for (int i = 0; i < D / NT; ++i) {
    const int k = tid + NT * i;
    const cf v = cmul(cmul(tab[k & 15], tab[16 + ((k >> 4) & 15)]), tab[32 + (k >> 8)]);
    const int j = pad(ring_fwd(k));
    pr[j] = v.x;
    pi[j] = v.y;
  }
}

// LDS carve (floats): psi planes | lambda planes (backward) | scratch; a plane holds DP = D + D / 16 floats (pad)
constexpr int DP = D + D / 16;
constexpr int F_PSI = 0, F_LAM = 2 * DP, F_SCR = 4 * DP;

// grid: samples looped; block 256.  x (B, 12) angles, w (G, L, 12, 2) (group of sample s = s / wgroup; wgroup 0:
// one group), img from prep_kernel, E (B, 12), psave (B, 2, 4096) or null.
__global__ void __launch_bounds__(NT, 2) fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                    const h8* __restrict__ img, float* __restrict__ E, int B, int L,
                                                    int wgroup, float* __restrict__ psave) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* pr = sm + F_PSI;
  float* pi = pr + DP;
  float* red = sm + 2 * DP;                            // 4 waves x 12
  cf* tab = reinterpret_cast<cf*>(sm + 2 * DP + 64);   // 48 complex
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  for (int s = blockIdx.x; s < B; s += gridDim.x) {
    const int grp = wgroup > 0 ? s / wgroup : 0;
    const float* wg = w + (size_t)grp * L * 2 * N;
    float xs[N];
#pragma unroll
    for (int q = 0; q < N; ++q) xs[q] = x[(size_t)s * N + q];
    layer0(pr, pi, tab, xs, wg, tid);
    __syncthreads();
    for (int l = 1; l < L; ++l) {
      const h8* li = img + ((size_t)grp * (L - 1) + (l - 1)) * LAYER_H8;
      const Op a0 = load_op(li + (0 * 2 + 0) * IMG_H8, lane);
      const Op a1 = load_op(li + (1 * 2 + 0) * IMG_H8, lane);
      const Op a2 = load_op(li + (2 * 2 + 0) * IMG_H8, lane);
      mode_apply<0, false>(pr, pi, a0, wv, lane);
      __syncthreads();
      mode_apply<1, false>(pr, pi, a1, wv, lane);
      __syncthreads();
      mode_apply<2, true>(pr, pi, a2, wv, lane);
      __syncthreads();
    }
    // <Z_q>: thread tid owns k = tid + 256 i, so bit q < 8 of k is bit q of tid, bit q >= 8 is bit q - 8 of i
    float ptot = 0.f, ph[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < D / NT; ++i) {
      const int k = tid + NT * i;
      const float re = pr[pad(k)], im = pi[pad(k)];
      const float p = re * re + im * im;
      ptot += p;
#pragma unroll
      for (int b = 0; b < 4; ++b) ph[b] += ((i >> b) & 1) ? -p : p;
      if (psave != nullptr) {
        psave[(size_t)s * 2 * D + k] = re;
        psave[(size_t)s * 2 * D + D + k] = im;
      }
    }
#pragma unroll
    for (int q = 0; q < N; ++q) {
      float v = q < 8 ? (((tid >> q) & 1) ? -ptot : ptot) : ph[q - 8];
      v = wave_sum(v);
      if (lane == 0) red[wv * N + q] = v;
    }
    __syncthreads();
    if (tid < N) E[(size_t)s * N + tid] = (red[tid] + red[N + tid]) + (red[2 * N + tid] + red[3 * N + tid]);
    __syncthreads();   // (the next sample rewrites the planes and red)
  }
}

// C_M partial of this wave: K steps ks = 4 wv .. 4 wv + 3 (16 other-indices o each) of
//   Cr[alpha][beta] = sum_o lr[o,alpha] pr[o,beta] + li[o,alpha] pi[o,beta],
//   Ci[alpha][beta] = sum_o lr[o,alpha] pi[o,beta] - li[o,alpha] pr[o,beta]
// A operand (lambda): lane (alpha, g) slot k = 8 g + j = plane g >> 1 at o = 16 ks + 8 (g & 1) + j; B operands (psi):
// lane (beta, g) the same slots of psi (-> Cr) and of (pi, -pr) (-> Ci).
template <int M>
__device__ __forceinline__ void cross_partial(const float* pr, const float* pi, const float* lr, const float* li,
                                              int wv, int lane, f4& cr, f4& ci) {
  const int jj = lane & 15, gq = lane >> 4;
  const f4 z = {0.f, 0.f, 0.f, 0.f};
  cr = z;
  ci = z;
  f4 crc = z, cic = z;
  const float* la = (gq >> 1) ? li : lr;
  const float* pb = (gq >> 1) ? pi : pr;   // -> Cr
  const float* qb = (gq >> 1) ? pr : pi;   // -> Ci (negated for the im half)
  const float sq = (gq >> 1) ? -1.f : 1.f;
#pragma unroll 1
  for (int kt = 0; kt < 4; ++kt) {
    const int o0 = (wv * 4 + kt) * 16 + 8 * (gq & 1);
    h8 ah, al, bh, bl, ch, cl;
    float va[8], vb[8], vc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int ka = pad(sidx<M>(o0 + j, jj));   // (alpha = jj for the A operand, beta = jj for the B operands)
      va[j] = la[ka];
      vb[j] = pb[ka];
      vc[j] = sq * qb[ka];
    }
    split8(va, ah, al);
    split8(vb, bh, bl);
    split8(vc, ch, cl);
    cr = mfma(ah, bh, cr);
    crc = mfma(al, bh, mfma(ah, bl, crc));
    ci = mfma(ah, ch, ci);
    cic = mfma(al, ch, mfma(ah, cl, cic));
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    cr[r] += crc[r] * LO_INV;
    ci[r] += cic[r] * LO_INV;
  }
}

// grid = slab rows; block 256.  gE (B, 12) = dL/dE; dx (B, 12); slab (gridDim.x, 2 n L); psave from fwd_kernel.
__global__ void __launch_bounds__(NT, 2) bwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                    const h8* __restrict__ img, const float* __restrict__ gE,
                                                    float* __restrict__ dx, float* __restrict__ slab, int B, int L,
                                                    int wgroup, const float* __restrict__ psave) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* pr = sm + F_PSI;
  float* pi = pr + DP;
  float* lr = sm + F_LAM;
  float* li = lr + DP;
  float* scr = sm + F_SCR;             // 4 waves x {Cr, Ci} x 256
  float* rho = scr + 4 * 2 * 256;      // 3 modes x 4 qubits x (x, y) 4 x {re, im}
  float* acc = rho + 96;               // 2 n L <= 192
  const int P = 2 * N * L;
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  for (int p = tid; p < P; p += NT) acc[p] = 0.f;
  for (int s = blockIdx.x; s < B; s += gridDim.x) {
    const int grp = wgroup > 0 ? s / wgroup : 0;
    const float* wg = w + (size_t)grp * L * 2 * N;
    float g[N];
#pragma unroll
    for (int q = 0; q < N; ++q) g[q] = gE[(size_t)s * N + q];
    // psi = the forward's final state; lambda = (sum_q g_q Z_q) psi
#pragma unroll 4
    for (int i = 0; i < D / NT; ++i) {
      const int k = tid + NT * i;
      const float a = psave[(size_t)s * 2 * D + k], b = psave[(size_t)s * 2 * D + D + k];
      float o = 0.f;
#pragma unroll
      for (int q = 0; q < N; ++q) o += ((k >> q) & 1) ? -g[q] : g[q];
      pr[pad(k)] = a;
      pi[pad(k)] = b;
      lr[pad(k)] = o * a;
      li[pad(k)] = o * b;
    }
    __syncthreads();
    for (int l = L - 1; l >= 0; --l) {
      // undo the ring: state[k] <- state[f(k)]
      {
        float v[4][D / NT];
#pragma unroll
        for (int i = 0; i < D / NT; ++i) {
          const int j = pad(ring_fwd(tid + NT * i));
          v[0][i] = pr[j];
          v[1][i] = pi[j];
          v[2][i] = lr[j];
          v[3][i] = li[j];
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < D / NT; ++i) {
          const int k = pad(tid + NT * i);
          pr[k] = v[0][i];
          pi[k] = v[1][i];
          lr[k] = v[2][i];
          li[k] = v[3][i];
        }
        __syncthreads();
      }
      // the layer's gradients from the cross densities of its output states, one mode at a time
      static_for<0, 3>([&](auto mc) {
        constexpr int M = decltype(mc)::value;
        f4 cr, ci;
        cross_partial<M>(pr, pi, lr, li, wv, lane, cr, ci);
        const int jj = lane & 15, gq = lane >> 4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {   // partial tile [alpha = 4 gq + r][beta = jj]
          scr[(wv * 2 + 0) * 256 + (4 * gq + r) * 16 + jj] = cr[r];
          scr[(wv * 2 + 1) * 256 + (4 * gq + r) * 16 + jj] = ci[r];
        }
        __syncthreads();
        if (tid < 32) {   // rho[M][ql][x][y][c] = sum over the other 3 bits and the 4 waves (fixed order)
          const int ql = tid >> 3, xy = (tid >> 1) & 3, c = tid & 1;
          const int xb = xy >> 1, yb = xy & 1;
          float t = 0.f;
#pragma unroll
          for (int o3 = 0; o3 < 8; ++o3) {
            const int lo = o3 & ((1 << ql) - 1), hi = (o3 >> ql) << (ql + 1);
            const int al = hi | (xb << ql) | lo, be = hi | (yb << ql) | lo;
#pragma unroll
            for (int ww = 0; ww < 4; ++ww) t += scr[(ww * 2 + c) * 256 + al * 16 + be];
          }
          rho[((M * 4 + ql) * 4 + xy) * 2 + c] = t;
        }
        __syncthreads();
      });
      if (tid < N) {
        const int q = tid;
        const float* rq = rho + q * 8;   // (x, y) = 00, 01, 10, 11 x {re, im}
        float sp, cp;
        __sincosf(wg[2 * N * l + 2 * q + 1], &sp, &cp);   // e^{i phi}
        const float dphi = rq[1] - rq[7];
        // Re(e^{i phi} rho_10) - Re(e^{-i phi} rho_01)
        const float dth = (cp * rq[4] - sp * rq[5]) - (cp * rq[2] + sp * rq[3]);
        acc[(l * N + q) * 2] += dth;
        acc[(l * N + q) * 2 + 1] += dphi;
        if (l == 0) dx[(size_t)s * N + q] = dth;
      }
      if (l > 0) {
        const h8* lm = img + ((size_t)grp * (L - 1) + (l - 1)) * LAYER_H8;
        const Op a0 = load_op(lm + (0 * 2 + 1) * IMG_H8, lane);
        mode_apply<0, false>(pr, pi, a0, wv, lane);
        mode_apply<0, false>(lr, li, a0, wv, lane);
        __syncthreads();
        const Op a1 = load_op(lm + (1 * 2 + 1) * IMG_H8, lane);
        mode_apply<1, false>(pr, pi, a1, wv, lane);
        mode_apply<1, false>(lr, li, a1, wv, lane);
        __syncthreads();
        const Op a2 = load_op(lm + (2 * 2 + 1) * IMG_H8, lane);
        mode_apply<2, false>(pr, pi, a2, wv, lane);
        mode_apply<2, false>(lr, li, a2, wv, lane);
        __syncthreads();
      }
    }
    __syncthreads();   // (acc / the planes before the next sample)
  }
  for (int p = tid; p < P; p += NT) slab[(size_t)blockIdx.x * P + p] = acc[p];
}

// ---------------------------------------------------------------------------------------------------------------
// 8 qubits: the adjoint backward of the flagship's circuit (its forward is csrc/hip/qsim_mfma.hip) in the same
// formulation with two modes, X[b][a] (k = b << 4 | a), ONE WAVE PER SAMPLE (a mode product or a cross density
// is a single 16 x 16 tile): per layer in reverse the ring undone through the wave's LDS planes, C_0 and C_1 (one
// K step each, 6 MFMAs), the 16 gate gradients from their partial traces, and psi, lambda <- U^dagger (two mode
// products each).  Replaces qsim.hip's register-resident VALU adjoint (qsim_bwd_kernel<8>); same contract as
// qd_qsim_bwd_saved: psave in qsim.hip's layout (written by either forward), one slab row per wave.
// ---------------------------------------------------------------------------------------------------------------
namespace k8 {
constexpr int N8 = 8, D8 = 256;
constexpr int DP8 = D8 + D8 / 16;           // padded plane (pad)
constexpr int WAVE_F = 4 * DP8 + 4 * D8 + 64 + 128;   // per-wave LDS floats: psi / lambda planes, C_0 / C_1, rho, acc
template <int M>
__device__ __forceinline__ int sidx8(int o, int e) {
  if constexpr (M == 0) return (o << 4) | e;
  else return (e << 4) | o;
}
__device__ __forceinline__ int ring8(int k) {
#pragma unroll
  for (int i = 0; i < N8 - 1; ++i) k ^= ((k >> i) & 1) << (i + 1);
  k ^= (k >> (N8 - 1)) & 1;
  return k;
}
// psi <- A psi along mode M (in place: the wave's one tile)
template <int M>
__device__ __forceinline__ void mode8(float* pr, float* pi, const Op& A, int lane) {
  const int jj = lane & 15, gq = lane >> 4;
  const f4 z = {0.f, 0.f, 0.f, 0.f};
  const float* pl = (gq >> 1) ? pi : pr;
  h8 bh, bl;
  float vv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) vv[j] = pl[pad(sidx8<M>(jj, 8 * (gq & 1) + j))];
  split8(vv, bh, bl);
  const f4 rc = mfma(A.rl, bh, mfma(A.rh, bl, z));
  const f4 ic = mfma(A.il, bh, mfma(A.ih, bl, z));
  f4 yr = mfma(A.rh, bh, z), yi = mfma(A.ih, bh, z);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int k = pad(sidx8<M>(jj, 4 * gq + r));
    pr[k] = yr[r] + rc[r] * LO_INV;
    pi[k] = yi[r] + ic[r] * LO_INV;
  }
}
// C_M = sum_o conj(lambda[o, alpha]) psi[o, beta] -> c (Cr at +0, Ci at +256, [alpha][beta])
template <int M>
__device__ __forceinline__ void cross8(const float* pr, const float* pi, const float* lr, const float* li, float* c,
                                       int lane) {
  const int jj = lane & 15, gq = lane >> 4;
  const f4 z = {0.f, 0.f, 0.f, 0.f};
  const float* la = (gq >> 1) ? li : lr;
  const float* pb = (gq >> 1) ? pi : pr;
  const float* qb = (gq >> 1) ? pr : pi;
  const float sq = (gq >> 1) ? -1.f : 1.f;
  h8 ah, al, bh, bl, ch, cl;
  float va[8], vb[8], vc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = pad(sidx8<M>(8 * (gq & 1) + j, jj));
    va[j] = la[k];
    vb[j] = pb[k];
    vc[j] = sq * qb[k];
  }
  split8(va, ah, al);
  split8(vb, bh, bl);
  split8(vc, ch, cl);
  const f4 crc = mfma(al, bh, mfma(ah, bl, z)), cic = mfma(al, ch, mfma(ah, cl, z));
  const f4 cr = mfma(ah, bh, z), ci = mfma(ah, ch, z);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    c[(4 * gq + r) * 16 + jj] = cr[r] + crc[r] * LO_INV;
    c[256 + (4 * gq + r) * 16 + jj] = ci[r] + cic[r] * LO_INV;
  }
}

// block 256 = 4 waves; global wave gw < rows takes samples gw, gw + rows, ... and writes slab row gw.
__global__ void __launch_bounds__(256) bwd8_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                   const h8* __restrict__ img, const float* __restrict__ gE,
                                                   float* __restrict__ dx, float* __restrict__ slab, int B, int L,
                                                   int wgroup, const cf* __restrict__ psave, int rows) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int gw = blockIdx.x * 4 + wv;
  if (gw >= rows) return;   // (whole wave; the kernel has no workgroup barrier)
  float* base = sm + wv * WAVE_F;
  float *pr = base, *pi = base + DP8, *lr = base + 2 * DP8, *li = base + 3 * DP8;
  float* cm = base + 4 * DP8;           // C_0 (512) | C_1 (512)
  float* rho = cm + 4 * D8;             // 64
  float* acc = rho + 64;                // 2 n L <= 128
  const int P = 2 * N8 * L;
  for (int p = lane; p < P; p += 64) acc[p] = 0.f;
  for (int s = gw; s < B; s += rows) {
    const int grp = wgroup > 0 ? s / wgroup : 0;
    const float* wg = w + (size_t)grp * L * 2 * N8;
    float g[N8];
#pragma unroll
    for (int q = 0; q < N8; ++q) g[q] = gE[(size_t)s * N8 + q];
    // psi_final in qsim.hip's layout: element r * 64 + lane is amplitude k = r | lane << 2
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = r | (lane << 2);
      const cf v = psave[(size_t)s * D8 + r * 64 + lane];
      float o = 0.f;
#pragma unroll
      for (int q = 0; q < N8; ++q) o += ((k >> q) & 1) ? -g[q] : g[q];
      pr[pad(k)] = v.x;
      pi[pad(k)] = v.y;
      lr[pad(k)] = o * v.x;
      li[pad(k)] = o * v.y;
    }
    wave_lds_fence();
    // (round 6: every global load of the layer loop issued ahead of its use -- the gate angles of all layers here,
    // each layer's two operand images at the layer's top, behind the ring / cross-density work; loaded where
    // they were used, each was one exposed round trip, seven per sample at L = 3)
    float th[8];
    if (lane < N8) {
#pragma unroll
      for (int l = 0; l < 8; ++l) th[l] = l < L ? wg[2 * N8 * l + 2 * lane + 1] : 0.f;
    }
    for (int l = L - 1; l >= 0; --l) {
      Op a0, a1;
      if (l > 0) {
        const h8* lm = img + ((size_t)grp * (L - 1) + (l - 1)) * (2 * 2 * IMG_H8);
        a0 = load_op(lm + (0 * 2 + 1) * IMG_H8, lane);
        a1 = load_op(lm + (1 * 2 + 1) * IMG_H8, lane);
      }
      float v[4][4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = pad(ring8(lane + 64 * r));
        v[0][r] = pr[j];
        v[1][r] = pi[j];
        v[2][r] = lr[j];
        v[3][r] = li[j];
      }
      wave_lds_fence();
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = pad(lane + 64 * r);
        pr[k] = v[0][r];
        pi[k] = v[1][r];
        lr[k] = v[2][r];
        li[k] = v[3][r];
      }
      wave_lds_fence();
      cross8<0>(pr, pi, lr, li, cm, lane);
      cross8<1>(pr, pi, lr, li, cm + 512, lane);
      wave_lds_fence();
      {   // rho[m][ql][xy][c]: lane = m * 32 + ql * 8 + xy * 2 + c
        const int m = lane >> 5, ql = (lane >> 3) & 3, xy = (lane >> 1) & 3, c = lane & 1;
        const int xb = xy >> 1, yb = xy & 1;
        const float* cc = cm + m * 512 + c * 256;
        float t = 0.f;
#pragma unroll
        for (int o3 = 0; o3 < 8; ++o3) {
          const int lo = o3 & ((1 << ql) - 1), hi = (o3 >> ql) << (ql + 1);
          t += cc[(hi | (xb << ql) | lo) * 16 + (hi | (yb << ql) | lo)];
        }
        rho[lane] = t;
      }
      wave_lds_fence();
      if (lane < N8) {
        const int q = lane;
        const float* rq = rho + q * 8;
        float sp, cp, t = th[0];
#pragma unroll
        for (int k = 1; k < 8; ++k) t = l == k ? th[k] : t;   // (static register index: no scratch)
        __sincosf(t, &sp, &cp);
        const float dphi = rq[1] - rq[7];
        const float dth = (cp * rq[4] - sp * rq[5]) - (cp * rq[2] + sp * rq[3]);
        acc[(l * N8 + q) * 2] += dth;
        acc[(l * N8 + q) * 2 + 1] += dphi;
        if (l == 0) dx[(size_t)s * N8 + q] = dth;
      }
      wave_lds_fence();
      if (l > 0) {
        mode8<0>(pr, pi, a0, lane);
        mode8<0>(lr, li, a0, lane);
        wave_lds_fence();
        mode8<1>(pr, pi, a1, lane);
        mode8<1>(lr, li, a1, lane);
        wave_lds_fence();
      }
    }
  }
  for (int p = lane; p < P; p += 64) slab[(size_t)gw * P + p] = acc[p];
}
}  // namespace k8

constexpr size_t FWD_SMEM = (2 * DP + 64 + 2 * 48) * sizeof(float);
constexpr size_t BWD_SMEM = (4 * DP + 4 * 2 * 256 + 96 + 192) * sizeof(float);

}  // namespace qm12
}  // namespace qd

using namespace qd::qm12;

// bytes of the operand-image workspace for G weight groups and L layers
QD_API long long qd_qsim_mfma12_workspace(int G, int L) {
  return (long long)(G < 1 ? 1 : G) * (L > 1 ? L - 1 : 0) * LAYER_H8 * (long long)sizeof(h8);
}

// The same contract as qd_qsim_big_fwd at n = 12 (ws = the qd_qsim_mfma12_workspace images, rebuilt here from w;
// psave (B, 2, 4096) fp32 for qd_qsim_mfma12_bwd).  grid: one workgroup per sample up to 512.
QD_API int qd_qsim_mfma12_fwd(const float* x, const float* w, float* E, int B, int n, int L, int wgroup, void* ws,
                              void* psave, void* stream) {
  if (wgroup > 0 && B % wgroup != 0) return (int)hipErrorInvalidValue;   // (G = B / wgroup weight groups, workspace)
  if (B < 1 || n != N || L < 1 || L > 8 || (L > 1 && ws == nullptr)) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const int G = wgroup > 0 ? (B + wgroup - 1) / wgroup : 1;
  if (L > 1) {
    hipLaunchKernelGGL(prep_kernel<N>, dim3(G, L - 1), dim3(64), 0, st, w, (h8*)ws, L);
    if (hipError_t e = hipGetLastError()) return (int)e;
  }
  if (hipError_t e = qd::allow_lds(fwd_kernel, FWD_SMEM)) return (int)e;
  const int grid = B < 512 ? B : 512;
  hipLaunchKernelGGL(fwd_kernel, dim3(grid), dim3(NT), FWD_SMEM, st, x, w, (const h8*)ws, E, B, L, wgroup,
                     (float*)psave);
  return (int)hipGetLastError();
}

// The same contract as qd_qsim_big_bwd at n = 12: dx (B, 12), slab (qd_qsim_big_grid(B), 2 n L) rows; ws / psave
// as the forward left them (same x, w).
QD_API int qd_qsim_mfma12_bwd(const float* x, const float* w, const float* gE, float* dx, float* slab, int B, int n,
                              int L, int wgroup, void* ws, void* psave, void* stream) {
  if (wgroup > 0 && B % wgroup != 0) return (int)hipErrorInvalidValue;   // (G = B / wgroup weight groups, workspace)
  if (B < 1 || n != N || L < 1 || L > 8 || psave == nullptr || (L > 1 && ws == nullptr)) return (int)hipErrorInvalidValue;
  if (hipError_t e = qd::allow_lds(bwd_kernel, BWD_SMEM)) return (int)e;
  const int grid = B < 512 ? B : 512;   // = qd_qsim_big_grid(B): the slab rows the caller sums
  hipLaunchKernelGGL(bwd_kernel, dim3(grid), dim3(NT), BWD_SMEM, (hipStream_t)stream, x, w, (const h8*)ws, gE, dx,
                     slab, B, L, wgroup, (const float*)psave);
  return (int)hipGetLastError();
}

// bytes of the 8-qubit adjoint's operand images (2 modes x {forward, adjoint} per (group, layer >= 1))
QD_API long long qd_qsim_mfma8_workspace(int G, int L) {
  return (long long)(G < 1 ? 1 : G) * (L > 1 ? L - 1 : 0) * (2 * 2 * IMG_H8) * (long long)sizeof(h8);
}

// The 8-qubit adjoint backward on the matrix cores: the contract of qd_qsim_bwd_saved (psave = the forward's
// final states in qsim.hip's layout, dx (B, 8), slab rows = qd_qsim_bwd_grid(8, B)) plus ws for the operand
// images, rebuilt here from w.
QD_API int qd_qsim_mfma8_bwd(const float* x, const float* w, const float* gE, float* dx, float* slab, int B, int n,
                             int L, int wgroup, void* ws, const void* psave, void* stream) {
  if (wgroup > 0 && B % wgroup != 0) return (int)hipErrorInvalidValue;   // (G = B / wgroup weight groups, workspace)
  if (B < 1 || n != 8 || L < 1 || L > 8 || psave == nullptr || (L > 1 && ws == nullptr)) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (L > 1) {
    const int G = wgroup > 0 ? (B + wgroup - 1) / wgroup : 1;
    hipLaunchKernelGGL(prep_kernel<8>, dim3(G, L - 1), dim3(64), 0, st, w, (h8*)ws, L);
    if (hipError_t e = hipGetLastError()) return (int)e;
  }
  const int rows = B < 4096 ? B : 4096;   // = qd_qsim_bwd_grid(8, B)
  const size_t smem = 4 * k8::WAVE_F * sizeof(float);
  hipLaunchKernelGGL(k8::bwd8_kernel, dim3((rows + 3) / 4), dim3(256), smem, st, x, w, (const h8*)ws, gE, dx, slab, B,
                     L, wgroup, (const cf*)psave, rows);
  return (int)hipGetLastError();
}
