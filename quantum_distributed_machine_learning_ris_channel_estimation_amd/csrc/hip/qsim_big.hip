// Batched VQC simulator for LARGE qubit counts (n = 11 .. 16): one workgroup per sample.
//
// Same circuit and adjoint method as csrc/hip/qsim.hip (reference E:125-142); that kernel keeps a
// sample's state in one wave's registers, which stops at n = 10 (16 amplitudes per lane).  Here a
// 512-thread workgroup owns a sample and applies the gates as passes over the state:
//   * state in LDS when it fits (forward: 2 buffers, backward: 4 buffers of 2^n complex fp32 --
//     n <= 12 backward / n <= 13 forward), otherwise in a per-workgroup HBM workspace (n = 16:
//     512 KiB per state; at one workgroup per CU the working set is L2/MALL-resident);
//   * one pass per fused RZ.RY wire rotation (amplitude pairs, no divergence), one gather pass per
//     CNOT ring (ping-pong buffers: the ring is a GF(2)-linear basis permutation);
//   * adjoint backward: each gate's two parameter-gradient partials are block-reduced as part of
//     the pass barrier; layer-0 RY gradients are the per-sample d(angles), the weight gradients are
//     accumulated over the workgroup's samples and written as one slab row per workgroup.
#include "common.h"

namespace qd {
namespace qsimbig {

struct cf {
  float x, y;
};
__device__ __forceinline__ cf cmul(cf a, cf b) { return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }

constexpr int NT = 512;
constexpr int NW = NT / 64;

__device__ __forceinline__ int ring_fwd(int k, int n) {
  for (int i = 0; i < n - 1; ++i) k ^= ((k >> i) & 1) << (i + 1);
  k ^= (k >> (n - 1)) & 1;
  return k;
}
__device__ __forceinline__ int ring_inv(int k, int n) {
  k ^= (k >> (n - 1)) & 1;
  for (int i = n - 2; i >= 0; --i) k ^= ((k >> i) & 1) << (i + 1);
  return k;
}
// insert a zero bit at position q
__device__ __forceinline__ int ins0(int p, int q) { return ((p >> q) << (q + 1)) | (p & ((1 << q) - 1)); }

// Block-wide sum of two values; every thread gets the result.  red: >= 2*NW floats.
__device__ __forceinline__ float2 block_sum2(float a, float b, float* red) {
  a = wave_sum(a);
  b = wave_sum(b);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[2 * w] = a;
    red[2 * w + 1] = b;
  }
  __syncthreads();
  float2 r = {0.f, 0.f};
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    r.x += red[2 * i];
    r.y += red[2 * i + 1];
  }
  __syncthreads();
  return r;
}

__device__ void product_state(cf* s, const float* xs, const float* w, int n, float* cs) {
  // cs: 4n floats of LDS: (ch, sh, cp, sp) per wire
  for (int q = threadIdx.x; q < n; q += NT) {
    float sh, ch, sp, cp;
    __sincosf(0.5f * (xs[q] + w[2 * q]), &sh, &ch);
    __sincosf(0.5f * w[2 * q + 1], &sp, &cp);
    cs[4 * q] = ch;
    cs[4 * q + 1] = sh;
    cs[4 * q + 2] = cp;
    cs[4 * q + 3] = sp;
  }
  __syncthreads();
  const int D = 1 << n;
  for (int k = threadIdx.x; k < D; k += NT) {
    cf a = {1.f, 0.f};
    for (int q = 0; q < n; ++q) {
      const float* c = cs + 4 * q;
      const bool b = (k >> q) & 1;
      const cf f = b ? cf{c[1] * c[2], c[1] * c[3]} : cf{c[0] * c[2], -c[0] * c[3]};
      a = cmul(a, f);
    }
    s[k] = a;
  }
  __syncthreads();
}

// dst[j] = src[f^-1(j)] (forward ring) or src[f(j)] (inverse)
__device__ __forceinline__ void permute(const cf* src, cf* dst, int n, bool inverse) {
  const int D = 1 << n;
  for (int j = threadIdx.x; j < D; j += NT) dst[j] = src[inverse ? ring_fwd(j, n) : ring_inv(j, n)];
  __syncthreads();
}

__device__ __forceinline__ void rotate(cf* s, int n, int q, float theta, float phi) {
  float sn, c, sp, cp;
  __sincosf(0.5f * theta, &sn, &c);
  __sincosf(0.5f * phi, &sp, &cp);
  const int half = 1 << (n - 1);
  for (int p = threadIdx.x; p < half; p += NT) {
    const int k0 = ins0(p, q), k1 = k0 | (1 << q);
    const cf a0 = s[k0], a1 = s[k1];
    s[k0] = cmul(cf{c * a0.x - sn * a1.x, c * a0.y - sn * a1.y}, cf{cp, -sp});
    s[k1] = cmul(cf{sn * a0.x + c * a1.x, sn * a0.y + c * a1.y}, cf{cp, sp});
  }
  __syncthreads();
}

// Forward circuit; returns the buffer holding psi_final (a or b).
__device__ cf* run_circuit(cf* a, cf* b, const float* xs, const float* w, int n, int L, float* cs) {
  product_state(a, xs, w, n, cs);
  permute(a, b, n, false);
  cf* cur = b;
  cf* oth = a;
  for (int l = 1; l < L; ++l) {
    for (int q = 0; q < n; ++q) rotate(cur, n, q, w[2 * (l * n + q)], w[2 * (l * n + q) + 1]);
    permute(cur, oth, n, false);
    cf* t = cur;
    cur = oth;
    oth = t;
  }
  return cur;
}

__global__ void __launch_bounds__(NT) qsim_big_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                          float* __restrict__ E, int B, int n, int L, int wgroup,
                                                          cf* __restrict__ ws, int use_lds) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* red = reinterpret_cast<float*>(smem);            // 64 floats
  float* cs = red + 64;                                   // 64 floats
  const int D = 1 << n;
  cf* a = use_lds ? reinterpret_cast<cf*>(smem + 512) : ws + (size_t)blockIdx.x * 2 * D;
  cf* b = a + D;
  for (int s = blockIdx.x; s < B; s += gridDim.x) {
    const float* ws_ = w + (wgroup > 0 ? (size_t)(s / wgroup) * 2 * n * L : 0);
    cf* psi = run_circuit(a, b, x + (size_t)s * n, ws_, n, L, cs);
    float part[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) part[q] = 0.f;
    for (int k = threadIdx.x; k < D; k += NT) {
      const float p = psi[k].x * psi[k].x + psi[k].y * psi[k].y;
#pragma unroll
      for (int q = 0; q < 16; ++q) part[q] += ((k >> q) & 1) ? -p : p;
    }
#pragma unroll
    for (int q = 0; q < 16; q += 2) {  // constant indices keep part[] in registers
      if (q < n) {                      // uniform branch: every thread reaches the barrier
        const float2 r = block_sum2(part[q], part[q + 1], red);
        if (threadIdx.x == 0) {
          E[(size_t)s * n + q] = r.x;
          if (q + 1 < n) E[(size_t)s * n + q + 1] = r.y;
        }
      }
    }
  }
}

// slab: (gridDim.x, 2*n*L) partial weight grads; dx: (B, n)
__global__ void __launch_bounds__(NT) qsim_big_bwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                          const float* __restrict__ gE, float* __restrict__ dx,
                                                          float* __restrict__ slab, int B, int n, int L, int wgroup,
                                                          cf* __restrict__ ws, int use_lds) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* red = reinterpret_cast<float*>(smem);            // 64
  float* cs = red + 64;                                   // 64
  float* acc = red + 128;                                 // 2*n*L <= 256 (weight grads)
  float* gq = red + 384;                                  // n <= 16 output cotangents
  const int D = 1 << n;
  const int P = 2 * n * L;
  cf* base = use_lds ? reinterpret_cast<cf*>(smem + 2048) : ws + (size_t)blockIdx.x * 4 * D;
  cf *pa = base, *pb = base + D, *la = base + 2 * D, *lb = base + 3 * D;
  for (int i = threadIdx.x; i < P; i += NT) acc[i] = 0.f;
  __syncthreads();
  for (int s = blockIdx.x; s < B; s += gridDim.x) {
    const float* wsmp = w + (wgroup > 0 ? (size_t)(s / wgroup) * 2 * n * L : 0);
    const float* xs = x + (size_t)s * n;
    cf* psi = run_circuit(pa, pb, xs, wsmp, n, L, cs);
    cf* psi_o = (psi == pa) ? pb : pa;
    cf* lam = la;
    cf* lam_o = lb;
    // lambda = (sum_q g_q Z_q) psi
    if (threadIdx.x < n) gq[threadIdx.x] = gE[(size_t)s * n + threadIdx.x];
    __syncthreads();
    for (int k = threadIdx.x; k < D; k += NT) {
      float o = 0.f;
      for (int q = 0; q < n; ++q) o += ((k >> q) & 1) ? -gq[q] : gq[q];
      lam[k] = {psi[k].x * o, psi[k].y * o};
    }
    __syncthreads();
    const int half = 1 << (n - 1);
    for (int l = L - 1; l >= 0; --l) {
      permute(psi, psi_o, n, true);
      permute(lam, lam_o, n, true);
      cf* t = psi; psi = psi_o; psi_o = t;
      t = lam; lam = lam_o; lam_o = t;
      for (int q = n - 1; q >= 0; --q) {
        const float theta = wsmp[2 * (l * n + q)] + (l == 0 ? xs[q] : 0.f);
        const float phi = wsmp[2 * (l * n + q) + 1];
        float sn, c, sp, cp;
        __sincosf(0.5f * theta, &sn, &c);
        __sincosf(0.5f * phi, &sp, &cp);
        float dphi = 0.f, dth = 0.f;
        for (int p = threadIdx.x; p < half; p += NT) {
          const int k0 = ins0(p, q), k1 = k0 | (1 << q);
          cf p0 = psi[k0], p1 = psi[k1], l0 = lam[k0], l1 = lam[k1];
          // RZ^dagger with dphi = Im <lam| Z |psi>
          dphi += (l0.x * p0.y - l0.y * p0.x) - (l1.x * p1.y - l1.y * p1.x);
          p0 = cmul(p0, cf{cp, sp}); l0 = cmul(l0, cf{cp, sp});
          p1 = cmul(p1, cf{cp, -sp}); l1 = cmul(l1, cf{cp, -sp});
          // RY^dagger with dtheta = Im <lam| Y |psi>
          dth += -(l0.x * p1.x + l0.y * p1.y) + (l1.x * p0.x + l1.y * p0.y);
          psi[k0] = {c * p0.x + sn * p1.x, c * p0.y + sn * p1.y};
          psi[k1] = {c * p1.x - sn * p0.x, c * p1.y - sn * p0.y};
          lam[k0] = {c * l0.x + sn * l1.x, c * l0.y + sn * l1.y};
          lam[k1] = {c * l1.x - sn * l0.x, c * l1.y - sn * l0.y};
        }
        const float2 r = block_sum2(dth, dphi, red);   // includes the pass barrier
        if (threadIdx.x == 0) {
          acc[2 * (l * n + q)] += r.x;
          acc[2 * (l * n + q) + 1] += r.y;
          if (l == 0) dx[(size_t)s * n + q] = r.x;
        }
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < P; i += NT) slab[(size_t)blockIdx.x * P + i] = acc[i];
}

}  // namespace qsimbig
}  // namespace qd

using namespace qd::qsimbig;

// Workspace (bytes) the large-n kernels need for a given grid when the state does not fit LDS.
static bool fwd_lds(int n) { return 512 + 2 * (size_t(8) << n) <= 160 * 1024; }
static bool bwd_lds(int n) { return 2048 + 4 * (size_t(8) << n) <= 160 * 1024; }

QD_API long long qd_qsim_big_workspace(int n, int grid, int backward) {
  if (backward) return bwd_lds(n) ? 0 : (long long)grid * 4 * (8ll << n);
  return fwd_lds(n) ? 0 : (long long)grid * 2 * (8ll << n);
}

QD_API int qd_qsim_big_grid(int B) { return B < 1024 ? B : 1024; }

QD_API int qd_qsim_big_fwd(const float* x, const float* w, float* E, int B, int n, int L, int wgroup, void* ws,
                           void* stream) {
  if (n < 2 || n > 16 || L < 1 || 2 * n * L > 256) return (int)hipErrorInvalidValue;
  const int grid = qd_qsim_big_grid(B);
  const int lds = fwd_lds(n);
  if (!lds && ws == nullptr) return (int)hipErrorInvalidValue;
  const size_t sm = lds ? 512 + 2 * (size_t(8) << n) : 512;
  if (hipError_t e = qd::allow_lds(qsim_big_fwd_kernel, sm)) return (int)e;
  hipLaunchKernelGGL(qsim_big_fwd_kernel, dim3(grid), dim3(NT), sm, (hipStream_t)stream, x, w, E, B, n, L, wgroup,
                     (cf*)ws, lds);
  return (int)hipGetLastError();
}

QD_API int qd_qsim_big_bwd(const float* x, const float* w, const float* gE, float* dx, float* slab, int B, int n, int L,
                           int wgroup, void* ws, void* stream) {
  if (n < 2 || n > 16 || L < 1 || 2 * n * L > 256) return (int)hipErrorInvalidValue;
  const int grid = qd_qsim_big_grid(B);
  const int lds = bwd_lds(n);
  if (!lds && ws == nullptr) return (int)hipErrorInvalidValue;
  const size_t sm = lds ? 2048 + 4 * (size_t(8) << n) : 2048;
  if (hipError_t e = qd::allow_lds(qsim_big_bwd_kernel, sm)) return (int)e;
  hipLaunchKernelGGL(qsim_big_bwd_kernel, dim3(grid), dim3(NT), sm, (hipStream_t)stream, x, w, gE, dx, slab, B, n, L,
                     wgroup, (cf*)ws, lds);
  return (int)hipGetLastError();
}
