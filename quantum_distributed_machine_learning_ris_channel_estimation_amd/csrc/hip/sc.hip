// Classical scenario classifier SC_P128 on gfx950: forward (training / inference) and backward.
//
// Reference: SC_P128 (Estimators_QuantumNAT_onchipQNN.py:79-101)
//   Conv2d(2, 32, 3, p=1, no bias) -> ReLU -> MaxPool2 -> Conv2d(32, 32, 3, p=1, no bias) -> ReLU
//   -> MaxPool2 -> Flatten (C, H/4, W/4) -> Linear(F, 3) -> log_softmax,
// trained with the mean NLL over the 9 (scenario, user) streams (helpers R:285-302; Test.py:158 runs
// it in eval for the classical routing).  F = 32 * H/4 * W/4 (256 for P128's 16 x 8 grid).
//
// One 256-thread workgroup per group of samples, the whole network per sample in LDS (0.74 MFLOP
// forward per sample: VALU fp32, exact like the reference; no library call anywhere):
//   sc_fwd_kernel  conv1 + ReLU + pool1 (a thread per pooled output: the 4 conv outputs of its window,
//                  the max, its argmax), conv2 + ReLU + pool2 likewise, the linear layer as a block
//                  reduction, log_softmax, NLL, argmax; training also saves the pooled maps, their
//                  argmax codes and dlogits = (softmax - onehot) / B for the backward.
//   sc_bwd_kernel  routes gradients through the saved argmax positions (ReLU: pooled value > 0):
//                  dW_fc, db, dW2 (a thread owns 4 (co, ci) pairs x 9 taps across its samples), dp1 by
//                  the transposed conv2, dW1 (a thread owns one (co, ci, ky) row); every weight
//                  gradient lands in ONE slab row per workgroup in the flat-parameter layout, summed
//                  in a fixed order afterwards (deterministic, no float atomics).
//   sc_finish      loss = sum of per-workgroup NLL partials / B, correct count, NaN-guard flag.
// ReLU(max(window)) = max(ReLU(window)), so a window's gradient goes to its first maximal position
// (PyTorch's max_pool2d tie rule) when the pooled value is positive, else nowhere.
#include "common.h"

namespace qd {
namespace sc {

constexpr int NT = 256;
constexpr int C = 32;          // channels of both convolutions
constexpr int NCLS = 3;

template <int H, int W>
struct G {
  static constexpr int XP = (H + 2) * (W + 2);           // padded input plane
  static constexpr int H2 = H / 2, W2 = W / 2, HW2 = H2 * W2;
  static constexpr int PP = (H2 + 2) * (W2 + 2);         // padded pool-1 plane
  static constexpr int H4 = H / 4, W4 = W / 4, HW4 = H4 * W4;
  static constexpr int F = C * HW4;
  static constexpr int NW1 = C * 2 * 9, NW2 = C * C * 9, NWF = NCLS * F;
  // LDS (floats): W1 | W2 | Wfc | bfc(4) | x (2 XP) | p1 padded (C PP) | p2 (F) | dc2 padded (C PP) | misc
  static constexpr int o_w1 = 0, o_w2 = o_w1 + NW1, o_wf = o_w2 + NW2, o_bf = o_wf + NWF, o_x = o_bf + 4;
  static constexpr int o_p1 = o_x + 2 * XP, o_p2 = o_p1 + C * PP, o_d2 = o_p2 + F, o_misc = o_d2 + C * PP;
  static constexpr int LDS = (o_misc + 64) * 4;
};

// flat-parameter offsets of SC_P128 (FlatParamSpace order: conv1.weight, conv2.weight, FC.weight, FC.bias)
struct Offs {
  int w1, w2, wf, bf;
  int row;   // slab row width (= the flat space's numel)
};

__device__ __forceinline__ void stage(float* dst, const float* __restrict__ src, int n) {
  for (int i = threadIdx.x; i < n; i += NT) dst[i] = src[i];
}

// x (2, H, W) of one sample -> zero-padded planes
template <int H, int W>
__device__ __forceinline__ void load_x(float* xs, const float* __restrict__ x) {
  using g = G<H, W>;
  for (int i = threadIdx.x; i < 2 * g::XP; i += NT) {
    const int c = i / g::XP, r = i % g::XP, y = r / (W + 2) - 1, xx = r % (W + 2) - 1;
    xs[i] = (y >= 0 && y < H && xx >= 0 && xx < W) ? x[(c * H + y) * W + xx] : 0.f;
  }
}

// block reduction of NCLS values per thread -> out[0..NCLS) (thread 0 reads them after the call)
__device__ __forceinline__ void block_sum3(float (&v)[NCLS], float* red) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int c = 0; c < NCLS; ++c) {
    const float s = wave_sum(v[c]);
    if (lane == 0) red[w * 4 + c] = s;
  }
  __syncthreads();
  if (threadIdx.x < NCLS) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NT / 64; ++k) s += red[k * 4 + threadIdx.x];
    red[16 + threadIdx.x] = s;
  }
  __syncthreads();
}

// Forward.  train: saves p1 (B, C*HW2), code1 (B, C*HW2) u8, p2 (B, F), code2 (B, F) u8,
// dlogit (B, 4) and the per-workgroup (NLL sum, correct) partials; logp (B, 3) nullable, pred (B,) nullable.
template <int H, int W>
__global__ void __launch_bounds__(NT) sc_fwd_kernel(const float* __restrict__ x, const float* __restrict__ flat, Offs o,
                                                    const long* __restrict__ labels, int B, int spb, float inv_b,
                                                    float* __restrict__ p1s, uint8_t* __restrict__ c1s,
                                                    float* __restrict__ p2s, uint8_t* __restrict__ c2s,
                                                    float* __restrict__ dlogit, float* __restrict__ part,
                                                    float* __restrict__ logp, long* __restrict__ pred) {
  using g = G<H, W>;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float *w1 = sm + g::o_w1, *w2 = sm + g::o_w2, *wf = sm + g::o_wf, *bf = sm + g::o_bf;
  float *xs = sm + g::o_x, *p1 = sm + g::o_p1, *p2 = sm + g::o_p2, *red = sm + g::o_misc;
  stage(w1, flat + o.w1, g::NW1);
  stage(w2, flat + o.w2, g::NW2);
  stage(wf, flat + o.wf, g::NWF);
  if (threadIdx.x < NCLS) bf[threadIdx.x] = flat[o.bf + threadIdx.x];
  for (int i = threadIdx.x; i < C * g::PP; i += NT) p1[i] = 0.f;   // (pad ring stays zero)
  float nll = 0.f, correct = 0.f;
  const int s0 = blockIdx.x * spb;
  for (int s = s0; s < s0 + spb && s < B; ++s) {
    __syncthreads();
    load_x<H, W>(xs, x + (size_t)s * 2 * H * W);
    __syncthreads();
    // conv1 + ReLU + pool1: thread per pooled output (co, py, px)
    for (int i = threadIdx.x; i < C * g::HW2; i += NT) {
      const int co = i / g::HW2, pp = i % g::HW2, py = pp / g::W2, px = pp % g::W2;
      float best = -INFINITY;
      int code = 0;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int y = 2 * py + (d >> 1), xx = 2 * px + (d & 1);
        float a = 0.f;
#pragma unroll
        for (int ci = 0; ci < 2; ++ci)
#pragma unroll
          for (int k = 0; k < 9; ++k) a += w1[(co * 2 + ci) * 9 + k] * xs[ci * g::XP + (y + k / 3) * (W + 2) + xx + k % 3];
        if (a > best || a != a) {   // (first maximum; NaN propagates)
          best = a;
          code = d;
        }
      }
      const float v = relu_nan(best);
      p1[co * g::PP + (py + 1) * (g::W2 + 2) + px + 1] = v;
      if (p1s) {
        p1s[(size_t)s * C * g::HW2 + i] = v;
        c1s[(size_t)s * C * g::HW2 + i] = (uint8_t)code;
      }
    }
    __syncthreads();
    // conv2 + ReLU + pool2
    for (int i = threadIdx.x; i < g::F; i += NT) {
      const int co = i / g::HW4, pp = i % g::HW4, py = pp / g::W4, px = pp % g::W4;
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
      for (int ci = 0; ci < C; ++ci) {
        // the 4 x 4 input patch of the 2 x 2 window's four 3 x 3 receptive fields
        float pt[16];
        const float* src = p1 + ci * g::PP + (2 * py) * (g::W2 + 2) + 2 * px;
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int c = 0; c < 4; ++c) pt[r * 4 + c] = src[r * (g::W2 + 2) + c];
        const float* wk = w2 + (co * C + ci) * 9;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
          const float wv = wk[k];
          const int ky = k / 3, kx = k % 3;
#pragma unroll
          for (int d = 0; d < 4; ++d) acc[d] += wv * pt[((d >> 1) + ky) * 4 + (d & 1) + kx];
        }
      }
      float best = acc[0];
      int code = 0;
#pragma unroll
      for (int d = 1; d < 4; ++d)
        if (acc[d] > best || (acc[d] != acc[d] && best == best)) {
          best = acc[d];
          code = d;
        }
      const float v = relu_nan(best);
      p2[i] = v;
      if (p2s) {
        p2s[(size_t)s * g::F + i] = v;
        c2s[(size_t)s * g::F + i] = (uint8_t)code;
      }
    }
    __syncthreads();
    // linear layer + log_softmax (+ NLL, dlogits)
    float z[NCLS] = {0.f, 0.f, 0.f};
    for (int f = threadIdx.x; f < g::F; f += NT) {
      const float v = p2[f];
#pragma unroll
      for (int c = 0; c < NCLS; ++c) z[c] += wf[c * g::F + f] * v;
    }
    block_sum3(z, red);
    if (threadIdx.x == 0) {
      float l[NCLS], m = -INFINITY;
#pragma unroll
      for (int c = 0; c < NCLS; ++c) {
        l[c] = red[16 + c] + bf[c];
        m = fmaxf(m, l[c]);
      }
      float se = 0.f;
#pragma unroll
      for (int c = 0; c < NCLS; ++c) se += __expf(l[c] - m);
      const float lse = m + __logf(se);
      int am = 0;
#pragma unroll
      for (int c = 1; c < NCLS; ++c)
        if (l[c] > l[am]) am = c;
      if (logp) {
#pragma unroll
        for (int c = 0; c < NCLS; ++c) logp[(size_t)s * NCLS + c] = l[c] - lse;
      }
      if (pred) pred[s] = am;
      if (labels) {
        const int y = (int)labels[s];
        nll -= l[y] - lse;
        correct += (am == y) ? 1.f : 0.f;
        if (dlogit) {
#pragma unroll
          for (int c = 0; c < NCLS; ++c) dlogit[(size_t)s * 4 + c] = (__expf(l[c] - lse) - (c == y ? 1.f : 0.f)) * inv_b;
        }
      }
    }
  }
  if (part && threadIdx.x == 0) {
    part[blockIdx.x * 2 + 0] = nll;
    part[blockIdx.x * 2 + 1] = correct;
  }
}

// Backward: one slab row per workgroup (flat layout: conv1.weight | conv2.weight | FC.weight | FC.bias
// + its 13 alignment floats, written as zero).
template <int H, int W>
__global__ void __launch_bounds__(NT) sc_bwd_kernel(const float* __restrict__ x, const float* __restrict__ flat, Offs o,
                                                    int B, int spb, const float* __restrict__ p1s,
                                                    const uint8_t* __restrict__ c1s, const float* __restrict__ p2s,
                                                    const uint8_t* __restrict__ c2s, const float* __restrict__ dlogit,
                                                    float* __restrict__ slab) {
  using g = G<H, W>;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  // LDS: W2 | Wfc | x | p1 padded | dc2 padded | dp2 (F) | dc1 (C HW2) | misc
  float* w2 = sm;
  float* wf = w2 + g::NW2;
  float* xs = wf + g::NWF;
  float* p1 = xs + 2 * g::XP;
  float* d2 = p1 + C * g::PP;
  float* dp2 = d2 + C * g::PP;
  float* dc1 = dp2 + g::F;
  float* misc = dc1 + C * g::HW2;
  stage(w2, flat + o.w2, g::NW2);
  stage(wf, flat + o.wf, g::NWF);
  for (int i = threadIdx.x; i < C * g::PP; i += NT) {
    p1[i] = 0.f;
    d2[i] = 0.f;
  }
  constexpr int FR = (g::F + NT - 1) / NT;
  float a2[4][9], a1[3] = {0.f, 0.f, 0.f}, af[FR][NCLS], ab = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int k = 0; k < 9; ++k) a2[r][k] = 0.f;
#pragma unroll
  for (int r = 0; r < FR; ++r)
#pragma unroll
    for (int c = 0; c < NCLS; ++c) af[r][c] = 0.f;
  const int tid = threadIdx.x;
  const int w1_co = tid / 6, w1_ci = (tid / 3) % 2, w1_ky = tid % 3;   // (threads < 192)
  const int s0 = blockIdx.x * spb;
  for (int s = s0; s < s0 + spb && s < B; ++s) {
    __syncthreads();   // (the previous sample's readers are done)
    load_x<H, W>(xs, x + (size_t)s * 2 * H * W);
    for (int i = tid; i < C * g::HW2; i += NT) {
      const int c = i / g::HW2, pp = i % g::HW2, o1 = c * g::PP + (pp / g::W2 + 1) * (g::W2 + 2) + pp % g::W2 + 1;
      p1[o1] = p1s[(size_t)s * C * g::HW2 + i];
      d2[o1] = 0.f;
    }
    if (tid < 4) misc[tid] = dlogit[(size_t)s * 4 + tid];
    __syncthreads();
    const float dl0 = misc[0], dl1 = misc[1], dl2 = misc[2];
    if (tid < NCLS) ab += misc[tid];
    // dp2 (ReLU-masked), dWfc; dc2 at the pool-2 argmax positions of the padded map
#pragma unroll
    for (int r = 0; r < FR; ++r) {
      const int f = tid + NT * r;
      if (f >= g::F) break;
      const float v = p2s[(size_t)s * g::F + f];
      af[r][0] += dl0 * v;
      af[r][1] += dl1 * v;
      af[r][2] += dl2 * v;
      const float d = v > 0.f ? wf[f] * dl0 + wf[g::F + f] * dl1 + wf[2 * g::F + f] * dl2 : 0.f;
      dp2[f] = d;
      const int co = f / g::HW4, pp = f % g::HW4, code = c2s[(size_t)s * g::F + f];
      const int y = 2 * (pp / g::W4) + (code >> 1), xx = 2 * (pp % g::W4) + (code & 1);
      d2[co * g::PP + (y + 1) * (g::W2 + 2) + xx + 1] = d;
    }
    __syncthreads();
    // dW2[co][ci][tap] += dc2 x the p1 patch at each of co's argmax positions
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = tid + NT * r, co = q / C, ci = q % C;
      for (int pp = 0; pp < g::HW4; ++pp) {
        const float d = dp2[co * g::HW4 + pp];
        if (d == 0.f) continue;
        const int code = c2s[(size_t)s * g::F + co * g::HW4 + pp];
        const int y = 2 * (pp / g::W4) + (code >> 1), xx = 2 * (pp % g::W4) + (code & 1);
        const float* src = p1 + ci * g::PP + y * (g::W2 + 2) + xx;
#pragma unroll
        for (int k = 0; k < 9; ++k) a2[r][k] += d * src[(k / 3) * (g::W2 + 2) + k % 3];
      }
    }
    // dp1 = conv2^T(dc2) at every pool-1 output, ReLU-masked -> dc1 (goes to conv1's argmax position)
    for (int i = tid; i < C * g::HW2; i += NT) {
      const int ci = i / g::HW2, pp = i % g::HW2, y = pp / g::W2, xx = pp % g::W2;
      const float pv = p1[ci * g::PP + (y + 1) * (g::W2 + 2) + xx + 1];
      float a = 0.f;
      if (pv > 0.f) {
        for (int co = 0; co < C; ++co) {
          const float* wk = w2 + (co * C + ci) * 9;
          const float* dsrc = d2 + co * g::PP + y * (g::W2 + 2) + xx;   // padded (y + 1 - ky', x + 1 - kx')
#pragma unroll
          for (int k = 0; k < 9; ++k) a += wk[k] * dsrc[(2 - k / 3) * (g::W2 + 2) + 2 - k % 3];
        }
      }
      dc1[i] = a;
    }
    __syncthreads();
    // dW1[co][ci][ky][kx] += dc1 x the input patch at each of co's pool-1 argmax positions
    if (tid < C * 2 * 3) {
      for (int pp = 0; pp < g::HW2; ++pp) {
        const float d = dc1[w1_co * g::HW2 + pp];
        if (d == 0.f) continue;
        const int code = c1s[(size_t)s * C * g::HW2 + w1_co * g::HW2 + pp];
        const int y = 2 * (pp / g::W2) + (code >> 1), xx = 2 * (pp % g::W2) + (code & 1);
        const float* src = xs + w1_ci * g::XP + (y + w1_ky) * (W + 2) + xx;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) a1[kx] += d * src[kx];
      }
    }
  }
  float* row = slab + (size_t)blockIdx.x * o.row;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int q = tid + NT * r;
#pragma unroll
    for (int k = 0; k < 9; ++k) row[o.w2 + q * 9 + k] = a2[r][k];
  }
  if (tid < C * 2 * 3) {
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) row[o.w1 + (w1_co * 2 + w1_ci) * 9 + w1_ky * 3 + kx] = a1[kx];
  }
#pragma unroll
  for (int r = 0; r < FR; ++r) {
    const int f = tid + NT * r;
    if (f < g::F) {
#pragma unroll
      for (int c = 0; c < NCLS; ++c) row[o.wf + c * g::F + f] = af[r][c];
    }
  }
  if (tid < 16) row[o.bf + tid] = tid < NCLS ? ab : 0.f;
}

// loss = sum(part[:, 0]) / B, correct = sum(part[:, 1]) (fixed-order sums); loss_acc += loss; skip
// = (or, skip_add: +=) loss not finite
__global__ void __launch_bounds__(NT) sc_finish_kernel(const float* __restrict__ part, int nblk, float inv_b,
                                                       float* __restrict__ out, float* __restrict__ loss_acc,
                                                       float* __restrict__ skip, int skip_add) {
  __shared__ float red[2 * NT / 64];
  float a = 0.f, c = 0.f;
  for (int k = threadIdx.x; k < nblk; k += NT) {
    a += part[2 * k];
    c += part[2 * k + 1];
  }
  a = wave_sum(a);
  c = wave_sum(c);
  if ((threadIdx.x & 63) == 0) {
    red[2 * (threadIdx.x >> 6)] = a;
    red[2 * (threadIdx.x >> 6) + 1] = c;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float l = 0.f, cc = 0.f;
    for (int w = 0; w < NT / 64; ++w) {
      l += red[2 * w];
      cc += red[2 * w + 1];
    }
    out[0] = l * inv_b;
    out[1] = cc;
    if (loss_acc) *loss_acc += out[0];
    const float bad = isfinite(out[0]) ? 0.f : 1.f;
    if (skip) *skip = skip_add ? *skip + bad : bad;
  }
}

template <int H, int W>
size_t bwd_lds() {
  using g = G<H, W>;
  return sizeof(float) * (g::NW2 + g::NWF + 2 * g::XP + 2 * C * g::PP + g::F + C * g::HW2 + 64);
}

}  // namespace sc
}  // namespace qd

using namespace qd::sc;

// grid (samples per workgroup) chosen by the caller; shapes: (H, W) = (16, 8) P128 or (16, 16) P256.
// Training forward: saved maps + dlogits + per-workgroup (NLL, correct) partials; inference forward:
// logp (B, 3) and/or pred (B,) only (labels nullable: no loss).
QD_API int qd_sc_fwd(const float* x, const float* flat, const int* offs, const long* labels, int B, int spb, int H,
                     int W, float* p1s, uint8_t* c1s, float* p2s, uint8_t* c2s, float* dlogit, float* part,
                     float* logp, long* pred, void* stream) {
  if (spb < 1 || B < 1) return (int)hipErrorInvalidValue;
  Offs o{offs[0], offs[1], offs[2], offs[3], offs[4]};
  const int grid = (B + spb - 1) / spb;
  hipStream_t st = (hipStream_t)stream;
  const float inv_b = 1.f / (float)B;
#define QD_L(HH, WW)                                                                                             \
  {                                                                                                              \
    auto k = &sc_fwd_kernel<HH, WW>;                                                                             \
    const size_t lds = G<HH, WW>::LDS;                                                                           \
    if (qd::allow_lds(k, lds) != hipSuccess) return (int)hipErrorInvalidValue;                                   \
    hipLaunchKernelGGL(k, dim3(grid), dim3(NT), lds, st, x, flat, o, labels, B, spb, inv_b, p1s, c1s,            \
                       p2s, c2s, dlogit, part, logp, pred);                                                      \
  }
  if (H == 16 && W == 8) QD_L(16, 8)
  else if (H == 16 && W == 16) QD_L(16, 16)
  else return (int)hipErrorInvalidValue;
#undef QD_L
  return (int)hipGetLastError();
}

QD_API int qd_sc_bwd(const float* x, const float* flat, const int* offs, int B, int spb, int H, int W, const float* p1s,
                     const uint8_t* c1s, const float* p2s, const uint8_t* c2s, const float* dlogit, float* slab,
                     void* stream) {
  if (spb < 1 || B < 1) return (int)hipErrorInvalidValue;
  Offs o{offs[0], offs[1], offs[2], offs[3], offs[4]};
  const int grid = (B + spb - 1) / spb;
  hipStream_t st = (hipStream_t)stream;
#define QD_L(HH, WW)                                                                                       \
  {                                                                                                        \
    auto k = &sc_bwd_kernel<HH, WW>;                                                                       \
    const size_t lds = bwd_lds<HH, WW>();                                                                  \
    if (qd::allow_lds(k, lds) != hipSuccess) return (int)hipErrorInvalidValue;                                 \
    hipLaunchKernelGGL(k, dim3(grid), dim3(NT), lds, st, x, flat, o, B, spb, p1s, c1s, p2s, c2s, dlogit, slab); \
  }
  if (H == 16 && W == 8) QD_L(16, 8)
  else if (H == 16 && W == 16) QD_L(16, 16)
  else return (int)hipErrorInvalidValue;
#undef QD_L
  return (int)hipGetLastError();
}

QD_API int qd_sc_finish(const float* part, int nblk, int B, float* out, float* loss_acc, float* skip, int skip_add,
                        void* stream) {
  hipLaunchKernelGGL(sc_finish_kernel, dim3(1), dim3(NT), 0, (hipStream_t)stream, part, nblk, 1.f / (float)B, out,
                     loss_acc, skip, skip_add);
  return (int)hipGetLastError();
}
