// Classical parts of the quantum scenario classifier (QSC) as fused per-sample kernels.
//
// Reference: QSC_P128.preprocess (Estimators_QuantumNAT_onchipQNN.py:152-162)
//   Conv2d(2,16,3,p=1) -> ReLU -> MaxPool2 -> Conv2d(16,32,3,p=1) -> ReLU -> MaxPool2 -> Flatten
//   -> Linear(32*H/4*W/4, n) -> Tanh            (angles for the VQC, csrc/hip/qsim.hip)
// and the head (E:165, E:201-203) Linear(n, C) -> log_softmax, trained with nll_loss (R:362).
// In PyTorch these are ~40 small launches (MIOpen convs, pooling, reductions) per step.
//
// MI355X design: one 256-thread workgroup owns a sample at a time, with every activation in
// LDS (the whole per-sample working set is < 40 KB), all weights staged once per workgroup
// in LDS, fp32 VALU math (0.4 MFLOP/sample: matrix cores do not pay at these shapes), and
// weight gradients accumulated in REGISTERS across the workgroup's samples (every thread
// owns a fixed set of weights), written once per workgroup to a slab whose row layout is the
// model's flat gradient layout -> one deterministic column-sum adds it into the flat buffer.
// The backward kernel recomputes the forward activations of its sample instead of storing
// them (cheaper than the HBM round trip).
#include "common.h"

namespace qd {
namespace qsc {

constexpr int C1 = 16, C2 = 32;
constexpr int NT = 256;

template <int H, int W>
struct QGeo {
  static constexpr int HW = H * W;
  static constexpr int H2 = H / 2, W2 = W / 2, HW2 = H2 * W2;  // after pool 1
  static constexpr int H4 = H / 4, W4 = W / 4, HW4 = H4 * W4;  // after pool 2
  static constexpr int F = C2 * HW4;                          // flattened features
};

// Parameter layout of one slab row / the flat gradient (offsets in floats, given by the host):
struct Offs {
  int w1, b1, w2, b2, wl, bl, row;
};

// LDS images (floats)
template <int H, int W>
struct Lds {
  using G = QGeo<H, W>;
  static constexpr int W1 = C1 * 2 * 9, B1 = C1, W2S = C2 * C1 * 9, B2 = C2;
  static constexpr int o_w1 = 0, o_b1 = o_w1 + W1, o_w2 = o_b1 + B1, o_b2 = o_w2 + W2S, o_wl = o_b2 + B2;
  static constexpr int XP = (H + 2) * (W + 2);               // padded input plane
  static constexpr int P1P = (G::H2 + 2) * (G::W2 + 2);      // padded pool-1 plane
  static constexpr int o_x = 0;                              // (relative to activation base)
  static constexpr int o_a1 = o_x + 2 * XP;                  // conv1 pre-activation C1 x HW
  static constexpr int o_p1 = o_a1 + C1 * G::HW;             // pool1 (padded) C1 x P1P
  static constexpr int o_a2 = o_p1 + C1 * P1P;               // conv2 pre-activation C2 x HW2
  static constexpr int o_p2 = o_a2 + C2 * G::HW2;            // pool2 F
  static constexpr int o_red = o_p2 + G::F;                  // reduction scratch: 16 x 4 partials, 16 angles
  static constexpr int o_ang = o_red + 64;
  static constexpr int ACT = o_red + 80;
  // backward scratch
  static constexpr int o_da2 = ACT;                          // C2 x HW2
  static constexpr int o_dp1 = o_da2 + C2 * G::HW2;          // C1 x HW2 (unpadded)
  static constexpr int o_dz1 = o_dp1 + C1 * G::HW2;          // C1 x HW
  static constexpr int o_dz2p = o_dz1 + C1 * G::HW;          // padded dz2 C2 x P1P (for the dgrad)
  static constexpr int o_misc = o_dz2p + C2 * P1P;           // 64 floats: dpre etc.
  static constexpr int o_gwl = o_misc + 64;                  // linear-weight grad accumulators n x F
  static constexpr int BWD = o_gwl;                          // + n * F floats (sized at launch)
};

__device__ __forceinline__ float relu(float v) { return relu_nan(v); }

// ---------------------------------------------------------------------------------------------
// Forward activations of one sample into LDS (all 256 threads).  Returns nothing; angles (tanh)
// land in act[o_red + j] for j < n.
// ---------------------------------------------------------------------------------------------
template <int H, int W>
__device__ void sample_forward(const float* __restrict__ xs, const float* wsm, const float* wl, const float* bl,
                               float* act, int n) {
  using G = QGeo<H, W>;
  using S = Lds<H, W>;
  const int t = threadIdx.x;
  constexpr int WP = W + 2, W2P = G::W2 + 2;
  // input (zero halo preset by the caller)
  for (int i = t; i < 2 * G::HW; i += NT) {
    const int c = i / G::HW, p = i % G::HW;
    act[S::o_x + c * S::XP + (p / W + 1) * WP + p % W + 1] = xs[i];
  }
  __syncthreads();
  // conv1 (+bias), pre-activation: thread = (co, image row), one register-tiled row of W outputs
  for (int i = t; i < C1 * H; i += NT) {
    const int co = i / H, ph = i % H;
    float acc[W];
#pragma unroll
    for (int q = 0; q < W; ++q) acc[q] = wsm[S::o_b1 + co];
#pragma unroll
    for (int ci = 0; ci < 2; ++ci) {
      const float* wk = wsm + S::o_w1 + (co * 2 + ci) * 9;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        float xr[W + 2];
        const float* xp = act + S::o_x + ci * S::XP + (ph + kh) * WP;
#pragma unroll
        for (int q = 0; q < W + 2; ++q) xr[q] = xp[q];
        const float w0 = wk[kh * 3], w1 = wk[kh * 3 + 1], w2 = wk[kh * 3 + 2];
#pragma unroll
        for (int q = 0; q < W; ++q) acc[q] += w0 * xr[q] + w1 * xr[q + 1] + w2 * xr[q + 2];
      }
    }
#pragma unroll
    for (int q = 0; q < W; ++q) act[S::o_a1 + co * G::HW + ph * W + q] = acc[q];
  }
  __syncthreads();
  // relu + maxpool 2x2 -> padded p1
  for (int i = t; i < C1 * G::HW2; i += NT) {
    const int c = i / G::HW2, q = i % G::HW2, qh = q / G::W2, qw = q % G::W2;
    const float* a = act + S::o_a1 + c * G::HW + (2 * qh) * W + 2 * qw;
    const float m = max_nan(max_nan(relu(a[0]), relu(a[1])), max_nan(relu(a[W]), relu(a[W + 1])));
    act[S::o_p1 + c * S::P1P + (qh + 1) * W2P + qw + 1] = m;
  }
  __syncthreads();
  // conv2 (+bias): thread = (co, pooled row), one register-tiled row of W/2 outputs
  for (int i = t; i < C2 * G::H2; i += NT) {
    const int co = i / G::H2, ph = i % G::H2;
    float acc[G::W2];
#pragma unroll
    for (int q = 0; q < G::W2; ++q) acc[q] = wsm[S::o_b2 + co];
    for (int ci = 0; ci < C1; ++ci) {
      const float* wk = wsm + S::o_w2 + (co * C1 + ci) * 9;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        float xr[G::W2 + 2];
        const float* xp = act + S::o_p1 + ci * S::P1P + (ph + kh) * W2P;
#pragma unroll
        for (int q = 0; q < G::W2 + 2; ++q) xr[q] = xp[q];
        const float w0 = wk[kh * 3], w1 = wk[kh * 3 + 1], w2 = wk[kh * 3 + 2];
#pragma unroll
        for (int q = 0; q < G::W2; ++q) acc[q] += w0 * xr[q] + w1 * xr[q + 1] + w2 * xr[q + 2];
      }
    }
#pragma unroll
    for (int q = 0; q < G::W2; ++q) act[S::o_a2 + co * G::HW2 + ph * G::W2 + q] = acc[q];
  }
  __syncthreads();
  // relu + maxpool -> p2 (flatten order c, h, w)
  for (int i = t; i < G::F; i += NT) {
    const int c = i / G::HW4, q = i % G::HW4, qh = q / G::W4, qw = q % G::W4;
    const float* a = act + S::o_a2 + c * G::HW2 + (2 * qh) * G::W2 + 2 * qw;
    act[S::o_p2 + i] = max_nan(max_nan(relu(a[0]), relu(a[1])), max_nan(relu(a[G::W2]), relu(a[G::W2 + 1])));
  }
  __syncthreads();
  // linear F -> n, tanh.  Each wave reduces a strided slice of features for every output.
  const int lane = t & 63, wv = t >> 6;
  for (int j = 0; j < n; ++j) {
    float s = 0.f;
    for (int f = t; f < G::F; f += NT) s += wl[(size_t)j * G::F + f] * act[S::o_p2 + f];
    s = wave_sum(s);
    if (lane == 0) act[S::o_red + j * 4 + wv] = s;
  }
  __syncthreads();
  if (t < n) {
    const float s = act[S::o_red + t * 4] + act[S::o_red + t * 4 + 1] + act[S::o_red + t * 4 + 2] +
                    act[S::o_red + t * 4 + 3] + bl[t];
    act[S::o_ang + t] = tanhf(s);
  }
  __syncthreads();
}

template <int H, int W>
__device__ void stage_weights(const float* __restrict__ flat, Offs o, float* wsm) {
  using S = Lds<H, W>;
  for (int i = threadIdx.x; i < S::W1; i += NT) wsm[S::o_w1 + i] = flat[o.w1 + i];
  for (int i = threadIdx.x; i < S::B1; i += NT) wsm[S::o_b1 + i] = flat[o.b1 + i];
  for (int i = threadIdx.x; i < S::W2S; i += NT) wsm[S::o_w2 + i] = flat[o.w2 + i];
  for (int i = threadIdx.x; i < S::B2; i += NT) wsm[S::o_b2 + i] = flat[o.b2 + i];
}

// angles (B, n) = tanh(preprocess(x)).  grid = min(B, ...), each block loops over samples.
template <int H, int W>
__global__ void __launch_bounds__(NT) qsc_pre_fwd_kernel(const float* __restrict__ x, const float* __restrict__ flat,
                                                         Offs o, float* __restrict__ angles, int B, int n) {
  using S = Lds<H, W>;
  using G = QGeo<H, W>;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* wsm = sm;
  float* act = sm + S::o_wl;
  stage_weights<H, W>(flat, o, wsm);
  for (int i = threadIdx.x; i < S::ACT; i += NT) act[i] = 0.f;
  __syncthreads();
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    sample_forward<H, W>(x + (size_t)b * 2 * G::HW, wsm, flat + o.wl, flat + o.bl, act, n);
    if (threadIdx.x < n) angles[(size_t)b * n + threadIdx.x] = act[S::o_ang + threadIdx.x];
  }
}

// Backward through the preprocess; dang (B, n) = dL/d(angles).  slab row per block (layout Offs).
template <int H, int W>
__global__ void __launch_bounds__(NT) qsc_pre_bwd_kernel(const float* __restrict__ x, const float* __restrict__ flat,
                                                         Offs o, const float* __restrict__ dang,
                                                         float* __restrict__ slab, int B, int n) {
  using S = Lds<H, W>;
  using G = QGeo<H, W>;
  constexpr int W2P = G::W2 + 2;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* wsm = sm;
  float* act = sm + S::o_wl;
  const float* wl = flat + o.wl;
  const int t = threadIdx.x;
  stage_weights<H, W>(flat, o, wsm);
  for (int i = t; i < S::BWD + n * G::F; i += NT) act[i] = 0.f;
  // register-resident gradient accumulators (fixed ownership per thread)
  constexpr int NWL = (G::F + NT - 1) / NT;       // features per thread for the linear layer
  float* gwl = act + S::o_gwl;                    // [n][F] in LDS, column f owned by one thread
  float gbl = 0.f, gb2 = 0.f, gb1 = 0.f;
  constexpr int W2PER = C2 * C1 * 9 / NT;         // 18 conv2 weights per thread
  float gw2[W2PER];
  float gw1[18];
#pragma unroll
  for (int k = 0; k < 18; ++k) gw1[k] = 0.f;
#pragma unroll
  for (int k = 0; k < W2PER; ++k) gw2[k] = 0.f;
  __syncthreads();

  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    sample_forward<H, W>(x + (size_t)b * 2 * G::HW, wsm, wl, flat + o.bl, act, n);
    float* misc = act + S::o_misc;
    // d pre-tanh
    if (t < n) {
      const float th = act[S::o_ang + t];
      const float d = dang[(size_t)b * n + t] * (1.f - th * th);
      misc[t] = d;
      gbl += d;
    }
    __syncthreads();
    // linear: grads + d p2 (thread f owns feature f [+ NT ...])
#pragma unroll
    for (int k = 0; k < NWL; ++k) {
      const int f = t + k * NT;
      if (f < G::F) {
        const float pv = act[S::o_p2 + f];
        float dp = 0.f;
        for (int j = 0; j < n; ++j) {
          gwl[j * G::F + f] += misc[j] * pv;
          dp += wl[(size_t)j * G::F + f] * misc[j];
        }
        // pool2 backward: route to the first max of relu(a2) in the 2x2 window, relu mask
        const int c = f / G::HW4, q = f % G::HW4, qh = q / G::W4, qw = q % G::W4;
        const int base = c * G::HW2 + (2 * qh) * G::W2 + 2 * qw;
        const int idx[4] = {base, base + 1, base + G::W2, base + G::W2 + 1};
        int am = idx[0];
        float mv = relu(act[S::o_a2 + idx[0]]);
#pragma unroll
        for (int r = 1; r < 4; ++r) {
          const float v = relu(act[S::o_a2 + idx[r]]);
          if (v > mv) { mv = v; am = idx[r]; }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) act[S::o_da2 + idx[r]] = (idx[r] == am && act[S::o_a2 + am] > 0.f) ? dp : 0.f;
      }
    }
    __syncthreads();
    // dz2 (padded copy for the dgrad) and bias grad
    for (int i = t; i < C2 * G::HW2; i += NT) {
      const int c = i / G::HW2, p = i % G::HW2;
      act[S::o_dz2p + c * S::P1P + (p / G::W2 + 1) * W2P + p % G::W2 + 1] = act[S::o_da2 + i];
    }
    if (t < C2) {
      float s = 0.f;
      for (int p = 0; p < G::HW2; ++p) s += act[S::o_da2 + t * G::HW2 + p];
      gb2 += s;
    }
    __syncthreads();
    // conv2 weight grads: thread owns (co, ci pair) x 9 taps; one output row at a time so every
    // loaded input window row is reused by the W/2 positions of the row.
    {
      const int co = t / 8, cp = (t % 8) * 2;
      for (int r = 0; r < G::H2; ++r) {
        float dz[G::W2];
#pragma unroll
        for (int q = 0; q < G::W2; ++q) dz[q] = act[S::o_da2 + co * G::HW2 + r * G::W2 + q];
#pragma unroll
        for (int cc = 0; cc < 2; ++cc) {
#pragma unroll
          for (int kh = 0; kh < 3; ++kh) {
            const float* xp = act + S::o_p1 + (cp + cc) * S::P1P + (r + kh) * W2P;
            float xr[G::W2 + 2];
#pragma unroll
            for (int q = 0; q < G::W2 + 2; ++q) xr[q] = xp[q];
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
              float s2 = 0.f;
#pragma unroll
              for (int q = 0; q < G::W2; ++q) s2 += dz[q] * xr[q + kw];
              gw2[cc * 9 + kh * 3 + kw] += s2;
            }
          }
        }
      }
    }
    // conv2 data grad -> d p1 (unpadded): thread = (ci, row, co half); halves combined by a lane swap
    {
      const int ci = t / 16, r = (t % 16) / 2, half = t & 1;
      float acc[G::W2];
#pragma unroll
      for (int q = 0; q < G::W2; ++q) acc[q] = 0.f;
      for (int co = half * (C2 / 2); co < (half + 1) * (C2 / 2); ++co) {
        const float* wk = wsm + S::o_w2 + (co * C1 + ci) * 9;
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
          const float* dzp = act + S::o_dz2p + co * S::P1P + (r + kh) * W2P;
          float dr[G::W2 + 2];
#pragma unroll
          for (int q = 0; q < G::W2 + 2; ++q) dr[q] = dzp[q];
          const float w0 = wk[(2 - kh) * 3 + 2], w1 = wk[(2 - kh) * 3 + 1], w2 = wk[(2 - kh) * 3];
#pragma unroll
          for (int q = 0; q < G::W2; ++q) acc[q] += w0 * dr[q] + w1 * dr[q + 1] + w2 * dr[q + 2];
        }
      }
#pragma unroll
      for (int q = 0; q < G::W2; ++q) acc[q] += __shfl_xor(acc[q], 1);
      if (half == 0) {
#pragma unroll
        for (int q = 0; q < G::W2; ++q) act[S::o_dp1 + ci * G::HW2 + r * G::W2 + q] = acc[q];
      }
    }
    __syncthreads();
    // pool1 backward + relu mask -> dz1 (C1 x HW)
    for (int i = t; i < C1 * G::HW2; i += NT) {
      const int c = i / G::HW2, q = i % G::HW2, qh = q / G::W2, qw = q % G::W2;
      const int base = c * G::HW + (2 * qh) * W + 2 * qw;
      const int idx[4] = {base, base + 1, base + W, base + W + 1};
      int am = idx[0];
      float mv = relu(act[S::o_a1 + idx[0]]);
#pragma unroll
      for (int r = 1; r < 4; ++r) {
        const float v = relu(act[S::o_a1 + idx[r]]);
        if (v > mv) { mv = v; am = idx[r]; }
      }
      const float g = act[S::o_dp1 + i];
#pragma unroll
      for (int r = 0; r < 4; ++r) act[S::o_dz1 + idx[r]] = (idx[r] == am && act[S::o_a1 + am] > 0.f) ? g : 0.f;
    }
    __syncthreads();
    // conv1 weight grads: thread = (co, image row); per-row partials of all 2 x 9 (ci, tap) weights,
    // summed over the 16 rows of a channel once, at the end (lane shuffles)
    for (int i = t; i < C1 * H; i += NT) {
      const int co = i / H, ph = i % H;
      float dz[W];
      float rs = 0.f;
#pragma unroll
      for (int q = 0; q < W; ++q) {
        dz[q] = act[S::o_dz1 + co * G::HW + ph * W + q];
        rs += dz[q];
      }
      gb1 += rs;
#pragma unroll
      for (int ci = 0; ci < 2; ++ci) {
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
          const float* xp = act + S::o_x + ci * S::XP + (ph + kh) * (W + 2);
          float xr[W + 2];
#pragma unroll
          for (int q = 0; q < W + 2; ++q) xr[q] = xp[q];
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) {
            float s1 = 0.f;
#pragma unroll
            for (int q = 0; q < W; ++q) s1 += dz[q] * xr[q + kw];
            gw1[ci * 9 + kh * 3 + kw] += s1;
          }
        }
      }
    }
    __syncthreads();
  }
  // write this block's slab row (zero the alignment gaps first: the row is summed whole)
  float* row = slab + (size_t)blockIdx.x * o.row;
  for (int i = t; i < o.row; i += NT) row[i] = 0.f;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NWL; ++k) {
    const int f = t + k * NT;
    if (f < G::F)
      for (int j = 0; j < n; ++j) row[o.wl - o.w1 + j * G::F + f] = gwl[j * G::F + f];
  }
  if (t < n) row[o.bl - o.w1 + t] = gbl;
  if (t < C2) row[o.b2 - o.w1 + t] = gb2;
  {
    const int co = t / 8, cp = (t % 8) * 2;
#pragma unroll
    for (int cc = 0; cc < 2; ++cc)
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) row[o.w2 - o.w1 + (co * C1 + cp + cc) * 9 + tap] = gw2[cc * 9 + tap];
  }
  {
    // conv1: threads (co, row) hold per-row partials; rows of one channel are H consecutive
    // threads (H = 16 lanes): butterfly-sum them, the row-0 thread writes.
    static_assert(C1 * H == NT, "conv1 grad ownership assumes C1*H == blockDim");
    const int co1 = t / H;
#pragma unroll
    for (int k = 0; k < 18; ++k) {
#pragma unroll
      for (int m = 1; m < H; m <<= 1) gw1[k] += __shfl_xor(gw1[k], m);
    }
#pragma unroll
    for (int m = 1; m < H; m <<= 1) gb1 += __shfl_xor(gb1, m);
    if (t % H == 0) {
#pragma unroll
      for (int k = 0; k < 18; ++k) row[co1 * 18 + k] = gw1[k];
      row[o.b1 - o.w1 + co1] = gb1;
    }
  }
}

// Classifier head: logits = E Wc^T + bc, log_softmax, mean NLL; writes loss, dE and the head
// parameter grads.  One block of 1024 threads; deterministic block reductions.
template <int N, int C>
__global__ void __launch_bounds__(1024) qsc_head_kernel(const float* __restrict__ E, const float* __restrict__ wc,
                                                        const float* __restrict__ bc, const long* __restrict__ labels,
                                                        float* __restrict__ dE, float* __restrict__ dwc,
                                                        float* __restrict__ dbc, float* __restrict__ loss,
                                                        float* __restrict__ loss_acc, float* __restrict__ skip,
                                                        int skip_add, int accumulate, int B) {
  constexpr int P = C * N + C;
  __shared__ float red[16][P + 1];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  float gw[P];
#pragma unroll
  for (int k = 0; k < P; ++k) gw[k] = 0.f;
  float lsum = 0.f;
  const float invB = 1.f / (float)B;
  for (int b = t; b < B; b += 1024) {
    float e[N], lg[C];
#pragma unroll
    for (int j = 0; j < N; ++j) e[j] = E[(size_t)b * N + j];
    float mx = -INFINITY;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      float s = bc[c];
#pragma unroll
      for (int j = 0; j < N; ++j) s += wc[c * N + j] * e[j];
      lg[c] = s;
      mx = fmaxf(mx, s);
    }
    float se = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) se += __expf(lg[c] - mx);
    const float lse = mx + __logf(se);
    const int y = (int)labels[b];
    float ly = 0.f, de[N];
#pragma unroll
    for (int j = 0; j < N; ++j) de[j] = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      ly += (c == y) ? lg[c] : 0.f;
      const float g = (__expf(lg[c] - lse) - (c == y ? 1.f : 0.f)) * invB;
#pragma unroll
      for (int j = 0; j < N; ++j) {
        de[j] += g * wc[c * N + j];
        gw[c * N + j] += g * e[j];
      }
      gw[C * N + c] += g;
    }
    lsum += lse - ly;
#pragma unroll
    for (int j = 0; j < N; ++j) dE[(size_t)b * N + j] = de[j];
  }
#pragma unroll
  for (int k = 0; k < P; ++k) {
    const float v = wave_sum(gw[k]);
    if (lane == 0) red[wv][k] = v;
  }
  {
    const float v = wave_sum(lsum);
    if (lane == 0) red[wv][P] = v;
  }
  __syncthreads();
  if (t <= P) {
    float s = 0.f;
    for (int w = 0; w < 16; ++w) s += red[w][t];
    if (t < C * N) dwc[t] = (accumulate ? dwc[t] : 0.f) + s;
    else if (t < P) dbc[t - C * N] = (accumulate ? dbc[t - C * N] : 0.f) + s;
    else {
      loss[0] = s * invB;
      if (loss_acc) loss_acc[0] += s * invB;
      if (skip) {  // NaN guard: a non-finite loss turns the optimizer step into a no-op
        const float bad = isfinite(s) ? 0.f : 1.f;
        skip[0] = skip_add ? skip[0] + bad : bad;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// QuantumNAT noise injection (E:175-199: w + noise_level * randn per forward call), for G weight
// groups (one per data stream) in ONE single-block launch: out[g] = w + sigma * N(0, 1), normals
// from a counter-based hash of (seed, counter, g, k) -- no RNG state, graph-replay safe.  The
// device counter is read by every thread and then advanced by thread 0, so every replay draws
// fresh noise, and forward and backward of the same step see the same noisy weights.
// ---------------------------------------------------------------------------------------------
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

__global__ void __launch_bounds__(256) qnoise_kernel(const float* __restrict__ w, float* __restrict__ out, int G,
                                                     int P, float sigma, unsigned long long seed,
                                                     unsigned long long* __restrict__ counter) {
  const unsigned long long ctr = *counter;
  for (int i = threadIdx.x; i < G * P; i += blockDim.x) out[i] = w[i % P] + sigma * hash_normal(seed, ctr, i);
  __syncthreads();
  if (threadIdx.x == 0) *counter = ctr + 1;
}

}  // namespace qsc
}  // namespace qd

using namespace qd::qsc;

QD_API int qd_qnoise(const float* w, float* out, int G, int P, float sigma, unsigned long long seed,
                     unsigned long long* counter, void* stream) {
  if (G < 1 || P < 1 || counter == nullptr) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(qnoise_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, w, out, G, P, sigma, seed, counter);
  return (int)hipGetLastError();
}

static size_t qsc_smem(int H, int W, bool bwd, int n) {
  if (H == 16 && W == 8)
    return sizeof(float) * (Lds<16, 8>::o_wl + (bwd ? Lds<16, 8>::BWD + n * QGeo<16, 8>::F : Lds<16, 8>::ACT));
  return sizeof(float) * (Lds<16, 16>::o_wl + (bwd ? Lds<16, 16>::BWD + n * QGeo<16, 16>::F : Lds<16, 16>::ACT));
}

// offs: [w1, b1, w2, b2, wl, bl, row_width] float offsets into the flat parameter buffer.
template <int H, int W>
static int launch_pre_fwd(const float* x, const float* flat, Offs o, float* angles, int B, int n, int grid,
                          hipStream_t s) {
  const size_t sm = qsc_smem(H, W, false, n);
  if (hipError_t e = qd::allow_lds(qsc_pre_fwd_kernel<H, W>, sm)) return (int)e;
  hipLaunchKernelGGL((qsc_pre_fwd_kernel<H, W>), dim3(grid), dim3(NT), sm, s, x, flat, o, angles, B, n);
  return (int)hipGetLastError();
}

template <int H, int W>
static int launch_pre_bwd(const float* x, const float* flat, Offs o, const float* dang, float* slab, int B, int n,
                          int grid, hipStream_t s) {
  const size_t sm = qsc_smem(H, W, true, n);
  if (hipError_t e = qd::allow_lds(qsc_pre_bwd_kernel<H, W>, sm)) return (int)e;
  hipLaunchKernelGGL((qsc_pre_bwd_kernel<H, W>), dim3(grid), dim3(NT), sm, s, x, flat, o, dang, slab, B, n);
  return (int)hipGetLastError();
}

QD_API int qd_qsc_pre_fwd(const float* x, const float* flat, const int* offs, float* angles, int B, int n, int H, int W,
                          int grid, void* stream) {
  if (n > 16 || B <= 0) return (int)hipErrorInvalidValue;
  Offs o{offs[0], offs[1], offs[2], offs[3], offs[4], offs[5], offs[6]};
  hipStream_t s = (hipStream_t)stream;
  if (H == 16 && W == 8) return launch_pre_fwd<16, 8>(x, flat, o, angles, B, n, grid, s);
  if (H == 16 && W == 16) return launch_pre_fwd<16, 16>(x, flat, o, angles, B, n, grid, s);
  return (int)hipErrorInvalidValue;
}

// slab: (grid, offs[6]) floats; row layout = flat layout starting at offs[0].
QD_API int qd_qsc_pre_bwd(const float* x, const float* flat, const int* offs, const float* dang, float* slab, int B,
                          int n, int H, int W, int grid, void* stream) {
  if (n > 16 || B <= 0 || qsc_smem(H, W, true, n) > 160 * 1024) return (int)hipErrorInvalidValue;
  Offs o{offs[0], offs[1], offs[2], offs[3], offs[4], offs[5], offs[6]};
  hipStream_t s = (hipStream_t)stream;
  if (H == 16 && W == 8) return launch_pre_bwd<16, 8>(x, flat, o, dang, slab, B, n, grid, s);
  if (H == 16 && W == 16) return launch_pre_bwd<16, 16>(x, flat, o, dang, slab, B, n, grid, s);
  return (int)hipErrorInvalidValue;
}

QD_API int qd_qsc_head(const float* E, const float* wc, const float* bc, const long* labels, float* dE, float* dwc,
                       float* dbc, float* loss, float* loss_acc, float* skip, int skip_add, int accumulate, int B,
                       int n, int C, void* stream) {
  hipStream_t s = (hipStream_t)stream;
#define QD_HEAD(NN, CC)                                                                                      \
  if (n == NN && C == CC) {                                                                                 \
    hipLaunchKernelGGL((qsc_head_kernel<NN, CC>), dim3(1), dim3(1024), 0, s, E, wc, bc, labels, dE, dwc, dbc, \
                       loss, loss_acc, skip, skip_add, accumulate, B);                                                               \
    return (int)hipGetLastError();                                                                          \
  }
#define QD_HEAD_N(NN) QD_HEAD(NN, 2) QD_HEAD(NN, 3) QD_HEAD(NN, 4)
  QD_HEAD_N(2) QD_HEAD_N(3) QD_HEAD_N(4) QD_HEAD_N(5) QD_HEAD_N(6) QD_HEAD_N(7) QD_HEAD_N(8) QD_HEAD_N(9)
  QD_HEAD_N(10) QD_HEAD_N(11) QD_HEAD_N(12) QD_HEAD_N(13) QD_HEAD_N(14) QD_HEAD_N(15) QD_HEAD_N(16)
#undef QD_HEAD_N
#undef QD_HEAD
  return (int)hipErrorInvalidValue;
}

// Inference head (eval / Test.py routing): per sample, logits = Wc E + bc -> log_softmax (logp, nullable)
// and the argmax (pred, nullable).  A thread per sample (the training head above is one workgroup: it
// also reduces the weight gradients).
namespace qd {
namespace qsc {
template <int N, int C>
__global__ void __launch_bounds__(256) qsc_infer_head_kernel(const float* __restrict__ E, const float* __restrict__ wc,
                                                             const float* __restrict__ bc, float* __restrict__ logp,
                                                             long* __restrict__ pred, int B) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  float e[N], lg[C], mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < N; ++j) e[j] = E[(size_t)b * N + j];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    float s = bc[c];
#pragma unroll
    for (int j = 0; j < N; ++j) s += wc[c * N + j] * e[j];
    lg[c] = s;
    mx = fmaxf(mx, s);
  }
  float se = 0.f;
  int am = 0;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    se += __expf(lg[c] - mx);
    if (lg[c] > lg[am]) am = c;
  }
  const float lse = mx + __logf(se);
  if (logp) {
#pragma unroll
    for (int c = 0; c < C; ++c) logp[(size_t)b * C + c] = lg[c] - lse;
  }
  if (pred) pred[b] = am;
}
}  // namespace qsc
}  // namespace qd

QD_API int qd_qsc_infer_head(const float* E, const float* wc, const float* bc, float* logp, long* pred, int B, int n,
                             int C, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int grid = (B + 255) / 256;
#define QD_IH(NN, CC)                                                                                      \
  if (n == NN && C == CC) {                                                                                \
    hipLaunchKernelGGL((qd::qsc::qsc_infer_head_kernel<NN, CC>), dim3(grid), dim3(256), 0, s, E, wc, bc, logp, \
                       pred, B);                                                                           \
    return (int)hipGetLastError();                                                                         \
  }
#define QD_IH_N(NN) QD_IH(NN, 2) QD_IH(NN, 3) QD_IH(NN, 4)
  QD_IH_N(2) QD_IH_N(3) QD_IH_N(4) QD_IH_N(5) QD_IH_N(6) QD_IH_N(7) QD_IH_N(8) QD_IH_N(9)
  QD_IH_N(10) QD_IH_N(11) QD_IH_N(12) QD_IH_N(13) QD_IH_N(14) QD_IH_N(15) QD_IH_N(16)
#undef QD_IH_N
#undef QD_IH
  return (int)hipErrorInvalidValue;
}

// The QSC preprocess linear layer's weight gradient when the MFMA backward cannot reduce it in its own slab
// (large n / P256 feature maps): dWl (n, F) = dpre^T p2 over the batch, dpre (B, n), p2 (B, F) fp32.  A tall-K
// outer-product sum (K = B = 2304, n <= 16): phase 1 here writes per-sample-chunk partials slab (S, n, F) --
// block (x, s) takes 256 columns of chunk s, each thread one column with n accumulators, the chunk's dpre rows
// staged in LDS -- and the caller's slab_rows_sum reduces over S in a fixed order (deterministic, no atomics).
namespace qd {
namespace qsc {
constexpr int OUTER_MAXN = 16;
__global__ void __launch_bounds__(256) outer_partial_kernel(const float* __restrict__ D, const float* __restrict__ P,
                                                            float* __restrict__ slab, int B, int n, int F, int bs) {
  __shared__ float ds[64 * OUTER_MAXN];
  const int s = blockIdx.y, f = blockIdx.x * 256 + threadIdx.x;
  const int b0 = s * bs, b1 = min(B, b0 + bs);
  float acc[OUTER_MAXN];
#pragma unroll
  for (int i = 0; i < OUTER_MAXN; ++i) acc[i] = 0.f;
  for (int c0 = b0; c0 < b1; c0 += 64) {
    const int cn = min(64, b1 - c0);
    __syncthreads();
    for (int t = threadIdx.x; t < cn * n; t += 256) ds[t] = D[(size_t)c0 * n + t];
    __syncthreads();
    if (f < F) {
      for (int b = 0; b < cn; ++b) {
        const float p = P[(size_t)(c0 + b) * F + f];
#pragma unroll
        for (int i = 0; i < OUTER_MAXN; ++i)
          if (i < n) acc[i] += ds[b * n + i] * p;
      }
    }
  }
  if (f < F) {
#pragma unroll
    for (int i = 0; i < OUTER_MAXN; ++i)
      if (i < n) slab[((size_t)s * n + i) * F + f] = acc[i];
  }
}
}  // namespace qsc
}  // namespace qd

// phase 1 of dWl = D^T P (see above): slab (S, n, F) with S = ceil(B / bs)
QD_API int qd_outer_partial(const float* D, const float* P, float* slab, int B, int n, int F, int bs, void* stream) {
  if (n < 1 || n > qd::qsc::OUTER_MAXN || bs < 1 || B < 1 || F < 1) return (int)hipErrorInvalidValue;
  const int S = (B + bs - 1) / bs;
  hipLaunchKernelGGL(qd::qsc::outer_partial_kernel, dim3((F + 255) / 256, S), dim3(256), 0, (hipStream_t)stream, D, P,
                     slab, B, n, F, bs);
  return (int)hipGetLastError();
}
