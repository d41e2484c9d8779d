// QSC preprocess CNN on fp32 MFMA: one wave per sample, no workgroup barriers in the sample loop.
//
// Reference: QSC_P128.preprocess (Estimators_QuantumNAT_onchipQNN.py:152-162)
//   Conv2d(2,16,3,p=1) -> ReLU -> MaxPool2 -> Conv2d(16,32,3,p=1) -> ReLU -> MaxPool2 -> Flatten
//   -> Linear(F, n) -> Tanh          (F = 32 * H/4 * W/4: 256 for P128, 512 for P256)
//
// The first version (csrc/hip/qsc.hip, kept as the reference path) ran a whole 256-thread
// workgroup per sample with ~12 barriers per sample and scalar LDS-bound convolutions (0.75 LDS
// loads per FMA): 46 us forward + 152 us backward for 2304 samples.  Here:
//   * conv2 (M = positions, N = 32 channels, K = 144) is an implicit GEMM on
//     v_mfma_f32_32x32x2_f32 (exact fp32, as the reference) from a channel-last LDS image of the
//     padded pool-1 map (two ds_read_b128 feed 8 MFMAs), conv2 weights in registers; conv1
//     (K = 18) stays on the VALU with a lane owning one row of a pool window x all 16 channels,
//     so every conv1 weight is wave-uniform (scalar loads) and pool 1 is one lane shuffle;
//   * backward: conv2 weight grads accumulate across the wave's samples in MFMA accumulators
//     (5 tiles of 32x32, K = positions), conv2 data grads are a 16x16x4 MFMA implicit GEMM over
//     the zero-padded dz2 image (K = 32 channels x 9 flipped taps), conv1 weight grads a 16x16x4
//     MFMA over positions; the linear layer's weight grads are one GEMM outside the kernel
//     (dpre^T . p2 over the batch), everything else lands in one slab row per workgroup, summed
//     in a fixed order (deterministic, no float atomics).
// Every wave owns its sample from input to output, so waves never wait for each other.
#include "common.h"

// pins a loaded value at its load site: without a use there, the compiler sinks a batch of loads into the guarded
// stores that consume them, one round trip each again
template <typename T>
__device__ __forceinline__ void keep_loaded(const T& v) {
  static_assert(sizeof(T) % 4 == 0, "dword values");
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&v);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); ++i) asm volatile("" ::"v"(w[i]));
}

namespace qd {
namespace qsc2 {

constexpr int C1 = 16, C2 = 32;
constexpr int K1 = 2 * 9;         // conv1 reduction size
constexpr int K2 = C1 * 9;        // conv2 reduction size (144)
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4_t;

// bf16x3: an fp32 value as hi + lo bf16 pair; a.b ~= ah.bh + ah.bl + al.bh (relative error ~1e-5)
__device__ __forceinline__ void split_bf16(float v, __bf16& hi, __bf16& lo) {
  hi = (__bf16)v;
  lo = (__bf16)(v - (float)hi);
}

struct Offs {
  int w1, b1, w2, b2, wl, bl, row;
  int base;   // flat offset of slab column 0 (min of the preprocess and quantum-weight offsets)
  int qw;     // flat offset of the quantum-layer weights (their slab columns: see qsc2_bwd_kernel)
};

// forward -> backward hand-off per sample (the backward routes gradients through the saved pool
// choices instead of recomputing conv1/conv2): see sample_forward
struct Saved {
  float* p1;      // (B, HW2, 16) pool-1 map, channel-last
  uint32_t* c1;   // (B, HW2) pool-1 argmax codes, 2 bits per channel
  uint8_t* c2;    // (B, F) pool-2 window-relative argmax
};

// the quantum layer's adjoint-pass slab (rows, width): each backward workgroup also sums its share
// of rows into the quantum-weight columns of its own slab row (one reduction launch fewer)
struct QSlab {
  const float* slab;
  int rows, width;
};

template <int H, int W>
struct Geo {
  static constexpr int HW = H * W;
  static constexpr int H2 = H / 2, W2 = W / 2, HW2 = H2 * W2;   // pool-1 grid (conv2 positions)
  static constexpr int H4 = H / 4, W4 = W / 4, HW4 = H4 * W4;   // pool-2 grid
  static constexpr int F = C2 * HW4;
  static constexpr int XW = W + 2, XP = (H + 2) * (W + 2);       // padded input plane
  static constexpr int PW = W2 + 2, PP = (H2 + 2) * (W2 + 2);    // padded pool-1 plane
  static constexpr int PC = 20;   // pool-1 map is channel-last: 16 channels (+4 pad: ds_read_b128 banks) per position
  static constexpr int MT2 = HW2 / 32;                           // conv2 32-position tiles
  static constexpr int MT1 = HW2 / 16;                           // dgrad 16-position tiles
  // per-wave LDS image (floats)
  static constexpr int o_x = 0;                                   // 2 x XP
  static constexpr int o_p1 = o_x + 2 * XP;                       // C1 x PP (padded pool-1 map)
  static constexpr int o_z2 = o_p1 + PC * PP;                     // C2 x HW2 (conv2 pre-activation)
  static constexpr int DC = 36;  // dz2 is channel-last too: 32 channels (+4 pad) per padded position
  static constexpr int o_dz2 = o_z2 + C2 * HW2;                   // PP x DC (padded conv2 grad)
  static constexpr int o_dp1 = o_dz2 + PP * DC;                   // C1 x HW2
  static constexpr int o_dz1 = o_z2;                              // C1 x HW, aliases z2 + dz2 (dead by then)
  static_assert(C1 * HW <= C2 * HW2 + PP * DC, "dz1 alias");
  static constexpr int o_misc = o_dp1 + C1 * HW2;                 // 32: dpre / angles
  static constexpr int o_p2f = o_dz2;                              // forward only: F pooled features
  static constexpr int FWD = o_p2f + F;                            // forward needs x, p1, z2, p2
  static constexpr int BWD = o_misc + 32;
};

// block-shared weights (floats): W1 [16][18] | b1 [16] | W2 [32][144] | b2 [32]
constexpr int S_W1 = 0, S_B1 = S_W1 + C1 * K1, S_W2 = S_B1 + C1, S_B2 = S_W2 + C2 * K2, S_WEND = S_B2 + C2;

__device__ __forceinline__ float relu(float v) { return relu_nan(v); }

// Diagnostic phase stamps (STAMP builds only): s_memtime with its own lgkmcnt wait, fenced by
// scheduling barriers so the compiler keeps each phase's work on its side of the stamp.
__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
constexpr int NSTAMP = 12;

// ... followed by the linear layer: wl [n][F + 4] (row pad: conflict-free 4-lanes-per-output reads)
// | bl [16] (LDS: a runtime-n loop over L2 loads of wl serialises one round trip per iteration)
__host__ __device__ constexpr int wl_stride(int F) { return F + 4; }
__host__ __device__ constexpr int act_base(int n, int F) { return S_WEND + ((n * wl_stride(F) + 16 + 3) & ~3); }
// backward only: W2 transposed to [tap][ci][co] (co contiguous, stride 36) after the linear layer
constexpr int W2T_CS = 36;
constexpr int W2T_SIZE = 9 * C1 * W2T_CS;
__host__ __device__ constexpr int act_base_bwd(int n, int F) { return act_base(n, F) + W2T_SIZE; }

// global -> LDS copy of n floats (both 16-byte aligned, n % 4 == 0): float4 loads, four in flight
// per thread (a plain strided loop serialises one L2 round trip per iteration)
__device__ __forceinline__ void stage4(float* dst, const float* __restrict__ src, int n) {
  const float4* s4 = reinterpret_cast<const float4*>(src);
  float4* d4 = reinterpret_cast<float4*>(dst);
  const int n4 = n >> 2, nt = blockDim.x;
  int i = threadIdx.x;
  for (; i + 3 * nt < n4; i += 4 * nt) {
    const float4 a = s4[i], b = s4[i + nt], c = s4[i + 2 * nt], d = s4[i + 3 * nt];
    d4[i] = a;
    d4[i + nt] = b;
    d4[i + 2 * nt] = c;
    d4[i + 3 * nt] = d;
  }
  for (; i < n4; i += nt) d4[i] = s4[i];
}

// forward kernel LDS: just the linear layer (wl [n][F+4] | bl), then the per-wave images
// ... then conv1's weights and bias (C1 * K1 + C1 floats: read as wave-uniform LDS broadcasts -- as scalar
// loads the 288 weights overflowed the SGPRs and the compiler spilled them through VGPR lanes, ~1800
// v_readlane / v_writelane per sample), then the per-wave images
__host__ __device__ constexpr int fwd_w1_base(int n, int F) { return (n * (F + 4) + 16 + 3) & ~3; }
__host__ __device__ constexpr int fwd_act_base(int n, int F) { return fwd_w1_base(n, F) + ((C1 * K1 + C1 + 3) & ~3); }
// (all offsets are multiples of 16 floats: FlatParamSpace ALIGN; LDS slots multiples of 4)
__device__ __forceinline__ void stage_weights(const float* __restrict__ flat, Offs o, float* ws, int n, int F) {
  stage4(ws + S_W1, flat + o.w1, C1 * K1);
  stage4(ws + S_B1, flat + o.b1, C1);
  stage4(ws + S_W2, flat + o.w2, C2 * K2);
  stage4(ws + S_B2, flat + o.b2, C2);
  {  // linear weights: one flat loop (a loop of per-row copies serialised ~2k cycles per row)
    const int q4 = F / 4;
    const float4* src = reinterpret_cast<const float4*>(flat + o.wl);
    for (int i = threadIdx.x; i < n * q4; i += blockDim.x) {
      const int j = i / q4, c = i % q4;
      *reinterpret_cast<float4*>(ws + S_WEND + j * wl_stride(F) + 4 * c) = src[i];
    }
  }
  if (threadIdx.x < n) ws[S_WEND + n * wl_stride(F) + threadIdx.x] = flat[o.bl + threadIdx.x];
}

// a wave-uniform value from the first active lane, in an SGPR (conv1's weights: see conv1_half; round 6: an
// optimisation now -- the SGPR operands take the weights out of the VGPR file -- the misread it masked is fixed at
// its cause, see conv1_half)
__device__ __forceinline__ float uniform(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
}

// conv1 pre-activations (+bias) of one ROW of pool window `win` (hw = 0 top, 1 bottom): all 16
// channels x 2 positions.  The whole wave walks the channels in lockstep, so every weight is
// wave-uniform: LDS broadcast reads of the workgroup's staged copy (w1g = W1 transposed [k][co], b1g),
// each value taken from lane 0 into an SGPR (uniform()).  Round 5 found that with the per-lane copies, under
// concurrent work in the graph plans, lanes 48-63 used a wrong channel-5 weight in 20-30 of 288 samples
// (profiles/r5_55_entries.txt).  Round 6 named the cause: the compiler fed those weights to v_pk_fma_f32 (packed
// FP32, op_sel picking one register of a pair, profiles/r6_qsc_conv1_prefix_isa.txt), and the next k's
// ds_read_b128 rewrote the registers while -- behind a co-resident wave's MFMAs -- the packed FMA's last
// quarter-wave had not read them yet.  csrc/hip/hazard_probe.hip reproduces exactly that (lanes 48-63, only with
// MFMA partners, never with plain v_fma_f32: profiles/r6_03_pkfma_war.txt), and the library is now built without
// packed-FP32 instructions (_native.NO_PACKED_F32, tests/test_no_packed_f32.py).  docs/CONCURRENCY.md.
template <int H, int W>
__device__ __forceinline__ void conv1_half(const float* act, const float* __restrict__ w1g,
                                           const float* __restrict__ b1g, int win, int hw, float (&acc)[16][2]) {
  using G = Geo<H, W>;
  const int qy = win / G::W2, qx = win % G::W2;
#pragma unroll
  for (int co = 0; co < C1; ++co) {
    const float b = uniform(b1g[co]);
    acc[co][0] = b;
    acc[co][1] = b;
  }
  // k = (ci, tap) outer as a rolled loop, channels inner: each k's 16 weights are four broadcast
  // ds_read_b128 of the transposed copy [k][co] and its two input values two LDS reads, consumed right
  // away (unrolled, the compiler hoisted all 288 weights into VGPRs and halved the occupancy).  3 k per
  // iteration since the weights live in SGPRs: 232 VGPRs (2 waves / SIMD as with 2), step 0.3841-0.3856 vs
  // 0.3856-0.3867 ms on one box (profiles/r5_62_ab.txt), level on another (r5_64_ab.txt); fully unrolled it spills
#pragma unroll 3
  for (int k = 0; k < K1; ++k) {
    const int ci = k / 9, t = k % 9;
    const float* px = act + G::o_x + ci * G::XP + (2 * qy + hw + t / 3) * G::XW + 2 * qx + t % 3;
    const float p0 = px[0], p1 = px[1];
    const float4* wk = reinterpret_cast<const float4*>(w1g + k * C1);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 wv = wk[q];
      const float4 w = make_float4(uniform(wv.x), uniform(wv.y), uniform(wv.z), uniform(wv.w));
      acc[4 * q][0] += w.x * p0;
      acc[4 * q][1] += w.x * p1;
      acc[4 * q + 1][0] += w.y * p0;
      acc[4 * q + 1][1] += w.y * p1;
      acc[4 * q + 2][0] += w.z * p0;
      acc[4 * q + 2][1] += w.z * p1;
      acc[4 * q + 3][0] += w.w * p0;
      acc[4 * q + 3][1] += w.w * p1;
    }
  }
}

// conv1 (+bias) + ReLU + pool 1 on f32 MFMAs (P128, W = 8; round 6).  Per band of two image rows one 16x16 tile:
// rows = the band's 16 positions (row r: image row 2 band + r / 8, column r % 8), columns = the 16 output channels,
// K = the 18 (ci, tap) in five 16x16x4 f32 steps (fp32 products, as the VALU loop: a bf16x3 form measured 2.4e-3
// max-rel on conv1's weight gradient against autograd at B = 300 through flipped near-tie pool choices) in place
// of conv1_half's 576 VALU FMAs and 288 readfirstlanes per lane.  The accumulator gives lane (channel
// c = lane & 15, group g = lane >> 4) the positions 4 g .. 4 g + 3 -- two horizontal pool pairs of one row -- and
// lanes l, l ^ 32 hold the two rows of the same windows.  Same outputs and tie rules as the conv1_half loop:
// the padded channel-last pool-1 image, p1g and the window codes c1g.  w1f: this lane's B operands
// W1[c][4 i + g] (zero past k = 17), i = 0..4; b1c = b1[c].
__device__ __forceinline__ uint32_t spread_even16(uint32_t x) {   // bit i -> bit 2 i (16 bits)
  x = (x | (x << 8)) & 0x00FF00FFu;
  x = (x | (x << 4)) & 0x0F0F0F0Fu;
  x = (x | (x << 2)) & 0x33333333u;
  return (x | (x << 1)) & 0x55555555u;
}
template <int H, int W>
__device__ __forceinline__ void conv1_mfma(float* act, int lane, const float (&w1f)[5], float b1c,
                                           float* __restrict__ p1g, uint32_t* __restrict__ c1g) {
  using G = Geo<H, W>;
  static_assert(W == 8 && H % 2 == 0, "bands of two 8-wide rows");
  constexpr int NB = H / 2;
  const int g = lane >> 4, c = lane & 15;
  const bool top = g < 2;
  const int ry = c >> 3, rx = c & 7;   // (A operand: this lane's position row = lane & 15)
  // every band's A operands first (40 LDS reads in flight), then the MFMA chains
  float av[NB][5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int k = 4 * i + g, ci = k / 9, t = k % 9;
    const int off = G::o_x + ci * G::XP + (ry + t / 3) * G::XW + rx + t % 3;
#pragma unroll
    for (int band = 0; band < NB; ++band) av[band][i] = k < K1 ? act[off + 2 * band * G::XW] : 0.f;
  }
#pragma unroll
  for (int band = 0; band < NB; ++band) {
    f32x4 acc = {b1c, b1c, b1c, b1c};
#pragma unroll
    for (int i = 0; i < 5; ++i) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[band][i], w1f[i], acc, 0, 0, 0);
#pragma unroll
    for (int w = 0; w < 2; ++w) {
      const float r0 = relu(acc[2 * w]), r1 = relu(acc[2 * w + 1]);
      const float v = max_nan(r0, r1);
      const uint32_t rt = (uint32_t)(r1 > r0);   // ties go to the left column
      // the other row of the window: lanes l and l ^ 32 swap (v_permlane32_swap, no LDS round trip)
      const auto sv = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(uint32_t, v),
                                                       __builtin_bit_cast(uint32_t, v), false, false);
      const auto sr = __builtin_amdgcn_permlane32_swap(rt, rt, false, false);
      const float pv = __builtin_bit_cast(float, top ? sv[1] : sv[0]);
      const uint32_t prt = top ? sr[1] : sr[0];
      const float m = top ? max_nan(v, pv) : max_nan(pv, v);
      const bool bottom = top ? pv > v : v > pv;   // ties go to the top row
      const uint32_t rtop = top ? rt : prt, rbot = top ? prt : rt;
      // window codes: 2 bits per channel = per lane of a group -- two ballots, the bits interleaved in SGPRs
      const unsigned long long b1 = __ballot(bottom);
      const unsigned long long b0 = __ballot(bottom ? rbot != 0u : rtop != 0u);
      if (top) {
        const int qx = 2 * g + w, win = band * G::W2 + qx;
        act[G::o_p1 + ((band + 1) * G::PW + qx + 1) * G::PC + c] = m;
        p1g[win * C1 + c] = m;
        if (c == 0) {
          const uint32_t sh = 16u * (uint32_t)g;
          c1g[win] = spread_even16((uint32_t)(b0 >> sh) & 0xFFFFu) |
                     (spread_even16((uint32_t)(b1 >> sh) & 0xFFFFu) << 1);
        }
      }
    }
  }
}

// conv1_mfma for P256 (W = 16): one 16x16 tile per image row (row = the row's 16 columns), so the two rows of a
// window are the same lane's accumulators in the tiles of rows 2 qy and 2 qy + 1: lane (c, g) holds columns
// 4 g .. 4 g + 3 of both, i.e. windows (qy, 2 g) and (qy, 2 g + 1) of channel c -- no exchange across lanes.
// The two rows' tiles are computed together, the row pairs in turn (accumulators of one pair live).
template <int H, int W>
__device__ __forceinline__ void conv1_mfma16(float* act, int lane, const float (&w1f)[5], float b1c,
                                             float* __restrict__ p1g, uint32_t* __restrict__ c1g) {
  using G = Geo<H, W>;
  static_assert(W == 16 && H % 2 == 0, "one 16-wide row per tile");
  const int g = lane >> 4, c = lane & 15;
  int aoff[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int k = 4 * i + g, ci = k / 9, t = k % 9;
    aoff[i] = k < K1 ? G::o_x + ci * G::XP + (t / 3) * G::XW + c + t % 3 : -1;   // (row 0; + y XW per row)
  }
#pragma unroll 2
  for (int qy = 0; qy < H / 2; ++qy) {
    float av[2][5];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 5; ++i) av[h][i] = aoff[i] >= 0 ? act[aoff[i] + (2 * qy + h) * G::XW] : 0.f;
    f32x4 acc[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      acc[h] = (f32x4){b1c, b1c, b1c, b1c};
#pragma unroll
      for (int i = 0; i < 5; ++i) acc[h] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[h][i], w1f[i], acc[h], 0, 0, 0);
    }
#pragma unroll
    for (int w = 0; w < 2; ++w) {
      const float t0 = relu(acc[0][2 * w]), t1 = relu(acc[0][2 * w + 1]);
      const float u0 = relu(acc[1][2 * w]), u1 = relu(acc[1][2 * w + 1]);
      const float v = max_nan(t0, t1), pv = max_nan(u0, u1);   // top / bottom row of the window
      const uint32_t rtop = (uint32_t)(t1 > t0), rbot = (uint32_t)(u1 > u0);   // ties go to the left column
      const float m = max_nan(v, pv);
      const bool bottom = pv > v;                                             // ties go to the top row
      const unsigned long long b1 = __ballot(bottom);
      const unsigned long long b0 = __ballot(bottom ? rbot != 0u : rtop != 0u);
      const int qx = 2 * g + w, win = qy * G::W2 + qx;
      act[G::o_p1 + ((qy + 1) * G::PW + qx + 1) * G::PC + c] = m;
      p1g[win * C1 + c] = m;
      if (c == 0) {
        const uint32_t sh = 16u * (uint32_t)g;
        c1g[win] = spread_even16((uint32_t)(b0 >> sh) & 0xFFFFu) | (spread_even16((uint32_t)(b1 >> sh) & 0xFFFFu) << 1);
      }
    }
  }
}

// Forward of one sample into the wave's LDS image: x -> p1 (padded) -> z2 (pre-activation).
// wreg (optional): this lane's 72 conv2 weights W2[co = lane&31][ci = 8*(lane>>5) + j][t] at
// [t*8 + j], register-resident across samples (forward kernel); null = read them from LDS.
// Saved for the backward (per sample): p1g = pool-1 map [window][16 ch]; c1g[window] = 2-bit
// window-relative argmax per channel (bits 2c..2c+1: 0 top-left, 1 top-right, 2 bottom-left,
// 3 bottom-right; first max in that scan order, the reference's max_pool2d choice).
// X3: conv2 on bf16x3 MFMAs (mfma_f32_32x32x16_bf16, K = one tap's 16 channels; wx3 = this lane's
// W2 column as bf16 hi [tap 0..8] | lo [9..17]) instead of the f32 32x32x2 form (1/16 of the rate).
template <int H, int W, bool WREG, bool STAMP = false, bool X3 = false>
__device__ __forceinline__ void sample_forward(const float* __restrict__ xs, const float* ws, float* act, int lane,
                                               const float (&wreg)[72], const float* __restrict__ w1g,
                                               const float* __restrict__ b1g, float bias2,
                                               float* __restrict__ p1g, uint32_t* __restrict__ c1g,
                                               unsigned long long* ts = nullptr, const bf16x8_t* wx3 = nullptr,
                                               const float4* xpre = nullptr, const float* w1f = nullptr,
                                               float b1c = 0.f) {
  using G = Geo<H, W>;
  static_assert(W % 4 == 0, "float4 rows");
  const float4* x4 = reinterpret_cast<const float4*>(xs);   // sample planes are 16-byte aligned
#pragma unroll
  for (int i = lane; i < 2 * G::HW / 4; i += 64) {
    const float4 v = (xpre && i < 64) ? *xpre : x4[i];   // (xpre: this lane's first float4, loaded early)
    const int c = (4 * i) / G::HW, p = (4 * i) % G::HW;
    float* d = act + G::o_x + c * G::XP + (p / W + 1) * G::XW + p % W + 1;
    d[0] = v.x;
    d[1] = v.y;
    d[2] = v.z;
    d[3] = v.w;
  }
  wave_lds_fence();
  if constexpr (STAMP) ts[2] = stamp();
  if constexpr (X3 && W == 8) {
    conv1_mfma<H, W>(act, lane, *reinterpret_cast<const float(*)[5]>(w1f), b1c, p1g, c1g);
  } else if constexpr (W == 16 && WREG) {
    conv1_mfma16<H, W>(act, lane, *reinterpret_cast<const float(*)[5]>(w1f), b1c, p1g, c1g);
  } else {
  // conv1 + ReLU + pool: lane = (window, row of the window); the two rows meet with one shuffle
  static_assert((2 * G::HW2) % 64 == 0, "whole waves per conv1 pass");
  for (int idx = lane; idx < 2 * G::HW2; idx += 64) {
    const int win = idx >> 1, hw = idx & 1;
    float acc[16][2];
    conv1_half<H, W>(act, w1g, b1g, win, hw, acc);
    float m[16];
    uint32_t right = 0, bottom = 0;   // per channel: right column wins in this row; bottom row wins
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const float r0 = relu(acc[c][0]), r1 = relu(acc[c][1]);
      const float v = max_nan(r0, r1), pv = __shfl_xor(v, 1);
      m[c] = max_nan(v, pv);
      right |= (uint32_t)(r1 > r0) << c;
      bottom |= (uint32_t)(hw ? (v > pv) : (pv > v)) << c;   // ties go to the top row
    }
    const uint32_t pright = __shfl_xor(right, 1);
    const int qy = win / G::W2, qx = win % G::W2;
    float4* d = reinterpret_cast<float4*>(act + G::o_p1 + ((qy + 1) * G::PW + qx + 1) * G::PC + 8 * hw);
    const float4 m0 = make_float4(m[8 * hw + 0], m[8 * hw + 1], m[8 * hw + 2], m[8 * hw + 3]);
    const float4 m1 = make_float4(m[8 * hw + 4], m[8 * hw + 5], m[8 * hw + 6], m[8 * hw + 7]);
    d[0] = m0;
    d[1] = m1;
    float4* g = reinterpret_cast<float4*>(p1g + win * C1 + 8 * hw);
    g[0] = m0;
    g[1] = m1;
    if (hw == 0) {
      uint32_t code = 0;
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const uint32_t b = (bottom >> c) & 1u;
        code |= (b ? 2u + ((pright >> c) & 1u) : (right >> c) & 1u) << (2 * c);
      }
      c1g[win] = code;
    }
  }
  }
  wave_lds_fence();
  if constexpr (STAMP) ts[3] = stamp();
  // conv2 on MFMA: rows = positions, cols = output channels.  MFMA step j of tap t sums the k-pair
  // (t, ci = j) [lane half 0] and (t, ci = 8 + j) [half 1]: a lane's 8 A operands of a tap are 8
  // consecutive channels of one position of the channel-last map = two ds_read_b128.
  const int col = lane & 31, kh = lane >> 5;
  for (int mt = 0; mt < G::MT2; ++mt) {
    const int pos = mt * 32 + col;
    const int py = pos / G::W2, px = pos % G::W2;
    f32x16 acc = {};
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const float4* ap =
          reinterpret_cast<const float4*>(act + G::o_p1 + ((py + t / 3) * G::PW + px + t % 3) * G::PC + 8 * kh);
      const float4 a0 = ap[0], a1 = ap[1];
      const float a[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
      if constexpr (X3) {   // k = 8 kh + j = channel: the same pairing as wx3's column
        bf16x8_t ah, al;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          __bf16 h, l;
          split_bf16(a[j], h, l);
          ah[j] = h;
          al[j] = l;
        }
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, wx3[t], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, wx3[9 + t], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, wx3[t], acc, 0, 0, 0);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float b = WREG ? wreg[t * 8 + j] : ws[S_W2 + col * K2 + (8 * kh + j) * 9 + t];
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[j], b, acc, 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * kh;
      act[G::o_z2 + col * G::HW2 + mt * 32 + row] = acc[r] + bias2;
    }
  }
  wave_lds_fence();
  if constexpr (STAMP) ts[4] = stamp();
}

// pool-2 (after ReLU) value and the winning position of feature f (first max, reference order)
template <int H, int W>
__device__ __forceinline__ float pool2(const float* act, int f, int& rel) {
  using G = Geo<H, W>;
  const int c = f / G::HW4, q = f % G::HW4, qy = q / G::W4, qx = q % G::W4;
  const int base = (2 * qy) * G::W2 + 2 * qx;
  const int idx[4] = {base, base + 1, base + G::W2, base + G::W2 + 1};
  const float* z = act + G::o_z2 + c * G::HW2;
  float m = relu(z[idx[0]]);
  rel = 0;
#pragma unroll
  for (int r = 1; r < 4; ++r) {
    const float v = relu(z[idx[r]]);
    if (v > m) {
      m = v;
      rel = r;
    }
  }
  return m;
}

// angles (B, n) = tanh(preprocess(x)); p2 (B, F) = flattened pool-2 features (for the linear
// layer's weight-gradient GEMM in the backward).  One wave per sample.
template <int H, int W, int NWV, bool STAMP = false, bool X3 = false>
__global__ void __launch_bounds__(64 * NWV) qsc2_fwd_kernel(const float* __restrict__ x, const float* __restrict__ flat,
                                                      Offs o, float* __restrict__ angles, float* __restrict__ p2,
                                                      Saved sv, int B, int n,
                                                      unsigned long long* __restrict__ stamps = nullptr,
                                                      __bf16* __restrict__ w2t_img = nullptr) {
  unsigned long long ts[NSTAMP] = {};
  if constexpr (STAMP) ts[0] = stamp();
  using G = Geo<H, W>;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* ws = sm;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // the first sample's input (one float4 per lane at P128) is loaded before the prologue: its
  // latency hides behind the weight staging instead of opening the sample
  float4 xpre = make_float4(0.f, 0.f, 0.f, 0.f);
  {
    const int s0 = blockIdx.x * NWV + wv;
    if (s0 < B) xpre = reinterpret_cast<const float4*>(x + (size_t)s0 * 2 * G::HW)[lane];
  }
  // LDS: only the linear layer is staged; conv1 weights are scalar loads, conv2 weights live in
  // registers (loaded straight from the flat buffer), conv2 bias is one value per lane
  float* act = sm + fwd_act_base(n, G::F) + wv * G::FWD;
  float* w1s = sm + fwd_w1_base(n, G::F);
  // Every weight load of the prologue in flight together, one round trip (round 6: the linear layer's copy loop,
  // conv1's transposing loop and the conv2 register loads waited for 4-5 round trips in turn, ~10k cycles per
  // workgroup: profiles/r2_18_qsc_fwd_conv1_lds.md "stage weights").
  constexpr int NTH = 64 * NWV;
  constexpr int WLQ = (16 * (G::F / 4) + NTH - 1) / NTH;   // linear-layer float4 per thread (n <= 16)
  constexpr int W1Q = (C1 * K1 + C1 + NTH - 1) / NTH;      // conv1 weights + bias per thread
  const int q4 = G::F / 4, wl_tot = n * q4;
  float4 vwl[WLQ];
  float vw1[W1Q];
  float vbl = 0.f;
  {
    const float4* src = reinterpret_cast<const float4*>(flat + o.wl);
#pragma unroll
    for (int k = 0; k < WLQ; ++k) {
      const int i = threadIdx.x + k * NTH;
      vwl[k] = src[i < wl_tot ? i : 0];
    }
#pragma unroll
    for (int k = 0; k < W1Q; ++k) {
      const int i = threadIdx.x + k * NTH;
      vw1[k] = flat[i < C1 * K1 ? o.w1 + i : (i < C1 * K1 + C1 ? o.b1 + i - C1 * K1 : o.w1)];
    }
    if (threadIdx.x < n) vbl = flat[o.bl + threadIdx.x];
  }
  // this lane's weights W2[co][8h .. 8h+7][0..8] are 72 contiguous floats: 18 float4 loads
  float wreg[72];
  float tmp[72];
  {
    const float4* wp = reinterpret_cast<const float4*>(flat + o.w2 + (lane & 31) * K2 + 72 * (lane >> 5));
#pragma unroll
    for (int q = 0; q < 18; ++q) {
      const float4 v = wp[q];
      tmp[4 * q] = v.x;
      tmp[4 * q + 1] = v.y;
      tmp[4 * q + 2] = v.z;
      tmp[4 * q + 3] = v.w;
    }
  }
  const float bias2 = flat[o.b2 + (lane & 31)];
  // conv1 on MFMAs (X3 at W = 8: conv1_mfma; W = 16: conv1_mfma16): this lane's B operands W1[c][4 i + g] and
  // b1[c], c = lane & 15
  constexpr bool C1M = (X3 && W == 8) || W == 16;
  [[maybe_unused]] float w1f[5], b1c = 0.f;
  if constexpr (C1M) {
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const int k = 4 * i + (lane >> 4);
      w1f[i] = k < K1 ? flat[o.w1 + (lane & 15) * K1 + k] : 0.f;
    }
    b1c = flat[o.b1 + (lane & 15)];
  }
#pragma unroll
  for (int k = 0; k < WLQ; ++k) keep_loaded(vwl[k]);
#pragma unroll
  for (int k = 0; k < WLQ; ++k) {
    const int i = threadIdx.x + k * NTH;
    if (i < wl_tot) *reinterpret_cast<float4*>(ws + (i / q4) * (G::F + 4) + 4 * (i % q4)) = vwl[k];
  }
  if (threadIdx.x < n) ws[n * (G::F + 4) + threadIdx.x] = vbl;
#pragma unroll
  for (int k = 0; k < W1Q; ++k) {   // W1 [co][k] -> [k][co] (+ bias)
    const int i = threadIdx.x + k * NTH;
    if (i < C1 * K1 + C1) w1s[i < C1 * K1 ? (i % K1) * C1 + i / K1 : i] = vw1[k];
  }
  static_assert(G::FWD % 4 == 0 && G::BWD % 4 == 0, "float4 image fills");
  for (int i = lane; i < G::FWD / 4; i += 64)   // zero halos once; interiors rewritten per sample
    reinterpret_cast<float4*>(act)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int t = 0; t < 9; ++t) wreg[t * 8 + j] = tmp[j * 9 + t];

  [[maybe_unused]] bf16x8_t wx3[X3 ? 18 : 1];
  if constexpr (X3) {
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        __bf16 h, l;
        split_bf16(wreg[t * 8 + j], h, l);
        wx3[t][j] = h;
        wx3[9 + t][j] = l;
      }
    // the backward's W2T hi / lo image [part][tap][ci (48)][co] (qsc2_bwd3_kernel copies it instead of
    // transposing W2 in every workgroup): block 0's first wave holds the whole W2, lane = (co, ci half)
    if (w2t_img && blockIdx.x == 0 && wv == 0) {
      const int co = lane & 31, c8 = 8 * (lane >> 5);
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          w2t_img[(t * C1 + c8 + j) * 48 + co] = wx3[t][j];
          w2t_img[9 * C1 * 48 + (t * C1 + c8 + j) * 48 + co] = wx3[9 + t][j];
        }
    }
  }
  __syncthreads();
  if constexpr (STAMP) ts[1] = stamp();
  const float* wl = ws;
  const float* bl = wl + n * wl_stride(G::F);
  bool first = true;
  for (int s = blockIdx.x * NWV + wv; s < B; s += gridDim.x * NWV) {
    float* p1g = sv.p1 + (size_t)s * C1 * G::HW2;
    uint32_t* c1g = sv.c1 + (size_t)s * G::HW2;
    const float4* xp = s == blockIdx.x * NWV + wv ? &xpre : nullptr;
    if (STAMP && first)
      sample_forward<H, W, true, true, X3>(x + (size_t)s * 2 * G::HW, ws, act, lane, wreg, w1s, w1s + C1 * K1,
                                           bias2, p1g, c1g, ts, wx3, xp, w1f, b1c);
    else
      sample_forward<H, W, true, false, X3>(x + (size_t)s * 2 * G::HW, ws, act, lane, wreg, w1s, w1s + C1 * K1,
                                            bias2, p1g, c1g, nullptr, wx3, xp, w1f, b1c);
    float* p2s = act + G::o_p2f;
#pragma unroll
    for (int i = 0; i < G::F / 64; ++i) {
      int rel;
      const float v = pool2<H, W>(act, lane + 64 * i, rel);
      p2s[lane + 64 * i] = v;
      p2[(size_t)s * G::F + lane + 64 * i] = v;
      sv.c2[(size_t)s * G::F + lane + 64 * i] = (uint8_t)rel;
    }
    wave_lds_fence();
    // linear: 4 lanes per output j (n <= 16), interleaved f (conflict-free), then 2 shuffles
    {
      const int j = lane >> 2, part = lane & 3;
      float acc = 0.f;
      if (j < n) {
        const float* wj = wl + j * wl_stride(G::F);
#pragma unroll 8
        for (int f = part; f < G::F; f += 4) acc += p2s[f] * wj[f];
      }
      acc += __shfl_xor(acc, 1);
      acc += __shfl_xor(acc, 2);
      if (j < n && part == 0) angles[(size_t)s * n + j] = tanhf(acc + bl[j]);
    }
    if (STAMP && first) {
      ts[5] = stamp();
      first = false;
    }
  }
  if constexpr (STAMP) {
    ts[6] = stamp();
    if (lane == 0)
      for (int k = 0; k < NSTAMP; ++k) stamps[(size_t)(blockIdx.x * NWV + wv) * NSTAMP + k] = ts[k];
  }
}

// The workgroup's slab row from its waves' partial rows (red: NWV rows of RW floats, w2 | w1 | b1 | b2 | bl (16 slots) |
// wl [n][F] from RW0 when wl_here) and the quantum-slab column sums (qred: 256 floats, zero past qs.width; null: summed
// here from the rows [q0, q1) of qs), four columns per thread and step (round 6: one column per step ran a ~90-instruction
// range search per column, ~17k cycles per workgroup, profiles/r6_07_*).  Every flat range starts on a 16-float boundary
// (FlatParamSpace ALIGN) and the partial rows hold zeros past a range's end up to its 4-float boundary, so a 4-column
// chunk never mixes two ranges; every sum runs in the order of the one-column loop (bit-identical slab rows).
template <int NWV>
__device__ __forceinline__ void slab_row_out(float* __restrict__ row, const float* red, int RW, int RW0,
                                             const float* qred, QSlab qs, int q0, int q1, Offs o, int n, int F,
                                             bool wl_here) {
  for (int i = 4 * threadIdx.x; i < o.row; i += 4 * 64 * NWV) {
    const int a = i + o.base;   // flat offset of the chunk's first column
    int src = -1;
    if (a >= o.w2 && a < o.w2 + C2 * K2) src = a - o.w2;
    else if (a >= o.w1 && a < o.w1 + C1 * K1) src = C2 * K2 + (a - o.w1);
    else if (a >= o.b1 && a < o.b1 + C1) src = C2 * K2 + C1 * K1 + (a - o.b1);
    else if (a >= o.b2 && a < o.b2 + C2) src = C2 * K2 + C1 * K1 + C1 + (a - o.b2);
    else if (a >= o.bl && a < o.bl + n) src = C2 * K2 + C1 * K1 + C1 + C2 + (a - o.bl);
    else if (wl_here && a >= o.wl && a < o.wl + n * F) src = RW0 + (a - o.wl);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (src >= 0) {
#pragma unroll
      for (int w = 0; w < NWV; ++w) {
        const float4 r = *reinterpret_cast<const float4*>(red + w * RW + src);
        v.x += r.x;
        v.y += r.y;
        v.z += r.z;
        v.w += r.w;
      }
    } else if (qs.slab && a >= o.qw && a < o.qw + qs.width) {
      if (qred) {
        v = *reinterpret_cast<const float4*>(qred + (a - o.qw));
      } else {
        float e[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (a + c < o.qw + qs.width) {
            const float* qc = qs.slab + (a + c - o.qw);
#pragma unroll 4
            for (int r = q0; r < q1; ++r) e[c] += qc[(size_t)r * qs.width];
          }
        v = make_float4(e[0], e[1], e[2], e[3]);
      }
    }
    *reinterpret_cast<float4*>(row + i) = v;
  }
}

// Backward.  dang (B, n) = dL/d(angles).  Outputs: dpre (B, n) = dL/d(pre-tanh), slab row per
// workgroup = grads of [w1 | b1 | w2 | b2 | wl | bl] in the flat layout starting at o.w1 (wl
// columns zero when n > 64 / (F / 64): the caller then forms dWl = dpre^T p2 with a GEMM).
template <int H, int W, int NWV, bool STAMP = false>
__global__ void __launch_bounds__(64 * NWV) qsc2_bwd_kernel(const float* __restrict__ x, const float* __restrict__ flat,
                                                      Offs o, const float* __restrict__ angles,
                                                      const float* __restrict__ dang, float* __restrict__ dpre_out,
                                                      float* __restrict__ slab, const float* __restrict__ p2,
                                                      Saved sv, int B, int n, int wlk, QSlab qs,
                                                      unsigned long long* __restrict__ stamps = nullptr) {
  unsigned long long ts[NSTAMP] = {};
  bool first = true;
  if constexpr (STAMP) ts[0] = stamp();
  using G = Geo<H, W>;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* ws = sm;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float* act = sm + act_base_bwd(n, G::F) + wv * G::BWD;
  float* w2t = sm + act_base(n, G::F);
  stage_weights(flat, o, ws, n, G::F);
  for (int i = lane; i < G::BWD / 4; i += 64) reinterpret_cast<float4*>(act)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  for (int i = threadIdx.x; i < C2 * K2; i += 64 * NWV) {   // W2 [co][ci][tap] -> W2T [tap][ci][co]
    const int co = i / K2, ci = (i % K2) / 9, t = i % 9;
    w2t[(t * C1 + ci) * W2T_CS + co] = ws[S_W2 + i];
  }
  __syncthreads();
  const float* wl = ws + S_WEND;
  const int col32 = lane & 31, kh = lane >> 5;     // 32x32x2 operand coordinates
  const int col16 = lane & 15, kq = lane >> 4;     // 16x16x4 operand coordinates
  f32x16 gw2[5];                                   // dW2 tiles: rows = co, cols = k in [32t, 32t+32)
#pragma unroll
  for (int t = 0; t < 5; ++t) gw2[t] = (f32x16){};
  f32x4 gw1[2];                                    // dW1 tiles: rows = co, cols = k in [16t, 16t+16)
  gw1[0] = (f32x4){};
  gw1[1] = (f32x4){};
  constexpr int FPL = G::F / 64;              // pool-2 features per lane (f = FPL * lane + i)
  constexpr int XQ = 2 * G::HW / 256;          // float4s of x per lane
  constexpr int P1Q = C1 * G::HW2 / 256;       // float4s of the saved pool-1 map per lane
  constexpr int CPL = C1 * G::HW2 / 64;        // pool-1 (channel, window) pairs per lane
  static_assert(FPL % 4 == 0 && XQ >= 1 && P1Q >= 1 && 64 % G::HW2 == 0, "lane mappings");
  float gb1[CPL], gb2 = 0.f, gbl = 0.f;
#pragma unroll
  for (int c = 0; c < CPL; ++c) gb1[c] = 0.f;
  // linear-layer weight gradient dWl[j][f] += dpre[j] * p2[f], accumulated in registers over the
  // wave's samples (lane = features FPL*lane ..) when n <= NWL: no separate GEMM launch
  constexpr int NWL = 64 / FPL;
  const bool wl_here = wlk != 0;   // host guarantees n <= NWL and the LDS reduction fits
  float gwl[NWL][FPL];
#pragma unroll
  for (int j = 0; j < NWL; ++j)
#pragma unroll
    for (int i = 0; i < FPL; ++i) gwl[j][i] = 0.f;

  // ---- one-sample-ahead register prefetch of everything a sample reads from global memory ----
  // ext-vector registers (float4 is a struct: arrays of it are copied by memcpy and land in scratch)
  f32x4 rx[XQ], rp1[P1Q], rp2[FPL / 4];
  uint32_t rc2[FPL / 4], rc1 = 0;
  float rth = 0.f, rda = 0.f;
  auto prefetch = [&](int s) {
    const f32x4* x4 = reinterpret_cast<const f32x4*>(x + (size_t)s * 2 * G::HW);
#pragma unroll
    for (int q = 0; q < XQ; ++q) rx[q] = x4[lane + 64 * q];
    const f32x4* p4 = reinterpret_cast<const f32x4*>(sv.p1 + (size_t)s * C1 * G::HW2);
#pragma unroll
    for (int q = 0; q < P1Q; ++q) rp1[q] = p4[lane + 64 * q];
    const f32x4* q4 = reinterpret_cast<const f32x4*>(p2 + (size_t)s * G::F + FPL * lane);
    const uint32_t* c4 = reinterpret_cast<const uint32_t*>(sv.c2 + (size_t)s * G::F + FPL * lane);
#pragma unroll
    for (int q = 0; q < FPL / 4; ++q) {
      rp2[q] = q4[q];
      rc2[q] = c4[q];
    }
    rc1 = sv.c1[(size_t)s * G::HW2 + lane % G::HW2];
    if (lane < n) {
      rth = angles[(size_t)s * n + lane];
      rda = dang[(size_t)s * n + lane];
    }
  };
  const int s0 = blockIdx.x * NWV + wv;
  if (s0 < B) prefetch(s0);

  for (int s = s0; s < B; s += gridDim.x * NWV) {
    if (STAMP && first) ts[1] = stamp();
    // ---- this sample's saved state -> LDS images (x padded, p1 padded channel-last) ----
#pragma unroll
    for (int q = 0; q < XQ; ++q) {
      const int i = lane + 64 * q, c = (4 * i) / G::HW, p = (4 * i) % G::HW;
      float* d = act + G::o_x + c * G::XP + (p / W + 1) * G::XW + p % W + 1;
      d[0] = rx[q][0];
      d[1] = rx[q][1];
      d[2] = rx[q][2];
      d[3] = rx[q][3];
    }
#pragma unroll
    for (int q = 0; q < P1Q; ++q) {
      const int i = lane + 64 * q, win = i >> 2, cq = i & 3;
      const int qy = win / G::W2, qx = win % G::W2;
      *reinterpret_cast<f32x4*>(act + G::o_p1 + ((qy + 1) * G::PW + qx + 1) * G::PC + 4 * cq) = rp1[q];
    }
    float* misc = act + G::o_misc;
    if (lane < n) {
      const float d = rda * (1.f - rth * rth);
      misc[lane] = d;
      dpre_out[(size_t)s * n + lane] = d;
      gbl += d;
    }
    float p2v[FPL];
    uint32_t c2v[FPL / 4], c1v = rc1;
#pragma unroll
    for (int q = 0; q < FPL / 4; ++q) {
      p2v[4 * q] = rp2[q][0];
      p2v[4 * q + 1] = rp2[q][1];
      p2v[4 * q + 2] = rp2[q][2];
      p2v[4 * q + 3] = rp2[q][3];
      c2v[q] = rc2[q];
    }
    if (s + gridDim.x * NWV < B) prefetch(s + gridDim.x * NWV);
    // dz2's zero halo is clobbered by the previous sample's dz1 (aliased): re-zero the image
    for (int i = lane; i < G::PP * G::DC / 4; i += 64)
      reinterpret_cast<float4*>(act + G::o_dz2)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    wave_lds_fence();
    if (STAMP && first) ts[2] = stamp();
    // linear backward -> dp2 (FPL consecutive features per lane: float4 weight reads), pool-2
    // backward through the saved window choice (+ReLU: passes iff the pooled value is > 0)
    {
      float dp[FPL];
#pragma unroll
      for (int i = 0; i < FPL; ++i) dp[i] = 0.f;
      for (int j = 0; j < n; ++j) {
        const float mj = misc[j];
        const float4* wr = reinterpret_cast<const float4*>(wl + j * wl_stride(G::F) + FPL * lane);
#pragma unroll
        for (int q = 0; q < FPL / 4; ++q) {
          const float4 w4 = wr[q];
          dp[4 * q] += w4.x * mj;
          dp[4 * q + 1] += w4.y * mj;
          dp[4 * q + 2] += w4.z * mj;
          dp[4 * q + 3] += w4.w * mj;
        }
      }
      if (wl_here) {
#pragma unroll
        for (int j = 0; j < NWL; ++j) {
          const float mj = j < n ? misc[j] : 0.f;
#pragma unroll
          for (int i = 0; i < FPL; ++i) gwl[j][i] += mj * p2v[i];
        }
      }
#pragma unroll
      for (int i = 0; i < FPL; ++i) {
        const int f = FPL * lane + i;
        const int c = f / G::HW4, q = f % G::HW4, qy = q / G::W4, qx = q % G::W4;
        const int rel = (c2v[i / 4] >> (8 * (i % 4))) & 0xff;
        const float g = p2v[i] > 0.f ? dp[i] : 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int py = 2 * qy + (r >> 1), px = 2 * qx + (r & 1);
          act[G::o_dz2 + ((py + 1) * G::PW + px + 1) * G::DC + c] = (r == rel) ? g : 0.f;
        }
      }
    }
    wave_lds_fence();
    if (STAMP && first) ts[3] = stamp();
    // conv2 bias grad: lane (co, half) sums half of the positions
    {
      const float* dz = act + G::o_dz2 + col32;
      for (int p = kh; p < G::HW2; p += 2) gb2 += dz[((p / G::W2 + 1) * G::PW + p % G::W2 + 1) * G::DC];
    }
    // conv2 weight grads: dW2[co][k] += sum_pos dz2[co][pos] * im2col(p1)[pos][k]  (K = positions)
#pragma unroll 2
    for (int kk = 0; kk < G::HW2 / 2; ++kk) {
      const int pos = 2 * kk + kh;
      const int py = pos / G::W2, px = pos % G::W2;
      const float a = act[G::o_dz2 + ((py + 1) * G::PW + px + 1) * G::DC + col32];
#pragma unroll
      for (int t = 0; t < 5; ++t) {
        const int k = 32 * t + col32;   // column = tap * 16 + ci (16 lanes read 16 contiguous channels)
        float b = 0.f;
        if (k < K2) {
          const int tp = k >> 4, ci = k & 15;
          b = act[G::o_p1 + ((py + tp / 3) * G::PW + px + tp % 3) * G::PC + ci];
        }
        gw2[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, gw2[t], 0, 0, 0);
      }
    }
    if (STAMP && first) ts[4] = stamp();
    // conv2 data grads: dp1[ci][pos] = sum_{tap,co} dz2_pad[pos + 2 - tap][co] * W2[co][ci][tap].
    // MFMA step j of tap t sums k = (t, co = 8*kq + j) over the four lane groups kq: a lane's 8 A
    // (dz2, channel-last) and 8 B (W2T, co-contiguous) operands of a tap are 2 + 2 ds_read_b128.
    for (int mt = 0; mt < G::MT1; ++mt) {
      const int pos = 16 * mt + col16;
      const int py = pos / G::W2, px = pos % G::W2;
      f32x4 acc = {};
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const float4* ap = reinterpret_cast<const float4*>(
            act + G::o_dz2 + ((py + 2 - t / 3) * G::PW + px + 2 - t % 3) * G::DC + 8 * kq);
        const float4* bp = reinterpret_cast<const float4*>(w2t + (t * C1 + col16) * W2T_CS + 8 * kq);
        const float4 a0 = ap[0], a1 = ap[1], b0 = bp[0], b1 = bp[1];
        const float a[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        const float b[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[j], acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) act[G::o_dp1 + col16 * G::HW2 + 16 * mt + 4 * kq + r] = acc[r];
    }
    wave_lds_fence();
    if (STAMP && first) ts[5] = stamp();
    // pool-1 backward through the saved window choices (+ReLU: passes iff p1 > 0): lane = window,
    // CPL channels; every 2x2 window of dz1 (C1 x HW) is written whole
    {
      const int win = lane % G::HW2, cb = (lane / G::HW2) * CPL;
      const int qy = win / G::W2, qx = win % G::W2;
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        const int co = cb + c;
        const float pv = act[G::o_p1 + ((qy + 1) * G::PW + qx + 1) * G::PC + co];
        const float g = pv > 0.f ? act[G::o_dp1 + co * G::HW2 + win] : 0.f;
        gb1[c] += g;
        const uint32_t code = (c1v >> (2 * co)) & 3u;
        float* dz = act + G::o_dz1 + co * G::HW + (2 * qy) * W + 2 * qx;
        dz[0] = code == 0 ? g : 0.f;
        dz[1] = code == 1 ? g : 0.f;
        dz[W] = code == 2 ? g : 0.f;
        dz[W + 1] = code == 3 ? g : 0.f;
      }
    }
    wave_lds_fence();
    if (STAMP && first) ts[6] = stamp();
    // conv1 weight grads: dW1[co][k] += sum_pos dz1[co][pos] * im2col(x)[pos][k]  (K = positions)
#pragma unroll 4
    for (int kk = 0; kk < G::HW / 4; ++kk) {
      const int pos = 4 * kk + kq;
      const int py = pos / W, px = pos % W;
      const float a = act[G::o_dz1 + col16 * G::HW + pos];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int k = 16 * t + col16;
        float b = 0.f;
        if (k < K1) {
          const int ci = k / 9, tp = k % 9;
          b = act[G::o_x + ci * G::XP + (py + tp / 3) * G::XW + px + tp % 3];
        }
        gw1[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, gw1[t], 0, 0, 0);
      }
    }
    wave_lds_fence();
    if (STAMP && first) {
      ts[7] = stamp();
      first = false;
    }
  }

  // ---- deterministic workgroup reduction -> slab row (w1 | b1 | w2 | b2 | wl = 0 | bl) ----
  __syncthreads();
  float* red = sm + S_WEND;   // reuse the activation images: NWV x RW
  constexpr int RW0 = C2 * K2 + C1 * K1 + C1 + C2 + 16;
  const int RW = RW0 + (wl_here ? n * G::F : 0);   // ... | wl [n][F]
  float* mine = red + wv * RW;
  if (wl_here) {
#pragma unroll
    for (int j = 0; j < NWL; ++j)
      if (j < n) {
#pragma unroll
        for (int q = 0; q < FPL / 4; ++q)
          *reinterpret_cast<float4*>(mine + RW0 + j * G::F + FPL * lane + 4 * q) =
              make_float4(gwl[j][4 * q], gwl[j][4 * q + 1], gwl[j][4 * q + 2], gwl[j][4 * q + 3]);
      }
  }
#pragma unroll
  for (int t = 0; t < 5; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = (r & 3) + 8 * (r >> 2) + 4 * kh, k = 32 * t + col32;
      if (k < K2) mine[co * K2 + (k & 15) * 9 + (k >> 4)] = gw2[t][r];   // (tap, ci) -> flat [ci][tap]
    }
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = 4 * kq + r, k = 16 * t + col16;
      if (k < K1) mine[C2 * K2 + co * K1 + k] = gw1[t][r];
    }
  // b1: lane (window, channel block cb) holds channels cb .. cb+CPL-1; sum over the windows
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    float v = gb1[c];
#pragma unroll
    for (int off = 1; off < G::HW2; off <<= 1) v += __shfl_xor(v, off);
    if (lane % G::HW2 == 0) mine[C2 * K2 + C1 * K1 + (lane / G::HW2) * CPL + c] = v;
  }
  {
    const float v = gb2 + __shfl_xor(gb2, 32);
    if (kh == 0) mine[C2 * K2 + C1 * K1 + C1 + col32] = v;
  }
  if (lane < 16) mine[C2 * K2 + C1 * K1 + C1 + C2 + lane] = lane < n ? gbl : 0.f;
  __syncthreads();
  float* row = slab + (size_t)blockIdx.x * o.row;
  if constexpr (STAMP) {
    ts[8] = stamp();
    if (lane == 0)
      for (int k = 0; k < NSTAMP; ++k) stamps[(size_t)(blockIdx.x * NWV + wv) * NSTAMP + k] = ts[k];
  }
  // this workgroup's share of the quantum-layer slab rows
  const int q0 = (int)((long long)qs.rows * blockIdx.x / gridDim.x);
  const int q1 = (int)((long long)qs.rows * (blockIdx.x + 1) / gridDim.x);
  slab_row_out<NWV>(row, red, RW, RW0, nullptr, qs, q0, q1, o, n, G::F, wl_here);
}

// ----------------------------------------------------------------------------------------------
// qsc2_bwd3_kernel (P128): the backward with every matrix product on bf16 MFMAs at fp32-grade
// accuracy ("bf16x3": each fp32 operand v = hi + lo, hi = bf16(v), lo = bf16(v - hi), and
// a.b ~= ah.bh + ah.bl + al.bh with fp32 accumulation; relative error ~1e-5).  The f32-input MFMA
// it replaces runs at 1/16 of the bf16 rate (64 cycles per 32x32x2): three bf16 products per fp32
// product are still 5x fewer MFMA cycles, and the operands come as whole 8/16-byte fragments
// instead of one float per lane per instruction.  Same phases, outputs and slab row as
// qsc2_bwd_kernel (the f32 kernel stays the P256 path and the reference of the GPU test).
// Per-wave LDS images, bf16 [part = hi | lo]:
//   XS  [2][kw][ci 2][18][8]    input x, three column-shifted copies      (conv1 wgrad B)
//   P1S [2][kw (644)][ci 16][10][4]  pool-1 map, three column-shifted copies (conv2 wgrad B, pool-1 mask)
//   DZT [2][co 32][40]          dz2 co-major                              (conv2 wgrad A)   } aliased
//   DZC [2][60][32]             dz2 channel-last, padded 10 x 6, 8-co chunk q at q ^ 2 (row & 1)
//                                                                          (conv2 dgrad A)   } by DZ1
//   DZ1 [2][ci 16][144]         dz1 co-major                              (conv1 wgrad A)
//   DP1 [16][32] fp32           conv2 data gradient
// block-shared: the linear layer (fp32, as qsc2_bwd_kernel) and W2T [2][tap][ci (48)][co 32] (dgrad B).
// Strides, pads and the DZC swizzle make every MFMA operand read conflict-free (modelled exhaustively
// with the ds_read_b64 / b128 lane groups before the build; the first layout measured 2.5 conflict
// cycles per LDS instruction).
// ----------------------------------------------------------------------------------------------
struct B3 {   // P128 geometry of the bf16 images (elements)
  static constexpr int XS_PART = 3 * 2 * 18 * 8, XS = 2 * XS_PART;
  static constexpr int P1S_CS = 644;   // kw-copy stride (16 * 40 + 4: the two taps of a 32-lane half apart)
  static constexpr int P1S_PART = 3 * P1S_CS, P1S = 2 * P1S_PART;
  static constexpr int DZT_RS = 40, DZT_PART = 32 * DZT_RS, DZT = 2 * DZT_PART;
  static constexpr int DZC_PART = 60 * 32, DZC = 2 * DZC_PART;
  static constexpr int DZ1_RS = 144, DZ1_PART = 16 * DZ1_RS, DZ1 = 2 * DZ1_PART;
  static_assert(DZ1 <= DZT + DZC, "dz1 alias");
  static constexpr int BF = XS + P1S + DZT + DZC;                   // bf16 elements per wave
  static constexpr int WAVE_BYTES = BF * 2 + 16 * 32 * 4 + 32 * 4;  // + DP1 + misc
  static constexpr int W2T_CS = 48, W2T_PART = 9 * 16 * W2T_CS, W2T = 2 * W2T_PART;
};
static_assert(B3::WAVE_BYTES % 16 == 0, "16-byte wave images");

__device__ __forceinline__ int dzc_off(int P, int c) {   // padded position P (= row * 6 + col), channel c
  return P * 32 + (((c >> 3) ^ (2 * ((P / 6) & 1))) << 3) + (c & 7);
}
template <int NWV, bool STAMP = false>
__global__ void __launch_bounds__(64 * NWV) qsc2_bwd3_kernel(const float* __restrict__ x, const float* __restrict__ flat,
                                                         Offs o, const float* __restrict__ angles,
                                                         const float* __restrict__ dang, float* __restrict__ dpre_out,
                                                         float* __restrict__ slab, const float* __restrict__ p2, Saved sv,
                                                         int B, int n, int wlk, QSlab qs,
                                                         unsigned long long* __restrict__ stamps = nullptr,
                                                         const __bf16* __restrict__ w2t_img = nullptr) {
  // STAMP (diagnostic builds): [0] start [1] prologue [2] staging [3] linear + pool-2 bwd [4] conv2 wgrad
  // [5] conv2 dgrad [6] pool-1 bwd [7] conv1 wgrad (first sample) [8] samples done [9] end
  unsigned long long ts[NSTAMP] = {};
  bool first = true;
  if constexpr (STAMP) ts[0] = stamp();
  using G = Geo<16, 8>;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // ---- one-sample-ahead register prefetch (the first sample's loads fly during the prologue) ----
  constexpr int FPL = G::F / 64;   // 4 pool-2 features per lane: channel lane / 2, cells 4 (lane & 1) + i
  f32x4 rx[2];           // lanes 0..31: x row (c = lane / 16, image row lane % 16)
  float rp1[2][4];       // (ci, pool-1 row) pairs lane, lane + 64: 4 columns
  f32x4 rp2;
  uint32_t rc2 = 0, rc1 = 0;
  float rth = 0.f, rda = 0.f;
  auto prefetch = [&](int s) {
    if (lane < 32) {
      const f32x4* x4 = reinterpret_cast<const f32x4*>(x + (size_t)s * 2 * G::HW + lane * 8);
      rx[0] = x4[0];
      rx[1] = x4[1];
    }
    const float* p1 = sv.p1 + (size_t)s * C1 * G::HW2;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int pr = lane + 64 * r, ci = pr >> 3, qy = pr & 7;
#pragma unroll
      for (int qx = 0; qx < 4; ++qx) rp1[r][qx] = p1[(qy * 4 + qx) * C1 + ci];
    }
    rp2 = *reinterpret_cast<const f32x4*>(p2 + (size_t)s * G::F + FPL * lane);
    rc2 = *reinterpret_cast<const uint32_t*>(sv.c2 + (size_t)s * G::F + FPL * lane);
    rc1 = sv.c1[(size_t)s * G::HW2 + (lane & 31)];
    if (lane < n) {
      rth = angles[(size_t)s * n + lane];
      rda = dang[(size_t)s * n + lane];
    }
  };
  const int s0 = blockIdx.x * NWV + wv;
  if (s0 < B) prefetch(s0);
  // ---- block-shared: linear layer (fp32) | W2T hi / lo ----
  float* wl = sm;
  const int wl_floats = (n * wl_stride(G::F) + 16 + 3) & ~3;
  __bf16* w2t = reinterpret_cast<__bf16*>(sm + wl_floats);
  char* wbase = reinterpret_cast<char*>(w2t + B3::W2T) + wv * B3::WAVE_BYTES;
  __bf16* XS = reinterpret_cast<__bf16*>(wbase);
  __bf16* P1S = XS + B3::XS;
  __bf16* DZT = P1S + B3::P1S;
  __bf16* DZC = DZT + B3::DZT;
  __bf16* DZ1 = DZT;   // (alias: dz2 images are dead once the conv2 data gradient is done)
  float* DP1 = reinterpret_cast<float*>(DZC + B3::DZC);
  float* misc = DP1 + 16 * 32;
  // this workgroup's share of the quantum layer's adjoint slab rows (summed into its slab row at the end): the
  // loads fly with the weight loads below -- at the end they cost the workgroup's last wave a round trip per
  // 4 rows (round 6)
  const int q0 = (int)((long long)qs.rows * blockIdx.x / gridDim.x);
  const int q1 = (int)((long long)qs.rows * (blockIdx.x + 1) / gridDim.x);
  constexpr int QPF = 16;   // rows prefetched; a longer share sums the rest at the end
  const bool q_mine = qs.slab && (int)threadIdx.x < qs.width;
  float qv[QPF];
  {
    const float* qc = qs.slab + (q_mine ? threadIdx.x : 0);
#pragma unroll
    for (int k = 0; k < QPF; ++k) qv[k] = q_mine && q0 + k < q1 ? qc[(size_t)(q0 + k) * qs.width] : 0.f;
  }
  {
    // the linear layer and (when the forward wrote it) the W2T image: every load in flight together, then the
    // stores -- one round trip (an index past the end re-loads element 0, not stored; round 6 merged the two
    // copies' round trips)
    const int q4 = G::F / 4, tot = n * q4;   // (n <= 16: tot <= 4 x 256)
    const float4* src = reinterpret_cast<const float4*>(flat + o.wl);
    float4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = threadIdx.x + k * 256;
      v[k] = src[i < tot ? i : 0];
    }
    constexpr int NCP = (B3::W2T * 2 / 16 + 255) / 256;
    uint4 vi[NCP];
    if (w2t_img) {
      const uint4* isrc = reinterpret_cast<const uint4*>(w2t_img);
#pragma unroll
      for (int k = 0; k < NCP; ++k) {
        const int i = threadIdx.x + 256 * k;
        vi[k] = isrc[i < B3::W2T * 2 / 16 ? i : 0];
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) keep_loaded(v[k]);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = threadIdx.x + k * 256;
      if (i < tot) *reinterpret_cast<float4*>(wl + (i / q4) * wl_stride(G::F) + 4 * (i % q4)) = v[k];
    }
    if (w2t_img) {   // this step's image from the forward (qd_qsc2_fwd3)
      uint4* dst = reinterpret_cast<uint4*>(w2t);
#pragma unroll
      for (int k = 0; k < NCP; ++k) keep_loaded(vi[k]);
#pragma unroll
      for (int k = 0; k < NCP; ++k) {
        const int i = threadIdx.x + 256 * k;
        if (i < B3::W2T * 2 / 16) dst[i] = vi[k];
      }
    } else
    // W2 [co][ci][tap] -> W2T [tap][ci][co]: iterate in DESTINATION order, two co per dword (in source
    // order the 2-byte writes of a wave landed 64 B apart: 32-way bank conflicts, ~5 us per workgroup)
#pragma unroll 3
    for (int i = threadIdx.x; i < 9 * C1 * 16; i += blockDim.x) {
      const int t = i / (C1 * 16), ci = (i / 16) % C1, cp = i % 16;
      __bf16 h0, l0, h1, l1;
      split_bf16(flat[o.w2 + ((2 * cp) * C1 + ci) * 9 + t], h0, l0);
      split_bf16(flat[o.w2 + ((2 * cp + 1) * C1 + ci) * 9 + t], h1, l1);
      const int d = ((t * C1 + ci) * B3::W2T_CS + 2 * cp) >> 1;
      reinterpret_cast<uint32_t*>(w2t)[d] = (uint32_t)__builtin_bit_cast(uint16_t, h0) |
                                            ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
      reinterpret_cast<uint32_t*>(w2t + B3::W2T_PART)[d] = (uint32_t)__builtin_bit_cast(uint16_t, l0) |
                                                           ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
    }
  }
  for (int i = lane; i < B3::WAVE_BYTES / 16; i += 64) reinterpret_cast<uint4*>(wbase)[i] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  if constexpr (STAMP) ts[1] = stamp();
  const int col32 = lane & 31, kh = lane >> 5;
  const int col16 = lane & 15, kq = lane >> 4;
  f32x16 gw2[5];
#pragma unroll
  for (int t = 0; t < 5; ++t) gw2[t] = (f32x16){};
  f32x4 gw1[2];
  gw1[0] = (f32x4){};
  gw1[1] = (f32x4){};
  float gb2 = 0.f, gbl = 0.f, gb1[4] = {0.f, 0.f, 0.f, 0.f};
  constexpr int NWL = 64 / FPL;
  const bool wl_here = wlk != 0;
  float gwl[NWL][FPL];
#pragma unroll
  for (int j = 0; j < NWL; ++j)
#pragma unroll
    for (int i = 0; i < FPL; ++i) gwl[j][i] = 0.f;


  for (int s = s0; s < B; s += gridDim.x * NWV) {
    // ---- saved state -> shifted bf16 copies ----
    if (lane < 32) {
      const int c = lane >> 4, ph = lane & 15;
      float v[10];
      v[0] = 0.f;
      v[9] = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v[1 + q] = rx[0][q];
        v[5 + q] = rx[1][q];
      }
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        bf16x8_t h, l;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          __bf16 a, b;
          split_bf16(v[j + kw], a, b);
          h[j] = a;
          l[j] = b;
        }
        const int off = ((kw * 2 + c) * 18 + ph + 1) * 8;
        *reinterpret_cast<bf16x8_t*>(XS + off) = h;
        *reinterpret_cast<bf16x8_t*>(XS + B3::XS_PART + off) = l;
      }
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int pr = lane + 64 * r, ci = pr >> 3, qy = pr & 7;
      float v[6] = {0.f, rp1[r][0], rp1[r][1], rp1[r][2], rp1[r][3], 0.f};
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        bf16x4_t h, l;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          __bf16 a, b;
          split_bf16(v[j + kw], a, b);
          h[j] = a;
          l[j] = b;
        }
        const int off = kw * B3::P1S_CS + (ci * 10 + qy + 1) * 4;
        *reinterpret_cast<bf16x4_t*>(P1S + off) = h;
        *reinterpret_cast<bf16x4_t*>(P1S + B3::P1S_PART + off) = l;
      }
    }
    if (lane < n) {
      const float d = rda * (1.f - rth * rth);
      misc[lane] = d;
      dpre_out[(size_t)s * n + lane] = d;
      gbl += d;
    }
    const f32x4 p2v = rp2;
    const uint32_t c2v = rc2, c1v = rc1;
    if (s + gridDim.x * NWV < B) prefetch(s + gridDim.x * NWV);
    // dz2's channel-last image is rewritten sparsely: clear it (dz1 of the previous sample aliased it)
    for (int i = lane; i < B3::DZC * 2 / 16; i += 64) reinterpret_cast<uint4*>(DZC)[i] = make_uint4(0, 0, 0, 0);
    wave_lds_fence();
    if (STAMP && first) ts[2] = stamp();
    // ---- linear backward -> dp2; pool-2 backward through the saved choice (+ReLU) -> dz2 ----
    {
      float dp[FPL];
#pragma unroll
      for (int i = 0; i < FPL; ++i) dp[i] = 0.f;
      for (int j = 0; j < n; ++j) {
        const float mj = misc[j];
        const float4 w4 = *reinterpret_cast<const float4*>(wl + j * wl_stride(G::F) + FPL * lane);
        dp[0] += w4.x * mj;
        dp[1] += w4.y * mj;
        dp[2] += w4.z * mj;
        dp[3] += w4.w * mj;
      }
      if (wl_here) {
#pragma unroll
        for (int j = 0; j < NWL; ++j) {
          const float mj = j < n ? misc[j] : 0.f;
#pragma unroll
          for (int i = 0; i < FPL; ++i) gwl[j][i] += mj * p2v[i];
        }
      }
      // lane: channel c = lane / 2, pool-1 rows 4 (lane & 1) .. +3 (16 positions, co-major contiguous)
      const int c = lane >> 1, hb = lane & 1;
      float v16[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) v16[k] = 0.f;
#pragma unroll
      for (int i = 0; i < FPL; ++i) {
        const int rel = (c2v >> (8 * i)) & 0xff;
        const float g = p2v[i] > 0.f ? dp[i] : 0.f;
        gb2 += g;
        const int lr = 2 * (i >> 1) + (rel >> 1), px = 2 * (i & 1) + (rel & 1);   // local pool-1 row, column
        v16[lr * 4 + px] = g;
        __bf16 h, l;
        split_bf16(g, h, l);
        const int py = 4 * hb + lr;
        DZC[dzc_off((py + 1) * 6 + px + 1, c)] = h;
        DZC[B3::DZC_PART + dzc_off((py + 1) * 6 + px + 1, c)] = l;
      }
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        bf16x8_t h, l;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          __bf16 a, b;
          split_bf16(v16[8 * hh + j], a, b);
          h[j] = a;
          l[j] = b;
        }
        const int off = c * B3::DZT_RS + 16 * hb + 8 * hh;
        *reinterpret_cast<bf16x8_t*>(DZT + off) = h;
        *reinterpret_cast<bf16x8_t*>(DZT + B3::DZT_PART + off) = l;
      }
    }
    wave_lds_fence();
    if (STAMP && first) ts[3] = stamp();
    // ---- conv2 weight grads: dW2[co][k] += sum_pos dz2[co][pos] * im2col(p1)[pos][k], K = positions;
    // A = DZT rows (co), B = P1S (k = tap * 16 + ci): two 8-byte rows of 4 positions per fragment ----
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int p0 = 16 * ks + 8 * kh;   // 8 positions = pool-1 rows p0 / 4, p0 / 4 + 1
      const bf16x8_t ah = *reinterpret_cast<const bf16x8_t*>(DZT + col32 * B3::DZT_RS + p0);
      const bf16x8_t al = *reinterpret_cast<const bf16x8_t*>(DZT + B3::DZT_PART + col32 * B3::DZT_RS + p0);
#pragma unroll
      for (int t = 0; t < 5; ++t) {
        const int k = 32 * t + col32;
        bf16x8_t bh = {}, bl = {};
        if (k < K2) {
          const int tp = k >> 4, ci = k & 15, ky = tp / 3, kx = tp % 3;
          const int off = kx * B3::P1S_CS + (ci * 10 + p0 / 4 + ky) * 4;
          const bf16x4_t h0 = *reinterpret_cast<const bf16x4_t*>(P1S + off);
          const bf16x4_t h1 = *reinterpret_cast<const bf16x4_t*>(P1S + off + 4);
          const bf16x4_t l0 = *reinterpret_cast<const bf16x4_t*>(P1S + B3::P1S_PART + off);
          const bf16x4_t l1 = *reinterpret_cast<const bf16x4_t*>(P1S + B3::P1S_PART + off + 4);
          bh = (bf16x8_t){h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
          bl = (bf16x8_t){l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
        }
        gw2[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, gw2[t], 0, 0, 0);
        gw2[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, gw2[t], 0, 0, 0);
        gw2[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, gw2[t], 0, 0, 0);
      }
    }
    if (STAMP && first) ts[4] = stamp();
    // ---- conv2 data grads: dp1[ci][pos] = sum_{tap, co} dz2_pad[pos + 2 - tap][co] W2[co][ci][tap];
    // 16x16x32: rows = 16 positions, cols = ci, K = one tap's 32 co ----
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int pos = 16 * mt + col16, py = pos >> 2, px = pos & 3;
      f32x4 acc = {};
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int ao = dzc_off((py + 2 - t / 3) * 6 + px + 2 - t % 3, 8 * kq);
        const int bo = (t * C1 + col16) * B3::W2T_CS + 8 * kq;
        const bf16x8_t ah = *reinterpret_cast<const bf16x8_t*>(DZC + ao);
        const bf16x8_t al = *reinterpret_cast<const bf16x8_t*>(DZC + B3::DZC_PART + ao);
        const bf16x8_t bh = *reinterpret_cast<const bf16x8_t*>(w2t + bo);
        const bf16x8_t bl = *reinterpret_cast<const bf16x8_t*>(w2t + B3::W2T_PART + bo);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) DP1[col16 * 32 + 16 * mt + 4 * kq + r] = acc[r];
    }
    wave_lds_fence();
    if (STAMP && first) ts[5] = stamp();
    // ---- pool-1 backward (+ReLU: passes iff p1 > 0): lane = (channel, image row) pairs, 8 positions
    // per pair written whole -> DZ1 (co-major); window codes from the lanes holding them ----
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int pr = lane + 64 * r, co = pr >> 4, row = pr & 15, qy = row >> 1, dy = row & 1;
      float v[8];
#pragma unroll
      for (int qx = 0; qx < 4; ++qx) {
        const int win = qy * 4 + qx;
        const float pv = (float)P1S[B3::P1S_CS + (co * 10 + qy + 1) * 4 + qx];   // kw = 1 copy, hi part
        const float g = pv > 0.f ? DP1[co * 32 + win] : 0.f;
        if (dy == 0) gb1[r] += g;
        const uint32_t code = (__shfl(c1v, win) >> (2 * co)) & 3u;
        v[2 * qx] = ((code >> 1) == (uint32_t)dy && (code & 1u) == 0u) ? g : 0.f;
        v[2 * qx + 1] = ((code >> 1) == (uint32_t)dy && (code & 1u) == 1u) ? g : 0.f;
      }
      bf16x8_t h, l;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        __bf16 a, b;
        split_bf16(v[j], a, b);
        h[j] = a;
        l[j] = b;
      }
      *reinterpret_cast<bf16x8_t*>(DZ1 + co * B3::DZ1_RS + row * 8) = h;
      *reinterpret_cast<bf16x8_t*>(DZ1 + B3::DZ1_PART + co * B3::DZ1_RS + row * 8) = l;
    }
    wave_lds_fence();
    if (STAMP && first) ts[6] = stamp();
    // ---- conv1 weight grads: dW1[co][k] += sum_pos dz1[co][pos] * im2col(x)[pos][k], k = ci * 9 + tap;
    // 16x16x32: K = 32 positions = 4 image rows, a lane's 8 = one row ----
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int row = 4 * ks + kq;
      const bf16x8_t ah = *reinterpret_cast<const bf16x8_t*>(DZ1 + col16 * B3::DZ1_RS + row * 8);
      const bf16x8_t al = *reinterpret_cast<const bf16x8_t*>(DZ1 + B3::DZ1_PART + col16 * B3::DZ1_RS + row * 8);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int k = 16 * t + col16;
        bf16x8_t bh = {}, bl = {};
        if (k < K1) {
          const int ci = k / 9, tp = k % 9;
          const int off = (((tp % 3) * 2 + ci) * 18 + row + tp / 3) * 8;
          bh = *reinterpret_cast<const bf16x8_t*>(XS + off);
          bl = *reinterpret_cast<const bf16x8_t*>(XS + B3::XS_PART + off);
        }
        gw1[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, gw1[t], 0, 0, 0);
        gw1[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, gw1[t], 0, 0, 0);
        gw1[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, gw1[t], 0, 0, 0);
      }
    }
    wave_lds_fence();
    if (STAMP && first) {
      ts[7] = stamp();
      first = false;
    }
  }
  if constexpr (STAMP) ts[8] = stamp();

  // ---- deterministic workgroup reduction -> slab row (w1 | b1 | w2 | b2 | wl | bl), as qsc2_bwd_kernel ----
  __syncthreads();
  float* red = sm;
  constexpr int RW0 = C2 * K2 + C1 * K1 + C1 + C2 + 16;
  const int RW = RW0 + (wl_here ? n * G::F : 0);
  float* mine = red + wv * RW;
  if (wl_here) {
#pragma unroll
    for (int j = 0; j < NWL; ++j)
      if (j < n)
        *reinterpret_cast<float4*>(mine + RW0 + j * G::F + FPL * lane) =
            make_float4(gwl[j][0], gwl[j][1], gwl[j][2], gwl[j][3]);
  }
#pragma unroll
  for (int t = 0; t < 5; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = (r & 3) + 8 * (r >> 2) + 4 * kh, k = 32 * t + col32;
      if (k < K2) mine[co * K2 + (k & 15) * 9 + (k >> 4)] = gw2[t][r];   // (tap, ci) -> flat [ci][tap]
    }
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = 4 * kq + r, k = 16 * t + col16;
      if (k < K1) mine[C2 * K2 + co * K1 + k] = gw1[t][r];
    }
  // b1: lanes 16k .. 16k+15 hold channel k + 4r's windows
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float v = gb1[r];
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) v += __shfl_xor(v, off);
    if (col16 == 0) mine[C2 * K2 + C1 * K1 + (lane >> 4) + 4 * r] = v;
  }
  {
    const float v = gb2 + __shfl_xor(gb2, 1);   // channel lane / 2 over both row halves
    if ((lane & 1) == 0) mine[C2 * K2 + C1 * K1 + C1 + (lane >> 1)] = v;
  }
  if (lane < 16) mine[C2 * K2 + C1 * K1 + C1 + C2 + lane] = lane < n ? gbl : 0.f;
  float* qred = red + NWV * RW;   // the quantum slab columns' sums by column, zero past qs.width (bwd3_smem: 256 floats)
  {
    float v = 0.f;
    if (q_mine) {
#pragma unroll
      for (int k = 0; k < QPF; ++k) v += qv[k];
      const float* qc = qs.slab + threadIdx.x;
      for (int r = q0 + QPF; r < q1; ++r) v += qc[(size_t)r * qs.width];
    }
    qred[threadIdx.x] = v;
  }
  __syncthreads();
  float* row = slab + (size_t)blockIdx.x * o.row;
  slab_row_out<NWV>(row, red, RW, RW0, qred, qs, q0, q1, o, n, G::F, wl_here);
  if constexpr (STAMP) {
    ts[9] = stamp();
    if (lane == 0)
      for (int k = 0; k < NSTAMP; ++k) stamps[(size_t)(blockIdx.x * NWV + wv) * NSTAMP + k] = ts[k];
  }
}

inline size_t bwd3_smem(int n) {
  using G = Geo<16, 8>;
  const size_t shared = (size_t)((n * wl_stride(G::F) + 16 + 3) & ~3) * 4 + (size_t)B3::W2T * 2;
  const size_t act = shared + 4 * (size_t)B3::WAVE_BYTES;
  const size_t red = sizeof(float) * (4 * (C2 * K2 + C1 * K1 + C1 + C2 + 16 + (size_t)n * G::F) + 256);   // (+ qred)
  return act > red ? act : red;
}

// waves per workgroup: 4 for P128; P256's backward images are twice as large -> 2
template <int W>
constexpr int fwd_waves() { return 4; }
template <int W>
constexpr int bwd_waves() { return W == 8 ? 4 : 2; }

template <int H, int W>
size_t fwd_smem(int n) {
  return sizeof(float) * (fwd_act_base(n, Geo<H, W>::F) + fwd_waves<W>() * Geo<H, W>::FWD);
}
// the backward also reduces the linear weight gradient when its register tile holds n outputs and
// the larger reduction image still fits the 160 KB of LDS
template <int H, int W>
bool wl_in_kernel(int n) {
  using G = Geo<H, W>;
  const size_t red = sizeof(float) * (S_WEND + bwd_waves<W>() * (C2 * K2 + C1 * K1 + C1 + C2 + 16 + (size_t)n * G::F));
  return n <= 64 / (G::F / 64) && red <= 160 * 1024;
}
template <int H, int W>
size_t bwd_smem(int n) {
  const size_t act = act_base_bwd(n, Geo<H, W>::F) + bwd_waves<W>() * Geo<H, W>::BWD;
  const size_t red = S_WEND + bwd_waves<W>() * (C2 * K2 + C1 * K1 + C1 + C2 + 16 + (wl_in_kernel<H, W>(n) ? n * Geo<H, W>::F : 0));
  return sizeof(float) * (act > red ? act : red);
}

template <int H, int W, bool X3 = false>
int launch_fwd(const float* x, const float* flat, Offs o, float* angles, float* p2, Saved sv, int B, int n, int grid,
               hipStream_t s, unsigned long long* stamps = nullptr, __bf16* w2t_img = nullptr) {
  constexpr int NW = fwd_waves<W>();
  const size_t sm = fwd_smem<H, W>(n);
  if (sm > 160 * 1024) return (int)hipErrorInvalidValue;
  if (stamps) {
    if (hipError_t e = allow_lds(qsc2_fwd_kernel<H, W, NW, true, X3>, sm)) return (int)e;
    hipLaunchKernelGGL((qsc2_fwd_kernel<H, W, NW, true, X3>), dim3(grid), dim3(64 * NW), sm, s, x, flat, o, angles, p2,
                       sv, B, n, stamps);
  } else {
    if (hipError_t e = allow_lds(qsc2_fwd_kernel<H, W, NW, false, X3>, sm)) return (int)e;
    hipLaunchKernelGGL((qsc2_fwd_kernel<H, W, NW, false, X3>), dim3(grid), dim3(64 * NW), sm, s, x, flat, o, angles,
                       p2, sv, B, n, nullptr, w2t_img);
  }
  return (int)hipGetLastError();
}

template <int H, int W>
int launch_bwd(const float* x, const float* flat, Offs o, const float* angles, const float* dang, float* dpre,
               float* slab, const float* p2, Saved sv, QSlab qs, int B, int n, int grid, hipStream_t s,
               unsigned long long* stamps = nullptr) {
  constexpr int NW = bwd_waves<W>();
  const size_t sm = bwd_smem<H, W>(n);
  if (sm > 160 * 1024) return (int)hipErrorInvalidValue;
  if (stamps) {
    if (hipError_t e = allow_lds(qsc2_bwd_kernel<H, W, NW, true>, sm)) return (int)e;
    hipLaunchKernelGGL((qsc2_bwd_kernel<H, W, NW, true>), dim3(grid), dim3(64 * NW), sm, s, x, flat, o, angles, dang,
                       dpre, slab, p2, sv, B, n, (int)wl_in_kernel<H, W>(n), qs, stamps);
  } else {
    if (hipError_t e = allow_lds(qsc2_bwd_kernel<H, W, NW>, sm)) return (int)e;
    hipLaunchKernelGGL((qsc2_bwd_kernel<H, W, NW>), dim3(grid), dim3(64 * NW), sm, s, x, flat, o, angles, dang, dpre,
                       slab, p2, sv, B, n, (int)wl_in_kernel<H, W>(n), qs, nullptr);
  }
  return (int)hipGetLastError();
}

}  // namespace qsc2
}  // namespace qd

using namespace qd::qsc2;

// offs: [w1, b1, w2, b2, wl, bl, row_width, base, qw] float offsets into the flat parameter buffer
// (slab rows cover [base, base + row_width)).
// Saved for the backward: p1s (B, HW/4, 16) f32, c1 (B, HW/4) u32, c2 (B, F) u8 (see sample_forward).
QD_API int qd_qsc2_fwd(const float* x, const float* flat, const int* offs, float* angles, float* p2, float* p1s,
                       uint32_t* c1, uint8_t* c2, int B, int n, int H, int W, int grid, void* stream) {
  if (n < 1 || n > 16 || B <= 0 || grid <= 0 || !p1s || !c1 || !c2) return (int)hipErrorInvalidValue;
  Offs o{offs[0], offs[1], offs[2], offs[3], offs[4], offs[5], offs[6], offs[7], offs[8]};
  Saved sv{p1s, c1, c2};
  hipStream_t s = (hipStream_t)stream;
  if (H == 16 && W == 8) return launch_fwd<16, 8>(x, flat, o, angles, p2, sv, B, n, grid, s);
  if (H == 16 && W == 16) return launch_fwd<16, 16>(x, flat, o, angles, p2, sv, B, n, grid, s);
  return (int)hipErrorInvalidValue;
}

// qd_qsc2_fwd with conv2 on bf16x3 MFMAs (sample_forward X3): same arguments and outputs.
// w2t_img (nullable): also write the backward's W2T hi / lo image (B3::W2T bf16) from these weights.
QD_API int qd_qsc2_fwd3(const float* x, const float* flat, const int* offs, float* angles, float* p2, float* p1s,
                        uint32_t* c1, uint8_t* c2, int B, int n, int H, int W, int grid, void* w2t_img, void* stream) {
  if (n < 1 || n > 16 || B <= 0 || grid <= 0 || !p1s || !c1 || !c2) return (int)hipErrorInvalidValue;
  Offs o{offs[0], offs[1], offs[2], offs[3], offs[4], offs[5], offs[6], offs[7], offs[8]};
  Saved sv{p1s, c1, c2};
  hipStream_t s = (hipStream_t)stream;
  if (H == 16 && W == 8)
    return launch_fwd<16, 8, true>(x, flat, o, angles, p2, sv, B, n, grid, s, nullptr, (__bf16*)w2t_img);
  if (H == 16 && W == 16) return launch_fwd<16, 16, true>(x, flat, o, angles, p2, sv, B, n, grid, s);
  return (int)hipErrorInvalidValue;
}

// slab: (grid, offs[6]) floats, row layout = flat layout from offs[0] (wl columns left zero).
// p2 / p1s / c1 / c2: what qd_qsc2_fwd saved for this batch.
QD_API int qd_qsc2_bwd(const float* x, const float* flat, const int* offs, const float* angles, const float* dang,
                       float* dpre, float* slab, const float* p2, float* p1s, uint32_t* c1, uint8_t* c2,
                       const float* qslab, int qrows, int qwidth, int B, int n, int H, int W, int grid, void* stream) {
  if (n < 1 || n > 16 || B <= 0 || grid <= 0 || !p2 || !p1s || !c1 || !c2) return (int)hipErrorInvalidValue;
  Offs o{offs[0], offs[1], offs[2], offs[3], offs[4], offs[5], offs[6], offs[7], offs[8]};
  Saved sv{p1s, c1, c2};
  hipStream_t s = (hipStream_t)stream;
  QSlab qs{qslab, qrows, qwidth};
  if (H == 16 && W == 8) return launch_bwd<16, 8>(x, flat, o, angles, dang, dpre, slab, p2, sv, qs, B, n, grid, s);
  if (H == 16 && W == 16) return launch_bwd<16, 16>(x, flat, o, angles, dang, dpre, slab, p2, sv, qs, B, n, grid, s);
  return (int)hipErrorInvalidValue;
}

// The P128 backward on bf16x3 MFMAs (qsc2_bwd3_kernel): same arguments and outputs as qd_qsc2_bwd.
// w2t_img (nullable): the W2T image the forward wrote this step (qd_qsc2_fwd3), else built in-kernel.
QD_API int qd_qsc2_bwd3(const float* x, const float* flat, const int* offs, const float* angles, const float* dang,
                        float* dpre, float* slab, const float* p2, float* p1s, uint32_t* c1, uint8_t* c2,
                        const float* qslab, int qrows, int qwidth, int B, int n, int H, int W, int grid,
                        const void* w2t_img, void* stream) {
  if (H != 16 || W != 8 || n < 1 || n > 16 || B <= 0 || grid <= 0 || !p2 || !p1s || !c1 || !c2)
    return (int)hipErrorInvalidValue;
  if (qslab && (qwidth < 1 || qwidth > 256)) return (int)hipErrorInvalidValue;   // (one column per thread: qred)
  Offs o{offs[0], offs[1], offs[2], offs[3], offs[4], offs[5], offs[6], offs[7], offs[8]};
  Saved sv{p1s, c1, c2};
  const size_t sm = bwd3_smem(n);
  if (sm > 160 * 1024) return (int)hipErrorInvalidValue;
  if (hipError_t e = qd::allow_lds(qsc2_bwd3_kernel<4>, sm)) return (int)e;
  hipLaunchKernelGGL((qsc2_bwd3_kernel<4>), dim3(grid), dim3(256), sm, (hipStream_t)stream, x, flat, o, angles, dang,
                     dpre, slab, p2, sv, B, n, (int)wl_in_kernel<16, 8>(n), QSlab{qslab, qrows, qwidth}, nullptr,
                     (const __bf16*)w2t_img);
  return (int)hipGetLastError();
}

// Diagnostic: qd_qsc2_bwd3 with per-wave phase stamps (stamps: grid * 4 * 12 u64; see qsc2_bwd3_kernel).
QD_API int qd_qsc2_bwd3_stamped(const float* x, const float* flat, const int* offs, const float* angles,
                                const float* dang, float* dpre, float* slab, const float* p2, float* p1s, uint32_t* c1,
                                uint8_t* c2, const float* qslab, int qrows, int qwidth, int B, int n, int grid,
                                unsigned long long* stamps, void* stream) {
  if (n < 1 || n > 16 || B <= 0 || grid <= 0 || (qslab && (qwidth < 1 || qwidth > 256))) return (int)hipErrorInvalidValue;
  Offs o{offs[0], offs[1], offs[2], offs[3], offs[4], offs[5], offs[6], offs[7], offs[8]};
  Saved sv{p1s, c1, c2};
  const size_t sm = bwd3_smem(n);
  if (sm > 160 * 1024 || !stamps) return (int)hipErrorInvalidValue;
  if (hipError_t e = qd::allow_lds(qsc2_bwd3_kernel<4, true>, sm)) return (int)e;
  hipLaunchKernelGGL((qsc2_bwd3_kernel<4, true>), dim3(grid), dim3(256), sm, (hipStream_t)stream, x, flat, o, angles,
                     dang, dpre, slab, p2, sv, B, n, (int)wl_in_kernel<16, 8>(n), QSlab{qslab, qrows, qwidth}, stamps);
  return (int)hipGetLastError();
}

// 1 if qd_qsc2_bwd also produces the linear-layer weight gradient (slab wl columns) for n qubits
QD_API int qd_qsc2_wl_in_kernel(int H, int W, int n) {
  if (H == 16 && W == 8) return wl_in_kernel<16, 8>(n) ? 1 : 0;
  if (H == 16 && W == 16) return wl_in_kernel<16, 16>(n) ? 1 : 0;
  return 0;
}

// waves (= samples in flight) per workgroup of the two kernels
QD_API int qd_qsc2_waves(int W, int backward) {
  if (W == 8) return backward ? bwd_waves<8>() : fwd_waves<8>();
  if (W == 16) return backward ? bwd_waves<16>() : fwd_waves<16>();
  return -1;
}

// Diagnostic: forward with per-wave phase stamps (stamps: grid * waves * 12 u64):
// [0] kernel start [1] weights staged [2] input tile [3] conv1+pool [4] conv2 [5] pool2+linear
// (first sample of the wave) [6] wave done.
QD_API int qd_qsc2_fwd_stamped(const float* x, const float* flat, const int* offs, float* angles, float* p2,
                               float* p1s, uint32_t* c1, uint8_t* c2, int B, int n, int H, int W, int grid,
                               unsigned long long* stamps, void* stream) {
  Offs o{offs[0], offs[1], offs[2], offs[3], offs[4], offs[5], offs[6], offs[7], offs[8]};
  Saved sv{p1s, c1, c2};
  hipStream_t s = (hipStream_t)stream;
  if (H == 16 && W == 8) return launch_fwd<16, 8, true>(x, flat, o, angles, p2, sv, B, n, grid, s, stamps);   // (bf16x3)
  if (H == 16 && W == 16) return launch_fwd<16, 16>(x, flat, o, angles, p2, sv, B, n, grid, s, stamps);
  return (int)hipErrorInvalidValue;
}

// Diagnostic: backward with per-wave phase stamps (stamps: grid * waves * 12 u64): [0] start
// [1] weights staged [2] saved state -> LDS [3] linear + pool-2 backward [4] conv2 weight grads
// [5] conv2 data grads [6] pool-1 backward [7] conv1 weight grads (first sample) [8] wave done.
QD_API int qd_qsc2_bwd_stamped(const float* x, const float* flat, const int* offs, const float* angles,
                               const float* dang, float* dpre, float* slab, const float* p2, float* p1s, uint32_t* c1,
                               uint8_t* c2, const float* qslab, int qrows, int qwidth, int B, int n, int H, int W,
                               int grid, unsigned long long* stamps, void* stream) {
  Offs o{offs[0], offs[1], offs[2], offs[3], offs[4], offs[5], offs[6], offs[7], offs[8]};
  Saved sv{p1s, c1, c2};
  hipStream_t s = (hipStream_t)stream;
  QSlab qs{qslab, qrows, qwidth};
  if (H == 16 && W == 8)
    return launch_bwd<16, 8>(x, flat, o, angles, dang, dpre, slab, p2, sv, qs, B, n, grid, s, stamps);
  if (H == 16 && W == 16)
    return launch_bwd<16, 16>(x, flat, o, angles, dang, dpre, slab, p2, sv, qs, B, n, grid, s, stamps);
  return (int)hipErrorInvalidValue;
}
