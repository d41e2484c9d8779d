// HDCE feature extractor (3 x [conv3x3 -> BatchNorm -> ReLU], 32 channels) for gfx950.
//
// Reference: Conv_P128 (Estimators_QuantumNAT_onchipQNN.py:237-268), applied per
// (scenario, user) stream with the scenario's own expert (Runner:109, R:194); PyTorch runs it
// through cuDNN conv + BN + ReLU kernels, and the grouped-expert form through MIOpen, whose
// grouped backward-weight kernel measured 4.7 ms per call on MI355X
// (profiles/r1_00_baseline_miopen_kernel_stats.md).
//
// Data: activations are (N, E*32, H, W) with N = users x batch samples and the E scenario
// experts folded into the channel axis; a "virtual sample" (n, e) is one sample through one
// expert.  BatchNorm statistics are per (group u = n / B, channel) -- ghost BN over each
// 256-sample stream batch, exactly what the reference's per-stream calls compute.
//
// Kernels (all MFMA bf16 32x32x16, fp32 accumulate):
//   conv3x3_kernel   implicit-GEMM conv: M = 32 positions, N = 32 channels, K = 9*CIN ordered
//                    (tap, channel) so an A fragment is ONE ds_read_b128 from a channel-last
//                    LDS tile (64-byte pixels, 16-byte channel chunks XOR-swizzled per pixel:
//                    conflict-free for every tap, see tile_swz).  Weights stay in
//                    VGPRs as B fragments for the whole launch.  Input transforms fused in the
//                    LDS staging: raw f32 pilots (layer 1), BN+ReLU of the previous layer's
//                    pre-BN output (forward), or the BN/ReLU backward (dz from dh and z) for the
//                    data-gradient pass (same kernel with flipped/transposed weights).
//                    Epilogue: bf16 z + per-(group, channel) sum / sum-of-squares partials, or
//                    fp32 dgrad output.
//   conv3x3_wgrad    dW = sum_{samples,positions} im2col(x)^T dz: the 4 waves of a workgroup
//                    split each sample's positions (K), keep all 9 tap tiles of accumulators
//                    in registers across samples, and reduce through LDS once per workgroup
//                    into a deterministic slab (no float atomics).  A operand rows come from 3
//                    column-shifted copies of the input tile so every read is an aligned
//                    ds_read_b128; rows are ordered (tap, channel) so the 32 rows of an MFMA tile
//                    are one tap's 32 channels at an odd 16-byte-slot stride (conflict-free).
//   bn_*             statistics finalisation (+ running-stat momentum updates in stream order),
//                    backward reductions, and the final BN+ReLU apply that feeds the FC GEMM.
#include <algorithm>
#include <cstdlib>

#include "common.h"

namespace qd {
namespace conv {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;

// two floats -> one word of two RNE bf16 (x low): a single v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t pack_bf16x2(f32x2 v) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
}
// the two floats of a packed bf16 word
__device__ __forceinline__ f32x2 unpack_bf16x2(uint32_t w) {
  return f32x2{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)};
}

constexpr int CO = 32;     // output channels of every layer (per expert)
constexpr int NST = 8;     // floats per (group, channel) BN state record

// BN state record per (u, channel): {mean, invstd, a=gamma*invstd, b=beta-mean*a, c1, c2, c3, 0}
enum { ST_MEAN = 0, ST_INV = 1, ST_A = 2, ST_B = 3, ST_C1 = 4, ST_C2 = 5, ST_C3 = 6 };

enum InMode { IN_RAW_F32 = 0, IN_BNRELU = 1, IN_BNBWD = 2 };
enum OutMode { OUT_Z_STATS = 0, OUT_F32 = 1, OUT_BF16 = 2 };

template <int H, int W>
struct Geo {
  static constexpr int HW = H * W;
  static constexpr int HP = H + 2;
  static constexpr int WP = W + 2;
  static constexpr int MT = HW / 32;  // 32-position M tiles
  static_assert(HW % 64 == 0 && W % 8 == 0, "geometry");
};

__device__ __forceinline__ float bf(uint16_t h) { return bf16_to_f32(h); }

// 32-channel conv tiles: padded pixel (R, C) is 64 bytes = four 16-byte channel chunks, chunk q stored
// at position q ^ tile_swz(R, C).  Pixel P's chunks sit in bank-row slot group P mod 4; the XOR makes
// the 16 lanes of every ds_read_b128 lane group ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ...) hit 16
// distinct 16-byte slots for every tap of both geometries (W = 8, 16).  The previous layout (pixels
// padded to 80 bytes) took 8 (W = 8) / 4 (W = 16) extra LDS cycles per 4-cycle read.
__device__ __forceinline__ int tile_swz(int R, int C) { return (2 * R + (C >> 2) + 2 * (C >> 3)) & 3; }

template <typename T>
__device__ __forceinline__ float ldf(const T* p, size_t i);
template <>
__device__ __forceinline__ float ldf<float>(const float* p, size_t i) { return p[i]; }
template <>
__device__ __forceinline__ float ldf<uint16_t>(const uint16_t* p, size_t i) { return bf16_to_f32(p[i]); }

// 8 consecutive values (16- or 32-byte aligned) -> floats
__device__ __forceinline__ void load8(const float* p, float* v) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void load8(const uint16_t* p, float* v) {
  const uint4 a = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

// Raw 16-byte vectors kept in registers between a prefetch and its use (no conversion at load
// time, so the compiler's wait for the data lands at the use, one sample later).
template <typename T>
struct PerQ;
template <>
struct PerQ<float> { static constexpr int N = 4; };
template <>
struct PerQ<uint16_t> { static constexpr int N = 8; };
__device__ __forceinline__ void unpack_q(const uint4 q, float* v, const float*) {
  v[0] = __uint_as_float(q.x); v[1] = __uint_as_float(q.y); v[2] = __uint_as_float(q.z); v[3] = __uint_as_float(q.w);
}
__device__ __forceinline__ void unpack_q(const uint4 q, float* v, const uint16_t*) {
  const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

// ------------------------------------------------------------------------------------------
// BatchNorm finalisation inside the consumer kernels.  A consumer workgroup of (group u, expert e)
// rebuilds the 32-channel BN records it needs straight from the producer's per-chunk partials
// (every workgroup gets bitwise-identical values: same order), so no separate finalisation launch
// sits between producer and consumer.  One designated workgroup per expert also does the
// once-per-step side effects (running statistics / dgamma, dbeta); chunk-0 workgroups publish the
// record for later kernels.  256 threads: channel c = tid / 8, part j = tid % 8.
// ------------------------------------------------------------------------------------------
struct BnFwd {            // forward: (mean, invstd, a, b) from conv statistics partials
  const float* stats;     // (U, chunks, 2, EC) sum / sum of squares; null: use the st record as is
  const float* gamma;
  const float* beta;
  float* run_mean;
  float* run_var;
  float* st_out;          // (U, EC, NST) record published by chunk-0 workgroups
  int chunks;
  float count, momentum, eps;
  int training;
};
struct BnBwd {            // backward: (c1, c2, c3) from the BN backward reduction partials
  const float* rslab;     // (U, chunks, 2, EC) sum g / sum g*xhat; null: use the st record as is
  const float* gamma;
  int chunks;
  float count;
};

// dgrad epilogue fusion: the BN backward reduction of the PREVIOUS layer (whose output h = relu(a z
// + b) is this pass's dx): per (u, chunk, channel) sum g and sum g*xhat, g = dx * [a z + b > 0],
// planar rows (U, chunks, 2, EC) -- what bn_bwd_reduce_kernel would compute in a launch of its own.
struct BnRed {
  const uint16_t* z;   // previous layer's pre-BN output (bf16, same layout as dx); null: no fusion
  const float* st;     // its published BN records (U, EC, NST)
  float* part;         // (U, chunks, 2, EC)
};

// COH: a value another workgroup of the SAME launch wrote (the persistent forward, conv_fwd_stack_kernel): an
// agent-scope atomic access (coherent across the XCDs' L2s, no cache-wide writeback / invalidate); else a plain one
template <bool COH>
__device__ __forceinline__ float ld_part(const float* p) {
  if constexpr (COH) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}
template <bool COH>
__device__ __forceinline__ void st_part(float* p, float v) {
  if constexpr (COH) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}

// sums of the two planar partial rows of channel ch over the chunks of group u (8 lanes per
// channel; up to 64 chunks with every load in flight at once)
template <bool COH = false>
__device__ __forceinline__ float2 bn_part_sums(const float* __restrict__ part, int u, int chunks, int EC, int ch,
                                               int j) {
  float a = 0.f, b = 0.f;
  const float* p = part + (size_t)u * chunks * 2 * EC + ch;
  // all 16 loads issued before the first add (a chunk past the end loads chunk 0 and is not added): guarded
  // loads compiled to 8 dependent round trips, each behind its own vmcnt(0) -- most of every consumer's prologue
  float pa[8], pb[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int k = j + 8 * i < chunks ? j + 8 * i : 0;
    pa[i] = ld_part<COH>(p + (size_t)k * 2 * EC);
    pb[i] = ld_part<COH>(p + (size_t)k * 2 * EC + EC);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (j + 8 * i < chunks) {   // (the same additions in the same order as before: bit-identical)
      a += pa[i];
      b += pb[i];
    }
  }
  for (int k = j + 64; k < chunks; k += 8) {
    a += ld_part<COH>(p + (size_t)k * 2 * EC);
    b += ld_part<COH>(p + (size_t)k * 2 * EC + EC);
  }
#pragma unroll
  for (int m = 1; m < 8; m <<= 1) {
    a += __shfl_xor(a, m);
    b += __shfl_xor(b, m);
  }
  return make_float2(a, b);
}

// rec[c * NST + ST_MEAN .. ST_B] for the 32 channels of (u, e); publish: also write the record to
// bn.st_out.  (The running statistics advance once per step in the BN tail launch.)
template <bool COH = false>
__device__ void bn_fwd_build(const BnFwd& bn, float* rec, int u, int e, int EC, bool publish) {
  const int tid = threadIdx.x, c = tid >> 3, j = tid & 7, ch = e * CO + c;
  // gamma / beta issued with the partial sums (loaded by lane j == 0 after the reduction they were one more
  // dependent round trip of every consumer's prologue)
  const float g = bn.gamma[ch], bt = bn.beta[ch];
  float mean, var;
  if (bn.training) {
    const float2 sm = bn_part_sums<COH>(bn.stats, u, bn.chunks, EC, ch, j);
    mean = sm.x / bn.count;
    var = fmaxf(sm.y / bn.count - mean * mean, 0.f);
  } else {
    mean = bn.run_mean[ch];
    var = bn.run_var[ch];
  }
  if (j == 0) {
    const float inv = rsqrtf(var + bn.eps);
    const float4 r = make_float4(mean, inv, g * inv, bt - mean * g * inv);
    *reinterpret_cast<float4*>(rec + c * NST) = r;
    if (publish) *reinterpret_cast<float4*>(bn.st_out + ((size_t)u * EC + ch) * NST) = r;
  }
}

// rec[c * NST + ...] = the published forward record of (u, e) with c1..c3 of the backward filled
// in.  (dgamma / dbeta: column sums of the same partials, in the step's batched slab reduction.)
__device__ void bn_bwd_build(const BnBwd& bn, const float* __restrict__ st, float* rec, int u, int e, int EC) {
  const int tid = threadIdx.x, c = tid >> 3, j = tid & 7, ch = e * CO + c;
  // the forward record and gamma issued with the partial sums (one round trip for the whole build)
  const float4 f = *reinterpret_cast<const float4*>(st + ((size_t)u * EC + ch) * NST);
  const float gm = bn.gamma[ch];
  const float2 sg = bn_part_sums(bn.rslab, u, bn.chunks, EC, ch, j);
  if (j == 0) {
    const float c1 = gm * f.y;
    *reinterpret_cast<float4*>(rec + c * NST) = f;
    *reinterpret_cast<float4*>(rec + c * NST + 4) = make_float4(c1, c1 * sg.x / bn.count, c1 * sg.y / bn.count, 0.f);
  }
}

// ------------------------------------------------------------------------------------------
// conv3x3_kernel: forward (and data-gradient) implicit GEMM
// grid: (U * chunks, E); block 256 (4 waves); each wave owns `spw` consecutive samples.
// CIN: input channels of THIS pass (layer-1 fwd: 2; else 32).
// DGRAD: weights used transposed + flipped (W[e*32+k][lane][8-tap]); output fp32.
// wt: B fragments pre-packed by pack_weights_kernel (fwd or dgrad order).
// ------------------------------------------------------------------------------------------
template <int CIN, int H, int W, int INM, int OUTM, bool DGRAD, typename TIN, bool STAMP = false, bool COH = false>
__device__ __forceinline__ void conv3x3_body(const TIN* __restrict__ xin, const uint16_t* __restrict__ zaux,
                                             const float* __restrict__ st_in, const uint16_t* __restrict__ wt,
                                             void* __restrict__ out, float* __restrict__ stats, int E, int B,
                                             int chunks, int spw, BnFwd bnf, BnBwd bnb, BnRed brd,
                                             unsigned long long* __restrict__ stamps, int bx, int by, int gdx) {
  // STAMP (diagnostic builds): per wave [0] start [1] weights + BN params staged [2] first sample
  // staged [3] first sample's MFMAs + epilogue [4] all samples [5] end
  unsigned long long ts[8] = {};
  if constexpr (STAMP) ts[0] = phase_stamp();
  using G = Geo<H, W>;
  constexpr int CINP = CIN;                                 // channel-last pixel stride (bf16)
  static_assert(CIN % 16 != 0 || CIN == 32, "the tile swizzle is for 4-chunk (32-channel) pixels");
  constexpr int KS = (9 * CIN + 15) / 16;                   // 16-deep k steps
  constexpr int TILE = G::HP * G::WP * CINP;                // bf16 elements per wave tile
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int hh = lane >> 5, l32 = lane & 31;
  const int u = bx / chunks, chunk = bx % chunks, e = by;
  const int EC_in = E * CIN;
  static_assert(TILE % 8 == 0, "16-byte tile fills");
  __bf16* tile = reinterpret_cast<__bf16*>(smem) + wv * TILE;
  for (int i = lane; i < TILE / 8; i += 64) reinterpret_cast<bf16x8*>(tile)[i] = bf16x8{};

  bf16x8* wl = reinterpret_cast<bf16x8*>(reinterpret_cast<__bf16*>(smem) + 4 * TILE);   // B fragments
  constexpr bool RAWIN = INM == IN_RAW_F32;
  float* stl = reinterpret_cast<float*>(wl + KS * 64);                                     // BN params
  // per-lane channel for the output/statistics: column of the MFMA tile
  float s1 = 0.f, s2 = 0.f;
  f32x2 s1v = {0.f, 0.f}, s2v = {0.f, 0.f};   // (OUT_Z_STATS: packed partial sums, even / odd positions)
  [[maybe_unused]] float ra = 0.f, rb = 0.f, rmu = 0.f, rinv = 0.f;
  const bool fuse_red = DGRAD && OUTM == OUT_BF16 && brd.part != nullptr;
  if (fuse_red) {
    const float4 r = *reinterpret_cast<const float4*>(brd.st + ((size_t)u * E * CO + e * CO + l32) * NST);
    rmu = r.x;
    rinv = r.y;
    ra = r.z;
    rb = r.w;
  }
  const int n0 = u * B + (chunk * 4 + wv) * spw;
  const int nend = min((u + 1) * B, n0 + spw);

  // ---- one-sample-ahead register prefetch of the raw input (converted at use, one sample later).
  // Where a whole sample does not fit the register budget (P256 dgrad), groups of GR items are
  // loaded and staged synchronously instead (batched: GR loads in flight per round trip). ----
  // staging item (non-raw input): 8 consecutive positions of a channel PAIR (c, c+1), so the
  // channel-last LDS tile is written as bf16x2 words -- 16 lanes of a pass write 16 consecutive
  // words of one pixel (a single-channel item wrote 2-byte values 640 bytes apart: 4-8-way bank
  // conflicts, profiles/r1_19_pmc.md)
  constexpr int CH8 = CIN * G::HW / 8;                  // 8-value (single channel) units per sample
  constexpr int NPAIR = CIN / 2;
  constexpr int ITER = RAWIN ? (CIN * G::HW) / 64 : CH8 / 128;
  static_assert(RAWIN ? (CIN * G::HW) % 64 == 0 : CH8 % 128 == 0, "whole waves per staging pass");
  constexpr int QV = RAWIN ? 1 : (int)sizeof(TIN) / 2;  // uint4s per 8-value unit (bf16: 1, f32: 2)
  constexpr int HOLD = ITER * (2 * QV + (INM == IN_BNBWD ? 2 : 0));   // 16-byte registers per sample
  // (dgrad: registers go to the fused BN-reduction operands; P256: to the MFMA pipeline)
  constexpr bool PREF = RAWIN || (!DGRAD && HOLD <= 16 && G::HW <= 128);
  constexpr int GR = PREF ? ITER : (INM == IN_BNBWD && ITER > 4 ? 2 : 4);
  static_assert(ITER % GR == 0, "staging groups");
  [[maybe_unused]] uint4 rv[RAWIN ? 1 : GR][2][QV];
  [[maybe_unused]] uint4 rz[INM == IN_BNBWD ? GR : 1][2];
  [[maybe_unused]] float rr[RAWIN ? GR : 1];
  auto load_group = [&](int n, int g0) {
    const size_t base = ((size_t)n * E + e) * CIN * G::HW;
#pragma unroll
    for (int k = 0; k < GR; ++k) {
      const int it = g0 + k;
      if constexpr (RAWIN) {
        rr[k] = ldf<TIN>(xin, base + lane + 64 * it);
      } else {
        // item i: channel pair i % NPAIR, positions [8 (i / NPAIR), +8)
        const int i = lane + 64 * it, pr = i % NPAIR, sg = i / NPAIR;
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          const size_t off = base + (size_t)(2 * pr + h2) * G::HW + 8 * sg;
          const uint4* src = reinterpret_cast<const uint4*>(xin + off);
#pragma unroll
          for (int q = 0; q < QV; ++q) rv[k][h2][q] = src[q];
          if constexpr (INM == IN_BNBWD) rz[k][h2] = *reinterpret_cast<const uint4*>(zaux + off);
        }
      }
    }
  };
  // transform + scatter a group into the channel-last LDS tile
  auto store_group = [&](int g0) {
#pragma unroll
    for (int k = 0; k < GR; ++k) {
      const int i = lane + 64 * (g0 + k);
      if constexpr (RAWIN) {
        const int c = i / G::HW, p = i % G::HW;
        tile[((p / W + 1) * G::WP + (p % W) + 1) * CINP + c] = (__bf16)rr[k];
      } else if constexpr (INM == IN_BNRELU && QV == 1) {
        // the forward's bf16 input, a channel pair at a time: one packed FMA per position for both channels,
        // a NaN-keeping max per value and one packed bf16 conversion per LDS word -- about half the vector
        // instructions of the per-value path below, which made the staging VALU-bound (the same values: RNE
        // rounding of relu(a z + b) either way)
        const int pr = i % NPAIR, p0 = (i / NPAIR) * 8;
        const float* s0 = stl + (2 * pr) * NST;
        const f32x2 a2 = {s0[ST_A], s0[NST + ST_A]}, b2 = {s0[ST_B], s0[NST + ST_B]};
        const uint32_t w0[4] = {rv[k][0][0].x, rv[k][0][0].y, rv[k][0][0].z, rv[k][0][0].w};
        const uint32_t w1[4] = {rv[k][1][0].x, rv[k][1][0].y, rv[k][1][0].z, rv[k][1][0].w};
        const int ph = p0 / W, pw = p0 % W;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t u0 = (j & 1) ? (w0[j >> 1] & 0xffff0000u) : (w0[j >> 1] << 16);
          const uint32_t u1 = (j & 1) ? (w1[j >> 1] & 0xffff0000u) : (w1[j >> 1] << 16);
          f32x2 y = f32x2{__uint_as_float(u0), __uint_as_float(u1)} * a2 + b2;
          y.x = relu_max(y.x);
          y.y = relu_max(y.y);
          const int R = ph + 1, C = pw + j + 1;
          *reinterpret_cast<uint32_t*>(tile + (R * G::WP + C) * CINP + 8 * ((pr >> 2) ^ tile_swz(R, C)) +
                                       2 * (pr & 3)) = pack_bf16x2(y);
        }
      } else {
        const int pr = i % NPAIR, p0 = (i / NPAIR) * 8;
        float v2[2][8];
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          const float* sc = stl + (2 * pr + h2) * NST;
          float* v = v2[h2];
#pragma unroll
          for (int q = 0; q < QV; ++q) unpack_q(rv[k][h2][q], v + q * (8 / QV), (const TIN*)nullptr);
          if constexpr (INM == IN_BNRELU) {
            const float a = sc[ST_A], b = sc[ST_B];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = relu_nan(a * v[j] + b);
          } else {  // IN_BNBWD: v = dh; dz = c1*g - c2 - c3*xhat, g = dh * [a z + b > 0]
            float z[8];
            unpack_q(rz[k][h2], z, (const uint16_t*)nullptr);
            const float a = sc[ST_A], b = sc[ST_B], mu = sc[ST_MEAN], inv = sc[ST_INV];
            const float c1 = sc[ST_C1], c2 = sc[ST_C2], c3 = sc[ST_C3];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float g = bn_gate(a, z[j], b) ? v[j] : 0.f;
              v[j] = bn_dz(g, bn_xhat(z[j], mu, inv), c1, c2, c3);
            }
          }
        }
        const int ph = p0 / W, pw = p0 % W;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t w2 = f32_to_bf16(v2[0][j]) | ((uint32_t)f32_to_bf16(v2[1][j]) << 16);
          const int R = ph + 1, C = pw + j + 1;
          *reinterpret_cast<uint32_t*>(tile + (R * G::WP + C) * CINP + 8 * ((pr >> 2) ^ tile_swz(R, C)) +
                                       2 * (pr & 3)) = w2;
        }
      }
    }
  };
  if (PREF && n0 < nend) load_group(n0, 0);   // the first sample's loads fly during the prologue
  // ---- prologue: weights -> B fragments in LDS, shared by the 4 waves (pre-packed [e][s][lane][8]
  // bf16 by pack_weights_kernel), and the BN parameters of this block's (group, expert) input
  // channels; every load in flight at once (a rolled copy loop waited one round trip per pass) ----
  {
    constexpr int WPT = (KS * 64 + 255) / 256;
    const bf16x8* wp = reinterpret_cast<const bf16x8*>(wt) + (size_t)e * KS * 64;
    bf16x8 tw[WPT];
#pragma unroll
    for (int k = 0; k < WPT; ++k)
      if ((KS * 64) % 256 == 0 || tid + 256 * k < KS * 64) tw[k] = wp[tid + 256 * k];
    [[maybe_unused]] float tp = 0.f;
    static_assert(CIN * NST <= 256, "one BN parameter per thread");
    // BN records of the input channels: rebuilt from the producer's partials (fused finalisation)
    // or read from the published record
    const bool build = (INM == IN_BNRELU && bnf.stats) || (INM == IN_BNBWD && bnb.rslab);
    if constexpr (!RAWIN)
      if (!build && tid < CIN * NST) tp = st_in[((size_t)u * EC_in + e * CIN) * NST + tid];
    // the BN build's loads go out behind the weight loads, before the weights' LDS stores wait for them (built
    // after the stores, the partial sums were a second dependent round trip of the prologue)
    if constexpr (INM == IN_BNRELU) {
      if (build) bn_fwd_build<COH>(bnf, stl, u, e, EC_in, chunk == 0);
    } else if constexpr (INM == IN_BNBWD) {
      if (build) bn_bwd_build(bnb, st_in, stl, u, e, EC_in);
    }
#pragma unroll
    for (int k = 0; k < WPT; ++k)
      if ((KS * 64) % 256 == 0 || tid + 256 * k < KS * 64) wl[tid + 256 * k] = tw[k];
    if constexpr (!RAWIN)
      if (!build && tid < CIN * NST) stl[tid] = tp;
  }
  __syncthreads();
  if constexpr (STAMP) ts[1] = phase_stamp();

  for (int n = n0; n < nend; ++n) {
    wave_lds_fence();
    // ---- stage the (transformed) input tile into LDS, channel-last, with zero halo ----
    if constexpr (PREF) {
      store_group(0);
      // the next sample's loads, branch-free (the last sample re-loads itself, unused): a guarded prefetch made
      // the compiler copy half-arrived registers at the branch join and wait for the loads right there, before
      // this sample's MFMAs -- no overlap at all (profiles/r4_12_stamp_conv.txt: ~3500 cycles per sample)
      load_group(n + 1 < nend ? n + 1 : n, 0);
    } else {
#pragma unroll 1
      for (int g0 = 0; g0 < ITER; g0 += GR) {
        load_group(n, g0);
        store_group(g0);
      }
    }
    wave_lds_fence();
    if (STAMP && n == n0) ts[2] = phase_stamp();
    // ---- MFMA: MG position tiles at once (independent accumulators) with the next k-step's
    // fragments in flight behind the current MFMAs (a one-tile loop waited out one LDS round trip
    // per MFMA: ds_read -> lgkmcnt(0) -> mfma) ----
    auto load_a = [&](int mt, int s) -> bf16x8 {
      const int p = mt * 32 + l32, ph = p / W, pw = p % W;
      bf16x8 a;
      if constexpr (CIN % 16 == 0) {
        const int tap = (16 * s) / CIN, q = ((16 * s) % CIN) / 8 + hh;
        const int R = ph + tap / 3, C = pw + tap % 3;
        a = *reinterpret_cast<const bf16x8*>(tile + (R * G::WP + C) * CINP + 8 * (q ^ tile_swz(R, C)));
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = 16 * s + 8 * hh + j;
          if (k < 9 * CIN) {
            const int tap = k / CIN, c = k % CIN;
            a[j] = tile[((ph + tap / 3) * G::WP + pw + tap % 3) * CINP + c];
          } else {
            a[j] = (__bf16)0.f;
          }
        }
      }
      return a;
    };
    // (with the prefetch in flight: 2 position tiles at a time -- 4 accumulator tiles plus the held next sample
    // exceed the 256-register budget of 2 workgroups per CU and spill, whose reload waits out the prefetch)
    constexpr int MGMAX = PREF ? 2 : 4;
    constexpr int MG = G::MT < MGMAX ? G::MT : MGMAX;
#pragma unroll
    for (int g0 = 0; g0 < G::MT; g0 += MG) {
      // fused BN reduction: the previous layer's z at this lane's output positions, loaded now so
      // the round trip hides behind the MFMAs
      [[maybe_unused]] uint2 zq[MG][4];
      if (fuse_red) {
#pragma unroll
        for (int j = 0; j < MG; ++j)
#pragma unroll
          for (int g = 0; g < 4; ++g)
            zq[j][g] = *reinterpret_cast<const uint2*>(
                brd.z + ((size_t)n * E + e) * CO * G::HW + (size_t)l32 * G::HW + (g0 + j) * 32 + 8 * g + 4 * hh);
      }
      f32x16 acc[MG];
      bf16x8 a_cur[MG], b_cur = wl[lane];
#pragma unroll
      for (int j = 0; j < MG; ++j) {
        acc[j] = f32x16{};
        a_cur[j] = load_a(g0 + j, 0);
      }
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        bf16x8 a_nxt[MG], b_nxt;
        if (s + 1 < KS) {
          b_nxt = wl[(s + 1) * 64 + lane];
#pragma unroll
          for (int j = 0; j < MG; ++j) a_nxt[j] = load_a(g0 + j, s + 1);
        }
        // pin the order: the next step's reads are issued before this step's MFMAs (left alone,
        // the scheduler drains the tiles one after another to save registers)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < MG; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_cur[j], b_cur, acc[j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (s + 1 < KS) {
          b_cur = b_nxt;
#pragma unroll
          for (int j = 0; j < MG; ++j) a_cur[j] = a_nxt[j];
        }
      }
#pragma unroll
      for (int j = 0; j < MG; ++j) {
        const int mt = g0 + j;
        // ---- epilogue: lane holds channel l32, positions mt*32 + 8g + 4hh + {0..3}.  bf16 outputs:
        // the two half-waves swap halves so each lane stores 8 consecutive positions (16 bytes) ----
        const size_t rbase = ((size_t)n * E + e) * CO * G::HW + (size_t)l32 * G::HW + mt * 32;
        if constexpr (OUTM == OUT_F32) {
#pragma unroll
          for (int g = 0; g < 4; ++g)
            *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + rbase + 8 * g + 4 * hh) =
                make_float4(acc[j][4 * g], acc[j][4 * g + 1], acc[j][4 * g + 2], acc[j][4 * g + 3]);
        } else {
          // packed conversions (one v_cvt_pk_bf16_f32 per two values) and packed statistics sums: the
          // epilogue's vector instructions sat outside the MFMA stream, one per value or more
          uint32_t pk[4][2];
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            pk[g][0] = pack_bf16x2(f32x2{acc[j][4 * g], acc[j][4 * g + 1]});
            pk[g][1] = pack_bf16x2(f32x2{acc[j][4 * g + 2], acc[j][4 * g + 3]});
            if constexpr (OUTM == OUT_Z_STATS) {   // statistics of the stored (bf16-rounded) values
              const f32x2 v01 = unpack_bf16x2(pk[g][0]), v23 = unpack_bf16x2(pk[g][1]);
              s1v += v01 + v23;
              s2v += v01 * v01 + v23 * v23;
            } else if constexpr (DGRAD && OUTM == OUT_BF16) {   // fused BN reduction (stored values)
              if (fuse_red) {
                const f32x2 d01 = unpack_bf16x2(pk[g][0]), d23 = unpack_bf16x2(pk[g][1]);
                const float d[4] = {d01.x, d01.y, d23.x, d23.y};
                const float zz[4] = {__uint_as_float(zq[j][g].x << 16), __uint_as_float(zq[j][g].x & 0xffff0000u),
                                     __uint_as_float(zq[j][g].y << 16), __uint_as_float(zq[j][g].y & 0xffff0000u)};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                  const float gg = bn_gate(ra, zz[q], rb) ? d[q] : 0.f;
                  bn_red(s1, s2, gg, bn_xhat(zz[q], rmu, rinv));
                }
              }
            }
          }
#pragma unroll
          for (int q = 0; q < 2; ++q) {   // pair (g = 2q, 2q + 1): half-wave hh stores g = 2q + hh
            // v_permlane32_swap: the upper half's group 2q goes down, the lower half's group 2q + 1 goes up, so
            // each lane then holds its 8 consecutive positions (no bpermute through LDS, no selects)
#pragma unroll
            for (int w = 0; w < 2; ++w) {
              const auto r = __builtin_amdgcn_permlane32_swap(pk[2 * q][w], pk[2 * q + 1][w], false, false);
              pk[2 * q][w] = r[0];
              pk[2 * q + 1][w] = r[1];
            }
            *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(out) + rbase + 8 * (2 * q + hh)) =
                make_uint4(pk[2 * q][0], pk[2 * q][1], pk[2 * q + 1][0], pk[2 * q + 1][1]);
          }
        }
      }
    }
    if (STAMP && n == n0) ts[3] = phase_stamp();
  }
  if constexpr (STAMP) ts[4] = phase_stamp();
  if (OUTM == OUT_Z_STATS || fuse_red) {
    // combine the two half-waves (same channel), then the 4 waves through LDS
    s1 += s1v.x + s1v.y;
    s2 += s2v.x + s2v.y;
    s1 += __shfl_xor(s1, 32);
    s2 += __shfl_xor(s2, 32);
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);
    if (hh == 0) {
      red[(wv * 32 + l32) * 2] = s1;
      red[(wv * 32 + l32) * 2 + 1] = s2;
    }
    __syncthreads();
    if (tid < 64) {
      const int c = tid >> 1, k = tid & 1;
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) t += red[(w * 32 + c) * 2 + k];
      float* dst = OUTM == OUT_Z_STATS ? stats : brd.part;
      st_part<COH>(dst + (((size_t)u * chunks + chunk) * 2 + k) * E * CO + e * CO + c, t);   // planar [2][EC] rows
    }
  }
  if constexpr (STAMP) {
    ts[5] = phase_stamp();
    if (lane == 0)
      for (int k = 0; k < 8; ++k) stamps[((size_t)(by * gdx + bx) * 4 + wv) * 8 + k] = ts[k];
  }
}

template <int CIN, int H, int W, int INM, int OUTM, bool DGRAD, typename TIN, bool STAMP = false>
__global__ void __launch_bounds__(256, 2) conv3x3_kernel(const TIN* __restrict__ xin, const uint16_t* __restrict__ zaux,
                                                      const float* __restrict__ st_in, const uint16_t* __restrict__ wt,
                                                      void* __restrict__ out, float* __restrict__ stats, int E, int B,
                                                      int chunks, int spw, BnFwd bnf, BnBwd bnb, BnRed brd,
                                                      unsigned long long* __restrict__ stamps = nullptr) {
  conv3x3_body<CIN, H, W, INM, OUTM, DGRAD, TIN, STAMP>(xin, zaux, st_in, wt, out, stats, E, B, chunks, spw, bnf, bnb,
                                                        brd, stamps, blockIdx.x, blockIdx.y, gridDim.x);
}

// ------------------------------------------------------------------------------------------
// conv3x3_fwd_db_kernel (round 6): the training forward of a 32-channel layer (2, 3) at P128, software-pipelined
// per wave over TWO LDS tiles.  conv3x3_body runs each sample's phases back to back -- stage (BN + ReLU of the
// previous layer's z, bf16 pack, 32 ds_write_b32 per lane), then 72 MFMAs, then the epilogue -- so with about one
// wave per SIMD the MFMA pipe idles through every staging (profiles/r4_28_stamp_conv.txt: ~2,800 cycles of vector
// issue beside 2,300 of MFMA per sample).  Here, while sample n's MFMAs run on tile[n & 1], the wave stages sample
// n + 1 into the other tile from the registers its loads landed in, a piece (2 positions of one channel-pair item:
// 2 packed FMAs, the NaN-keeping ReLU, 2 ds_write_b32) after each k-step's MFMA pair -- inside the MFMA shadow
// (an MFMA holds the SIMD's vector issue for 8 of its 32 cycles: MI355X_MICROARCH "vector-instruction ISSUE cost")
// -- and issues sample n + 2's global loads as soon as the last piece has consumed the registers.  Only the first
// sample's staging is exposed.  The arithmetic is conv3x3_body's (same k order, same accumulation, same statistics
// order): z and the BN partials are bit-identical to it.  One workgroup per CU (two tiles per wave: 111 KB of LDS).
// ------------------------------------------------------------------------------------------
template <int W>
__global__ void __launch_bounds__(256, 1) conv3x3_fwd_db_kernel(const uint16_t* __restrict__ xin,
                                                             const float* __restrict__ st_in,
                                                             const uint16_t* __restrict__ wt, uint16_t* __restrict__ out,
                                                             float* __restrict__ stats, int E, int B, int chunks,
                                                             int spw, BnFwd bnf) {
  using G = Geo<16, W>;
  constexpr int CIN = 32, KS = 18;                    // 16-deep k steps of K = 9 taps x 32 channels
  constexpr int TILE = G::HP * G::WP * CIN;           // bf16 elements per tile
  // staging items per lane: (channel pair, 8 positions) -- CIN * HW / 8 single-channel 8-position units, two per
  // item, 64 lanes
  constexpr int ITER = CIN * G::HW / 8 / 2 / 64;
  constexpr int NPIECE = ITER * 4;                    // pieces: 2 positions of one item
  constexpr int MG = 2, NG = G::MT / MG;               // position tiles per MFMA group, groups per sample
  static_assert(NPIECE < NG * KS, "the staging pieces and the next loads fit in one sample's k-steps");
  static_assert((CIN * G::HW / 8) % 128 == 0 && G::MT % MG == 0, "geometry");
  static_assert(32 * ITER == G::HW, "item k of lane l: positions 8 ((l >> 4) + 4 k) .. + 8 -- 4 lane groups x ITER");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int hh = lane >> 5, l32 = lane & 31;
  const int u = blockIdx.x / chunks, chunk = blockIdx.x % chunks, e = blockIdx.y;
  const int EC_in = E * CIN;
  __bf16* tiles = reinterpret_cast<__bf16*>(smem) + wv * 2 * TILE;
  for (int i = lane; i < 2 * TILE / 8; i += 64) reinterpret_cast<bf16x8*>(tiles)[i] = bf16x8{};
  bf16x8* wl = reinterpret_cast<bf16x8*>(reinterpret_cast<__bf16*>(smem) + 8 * TILE);   // B fragments
  float* stl = reinterpret_cast<float*>(wl + KS * 64);                                     // BN records
  const int n0 = u * B + (chunk * 4 + wv) * spw;
  const int nend = min((u + 1) * B, n0 + spw);
  const int nlast = nend - 1;

  // item k of this lane: channel pair pr = lane % 16 (the same for every k), positions [8 sg, 8 sg + 8)
  const int pr = lane & 15;
  // two register sets: the loads of sample n + 2 are issued during sample n, so every sample's data has a whole
  // sample period (~1 us) to arrive before its staging reads it (one sample ahead it waited out the HBM latency)
  uint4 ra[ITER][2], rb[ITER][2];
  auto load = [&](uint4 (&rv)[ITER][2], int n) {
    const size_t base = ((size_t)n * E + e) * CIN * G::HW;
#pragma unroll
    for (int k = 0; k < ITER; ++k) {
      const int sg = (lane >> 4) + 4 * k;
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2)
        rv[k][h2] = *reinterpret_cast<const uint4*>(xin + base + (size_t)(2 * pr + h2) * G::HW + 8 * sg);
    }
  };
  f32x2 a2, b2;   // this lane's channel pair's BN affine (after the prologue)
  // positions 2 jp, 2 jp + 1 of item k: BN + ReLU of both channels, one packed bf16 word per position
  auto piece = [&](const uint4 (&rv)[ITER][2], __bf16* tile, int k, int jp) {
    const int sg = (lane >> 4) + 4 * k, ph = (8 * sg) / W, pw = (8 * sg) % W;
    const uint32_t w0 = (&rv[k][0].x)[jp], w1 = (&rv[k][1].x)[jp];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const uint32_t u0 = q ? (w0 & 0xffff0000u) : (w0 << 16);
      const uint32_t u1 = q ? (w1 & 0xffff0000u) : (w1 << 16);
      f32x2 y = f32x2{__uint_as_float(u0), __uint_as_float(u1)} * a2 + b2;
      y.x = relu_max(y.x);
      y.y = relu_max(y.y);
      const int R = ph + 1, C = pw + 2 * jp + q + 1;
      *reinterpret_cast<uint32_t*>(tile + (R * G::WP + C) * CIN + 8 * ((pr >> 2) ^ tile_swz(R, C)) + 2 * (pr & 3)) =
          pack_bf16x2(y);
    }
  };

  // the first two samples' loads fly during the prologue (branch-free: past the wave's last sample, re-load it)
  if (n0 < nend) {
    load(ra, n0);
    load(rb, n0 + 1 <= nlast ? n0 + 1 : nlast);
  }
  {  // prologue: B fragments and the input BN records (conv3x3_body's)
    constexpr int WPT = (KS * 64 + 255) / 256;
    const bf16x8* wp = reinterpret_cast<const bf16x8*>(wt) + (size_t)e * KS * 64;
    bf16x8 tw[WPT];
#pragma unroll
    for (int k = 0; k < WPT; ++k)
      if (tid + 256 * k < KS * 64) tw[k] = wp[tid + 256 * k];
    float tp = 0.f;
    const bool build = bnf.stats != nullptr;
    if (!build) tp = st_in[((size_t)u * EC_in + e * CIN) * NST + tid];
    if (build) bn_fwd_build<false>(bnf, stl, u, e, EC_in, chunk == 0);
#pragma unroll
    for (int k = 0; k < WPT; ++k)
      if (tid + 256 * k < KS * 64) wl[tid + 256 * k] = tw[k];
    if (!build) stl[tid] = tp;
  }
  __syncthreads();
  a2 = f32x2{stl[(2 * pr) * NST + ST_A], stl[(2 * pr + 1) * NST + ST_A]};
  b2 = f32x2{stl[(2 * pr) * NST + ST_B], stl[(2 * pr + 1) * NST + ST_B]};
  if (n0 < nend) {   // the first sample staged up front (exposed), then set a takes sample n0 + 2
#pragma unroll
    for (int p = 0; p < NPIECE; ++p) piece(ra, tiles, p >> 2, p & 3);
    load(ra, n0 + 2 <= nlast ? n0 + 2 : nlast);
  }
  f32x2 s1v = {0.f, 0.f}, s2v = {0.f, 0.f};
  // sample n (tile cb): MFMAs over it; in their shadow sample n + 1 is staged from set `nx` into the other tile, and
  // set nx then takes sample n + 3
  auto sample = [&](int n, int cb, uint4 (&nx)[ITER][2]) {
    const __bf16* cur = tiles + cb * TILE;
    __bf16* nxt = tiles + (cb ^ 1) * TILE;
    wave_lds_fence();   // this sample's tile is written (by this wave alone) and the other one free to rewrite
    auto load_a = [&](int mt, int s) -> bf16x8 {
      const int p = mt * 32 + l32, ph = p / W, pw = p % W;
      const int tap = (16 * s) / CIN, q = ((16 * s) % CIN) / 8 + hh;
      const int R = ph + tap / 3, C = pw + tap % 3;
      return *reinterpret_cast<const bf16x8*>(cur + (R * G::WP + C) * CIN + 8 * (q ^ tile_swz(R, C)));
    };
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      f32x16 acc[MG];
      bf16x8 a_cur[MG], b_cur = wl[lane];
#pragma unroll
      for (int j = 0; j < MG; ++j) {
        acc[j] = f32x16{};
        a_cur[j] = load_a(g * MG + j, 0);
      }
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        bf16x8 a_nxt[MG], b_nxt;
        if (s + 1 < KS) {
          b_nxt = wl[(s + 1) * 64 + lane];
#pragma unroll
          for (int j = 0; j < MG; ++j) a_nxt[j] = load_a(g * MG + j, s + 1);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < MG; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_cur[j], b_cur, acc[j], 0, 0, 0);
        // the next sample's staging in this k-step's MFMA shadow, then (registers free) the loads after it
        const int p = g * KS + s;
        if (p < NPIECE) piece(nx, nxt, p >> 2, p & 3);
        if (p == NPIECE) load(nx, n + 3 <= nlast ? n + 3 : nlast);
        __builtin_amdgcn_sched_barrier(0);
        if (s + 1 < KS) {
          b_cur = b_nxt;
#pragma unroll
          for (int j = 0; j < MG; ++j) a_cur[j] = a_nxt[j];
        }
      }
#pragma unroll
      for (int j = 0; j < MG; ++j) {   // epilogue (conv3x3_body's OUT_Z_STATS)
        const int mt = g * MG + j;
        const size_t rbase = ((size_t)n * E + e) * CO * G::HW + (size_t)l32 * G::HW + mt * 32;
        uint32_t pk[4][2];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          pk[q][0] = pack_bf16x2(f32x2{acc[j][4 * q], acc[j][4 * q + 1]});
          pk[q][1] = pack_bf16x2(f32x2{acc[j][4 * q + 2], acc[j][4 * q + 3]});
          const f32x2 v01 = unpack_bf16x2(pk[q][0]), v23 = unpack_bf16x2(pk[q][1]);
          s1v += v01 + v23;
          s2v += v01 * v01 + v23 * v23;
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
#pragma unroll
          for (int w = 0; w < 2; ++w) {
            const auto r = __builtin_amdgcn_permlane32_swap(pk[2 * q][w], pk[2 * q + 1][w], false, false);
            pk[2 * q][w] = r[0];
            pk[2 * q + 1][w] = r[1];
          }
          *reinterpret_cast<uint4*>(out + rbase + 8 * (2 * q + hh)) =
              make_uint4(pk[2 * q][0], pk[2 * q][1], pk[2 * q + 1][0], pk[2 * q + 1][1]);
        }
      }
    }
  };
  for (int n = n0; n < nend; n += 2) {   // (by two: the register sets are named statically)
    sample(n, 0, rb);                    // stages n + 1 from b, b takes n + 3
    if (n + 1 < nend) sample(n + 1, 1, ra);   // stages n + 2 from a, a takes n + 4
  }
  float s1 = s1v.x + s1v.y, s2 = s2v.x + s2v.y;
  s1 += __shfl_xor(s1, 32);
  s2 += __shfl_xor(s2, 32);
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);
  if (hh == 0) {
    red[(wv * 32 + l32) * 2] = s1;
    red[(wv * 32 + l32) * 2 + 1] = s2;
  }
  __syncthreads();
  if (tid < 64) {
    const int c = tid >> 1, k = tid & 1;
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) t += red[(w * 32 + c) * 2 + k];
    stats[(((size_t)u * chunks + chunk) * 2 + k) * E * CO + e * CO + c] = t;   // planar [2][EC] rows
  }
}

// LDS writes of this workgroup visible to all its waves, WITHOUT waiting for outstanding global loads (a
// __syncthreads() drains vmcnt too, i.e. the next sample's prefetch)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ------------------------------------------------------------------------------------------
// conv3x3_split_kernel (round 6): the training forward of a layer (1: raw f32 pilots; 2, 3: BN + ReLU of the previous
// z) with every SAMPLE split over the workgroup's 4 waves.  conv3x3_body gives a wave whole samples -- the whole
// staging (BN + ReLU + bf16 pack + LDS writes) and all 72 MFMAs of each -- and at the step's 2,304 virtual samples
// that is about one wave per SIMD, which alternates its staging (vector issue), its MFMAs and its HBM waits with
// nothing beside it (profiles/r4_28_stamp_conv.txt).  Here the 4 waves stage a sample together (one channel-pair item
// per lane at P128), meet at ONE barrier, and each runs the MFMAs of its own position tile(s) -- a quarter of the
// sample -- while the next sample's loads fly; two tiles alternate, so that barrier is the only one per sample.  A
// workgroup is small (two sample tiles + the B fragments: 42 KB at P128) and short (sps samples), so three share a
// CU and its SIMDs interleave one workgroup's staging with another's MFMAs and HBM waits.  conv3x3_body's k order,
// MFMA shape and epilogue: z is bit-identical to it; the BN statistics partials come as ceil(B / sps) rows per group
// (another grouping of the same sums).
// ------------------------------------------------------------------------------------------
template <int CIN, int W, int INM, typename TIN, int SPS, int D>
__global__ void __launch_bounds__(256, W == 8 ? 3 : 2) conv3x3_split_kernel(const TIN* __restrict__ xin,
                                                                         const float* __restrict__ st_in,
                                                                         const uint16_t* __restrict__ wt,
                                                                         uint16_t* __restrict__ out,
                                                                         float* __restrict__ stats, int E, int B,
                                                                         int chunks, BnFwd bnf) {
  using G = Geo<16, W>;
  constexpr bool RAWIN = INM == IN_RAW_F32;
  static_assert(RAWIN ? CIN == 2 : (CIN == 32 && INM == IN_BNRELU), "layer 1 (raw pilots) or a 32-channel layer");
  static_assert(D >= 1 && D <= SPS, "prefetch depth");
  constexpr int KS = (9 * CIN + 15) / 16;             // 16-deep k steps
  constexpr int TILE = G::HP * G::WP * CIN;           // bf16 elements per sample tile
  constexpr int MTW = G::MT / 4;                      // 32-position tiles per wave
  // staging items per thread: raw input -- single values; else (channel pair, 8 positions) = two 16-byte vectors
  constexpr int IPT = RAWIN ? CIN * G::HW / 256 : 2 * G::HW / 256;
  static_assert(IPT >= 1 && G::MT % 4 == 0 && TILE % 8 == 0, "geometry");
  static_assert(2 * TILE * 2 >= 4 * 32 * 2 * (int)sizeof(float), "the statistics reduction reuses the tiles");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int hh = lane >> 5, l32 = lane & 31;
  const int u = blockIdx.x / chunks, chunk = blockIdx.x % chunks, e = blockIdx.y;
  const int EC_in = E * CIN;
  __bf16* tiles = reinterpret_cast<__bf16*>(smem);
  bf16x8* wl = reinterpret_cast<bf16x8*>(tiles + 2 * TILE);    // B fragments
  float* stl = reinterpret_cast<float*>(wl + KS * 64);          // BN records of the input channels
  const int n0 = u * B + chunk * SPS, cnt = min((u + 1) * B, n0 + SPS) - n0, nlast = n0 + cnt - 1;
  const int pr = tid & 15;   // (bf16 input) this thread's channel pair, the same for all its items

  // D samples' loads in flight (a ring of register sets, static indices: the sample loop is unrolled): one sample's
  // MFMAs are a quarter of conv3x3_body's, far shorter than an HBM round trip, so one sample ahead exposed it
  [[maybe_unused]] uint4 rv[RAWIN ? 1 : D][RAWIN ? 1 : IPT][2];
  [[maybe_unused]] float rr[RAWIN ? D : 1][RAWIN ? IPT : 1];
  auto load = [&](auto slot, int n) {
    constexpr int S = decltype(slot)::value;
    const size_t base = ((size_t)n * E + e) * CIN * G::HW;
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      const int i = tid + 256 * k;
      if constexpr (RAWIN) {
        rr[S][k] = xin[base + i];
      } else {
        const int sg = i >> 4;
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2)
          rv[S][k][h2] = *reinterpret_cast<const uint4*>(xin + base + (size_t)(2 * pr + h2) * G::HW + 8 * sg);
      }
    }
  };
  f32x2 a2 = {0.f, 0.f}, b2 = {0.f, 0.f};   // (bf16 input) this pair's BN affine, after the prologue
  auto stage = [&](auto slot, __bf16* tile) {
    constexpr int S = decltype(slot)::value;
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      const int i = tid + 256 * k;
      if constexpr (RAWIN) {
        const int c = i / G::HW, p = i % G::HW;
        tile[((p / W + 1) * G::WP + (p % W) + 1) * CIN + c] = (__bf16)rr[S][k];
      } else {   // conv3x3_body's channel-pair staging: packed FMA, NaN-keeping max, one packed bf16 word per position
        const int p0 = (i >> 4) * 8, ph = p0 / W, pw = p0 % W;
        const uint32_t w0[4] = {rv[S][k][0].x, rv[S][k][0].y, rv[S][k][0].z, rv[S][k][0].w};
        const uint32_t w1[4] = {rv[S][k][1].x, rv[S][k][1].y, rv[S][k][1].z, rv[S][k][1].w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t u0 = (j & 1) ? (w0[j >> 1] & 0xffff0000u) : (w0[j >> 1] << 16);
          const uint32_t u1 = (j & 1) ? (w1[j >> 1] & 0xffff0000u) : (w1[j >> 1] << 16);
          f32x2 y = f32x2{__uint_as_float(u0), __uint_as_float(u1)} * a2 + b2;
          y.x = relu_max(y.x);
          y.y = relu_max(y.y);
          const int R = ph + 1, C = pw + j + 1;
          *reinterpret_cast<uint32_t*>(tile + (R * G::WP + C) * CIN + 8 * ((pr >> 2) ^ tile_swz(R, C)) +
                                       2 * (pr & 3)) = pack_bf16x2(y);
        }
      }
    }
  };

  if (cnt > 0)   // the first D samples' loads fly during the prologue (past the last sample: re-load it, unused)
    static_for<0, D>([&](auto I) { load(I, min(n0 + (int)I, nlast)); });
  for (int i = tid; i < 2 * TILE / 8; i += 256) reinterpret_cast<bf16x8*>(tiles)[i] = bf16x8{};   // zero halos
  {  // prologue: B fragments -> LDS, the input BN records (built from the producer's partials or read as published)
    constexpr int WPT = (KS * 64 + 255) / 256;
    const bf16x8* wp = reinterpret_cast<const bf16x8*>(wt) + (size_t)e * KS * 64;
    bf16x8 tw[WPT];
#pragma unroll
    for (int k = 0; k < WPT; ++k)
      if ((KS * 64) % 256 == 0 || tid + 256 * k < KS * 64) tw[k] = wp[tid + 256 * k];
    if constexpr (!RAWIN) {
      if (bnf.stats) {
        bn_fwd_build<false>(bnf, stl, u, e, EC_in, chunk == 0);
      } else if (tid < CIN * NST) {
        stl[tid] = st_in[((size_t)u * EC_in + e * CIN) * NST + tid];
      }
    }
#pragma unroll
    for (int k = 0; k < WPT; ++k)
      if ((KS * 64) % 256 == 0 || tid + 256 * k < KS * 64) wl[tid + 256 * k] = tw[k];
  }
  __syncthreads();
  if constexpr (!RAWIN) {
    a2 = f32x2{stl[(2 * pr) * NST + ST_A], stl[(2 * pr + 1) * NST + ST_A]};
    b2 = f32x2{stl[(2 * pr) * NST + ST_B], stl[(2 * pr + 1) * NST + ST_B]};
  }
  f32x2 s1v = {0.f, 0.f}, s2v = {0.f, 0.f};
  static_for<0, SPS>([&](auto I) {
    constexpr int i = I;
    if (i < cnt) {   // (uniform over the workgroup)
      const int n = n0 + i;
      __bf16* tile = tiles + (i & 1) * TILE;
      stage(std::integral_constant<int, i % D>{}, tile);
      if constexpr (i + D < SPS) load(std::integral_constant<int, i % D>{}, min(n + D, nlast));   // refill the slot
      lds_barrier();
      auto load_a = [&](int mt, int s) -> bf16x8 {
        const int p = mt * 32 + l32, ph = p / W, pw = p % W;
        bf16x8 a;
        if constexpr (CIN % 16 == 0) {
          const int tap = (16 * s) / CIN, q = ((16 * s) % CIN) / 8 + hh;
          const int R = ph + tap / 3, C = pw + tap % 3;
          a = *reinterpret_cast<const bf16x8*>(tile + (R * G::WP + C) * CIN + 8 * (q ^ tile_swz(R, C)));
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int k = 16 * s + 8 * hh + j;
            if (k < 9 * CIN) {
              const int tap = k / CIN, c = k % CIN;
              a[j] = tile[((ph + tap / 3) * G::WP + pw + tap % 3) * CIN + c];
            } else {
              a[j] = (__bf16)0.f;
            }
          }
        }
        return a;
      };
      f32x16 acc[MTW];
      bf16x8 a_cur[MTW], b_cur = wl[lane];
#pragma unroll
      for (int j = 0; j < MTW; ++j) {
        acc[j] = f32x16{};
        a_cur[j] = load_a(wv + 4 * j, 0);
      }
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        bf16x8 a_nxt[MTW], b_nxt;
        if (s + 1 < KS) {
          b_nxt = wl[(s + 1) * 64 + lane];
#pragma unroll
          for (int j = 0; j < MTW; ++j) a_nxt[j] = load_a(wv + 4 * j, s + 1);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < MTW; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_cur[j], b_cur, acc[j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (s + 1 < KS) {
          b_cur = b_nxt;
#pragma unroll
          for (int j = 0; j < MTW; ++j) a_cur[j] = a_nxt[j];
        }
      }
#pragma unroll
      for (int j = 0; j < MTW; ++j) {   // epilogue (conv3x3_body's OUT_Z_STATS)
        const int mt = wv + 4 * j;
        const size_t rbase = ((size_t)n * E + e) * CO * G::HW + (size_t)l32 * G::HW + mt * 32;
        uint32_t pk[4][2];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          pk[q][0] = pack_bf16x2(f32x2{acc[j][4 * q], acc[j][4 * q + 1]});
          pk[q][1] = pack_bf16x2(f32x2{acc[j][4 * q + 2], acc[j][4 * q + 3]});
          const f32x2 v01 = unpack_bf16x2(pk[q][0]), v23 = unpack_bf16x2(pk[q][1]);
          s1v += v01 + v23;
          s2v += v01 * v01 + v23 * v23;
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
#pragma unroll
          for (int w = 0; w < 2; ++w) {
            const auto r = __builtin_amdgcn_permlane32_swap(pk[2 * q][w], pk[2 * q + 1][w], false, false);
            pk[2 * q][w] = r[0];
            pk[2 * q + 1][w] = r[1];
          }
          *reinterpret_cast<uint4*>(out + rbase + 8 * (2 * q + hh)) =
              make_uint4(pk[2 * q][0], pk[2 * q][1], pk[2 * q + 1][0], pk[2 * q + 1][1]);
        }
      }
    }
  });
  float s1 = s1v.x + s1v.y, s2 = s2v.x + s2v.y;
  s1 += __shfl_xor(s1, 32);
  s2 += __shfl_xor(s2, 32);
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);
  if (hh == 0) {
    red[(wv * 32 + l32) * 2] = s1;
    red[(wv * 32 + l32) * 2 + 1] = s2;
  }
  __syncthreads();
  if (tid < 64) {
    const int c = tid >> 1, k = tid & 1;
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) t += red[(w * 32 + c) * 2 + k];
    stats[(((size_t)u * chunks + chunk) * 2 + k) * E * CO + e * CO + c] = t;   // planar [2][EC] rows
  }
}

// ------------------------------------------------------------------------------------------
// conv_fwd_stack_kernel: the training forward of all three conv/BN/ReLU layers -- and the BN tail (layer 3's
// records, h3 = relu(bn3(z3)) for the FC GEMM, the running statistics) -- as ONE persistent launch.
// Workgroup (group u, chunk, expert e) runs conv3x3_body for layer 1, 2, 3 on the same samples, so each wave
// re-reads only the z it wrote itself (through its CU's L2: no cross-XCD traffic, no writeback between layers);
// between layers the `chunks` workgroups of stream (u, e) meet at a barrier, after which every one of them builds
// the next BN records from the stream's statistics partials (agent-scope atomic stores / loads: coherent across
// the XCDs).  Replaces 4 launches (3 conv + BN tail): no launch gaps, no per-kernel dispatch ramp and tail, no
// end-of-kernel L2 writeback of the activations between layers.  Bitwise the same z / h3 / records as the
// per-layer launches (same bodies, same partials, same summation order); the running statistics are summed in
// the consumers' order (bn_part_sums) instead of bn_fin_body's.
// Co-residency: the grid must fit the chip at once (checked on the host with the occupancy API, 2 workgroups per
// CU by launch bounds / LDS), and every barrier wait gives up after kStackSpin polls (the error word is set and
// the launch completes with wrong values instead of hanging).
// ------------------------------------------------------------------------------------------
constexpr int kStackSpin = 1 << 20;
struct StackSync {
  unsigned* bar;      // (U * E) x 2: arrivals, generation -- one barrier per stream (group u, expert e)
  unsigned* arrive;   // E x 3: streams of expert e past layer l (the last one updates the running statistics)
  int* err;           // set when a barrier wait gave up
};
struct StackFwd {
  const float* x1;              // (N, E*2, H, W) f32 pilots
  const uint16_t* w[3];         // packed forward B fragments (pack_weights)
  uint16_t* z[3];               // pre-BN outputs (bf16)
  float* stats[3];              // (U, chunks, 2, EC) statistics partials
  const float* gamma[3];
  const float* beta[3];
  float* run_mean[3];
  float* run_var[3];
  float* st[3];                 // (U, EC, NST) published records
  uint16_t* h3;                 // (N * E, 32 * HW) bf16: relu(bn3(z3)), the FC operand
  long long* nbt;               // (E * 3) num_batches_tracked, or null
  long long nbt_inc;
  float count, momentum, eps;
};

__device__ __forceinline__ unsigned ld_agent_u(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the n workgroups of one stream: sense-reversal barrier on (arrivals, generation), agent-scope atomics.  Every
// wave first waits for its own stores: the statistics partials are agent-scope atomic stores, complete = visible
// to the other XCDs (z needs nothing: only the wave that wrote it reads it back)
__device__ void stream_barrier(unsigned* bar, int n, int* err) {
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned* cnt = bar;
    unsigned* gen = bar + 1;
    const unsigned g = ld_agent_u(gen);
    __builtin_amdgcn_s_waitcnt(0);   // (the generation is read before this workgroup arrives)
    const unsigned old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == (unsigned)n - 1) {    // the last arrival resets the count, then releases the others
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_s_waitcnt(0);
      __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      int it = 0;
      while (ld_agent_u(gen) == g) {
        if (++it > kStackSpin) {
          __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
  }
  __syncthreads();
}

// running statistics of layer l, expert e, after every stream of the expert passed layer l's barrier: the groups'
// mean / var as the consumers computed them (bn_part_sums), momentum-updated in group order (the reference's
// per-stream BatchNorm calls); num_batches_tracked with layer 0
__device__ void stack_running_stats(const StackFwd& a, int l, int e, int U, int chunks, int EC) {
  const int tid = threadIdx.x, c = tid >> 3, j = tid & 7, ch = e * CO + c;
  float rm = a.run_mean[l][ch], rv = a.run_var[l][ch];
  for (int u = 0; u < U; ++u) {
    const float2 sm = bn_part_sums<true>(a.stats[l], u, chunks, EC, ch, j);
    const float mean = sm.x / a.count, var = fmaxf(sm.y / a.count - mean * mean, 0.f);
    rm = (1.f - a.momentum) * rm + a.momentum * mean;
    rv = (1.f - a.momentum) * rv + a.momentum * var * a.count / (a.count - 1.f);
  }
  if (j == 0) {
    a.run_mean[l][ch] = rm;
    a.run_var[l][ch] = rv;
  }
  if (l == 0 && a.nbt && tid < 3) a.nbt[e * 3 + tid] += a.nbt_inc;
}

// STAMP (diagnostic build, qd_conv_fwd_stack_stamped): per workgroup 8 s_memtime stamps -- start, after each layer's
// body, after each layer's barrier (+ running statistics), end
template <int W, bool STAMP = false>
__global__ void __launch_bounds__(256, 2) conv_fwd_stack_kernel(StackFwd a, StackSync sy, int E, int B, int U,
                                                                int chunks, int spw,
                                                                unsigned long long* __restrict__ stamps = nullptr) {
  __shared__ int last;
  unsigned long long ts[8] = {};
  if constexpr (STAMP) ts[0] = phase_stamp();
  const int bx = blockIdx.x, e = blockIdx.y, u = bx / chunks, chunk = bx % chunks;
  const int EC = E * CO;
  unsigned* bar = sy.bar + 2 * (u * E + e);
  auto bnf = [&](int l) {
    return BnFwd{a.stats[l], a.gamma[l], a.beta[l], a.run_mean[l], a.run_var[l], a.st[l], chunks, a.count, a.momentum,
                 a.eps, 1};
  };
  // after stream (u, e) passed layer l's barrier: its chunk-0 workgroup counts the stream in; the expert's last
  // stream updates the layer's running statistics
  auto arrive = [&](int l) {
    if (threadIdx.x == 0) {
      last = 0;
      if (chunk == 0) {
        unsigned* c = sy.arrive + e * 3 + l;
        if (__hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)U - 1) {
          __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          last = 1;
        }
      }
    }
    __syncthreads();
    if (last) stack_running_stats(a, l, e, U, chunks, EC);
  };
  conv3x3_body<2, 16, W, IN_RAW_F32, OUT_Z_STATS, false, float, false, true>(
      a.x1, nullptr, nullptr, a.w[0], a.z[0], a.stats[0], E, B, chunks, spw, BnFwd{}, BnBwd{}, BnRed{}, nullptr, bx, e,
      gridDim.x);
  if constexpr (STAMP) ts[1] = phase_stamp();
  stream_barrier(bar, chunks, sy.err);
  arrive(0);
  if constexpr (STAMP) ts[2] = phase_stamp();
  conv3x3_body<32, 16, W, IN_BNRELU, OUT_Z_STATS, false, uint16_t, false, true>(
      a.z[0], nullptr, nullptr, a.w[1], a.z[1], a.stats[1], E, B, chunks, spw, bnf(0), BnBwd{}, BnRed{}, nullptr, bx, e,
      gridDim.x);
  if constexpr (STAMP) ts[3] = phase_stamp();
  stream_barrier(bar, chunks, sy.err);
  arrive(1);
  if constexpr (STAMP) ts[4] = phase_stamp();
  conv3x3_body<32, 16, W, IN_BNRELU, OUT_Z_STATS, false, uint16_t, false, true>(
      a.z[1], nullptr, nullptr, a.w[2], a.z[2], a.stats[2], E, B, chunks, spw, bnf(1), BnBwd{}, BnRed{}, nullptr, bx, e,
      gridDim.x);
  if constexpr (STAMP) ts[5] = phase_stamp();
  stream_barrier(bar, chunks, sy.err);
  arrive(2);
  if constexpr (STAMP) ts[6] = phase_stamp();
  // ---- tail: layer 3's records (chunk 0 publishes them for the backward), then h3 = relu(a z3 + b) for every
  // wave's own samples (the z3 it wrote), 8 items of 8 values per lane and sample, all loads in flight ----
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* stl = reinterpret_cast<float*>(smem);
  bn_fwd_build<true>(bnf(2), stl, u, e, EC, chunk == 0);
  __syncthreads();
  constexpr int HW = 16 * W, ITEMS = CO * HW / 8, PER = ITEMS / 64;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int n0 = u * B + (chunk * 4 + wv) * spw, nend = min((u + 1) * B, n0 + spw);
  for (int n = n0; n < nend; ++n) {
    const size_t base = ((size_t)n * E + e) * CO * HW;
    uint4 raw[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) raw[k] = *reinterpret_cast<const uint4*>(a.z[2] + base + (size_t)(lane + 64 * k) * 8);
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = lane + 64 * k, c = (i * 8) / HW;
      const f32x2 a2 = {stl[c * NST + ST_A], stl[c * NST + ST_A]}, b2 = {stl[c * NST + ST_B], stl[c * NST + ST_B]};
      const uint32_t r4[4] = {raw[k].x, raw[k].y, raw[k].z, raw[k].w};
      uint32_t w4[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        f32x2 y = unpack_bf16x2(r4[q]) * a2 + b2;
        y.x = relu_nan(y.x);
        y.y = relu_nan(y.y);
        w4[q] = pack_bf16x2(y);
      }
      *reinterpret_cast<uint4*>(a.h3 + base + (size_t)i * 8) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
    }
  }
  if constexpr (STAMP) {
    ts[7] = phase_stamp();
    if (threadIdx.x == 0)
      for (int k = 0; k < 8; ++k) stamps[((size_t)e * gridDim.x + bx) * 8 + k] = ts[k];
  }
}

// ------------------------------------------------------------------------------------------
// conv3x3_f8_kernel: the fp8 estimator's 32-channel forward (layers 2, 3) on e4m3 operands.
// conv3x3_body's structure with an e4m3 channel-last tile -- 32-byte pixels, 8-byte chunks at
// q ^ tile8_swz(R, C): conflict-free ds_read_b64 fragment reads (lane halves of 32) for every tap
// of both geometries -- e4m3 B fragments (qd_conv_pack_f8) and mfma_f32_32x32x16_fp8_fp8 (lane l:
// A[row l&31][k = 8(l>>5) + j], the bf16 form's map; K order (tap, channel) as the bf16 pack), built in
// the prologue straight from the fp32 weights with the delayed weight factor (no pack launch: the
// separate pack sat on the critical path at 16 us); the bx == 0 block of each expert records the
// expert's max |W| (amax_w[e]) for the next step's factor.
// Input transform h = BN+ReLU(z_prev) -> e4m3(h * qs_a) with the delayed activation scale; the
// epilogue scales the accumulators by deq = scale_a * scale_w, then writes bf16 z + statistics
// exactly as the bf16 body (the BN backward still sees bf16 z).  amax_a[block] = max h of the
// block for the next step's scale.  W = 8: the next sample's loads fly during the MFMAs.
// ------------------------------------------------------------------------------------------
template <int W>
__device__ __forceinline__ int tile8_swz(int R, int C) {
  if constexpr (W == 8) return R & 3;
  else return (R + 2 * (C >> 3)) & 3;
}
constexpr int KS8 = 18;   // 16-deep k-steps of a 32-channel layer

template <int W>
__global__ void __launch_bounds__(256, 2) conv3x3_f8_kernel(const uint16_t* __restrict__ xin,
                                                         const float* __restrict__ w32, uint16_t* __restrict__ out,
                                                         float* __restrict__ stats, int E, int B, int chunks, int spw,
                                                         BnFwd bnf, const float* __restrict__ qs,
                                                         const float* __restrict__ scale, float* __restrict__ amax_a,
                                                         float* __restrict__ amax_w) {
  using G = Geo<16, W>;
  constexpr int CIN = 32, PIX = 32;
  constexpr int TILE = G::HP * G::WP * PIX;     // bytes per wave tile
  constexpr int ITER = 8 * G::HW / 8 / 64;      // staging items (channel quad x 8 positions) per lane
  constexpr bool PREF = G::HW <= 128;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int hh = lane >> 5, l32 = lane & 31;
  const int bx = blockIdx.x, e = blockIdx.y, u = bx / chunks, chunk = bx % chunks;
  const int EC_in = E * CIN;
  uint8_t* tile = reinterpret_cast<uint8_t*>(smem) + wv * TILE;
  for (int i = lane; i < TILE / 16; i += 64) reinterpret_cast<uint4*>(tile)[i] = make_uint4(0u, 0u, 0u, 0u);
  uint2* wl = reinterpret_cast<uint2*>(smem + 4 * TILE);   // [s][lane] 8-byte B fragments
  float* stl = reinterpret_cast<float*>(wl + KS8 * 64);    // BN records of the input channels
  const float qa = qs[0], deq = scale[0] * scale[1];
  const int n0 = u * B + (chunk * 4 + wv) * spw;
  const int nend = min((u + 1) * B, n0 + spw);

  // staging item: 8 positions x 4 channels (bf16), one dword per pixel in the e4m3 tile
  auto load_item = [&](int n, int it, uint4 (&r)[4]) {
    const size_t base = ((size_t)n * E + e) * CIN * G::HW;
    const int i = lane + 64 * it, qd = i & 7, sg = i >> 3;
#pragma unroll
    for (int c4 = 0; c4 < 4; ++c4)
      r[c4] = *reinterpret_cast<const uint4*>(xin + base + (size_t)(4 * qd + c4) * G::HW + 8 * sg);
  };
  float mx = 0.f;
  auto store_item = [&](int it, const uint4 (&r)[4]) {
    {
      const int i = lane + 64 * it, qd = i & 7, p0 = (i >> 3) * 8;
      float v[4][8];
#pragma unroll
      for (int c4 = 0; c4 < 4; ++c4) {
        const float* sc = stl + (4 * qd + c4) * NST;
        const float a = sc[ST_A], b = sc[ST_B];
        unpack_q(r[c4], v[c4], (const uint16_t*)nullptr);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          v[c4][j] = relu_nan(a * v[c4][j] + b);
          mx = fmaxf(mx, v[c4][j]);
        }
      }
      const int ph = p0 / W, pw = p0 % W;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int R = ph + 1, C = pw + j + 1;
        const uint32_t q4 = e4m3_pack4(v[0][j] * qa, v[1][j] * qa, v[2][j] * qa, v[3][j] * qa);
        *reinterpret_cast<uint32_t*>(tile + (R * G::WP + C) * PIX + 8 * ((qd >> 1) ^ tile8_swz<W>(R, C)) +
                                     4 * (qd & 1)) = q4;
      }
    }
  };
  uint4 rv[PREF ? ITER : 1][4];   // (P128) the next sample's items
  auto load = [&](int n) {
#pragma unroll
    for (int it = 0; it < ITER; ++it) load_item(n, it, rv[it]);
  };
  auto stage = [&](int n) {
    if constexpr (PREF) {
#pragma unroll
      for (int it = 0; it < ITER; ++it) store_item(it, rv[it]);
    } else {
#pragma unroll 1
      for (int it = 0; it < ITER; ++it) {   // one item in registers at a time (P256)
        load_item(n, it, rv[0]);
        store_item(it, rv[0]);
      }
    }
  };
  if (PREF && n0 < nend) load(n0);
  float wmx = 0.f;
  {
    constexpr int NF = KS8 * 64, FPT = (NF + 255) / 256;   // fragments (s, lane) per thread
    const float qw = qs[1];
    float tv[FPT][8];
#pragma unroll
    for (int t = 0; t < FPT; ++t) {
      const int f = tid + 256 * t, s8 = f >> 6, h = (f >> 5) & 1, col = f & 31;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 16 * s8 + 8 * h + j;   // (tap k / 32, input channel k % 32)
        tv[t][j] = f < NF ? w32[((size_t)(e * CO + col) * CO + k % CO) * 9 + k / CO] : 0.f;
      }
    }
    float tp = 0.f;
    if (!bnf.stats) tp = bnf.st_out[((size_t)u * EC_in + e * CIN) * NST + tid];   // (records given as is)
#pragma unroll
    for (int t = 0; t < FPT; ++t) {
      const int f = tid + 256 * t;
      if (f < NF) {
        const float* v = tv[t];
#pragma unroll
        for (int j = 0; j < 8; ++j) wmx = fmaxf(wmx, fabsf(v[j]));
        wl[f] = make_uint2(e4m3_pack4(v[0] * qw, v[1] * qw, v[2] * qw, v[3] * qw),
                           e4m3_pack4(v[4] * qw, v[5] * qw, v[6] * qw, v[7] * qw));
      }
    }
    if (bnf.stats) bn_fwd_build(bnf, stl, u, e, EC_in, chunk == 0);
    else stl[tid] = tp;
  }
  __syncthreads();

  float s1 = 0.f, s2 = 0.f;
  f32x2 s1v = {0.f, 0.f}, s2v = {0.f, 0.f};
  for (int n = n0; n < nend; ++n) {
    wave_lds_fence();
    stage(n);
    if (PREF && n + 1 < nend) load(n + 1);
    wave_lds_fence();
    auto load_a = [&](int mt, int s) -> long {
      const int p = mt * 32 + l32, ph = p / W, pw = p % W;
      const int tap = s >> 1, q = ((s & 1) << 1) + hh;
      const int R = ph + tap / 3, C = pw + tap % 3;
      const uint2 v = *reinterpret_cast<const uint2*>(tile + (R * G::WP + C) * PIX + 8 * (q ^ tile8_swz<W>(R, C)));
      return (long)(((unsigned long)v.y << 32) | v.x);
    };
    constexpr int MG = G::MT < 4 ? G::MT : 4;
#pragma unroll
    for (int g0 = 0; g0 < G::MT; g0 += MG) {
      f32x16 acc[MG];
#pragma unroll
      for (int j = 0; j < MG; ++j) acc[j] = f32x16{};
#pragma unroll
      for (int s = 0; s < KS8; ++s) {
        const uint2 bw = wl[s * 64 + lane];
        const long b = (long)(((unsigned long)bw.y << 32) | bw.x);
#pragma unroll
        for (int j = 0; j < MG; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_fp8_fp8(load_a(g0 + j, s), b, acc[j], 0, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < MG; ++j) {
        const int mt = g0 + j;
        const size_t rbase = ((size_t)n * E + e) * CO * G::HW + (size_t)l32 * G::HW + mt * 32;
        uint32_t pk[4][2];   // (conv3x3_body's packed epilogue)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          pk[g][0] = pack_bf16x2(f32x2{acc[j][4 * g], acc[j][4 * g + 1]} * deq);
          pk[g][1] = pack_bf16x2(f32x2{acc[j][4 * g + 2], acc[j][4 * g + 3]} * deq);
          const f32x2 v01 = unpack_bf16x2(pk[g][0]), v23 = unpack_bf16x2(pk[g][1]);
          s1v += v01 + v23;
          s2v += v01 * v01 + v23 * v23;
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
#pragma unroll
          for (int w = 0; w < 2; ++w) {
            const auto r = __builtin_amdgcn_permlane32_swap(pk[2 * q][w], pk[2 * q + 1][w], false, false);
            pk[2 * q][w] = r[0];
            pk[2 * q + 1][w] = r[1];
          }
          *reinterpret_cast<uint4*>(out + rbase + 8 * (2 * q + hh)) =
              make_uint4(pk[2 * q][0], pk[2 * q][1], pk[2 * q + 1][0], pk[2 * q + 1][1]);
        }
      }
    }
  }
  s1 += s1v.x + s1v.y;
  s2 += s2v.x + s2v.y;
  s1 += __shfl_xor(s1, 32);
  s2 += __shfl_xor(s2, 32);
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);
  if (hh == 0) {
    red[(wv * 32 + l32) * 2] = s1;
    red[(wv * 32 + l32) * 2 + 1] = s2;
  }
  __syncthreads();
  if (tid < 64) {
    const int c = tid >> 1, k = tid & 1;
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) t += red[(w * 32 + c) * 2 + k];
    stats[(((size_t)u * chunks + chunk) * 2 + k) * E * CO + e * CO + c] = t;
  }
  // the block's max h (h >= 0) -> its amax partial (index: the flat block id; < kAmaxParts); the
  // expert's max |W| from its bx == 0 block
  float m = mx, mw = wmx;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    m = fmaxf(m, __shfl_xor(m, o));
    mw = fmaxf(mw, __shfl_xor(mw, o));
  }
  __syncthreads();
  if (lane == 0) {
    red[wv] = m;
    red[4 + wv] = mw;
  }
  __syncthreads();
  if (tid == 0) {
    const float bm = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    float* ap = amax_a + (size_t)blockIdx.y * gridDim.x + blockIdx.x;
    *ap = fmaxf(*ap, bm);
    if (bx == 0) amax_w[e] = fmaxf(amax_w[e], fmaxf(fmaxf(red[4], red[5]), fmaxf(red[6], red[7])));
  }
}

// ------------------------------------------------------------------------------------------
// pack_weights_kernel: fp32 W (E*32, CIN, 3, 3) -> bf16 B fragments [e][s][lane][8] in the
// exact register order conv3x3_kernel consumes (16-byte coalesced loads per lane).
// dgrad = 1: transposed + spatially flipped (the data-gradient correlation).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void pack_weights_body(const float* __restrict__ w, uint16_t* __restrict__ out, int CIN,
                                                  int KS, int dgrad, int s, int e) {
  const int lane = threadIdx.x;
  const int hh = lane >> 5, col = lane & 31;
  uint16_t v8[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 16 * s + 8 * hh + j;
    float v = 0.f;
    if (!dgrad) {
      if (k < 9 * CIN) v = w[((size_t)(e * CO + col) * CIN + k % CIN) * 9 + k / CIN];
    } else {
      if (k < 9 * CO) v = w[((size_t)(e * CO + k % CO) * CO + col) * 9 + (8 - k / CO)];
    }
    v8[j] = f32_to_bf16(v);
  }
  uint4 pk = make_uint4(v8[0] | ((uint32_t)v8[1] << 16), v8[2] | ((uint32_t)v8[3] << 16),
                        v8[4] | ((uint32_t)v8[5] << 16), v8[6] | ((uint32_t)v8[7] << 16));
  *reinterpret_cast<uint4*>(out + (((size_t)e * KS + s) * 64 + lane) * 8) = pk;
}

__global__ void pack_weights_kernel(const float* __restrict__ w, uint16_t* __restrict__ out, int E, int CIN, int KS,
                                    int dgrad) {
  pack_weights_body(w, out, CIN, KS, dgrad, blockIdx.x, blockIdx.y);
}

// All packs of a step in one launch (weights only change at the optimizer step).
struct PackJobs {
  const float* w[8];
  uint16_t* out[8];
  int cin[8], ks[8], dgrad[8];
  int* cursor;      // optional: *cursor += cursor_inc (the step's batch cursor, advanced here when the
  int cursor_inc;   // pack runs at the END of a step, after everything that read the cursor)
};
__global__ void pack_weights_multi_kernel(PackJobs jobs) {
  const int j = blockIdx.z, s = blockIdx.x;
  if (jobs.cursor != nullptr && j == 0 && s == 0 && blockIdx.y == 0 && threadIdx.x == 0) *jobs.cursor += jobs.cursor_inc;
  if (s >= jobs.ks[j]) return;
  pack_weights_body(jobs.w[j], jobs.out[j], jobs.cin[j], jobs.ks[j], jobs.dgrad[j], s, blockIdx.y);
}

// ------------------------------------------------------------------------------------------
// conv3x3_wgrad: dW[e][co][ci][tap] partials.  grid (U*chunks, E), block 256, `spb` samples
// per workgroup; slab[(e * U*chunks + blockIdx.x)][co][ci][tap].
// x = layer input (raw f32 pilots, or BN+ReLU of the previous z); dz from (dh, z, st).
// ------------------------------------------------------------------------------------------
template <int CIN, int H, int W, int INM, typename TIN, typename TDH>
__device__ __forceinline__ void conv3x3_wgrad_body(const TIN* __restrict__ xin, const float* __restrict__ st_prev,
                                                   const TDH* __restrict__ dh, const uint16_t* __restrict__ z,
                                                   const float* __restrict__ st, float* __restrict__ slab, int E, int B,
                                                   int chunks, int spb, BnBwd bnb, int bx, int by, int gdx) {
  using G = Geo<H, W>;
  constexpr int MTW = (9 * CIN + 31) / 32;        // accumulator tiles (9 for CIN=32, 1 for CIN=2)
  constexpr int XCS = G::HP * W + 8;              // channel stride of the shifted copies (bf16)
  constexpr int DZS = G::HW + 8;                  // channel stride of the dz tile (bf16)
  constexpr int KSW = G::HW / 16 / 4;             // k-steps per wave per sample (positions split 4 ways)
  constexpr int XELEMS = 3 * CIN * XCS;
  // staging items per thread: x = one (channel, image row) of W values; dz = 8 positions of a channel
  constexpr int XN = CIN * H, XIT = (XN + 255) / 256, XQ = W / PerQ<TIN>::N;
  constexpr int DN = CO * G::HW / 8, DIT = DN / 256, DQ = 8 / PerQ<TDH>::N;
  static_assert(DN % 256 == 0, "dz staging items");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __bf16* X = reinterpret_cast<__bf16*>(smem);
  __bf16* DZ = X + XELEMS;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int hh = lane >> 5, l32 = lane & 31;
  const int u = bx / chunks, chunk = bx % chunks, e = by;
  // zero halo rows (0 and HP-1) of every shifted copy; interior rows are rewritten per sample
  for (int i = tid; i < 3 * CIN * 2 * (W / 8); i += 256) {
    const int cc = i / (2 * (W / 8)), r = (i / (W / 8)) & 1, q = i % (W / 8);
    *reinterpret_cast<bf16x8*>(X + cc * XCS + r * (G::HP - 1) * W + 8 * q) = bf16x8{};
  }

  f32x16 acc[MTW];
#pragma unroll
  for (int t = 0; t < MTW; ++t) acc[t] = f32x16{};
  const int n0 = u * B + chunk * spb, nend = min((u + 1) * B, n0 + spb);

  // ---- one-sample-ahead register prefetch: sample n+1's loads fly during sample n's MFMAs ----
  uint4 xr[XIT][XQ], dr[DIT][DQ], zr[DIT];
  auto prefetch = [&](int n) {
    const size_t xb = ((size_t)n * E + e) * CIN * G::HW;
#pragma unroll
    for (int k = 0; k < XIT; ++k) {
      const int i = tid + 256 * k;
      if (XN % 256 == 0 || i < XN) {
        const uint4* src = reinterpret_cast<const uint4*>(xin + xb + (size_t)(i / H) * G::HW + (i % H) * W);
#pragma unroll
        for (int q = 0; q < XQ; ++q) xr[k][q] = src[q];
      }
    }
    const size_t zb = ((size_t)n * E + e) * CO * G::HW;
#pragma unroll
    for (int k = 0; k < DIT; ++k) {
      const size_t off = zb + (size_t)(tid + 256 * k) * 8;   // item i covers elements [8i, 8i+8) of the sample
      const uint4* sd = reinterpret_cast<const uint4*>(dh + off);
#pragma unroll
      for (int q = 0; q < DQ; ++q) dr[k][q] = sd[q];
      zr[k] = *reinterpret_cast<const uint4*>(z + off);
    }
  };
  if (n0 < nend) prefetch(n0);   // (the first sample's loads fly while the BN records are built)

  // ---- BN parameters of this block's (group, expert) channels -> LDS once: [x: CIN][dz: CO] x NST ----
  float* prm = reinterpret_cast<float*>(DZ + CO * DZS);
  if constexpr (INM == IN_BNRELU) {
    const float* sp = st_prev + ((size_t)u * E * CIN + e * CIN) * NST;
    for (int i = tid; i < CIN * NST; i += 256) prm[i] = sp[i];
  }
  if (bnb.rslab) {   // fused BN backward finalisation
    bn_bwd_build(bnb, st, prm + CIN * NST, u, e, E * CO);
  } else {
    const float* sp = st + ((size_t)u * E * CO + e * CO) * NST;
    for (int i = tid; i < CO * NST; i += 256) prm[CIN * NST + i] = sp[i];
  }

  for (int n = n0; n < nend; ++n) {
    __syncthreads();   // the previous sample's MFMAs are done reading X / DZ
    // ---- x -> 3 column-shifted copies: X[kw][ci][row 0..HP-1][w] = x[ci][row-1][w+kw-1] ----
#pragma unroll
    for (int k = 0; k < XIT; ++k) {
      const int i = tid + 256 * k;
      if (XN % 256 == 0 || i < XN) {
        const int c = i / H, ph = i % H;
        float v[W + 2];
        v[0] = 0.f;
        v[W + 1] = 0.f;
#pragma unroll
        for (int q = 0; q < XQ; ++q) unpack_q(xr[k][q], v + 1 + q * PerQ<TIN>::N, (const TIN*)nullptr);
        if constexpr (INM == IN_BNRELU) {
          const float xa = prm[c * NST + ST_A], xb2 = prm[c * NST + ST_B];
#pragma unroll
          for (int q = 1; q <= W; ++q) v[q] = relu_nan(xa * v[q] + xb2);
        }
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          __bf16* dst = X + (kw * CIN + c) * XCS + (ph + 1) * W;
#pragma unroll
          for (int q = 0; q < W; q += 8) {
            bf16x8 o;
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = (__bf16)v[q + j + kw];  // column w holds x[w + kw - 1]
            *reinterpret_cast<bf16x8*>(dst + q) = o;
          }
        }
      }
    }
    // ---- dz = BN/ReLU backward of dh (bf16) [co][p] ----
#pragma unroll
    for (int k = 0; k < DIT; ++k) {
      const int i = tid + 256 * k;
      const int c = i / (G::HW / 8), p0 = (i % (G::HW / 8)) * 8;
      float d[8], zz[8];
#pragma unroll
      for (int q = 0; q < DQ; ++q) unpack_q(dr[k][q], d + q * PerQ<TDH>::N, (const TDH*)nullptr);
      unpack_q(zr[k], zz, (const uint16_t*)nullptr);
      const float* sc = prm + (CIN + c) * NST;
      const float da = sc[ST_A], db = sc[ST_B], dmu = sc[ST_MEAN], dinv = sc[ST_INV];
      const float dc1 = sc[ST_C1], dc2 = sc[ST_C2], dc3 = sc[ST_C3];
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float g = bn_gate(da, zz[j], db) ? d[j] : 0.f;
        o[j] = (__bf16)bn_dz(g, bn_xhat(zz[j], dmu, dinv), dc1, dc2, dc3);
      }
      *reinterpret_cast<bf16x8*>(DZ + c * DZS + p0) = o;
    }
    if (n + 1 < nend) prefetch(n + 1);
    __syncthreads();
    // ---- MFMA: this wave's positions p in [wv*HW/4, (wv+1)*HW/4) ----
#pragma unroll
    for (int ks = 0; ks < KSW; ++ks) {
      const int p0 = (wv * KSW + ks) * 16 + 8 * hh;   // 8 consecutive positions (aligned, one row)
      const int ph = p0 / W, pw0 = p0 % W;
      const bf16x8 bfr = *reinterpret_cast<const bf16x8*>(DZ + l32 * DZS + p0);
#pragma unroll
      for (int t = 0; t < MTW; ++t) {
        const int m = t * 32 + l32;
        bf16x8 a;
        if (m < 9 * CIN) {
          const int c = m % CIN, tap = m / CIN, kh = tap / 3, kw = tap % 3;   // row m = (tap, ci)
          a = *reinterpret_cast<const bf16x8*>(X + (kw * CIN + c) * XCS + (ph + kh) * W + pw0);
        } else {
          a = bf16x8{};
        }
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bfr, acc[t], 0, 0, 0);
      }
    }
  }
  // ---- reduce the 4 waves' accumulators through LDS (two transposed regions [co][m], odd row
  // stride: conflict-free), (w0 + w2) + (w1 + w3) in a fixed order, then one contiguous slab row ----
  constexpr int RS = 9 * CIN + 1;
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem) + (wv & 1) * 32 * RS;
#pragma unroll
  for (int round = 0; round < 2; ++round) {
    if ((wv >> 1) == round) {
#pragma unroll
      for (int t = 0; t < MTW; ++t) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = t * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;   // (tap, ci) -> slab column ci * 9 + tap
          if (m < 9 * CIN) {
            float* q = red + l32 * RS + (m % CIN) * 9 + m / CIN;
            *q = (round == 0 ? 0.f : *q) + acc[t][r];
          }
        }
      }
    }
    __syncthreads();
  }
  const float* r0 = reinterpret_cast<const float*>(smem);
  float* srow = slab + ((size_t)e * gdx + bx) * CO * CIN * 9;
  for (int i = tid; i < CO * CIN * 9; i += 256) {
    const int co = i / (CIN * 9), m = i % (CIN * 9);
    srow[i] = r0[co * RS + m] + r0[32 * RS + co * RS + m];
  }
}

template <int CIN, int H, int W, int INM, typename TIN, typename TDH>
__global__ void __launch_bounds__(256, 2) conv3x3_wgrad_kernel(const TIN* __restrict__ xin,
                                                            const float* __restrict__ st_prev,
                                                            const TDH* __restrict__ dh,
                                                            const uint16_t* __restrict__ z,
                                                            const float* __restrict__ st, float* __restrict__ slab,
                                                            int E, int B, int chunks, int spb, BnBwd bnb) {
  conv3x3_wgrad_body<CIN, H, W, INM, TIN, TDH>(xin, st_prev, dh, z, st, slab, E, B, chunks, spb, bnb, blockIdx.x,
                                               blockIdx.y, gridDim.x);
}

// One launch for a 32-channel layer's weight gradient AND data gradient (bf16 dh / dx): the two are
// independent (they share only their inputs), so their workgroups run side by side -- blocks
// [0, gx_w) take the wgrad body, the rest the dgrad body -- without a graph branch (whose cross-
// queue edges cost more than the overlap wins).  Each body is exactly its own kernel's.
template <int W>
__global__ void __launch_bounds__(256, 2) conv3x3_wd_kernel(const uint16_t* __restrict__ xin,
                                                         const float* __restrict__ st_prev,
                                                         const uint16_t* __restrict__ dh,
                                                         const uint16_t* __restrict__ z, const float* __restrict__ st,
                                                         float* __restrict__ slab, int chunks_w, int spb, BnBwd bnb,
                                                         const uint16_t* __restrict__ wt, uint16_t* __restrict__ dx,
                                                         int chunks_d, int spw, BnRed brd, int E, int B, int gx_w) {
  if ((int)blockIdx.x < gx_w) {
    conv3x3_wgrad_body<32, 16, W, IN_BNRELU, uint16_t, uint16_t>(xin, st_prev, dh, z, st, slab, E, B, chunks_w, spb,
                                                                 bnb, blockIdx.x, blockIdx.y, gx_w);
  } else {
    conv3x3_body<32, 16, W, IN_BNBWD, OUT_BF16, true, uint16_t>(dh, z, st, wt, dx, nullptr, E, B, chunks_d, spw,
                                                                 BnFwd{}, bnb, brd, nullptr, blockIdx.x - gx_w,
                                                                 blockIdx.y, gridDim.x - gx_w);
  }
}

// ------------------------------------------------------------------------------------------
// conv3x3_bwd_kernel: a 32-channel layer's weight gradient, data gradient and the previous layer's
// BN backward reduction from ONE staging of each sample.  conv3x3_wd_kernel runs the wgrad and dgrad
// bodies as separate workgroups, and each of them reads dh, z and z_prev of every sample: per layer
// at P128 / 9 streams that is 2 x 3 x 18.9 MB of reads + 18.9 MB of dx.  Here a workgroup stages a
// sample once --
//   dz = BN/ReLU backward of (dh, z) into two LDS images: channel-major rows (the wgrad B operand)
//        and the swizzled channel-last tile (the dgrad A operand, tile_swz);
//   x  = BN+ReLU(z_prev) into the three column-shifted copies (the wgrad A operand)
// -- and its 4 waves run both GEMMs on it, interleaved (the dependent dgrad chain beside the wgrad
// accumulators):
//   dgrad  wave w: position tiles w, w+4, ... (M = 32 positions, N = 32 input channels, K = 288),
//          epilogue = bf16 dx + the previous layer's BN backward partials (raw z_prev kept in LDS: a
//          global re-read there would wait out the next sample's prefetch, vmcnt being in order);
//   wgrad  dW rows are (tap, ci) tiles of 32: wave w owns taps w and w+4 over ALL positions (no
//          cross-wave sum) and a quarter of tap 8's positions -- 18 MFMAs per dgrad tile, same as
//          the dgrad, 3 accumulator tiles instead of 9; accumulated across the workgroup's samples.
// P128: the next sample's dh / z / z_prev loads are in flight during the MFMAs.
// grid (U * chunks, E), block 256, spb samples per workgroup.  Outputs are exactly the two bodies':
// dx, slab rows (e * gridDim.x + bx) and part rows (u, chunk) -- same arithmetic, same order.
// ------------------------------------------------------------------------------------------
template <int W>
struct BwdGeo {
  using G = Geo<16, W>;
  static constexpr int XCS = G::HP * W + 8;    // channel stride of the shifted x copies (bf16)
  static constexpr int DZS = G::HW + 8;        // channel stride of the channel-major dz rows (bf16)
  static constexpr int ZPS = G::HW + 4;        // raw z_prev rows [ci][p] (ds_read_b64: 66 dwords per row)
  static constexpr int X_EL = 3 * CO * XCS, DZ_EL = CO * DZS, T_EL = G::HP * G::WP * CO, ZP_EL = CO * ZPS;
  static constexpr int KSD = 18;               // dgrad k-steps (9 taps x 32 channels / 16)
  static constexpr size_t STAGE = (size_t)(X_EL + DZ_EL + T_EL + ZP_EL) * 2 + KSD * 64 * 16 + 2 * CO * NST * 4;
  static constexpr size_t RED = (CO * (size_t)(9 * CO + 1) + 4 * CO * (CO + 1)) * 4;   // dW rows | tap-8 partials
  static constexpr size_t SMEM = STAGE > RED ? STAGE : RED;
};

template <int W>
__global__ void __launch_bounds__(256, W == 8 ? 2 : 1) conv3x3_bwd_kernel(const uint16_t* __restrict__ zprev,
                                                          const float* __restrict__ st_prev,
                                                          const uint16_t* __restrict__ dh,
                                                          const uint16_t* __restrict__ z, const float* __restrict__ st,
                                                          float* __restrict__ slab, const uint16_t* __restrict__ wt,
                                                          uint16_t* __restrict__ dx, float* __restrict__ part, int E,
                                                          int B, int chunks, int spb, BnBwd bnb, LossFinish lf) {
  if ((int)blockIdx.y == E) {   // the extra row (lf.part set): block 0 hosts the HDCE loss finish (when layer 3's
    if (blockIdx.x == 0) loss_finish_body(lf);   // BN reduction rode in the FC data gradient, the launch that
    return;                                      // hosted it is gone)
  }
  using BG = BwdGeo<W>;
  using G = typename BG::G;
  constexpr int HW = G::HW, HP = G::HP, WP = G::WP, XCS = BG::XCS, DZS = BG::DZS;
  constexpr int KSA = HW / 16;                  // wgrad k-steps (16 positions) per sample
  constexpr int TPW = G::MT / 4;               // dgrad position tiles per wave
  constexpr int NDI = HW / 128;                // dz items (channel pair x 8 positions) per thread
  constexpr int NXI = CO * 16 / 256;           // x items (channel, image row) per thread
  constexpr int XQ = W / 8;                    // 16-byte vectors per image row
  constexpr bool PREF = HW <= 128;             // one-sample-ahead register prefetch (P128)
  static_assert(2 * KSA + KSA / 4 == 18 * TPW, "wgrad steps pair with dgrad k-steps");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __bf16* X = reinterpret_cast<__bf16*>(smem);       // [kw][ci][row][w]
  __bf16* DZ = X + BG::X_EL;                         // [co][p]
  __bf16* T = DZ + BG::DZ_EL;                        // [pixel][32] swizzled
  uint16_t* ZP = reinterpret_cast<uint16_t*>(T + BG::T_EL);   // [ci][p] raw z_prev
  bf16x8* WB = reinterpret_cast<bf16x8*>(ZP + BG::ZP_EL);
  float* prm = reinterpret_cast<float*>(WB + BG::KSD * 64);   // this layer's records (dz)
  float* prp = prm + CO * NST;                               // previous layer's records (x, reduction)
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int hh = lane >> 5, l32 = lane & 31;
  const int bx = blockIdx.x, e = blockIdx.y, u = bx / chunks, chunk = bx % chunks;
  const int EC = E * CO;
  const int n0 = u * B + chunk * spb, nend = min((u + 1) * B, n0 + spb);

  // ---- zero the tile (its halo stays zero) and the halo rows of the shifted copies ----
  for (int i = tid; i < BG::T_EL / 8; i += 256) reinterpret_cast<bf16x8*>(T)[i] = bf16x8{};
  for (int i = tid; i < 3 * CO * 2 * XQ; i += 256) {
    const int cc = i / (2 * XQ), r = (i / XQ) & 1, q = i % XQ;
    *reinterpret_cast<bf16x8*>(X + cc * XCS + r * (HP - 1) * W + 8 * q) = bf16x8{};
  }

  uint4 rd[NDI][2], rz[NDI][2], rx[NXI][XQ];
  auto load = [&](int n) {
    const size_t sb = ((size_t)n * E + e) * CO * HW;
#pragma unroll
    for (int j = 0; j < NDI; ++j) {
      const int i = tid + 256 * j, pr = i & 15, sg = i >> 4;
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const size_t off = sb + (size_t)(2 * pr + h2) * HW + 8 * sg;
        rd[j][h2] = *reinterpret_cast<const uint4*>(dh + off);
        rz[j][h2] = *reinterpret_cast<const uint4*>(z + off);
      }
    }
#pragma unroll
    for (int j = 0; j < NXI; ++j) {
      const int i = tid + 256 * j, c = i >> 4, ph = i & 15;
      const uint4* src = reinterpret_cast<const uint4*>(zprev + sb + (size_t)c * HW + ph * W);
#pragma unroll
      for (int q = 0; q < XQ; ++q) rx[j][q] = src[q];
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int j = 0; j < NDI; ++j) {
      const int i = tid + 256 * j, pr = i & 15, p0 = (i >> 4) * 8;
      float v[2][8];
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int c = 2 * pr + h2;
        const float* sc = prm + c * NST;
        const float a = sc[ST_A], b = sc[ST_B], mu = sc[ST_MEAN], inv = sc[ST_INV];
        const float c1 = sc[ST_C1], c2 = sc[ST_C2], c3 = sc[ST_C3];
        float d[8], zz[8];
        unpack_q(rd[j][h2], d, (const uint16_t*)nullptr);
        unpack_q(rz[j][h2], zz, (const uint16_t*)nullptr);
        uint32_t w4[4];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float g = bn_gate(a, zz[k], b) ? d[k] : 0.f;
          v[h2][k] = bn_dz(g, bn_xhat(zz[k], mu, inv), c1, c2, c3);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
          w4[k] = f32_to_bf16(v[h2][2 * k]) | ((uint32_t)f32_to_bf16(v[h2][2 * k + 1]) << 16);
        *reinterpret_cast<uint4*>(DZ + c * DZS + p0) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
      }
      const int ph = p0 / W, pw = p0 % W;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t w2 = f32_to_bf16(v[0][k]) | ((uint32_t)f32_to_bf16(v[1][k]) << 16);
        const int R = ph + 1, C = pw + k + 1;
        *reinterpret_cast<uint32_t*>(T + (R * WP + C) * CO + 8 * ((pr >> 2) ^ tile_swz(R, C)) + 2 * (pr & 3)) = w2;
      }
    }
#pragma unroll
    for (int j = 0; j < NXI; ++j) {
      const int i = tid + 256 * j, c = i >> 4, ph = i & 15;
      float v[W + 2];
      v[0] = 0.f;
      v[W + 1] = 0.f;
#pragma unroll
      for (int q = 0; q < XQ; ++q) {
        unpack_q(rx[j][q], v + 1 + 8 * q, (const uint16_t*)nullptr);
        uint2* zp = reinterpret_cast<uint2*>(ZP + c * BG::ZPS + ph * W + 8 * q);   // (8-byte aligned rows)
        zp[0] = make_uint2(rx[j][q].x, rx[j][q].y);
        zp[1] = make_uint2(rx[j][q].z, rx[j][q].w);
      }
      const float xa = prp[c * NST + ST_A], xb = prp[c * NST + ST_B];
#pragma unroll
      for (int q = 1; q <= W; ++q) v[q] = relu_nan(xa * v[q] + xb);
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        __bf16* dst = X + (kw * CO + c) * XCS + (ph + 1) * W;
#pragma unroll
        for (int q = 0; q < W; q += 8) {
          bf16x8 o;
#pragma unroll
          for (int k = 0; k < 8; ++k) o[k] = (__bf16)v[q + k + kw];   // column w holds x[w + kw - 1]
          *reinterpret_cast<bf16x8*>(dst + q) = o;
        }
      }
    }
  };

  // ---- prologue: first sample's loads, dgrad B fragments, both layers' BN records ----
  if (PREF && n0 < nend) load(n0);
  {
    constexpr int NW = BG::KSD * 64, WPT = (NW + 255) / 256;
    const bf16x8* wp = reinterpret_cast<const bf16x8*>(wt) + (size_t)e * NW;
    bf16x8 tw[WPT];
#pragma unroll
    for (int k = 0; k < WPT; ++k)
      if (tid + 256 * k < NW) tw[k] = wp[tid + 256 * k];
    const float pv = st_prev[((size_t)u * EC + e * CO) * NST + tid];   // 32 channels x NST = one per thread
    float cv = 0.f;
    if (bnb.rslab) bn_bwd_build(bnb, st, prm, u, e, EC);
    else cv = st[((size_t)u * EC + e * CO) * NST + tid];
#pragma unroll
    for (int k = 0; k < WPT; ++k)
      if (tid + 256 * k < NW) WB[tid + 256 * k] = tw[k];
    prp[tid] = pv;
    if (!bnb.rslab) prm[tid] = cv;
  }
  __syncthreads();
  const float rmu = prp[l32 * NST + ST_MEAN], rinv = prp[l32 * NST + ST_INV];
  const float ra = prp[l32 * NST + ST_A], rb = prp[l32 * NST + ST_B];
  bf16x8 wreg[BG::KSD];   // the dgrad B fragments stay in registers (each wave reads them once)
#pragma unroll
  for (int k = 0; k < BG::KSD; ++k) wreg[k] = WB[k * 64 + lane];

  f32x16 accw[3];   // taps wv, wv + 4, and this wave's share of tap 8
#pragma unroll
  for (int t = 0; t < 3; ++t) accw[t] = f32x16{};
  float s1 = 0.f, s2 = 0.f;
  for (int n = n0; n < nend; ++n) {
    __syncthreads();   // the previous sample's MFMAs are done reading X / DZ / T
    if (!PREF) load(n);
    store();
    if (PREF && n + 1 < nend) load(n + 1);
    __syncthreads();
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) {
      const int mt = wv + 4 * tt;
      // the previous layer's z at this lane's dx positions (for the reduction)
      uint2 zq[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) zq[g] = *reinterpret_cast<const uint2*>(ZP + l32 * BG::ZPS + mt * 32 + 8 * g + 4 * hh);
      const int p = mt * 32 + l32, ph = p / W, pw = p % W;
      f32x16 acc = f32x16{};
#pragma unroll
      for (int s = 0; s < BG::KSD; ++s) {
        const int tap = s >> 1, q = ((s & 1) << 1) + hh;
        const int R = ph + tap / 3, C = pw + tap % 3;
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(T + (R * WP + C) * CO + 8 * (q ^ tile_swz(R, C)));
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, wreg[s], acc, 0, 0, 0);
        // wgrad step ws: taps wv / wv + 4 at k-step ws / 2, then tap 8 at this wave's k-steps
        const int ws = tt * BG::KSD + s;
        const int j = ws < 2 * KSA ? (ws & 1) : 2;
        const int wt = j == 0 ? wv : (j == 1 ? wv + 4 : 8);
        const int ks = ws < 2 * KSA ? (ws >> 1) : wv * (KSA / 4) + ws - 2 * KSA;
        const int p0 = ks * 16 + 8 * hh, xh = p0 / W, xw = p0 % W;
        const bf16x8 bz = *reinterpret_cast<const bf16x8*>(DZ + l32 * DZS + p0);
        const bf16x8 ax =
            *reinterpret_cast<const bf16x8*>(X + ((wt % 3) * CO + l32) * XCS + (xh + wt / 3) * W + xw);
        accw[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ax, bz, accw[j], 0, 0, 0);
      }
      // ---- dgrad epilogue: lane holds input channel l32, positions mt*32 + 8g + 4hh + {0..3} ----
      const size_t rbase = ((size_t)n * E + e) * CO * HW + (size_t)l32 * HW + mt * 32;
      uint32_t pk[4][2];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        pk[g][0] = pack_bf16x2(f32x2{acc[4 * g], acc[4 * g + 1]});
        pk[g][1] = pack_bf16x2(f32x2{acc[4 * g + 2], acc[4 * g + 3]});
        const f32x2 d01 = unpack_bf16x2(pk[g][0]), d23 = unpack_bf16x2(pk[g][1]);
        const float d[4] = {d01.x, d01.y, d23.x, d23.y};
        const float zz[4] = {__uint_as_float(zq[g].x << 16), __uint_as_float(zq[g].x & 0xffff0000u),
                             __uint_as_float(zq[g].y << 16), __uint_as_float(zq[g].y & 0xffff0000u)};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float gg = bn_gate(ra, zz[k], rb) ? d[k] : 0.f;
          bn_red(s1, s2, gg, bn_xhat(zz[k], rmu, rinv));
        }
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {   // pair (g = 2q, 2q + 1): half-wave hh stores g = 2q + hh (conv3x3_body's swap)
#pragma unroll
        for (int w = 0; w < 2; ++w) {
          const auto r = __builtin_amdgcn_permlane32_swap(pk[2 * q][w], pk[2 * q + 1][w], false, false);
          pk[2 * q][w] = r[0];
          pk[2 * q + 1][w] = r[1];
        }
        *reinterpret_cast<uint4*>(dx + rbase + 8 * (2 * q + hh)) =
            make_uint4(pk[2 * q][0], pk[2 * q][1], pk[2 * q + 1][0], pk[2 * q + 1][1]);
      }
    }
  }

  // ---- the previous layer's BN backward partials: half-waves, then the 4 waves through LDS ----
  s1 += __shfl_xor(s1, 32);
  s2 += __shfl_xor(s2, 32);
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);
  if (hh == 0) {
    red[(wv * 32 + l32) * 2] = s1;
    red[(wv * 32 + l32) * 2 + 1] = s2;
  }
  __syncthreads();
  if (tid < 64) {
    const int c = tid >> 1, k = tid & 1;
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) t += red[(w * 32 + c) * 2 + k];
    part[(((size_t)u * chunks + chunk) * 2 + k) * EC + e * CO + c] = t;   // planar [2][EC] rows
  }
  // ---- weight gradient: [co][ci * 9 + tap] rows in LDS (taps wv, wv + 4 written by their owner;
  // tap 8 = the 4 waves' partials, summed in wave order), then one coalesced slab row ----
  constexpr int RS = 9 * CO + 1;
  __syncthreads();
  float* wr = reinterpret_cast<float*>(smem);
  float* p8 = wr + CO * RS;   // [wave][co][ci], rows padded to 33: the 32 lanes (co) on distinct banks
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int ci = (r & 3) + 8 * (r >> 2) + 4 * hh;   // accumulator row = ci, column = co = l32
    wr[l32 * RS + ci * 9 + wv] = accw[0][r];
    wr[l32 * RS + ci * 9 + wv + 4] = accw[1][r];
    p8[(wv * CO + l32) * (CO + 1) + ci] = accw[2][r];
  }
  __syncthreads();
  float* srow = slab + ((size_t)e * gridDim.x + bx) * CO * CO * 9;
  for (int i = tid; i < CO * CO * 9; i += 256) {
    const int co = i / (CO * 9), m = i % (CO * 9);
    float v;
    if (m % 9 == 8) {
      const int ci = m / 9;
      constexpr int P8 = CO + 1;
      v = ((p8[co * P8 + ci] + p8[(CO + co) * P8 + ci]) + p8[(2 * CO + co) * P8 + ci]) + p8[(3 * CO + co) * P8 + ci];
    } else {
      v = wr[co * RS + m];
    }
    srow[i] = v;
  }
}

// ------------------------------------------------------------------------------------------
// conv3x3_bwd_db_kernel (round 6): conv3x3_bwd_kernel (P128) software-pipelined over TWO stage buffers.  In
// conv3x3_bwd_kernel every sample is staged by the whole workgroup between two barriers, and only then do the 4
// waves run their 36 MFMAs; two workgroups per CU were meant to fill each other's gaps, but the kernel ran at
// ~2.4 TB/s of its ~75 MB (31 us per layer, profiles/r5_46_step_kernel_stats.md).  Here one workgroup per CU
// (136 KB of LDS) holds two buffers: while the MFMAs of sample n read buffer n & 1, every thread stages sample n + 1
// into the other one in six pieces placed between the k-steps' MFMA pairs (the dz item's two 4-position halves, the
// two x items' raw copy + transform and their shifted copies), and then issues sample n + 3's loads (two register
// sets: each sample's loads get two sample periods to land).  One barrier per sample instead of two.  The
// arithmetic and every summation order are conv3x3_bwd_kernel's: dx, the slab row and the BN partials are
// bit-identical to it at the same chunking.
// ------------------------------------------------------------------------------------------
template <int W>
struct BwdDbGeo {
  using BG = BwdGeo<W>;
  static constexpr int STG = BG::X_EL + BG::DZ_EL + BG::T_EL + BG::ZP_EL;   // 16-bit elements per stage buffer
  static constexpr size_t SMEM_STAGE = 2 * (size_t)STG * 2 + BG::KSD * 64 * 16 + 2 * CO * NST * 4;
  static constexpr size_t SMEM = SMEM_STAGE > BG::RED ? SMEM_STAGE : BG::RED;
};

template <int W>
__global__ void __launch_bounds__(256, 1) conv3x3_bwd_db_kernel(const uint16_t* __restrict__ zprev,
                                                             const float* __restrict__ st_prev,
                                                             const uint16_t* __restrict__ dh,
                                                             const uint16_t* __restrict__ z,
                                                             const float* __restrict__ st, float* __restrict__ slab,
                                                             const uint16_t* __restrict__ wt,
                                                             uint16_t* __restrict__ dx, float* __restrict__ part, int E,
                                                             int B, int chunks, int spb, BnBwd bnb, LossFinish lf) {
  if ((int)blockIdx.y == E) {   // (as conv3x3_bwd_kernel: the extra row hosts the HDCE loss finish)
    if (blockIdx.x == 0) loss_finish_body(lf);
    return;
  }
  using BG = BwdGeo<W>;
  using DB = BwdDbGeo<W>;
  using G = typename BG::G;
  constexpr int HW = G::HW, HP = G::HP, WP = G::WP, XCS = BG::XCS, DZS = BG::DZS;
  constexpr int KSA = HW / 16;                  // wgrad k-steps (16 positions) per sample
  static_assert(W == 8 && G::MT == 4, "P128: one dgrad position tile per wave, one dz item / two x items per thread");
  static_assert(2 * KSA + KSA / 4 == 18, "wgrad steps pair with dgrad k-steps");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  auto X_of = [&](int b) { return reinterpret_cast<__bf16*>(smem) + b * DB::STG; };        // [kw][ci][row][w]
  auto DZ_of = [&](int b) { return X_of(b) + BG::X_EL; };                                  // [co][p]
  auto T_of = [&](int b) { return DZ_of(b) + BG::DZ_EL; };                                 // [pixel][32] swizzled
  auto ZP_of = [&](int b) { return reinterpret_cast<uint16_t*>(T_of(b) + BG::T_EL); };     // [ci][p] raw z_prev
  bf16x8* WB = reinterpret_cast<bf16x8*>(reinterpret_cast<__bf16*>(smem) + 2 * DB::STG);
  float* prm = reinterpret_cast<float*>(WB + BG::KSD * 64);   // this layer's records (dz)
  float* prp = prm + CO * NST;                               // previous layer's records (x, reduction)
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int hh = lane >> 5, l32 = lane & 31;
  const int bx = blockIdx.x, e = blockIdx.y, u = bx / chunks, chunk = bx % chunks;
  const int EC = E * CO;
  const int n0 = u * B + chunk * spb, nend = min((u + 1) * B, n0 + spb), nlast = nend - 1;

  // ---- zero both buffers' tiles (halos stay zero) and the halo rows of their shifted copies ----
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    for (int i = tid; i < BG::T_EL / 8; i += 256) reinterpret_cast<bf16x8*>(T_of(b))[i] = bf16x8{};
    for (int i = tid; i < 3 * CO * 2; i += 256) {
      const int cc = i >> 1, r = i & 1;
      *reinterpret_cast<bf16x8*>(X_of(b) + cc * XCS + r * (HP - 1) * W) = bf16x8{};
    }
  }
  // this thread's staging items: dz (channels 2 pr, 2 pr + 1; positions [p0, p0 + 8)), x rows (channel cx[j], row
  // phx[j])
  const int pr = tid & 15, p0 = (tid >> 4) * 8;
  int cx[2], phx[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int i = tid + 256 * j;
    cx[j] = i >> 4;
    phx[j] = i & 15;
  }
  struct Set {
    uint4 rd[2], rz[2], rx[2];
  };
  Set sa, sb;
  auto load = [&](Set& r, int n) {
    const size_t sbase = ((size_t)n * E + e) * CO * HW;
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      const size_t off = sbase + (size_t)(2 * pr + h2) * HW + p0;
      r.rd[h2] = *reinterpret_cast<const uint4*>(dh + off);
      r.rz[h2] = *reinterpret_cast<const uint4*>(z + off);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) r.rx[j] = *reinterpret_cast<const uint4*>(zprev + sbase + (size_t)cx[j] * HW + phx[j] * W);
  };
  // piece 0 / 1: dz of positions [p0 + 4 q, + 4), both channels -> DZ (two 8-byte rows) and T (4 words)
  auto piece_dz = [&](const Set& r, int b, int q) {
    __bf16* DZ = DZ_of(b);
    __bf16* T = T_of(b);
    float v[2][4];
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      const int c = 2 * pr + h2;
      const float* sc = prm + c * NST;
      const float a = sc[ST_A], bb = sc[ST_B], mu = sc[ST_MEAN], inv = sc[ST_INV];
      const float c1 = sc[ST_C1], c2 = sc[ST_C2], c3 = sc[ST_C3];
      const uint32_t dw[2] = {(&r.rd[h2].x)[2 * q], (&r.rd[h2].x)[2 * q + 1]};
      const uint32_t zw[2] = {(&r.rz[h2].x)[2 * q], (&r.rz[h2].x)[2 * q + 1]};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t dk = dw[k >> 1], zk = zw[k >> 1];
        const float d = __uint_as_float((k & 1) ? (dk & 0xffff0000u) : (dk << 16));
        const float zz = __uint_as_float((k & 1) ? (zk & 0xffff0000u) : (zk << 16));
        const float g = bn_gate(a, zz, bb) ? d : 0.f;
        v[h2][k] = bn_dz(g, bn_xhat(zz, mu, inv), c1, c2, c3);
      }
      const uint32_t w0 = f32_to_bf16(v[h2][0]) | ((uint32_t)f32_to_bf16(v[h2][1]) << 16);
      const uint32_t w1 = f32_to_bf16(v[h2][2]) | ((uint32_t)f32_to_bf16(v[h2][3]) << 16);
      *reinterpret_cast<uint2*>(DZ + c * DZS + p0 + 4 * q) = make_uint2(w0, w1);
    }
    const int ph = p0 / W, pw = p0 % W;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t w2 = f32_to_bf16(v[0][k]) | ((uint32_t)f32_to_bf16(v[1][k]) << 16);
      const int R = ph + 1, C = pw + 4 * q + k + 1;
      *reinterpret_cast<uint32_t*>(T + (R * WP + C) * CO + 8 * ((pr >> 2) ^ tile_swz(R, C)) + 2 * (pr & 3)) = w2;
    }
  };
  // piece 2 + j: x item j -- the raw z_prev row (for the reduction) and BN + ReLU into the 3 column-shifted copies
  auto piece_x = [&](const Set& r, int b, int j) {
    __bf16* X = X_of(b);
    uint16_t* ZP = ZP_of(b);
    const int c = cx[j], ph = phx[j];
    float v[W + 2];
    v[0] = 0.f;
    v[W + 1] = 0.f;
    unpack_q(r.rx[j], v + 1, (const uint16_t*)nullptr);
    uint2* zp = reinterpret_cast<uint2*>(ZP + c * BG::ZPS + ph * W);
    zp[0] = make_uint2(r.rx[j].x, r.rx[j].y);
    zp[1] = make_uint2(r.rx[j].z, r.rx[j].w);
    const float xa = prp[c * NST + ST_A], xb = prp[c * NST + ST_B];
#pragma unroll
    for (int q = 1; q <= W; ++q) v[q] = relu_nan(xa * v[q] + xb);
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      bf16x8 o;
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = (__bf16)v[k + kw];   // column w holds x[w + kw - 1]
      *reinterpret_cast<bf16x8*>(X + (kw * CO + c) * XCS + (ph + 1) * W) = o;
    }
  };

  // ---- prologue: the first two samples' loads, the dgrad B fragments, both layers' BN records ----
  if (n0 < nend) {
    load(sa, n0);
    load(sb, n0 + 1 <= nlast ? n0 + 1 : nlast);
  }
  {
    constexpr int NW = BG::KSD * 64, WPT = (NW + 255) / 256;
    const bf16x8* wp = reinterpret_cast<const bf16x8*>(wt) + (size_t)e * NW;
    bf16x8 tw[WPT];
#pragma unroll
    for (int k = 0; k < WPT; ++k)
      if (tid + 256 * k < NW) tw[k] = wp[tid + 256 * k];
    const float pv = st_prev[((size_t)u * EC + e * CO) * NST + tid];   // 32 channels x NST = one per thread
    float cv = 0.f;
    if (bnb.rslab) bn_bwd_build(bnb, st, prm, u, e, EC);
    else cv = st[((size_t)u * EC + e * CO) * NST + tid];
#pragma unroll
    for (int k = 0; k < WPT; ++k)
      if (tid + 256 * k < NW) WB[tid + 256 * k] = tw[k];
    prp[tid] = pv;
    if (!bnb.rslab) prm[tid] = cv;
  }
  __syncthreads();
  const float rmu = prp[l32 * NST + ST_MEAN], rinv = prp[l32 * NST + ST_INV];
  const float ra = prp[l32 * NST + ST_A], rb = prp[l32 * NST + ST_B];
  bf16x8 wreg[BG::KSD];   // the dgrad B fragments stay in registers (each wave reads them once)
#pragma unroll
  for (int k = 0; k < BG::KSD; ++k) wreg[k] = WB[k * 64 + lane];
  if (n0 < nend) {   // the first sample staged up front (exposed), then set a takes sample n0 + 2
    piece_dz(sa, 0, 0);
    piece_dz(sa, 0, 1);
    piece_x(sa, 0, 0);
    piece_x(sa, 0, 1);
    load(sa, n0 + 2 <= nlast ? n0 + 2 : nlast);
  }

  f32x16 accw[3];   // taps wv, wv + 4, and this wave's share of tap 8
#pragma unroll
  for (int t = 0; t < 3; ++t) accw[t] = f32x16{};
  float s1 = 0.f, s2 = 0.f;
  const int mt = wv;                             // this wave's dgrad position tile
  auto sample = [&](int n, int cb, Set& nx) {
    __syncthreads();   // buffer cb staged by every thread; everyone is done reading buffer cb ^ 1 (sample n - 1)
    const __bf16* X = X_of(cb);
    const __bf16* DZ = DZ_of(cb);
    const __bf16* T = T_of(cb);
    const uint16_t* ZP = ZP_of(cb);
    uint2 zq[4];   // the previous layer's z at this lane's dx positions (for the reduction)
#pragma unroll
    for (int g = 0; g < 4; ++g) zq[g] = *reinterpret_cast<const uint2*>(ZP + l32 * BG::ZPS + mt * 32 + 8 * g + 4 * hh);
    const int p = mt * 32 + l32, ph = p / W, pw = p % W;
    f32x16 acc = f32x16{};
#pragma unroll
    for (int s = 0; s < BG::KSD; ++s) {
      const int tap = s >> 1, q = ((s & 1) << 1) + hh;
      const int R = ph + tap / 3, C = pw + tap % 3;
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(T + (R * WP + C) * CO + 8 * (q ^ tile_swz(R, C)));
      const int ws = s;   // (one dgrad tile per wave: the wgrad step index is the k-step's)
      const int j = ws < 2 * KSA ? (ws & 1) : 2;
      const int wtp = j == 0 ? wv : (j == 1 ? wv + 4 : 8);
      const int ks = ws < 2 * KSA ? (ws >> 1) : wv * (KSA / 4) + ws - 2 * KSA;
      const int q0 = ks * 16 + 8 * hh, xh = q0 / W, xw = q0 % W;
      const bf16x8 bz = *reinterpret_cast<const bf16x8*>(DZ + l32 * DZS + q0);
      const bf16x8 ax = *reinterpret_cast<const bf16x8*>(X + ((wtp % 3) * CO + l32) * XCS + (xh + wtp / 3) * W + xw);
      __builtin_amdgcn_sched_barrier(0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, wreg[s], acc, 0, 0, 0);
      accw[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ax, bz, accw[j], 0, 0, 0);
      // the next sample's staging in this k-step's MFMA shadow (writes the other buffer), then its registers reload
      if (s == 0) piece_dz(nx, cb ^ 1, 0);
      if (s == 3) piece_dz(nx, cb ^ 1, 1);
      if (s == 6) piece_x(nx, cb ^ 1, 0);
      if (s == 9) piece_x(nx, cb ^ 1, 1);
      if (s == 12) load(nx, n + 3 <= nlast ? n + 3 : nlast);
      __builtin_amdgcn_sched_barrier(0);
    }
    // ---- dgrad epilogue (conv3x3_bwd_kernel's): lane holds input channel l32, positions mt*32 + 8g + 4hh + {0..3}
    const size_t rbase = ((size_t)n * E + e) * CO * HW + (size_t)l32 * HW + mt * 32;
    uint32_t pk[4][2];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      pk[g][0] = pack_bf16x2(f32x2{acc[4 * g], acc[4 * g + 1]});
      pk[g][1] = pack_bf16x2(f32x2{acc[4 * g + 2], acc[4 * g + 3]});
      const f32x2 d01 = unpack_bf16x2(pk[g][0]), d23 = unpack_bf16x2(pk[g][1]);
      const float d[4] = {d01.x, d01.y, d23.x, d23.y};
      const float zz[4] = {__uint_as_float(zq[g].x << 16), __uint_as_float(zq[g].x & 0xffff0000u),
                           __uint_as_float(zq[g].y << 16), __uint_as_float(zq[g].y & 0xffff0000u)};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float gg = bn_gate(ra, zz[k], rb) ? d[k] : 0.f;
        bn_red(s1, s2, gg, bn_xhat(zz[k], rmu, rinv));
      }
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
#pragma unroll
      for (int w = 0; w < 2; ++w) {
        const auto r = __builtin_amdgcn_permlane32_swap(pk[2 * q][w], pk[2 * q + 1][w], false, false);
        pk[2 * q][w] = r[0];
        pk[2 * q + 1][w] = r[1];
      }
      *reinterpret_cast<uint4*>(dx + rbase + 8 * (2 * q + hh)) =
          make_uint4(pk[2 * q][0], pk[2 * q][1], pk[2 * q + 1][0], pk[2 * q + 1][1]);
    }
  };
  for (int n = n0; n < nend; n += 2) {          // (by two: the register sets are named statically)
    sample(n, 0, sb);                           // stages n + 1 from b, b takes n + 3
    if (n + 1 < nend) sample(n + 1, 1, sa);     // stages n + 2 from a, a takes n + 4
  }

  // ---- the previous layer's BN backward partials: half-waves, then the 4 waves through LDS ----
  s1 += __shfl_xor(s1, 32);
  s2 += __shfl_xor(s2, 32);
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);
  if (hh == 0) {
    red[(wv * 32 + l32) * 2] = s1;
    red[(wv * 32 + l32) * 2 + 1] = s2;
  }
  __syncthreads();
  if (tid < 64) {
    const int c = tid >> 1, k = tid & 1;
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) t += red[(w * 32 + c) * 2 + k];
    part[(((size_t)u * chunks + chunk) * 2 + k) * EC + e * CO + c] = t;   // planar [2][EC] rows
  }
  // ---- weight gradient rows (conv3x3_bwd_kernel's) ----
  constexpr int RS = 9 * CO + 1;
  __syncthreads();
  float* wr = reinterpret_cast<float*>(smem);
  float* p8 = wr + CO * RS;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int ci = (r & 3) + 8 * (r >> 2) + 4 * hh;
    wr[l32 * RS + ci * 9 + wv] = accw[0][r];
    wr[l32 * RS + ci * 9 + wv + 4] = accw[1][r];
    p8[(wv * CO + l32) * (CO + 1) + ci] = accw[2][r];
  }
  __syncthreads();
  float* srow = slab + ((size_t)e * gridDim.x + bx) * CO * CO * 9;
  for (int i = tid; i < CO * CO * 9; i += 256) {
    const int co = i / (CO * 9), m = i % (CO * 9);
    float v;
    if (m % 9 == 8) {
      const int ci = m / 9;
      constexpr int P8 = CO + 1;
      v = ((p8[co * P8 + ci] + p8[(CO + co) * P8 + ci]) + p8[(2 * CO + co) * P8 + ci]) + p8[(3 * CO + co) * P8 + ci];
    } else {
      v = wr[co * RS + m];
    }
    srow[i] = v;
  }
}

// ------------------------------------------------------------------------------------------
// BatchNorm pieces
// ------------------------------------------------------------------------------------------
// Forward statistics: per (u, ch) mean/invstd/(a,b); running stats updated in u order.
// One 64-lane block per channel: lanes sum the chunk partials, lane 0 finishes.
constexpr int kMaxGroups = 8;   // statistics groups (users) per finalisation launch
// up to 3 BN layers per launch (blockIdx.y): the step's one BN tail launch advances every layer's
// running statistics (layers 1/2 had their records built by their consumers) and publishes the last
// layer's records
struct FinJobs {
  const float* stats[3];
  const float* gamma[3];
  const float* beta[3];
  float* run_mean[3];
  float* run_var[3];
  float* st[3];
};
// one (layer l, channel ch) per wave; st[l] null: running statistics only (no records)
__device__ __forceinline__ void bn_fin_body(const FinJobs& jobs, int ch, int l, int lane, int U, int chunks, int EC,
                                            float count, float momentum, float eps, int training,
                                            long long* __restrict__ nbt, int n_nbt, long long nbt_inc) {
  // every global load is issued up front (the per-group loop paid one round trip per group)
  const float* __restrict__ stats = jobs.stats[l];
  const float* __restrict__ gamma = jobs.gamma[l];
  const float* __restrict__ beta = jobs.beta[l];
  float* __restrict__ run_mean = jobs.run_mean[l];
  float* __restrict__ run_var = jobs.run_var[l];
  float* __restrict__ st = jobs.st[l];
  if (nbt && ch == 0 && l == 0 && lane < n_nbt) nbt[lane] += nbt_inc;   // BatchNorm num_batches_tracked
  const float g = gamma[ch], bt = beta[ch];
  float rm = run_mean[ch], rv = run_var[ch];
  float a[kMaxGroups], b[kMaxGroups];
#pragma unroll
  for (int u = 0; u < kMaxGroups; ++u) {
    a[u] = 0.f;
    b[u] = 0.f;
    if (training && u < U) {
      for (int k = lane; k < chunks; k += 64) {
        a[u] += stats[((size_t)u * chunks + k) * 2 * EC + ch];
        b[u] += stats[((size_t)u * chunks + k) * 2 * EC + EC + ch];
      }
    }
  }
#pragma unroll
  for (int u = 0; u < kMaxGroups; ++u) {
    if (training && u < U) {
      a[u] = wave_sum(a[u]);
      b[u] = wave_sum(b[u]);
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int u = 0; u < kMaxGroups; ++u) {
      if (u >= U) break;
      float mean, var;
      if (training) {
        mean = a[u] / count;
        var = fmaxf(b[u] / count - mean * mean, 0.f);
        rm = (1.f - momentum) * rm + momentum * mean;
        rv = (1.f - momentum) * rv + momentum * var * count / (count - 1.f);
      } else {
        mean = rm;
        var = rv;
      }
      const float inv = rsqrtf(var + eps);
      if (st) {
        float4* r = reinterpret_cast<float4*>(st + ((size_t)u * EC + ch) * NST);
        r[0] = make_float4(mean, inv, g * inv, bt - mean * g * inv);   // ST_MEAN, ST_INV, ST_A, ST_B
      }
    }
    if (training) {
      run_mean[ch] = rm;
      run_var[ch] = rv;
    }
  }
}

__global__ void __launch_bounds__(64) bn_stats_finalize_kernel(FinJobs jobs, int U, int chunks, int EC, float count,
                                                               float momentum, float eps, int training,
                                                               long long* __restrict__ nbt, int n_nbt,
                                                               long long nbt_inc) {
  bn_fin_body(jobs, blockIdx.x, blockIdx.y, threadIdx.x, U, chunks, EC, count, momentum, eps, training, nbt, n_nbt,
              nbt_inc);
}

// Backward reductions: per (u, chunk, ch): sum g, sum g*xhat.  grid (U*chunks, E), block 256.
// 16-lane groups each own one (sample, channel) row of HW values (8 per lane per pass); a
// group's rows alternate between channels g and g+16, so every lane keeps 2 x 2 partials.
template <int HW, typename TDH, int UNR = (HW == 128 ? 4 : 2)>
__global__ void __launch_bounds__(256) bn_bwd_reduce_kernel(const TDH* __restrict__ dh, const uint16_t* __restrict__ z,
                                                            const float* __restrict__ st, float* __restrict__ slab,
                                                            int E, int B, int chunks, int spb, LossFinish lf) {
  if ((int)blockIdx.y == E) {   // the extra row (lf.part set): block 0 hosts the HDCE loss finish
    if (blockIdx.x == 0) loss_finish_body(lf);
    return;
  }
  const int tid = threadIdx.x, grp = tid >> 4, gl = tid & 15;
  const int u = blockIdx.x / chunks, chunk = blockIdx.x % chunks, e = blockIdx.y;
  const int EC = E * CO;
  const int n0 = u * B + chunk * spb, nend = min((u + 1) * B, n0 + spb);
  const int rows = (nend - n0) * CO;
  float sg0 = 0.f, sgx0 = 0.f, sg1 = 0.f, sgx1 = 0.f;  // channels grp and grp+16
  // rows in rounds of UNR with every load of a round issued before its math (one row per round trip kept the
  // kernel latency-bound); the per-row sums and their order into sg / sgx are the one-row loop's
  constexpr int QN = HW / 128;   // 8-value passes per lane per row
  const int nit = (rows + 15) / 16;
  for (int it0 = 0; it0 < nit; it0 += UNR) {
    float d[UNR][QN][8], zz[UNR][QN][8], a[UNR], b[UNR], mu[UNR], inv[UNR];
    bool ok[UNR];
#pragma unroll
    for (int k = 0; k < UNR; ++k) {
      // (branch-free: a row past the end loads row grp -- rows >= CO > grp -- and is not added; guarded loads
      // compiled to one round trip per row)
      const int rr = (it0 + k) * 16 + grp;
      ok[k] = it0 + k < nit && rr < rows;
      const int r = ok[k] ? rr : grp;
      const int n = n0 + r / CO, c = r % CO, ch = e * CO + c;
      const float* sc = st + ((size_t)u * EC + ch) * NST;
      a[k] = sc[ST_A];
      b[k] = sc[ST_B];
      mu[k] = sc[ST_MEAN];
      inv[k] = sc[ST_INV];
      const size_t rb = ((size_t)n * EC + ch) * HW;
#pragma unroll
      for (int qi = 0; qi < QN; ++qi) {
        load8(dh + rb + gl * 8 + 128 * qi, d[k][qi]);
        load8(z + rb + gl * 8 + 128 * qi, zz[k][qi]);
      }
    }
#pragma unroll
    for (int k = 0; k < UNR; ++k) {
      // (the row sums unconditionally -- a row past the end sums its stand-in and is dropped below: a guarded
      // body let the compiler sink each row's loads into it, one round trip per row again)
      float tg = 0.f, tgx = 0.f;
#pragma unroll
      for (int qi = 0; qi < QN; ++qi)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float g = bn_gate(a[k], zz[k][qi][j], b[k]) ? d[k][qi][j] : 0.f;
          bn_red(tg, tgx, g, bn_xhat(zz[k][qi][j], mu[k], inv[k]));
        }
      if (!ok[k]) continue;
      if ((it0 + k) & 1) {
        sg1 += tg;
        sgx1 += tgx;
      } else {
        sg0 += tg;
        sgx0 += tgx;
      }
    }
  }
#pragma unroll
  for (int m = 8; m >= 1; m >>= 1) {
    sg0 += __shfl_xor(sg0, m);
    sgx0 += __shfl_xor(sgx0, m);
    sg1 += __shfl_xor(sg1, m);
    sgx1 += __shfl_xor(sgx1, m);
  }
  if (gl == 0) {
    float* o = slab + ((size_t)u * chunks + chunk) * 2 * EC + e * CO + grp;   // planar [2][EC] rows
    o[0] = sg0;
    o[EC] = sgx0;
    o[16] = sg1;   // channel grp + 16
    o[EC + 16] = sgx1;
  }
}

// c1 = gamma*invstd, c2 = c1*Sg/M, c3 = c1*Sgx/M per (u, ch); dgamma += sum_u Sgx, dbeta += sum_u Sg.
__global__ void __launch_bounds__(64) bn_bwd_finalize_kernel(const float* __restrict__ slab,
                                                             const float* __restrict__ gamma, float* __restrict__ st,
                                                             float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                             int U, int chunks, int EC, float count, int accumulate) {
  const int ch = blockIdx.x, lane = threadIdx.x;
  const float gm = gamma[ch];
  const float od = accumulate ? dgamma[ch] : 0.f, ob = accumulate ? dbeta[ch] : 0.f;
  float sg[kMaxGroups], sgx[kMaxGroups], inv[kMaxGroups];
#pragma unroll
  for (int u = 0; u < kMaxGroups; ++u) {
    sg[u] = 0.f;
    sgx[u] = 0.f;
    inv[u] = 0.f;
    if (u < U) {
      inv[u] = st[((size_t)u * EC + ch) * NST + ST_INV];
      for (int k = lane; k < chunks; k += 64) {
        sg[u] += slab[((size_t)u * chunks + k) * 2 * EC + ch];
        sgx[u] += slab[((size_t)u * chunks + k) * 2 * EC + EC + ch];
      }
    }
  }
  float tg = 0.f, tgx = 0.f;
#pragma unroll
  for (int u = 0; u < kMaxGroups; ++u) {
    if (u < U) {
      sg[u] = wave_sum(sg[u]);
      sgx[u] = wave_sum(sgx[u]);
      tg += sg[u];
      tgx += sgx[u];
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int u = 0; u < kMaxGroups; ++u) {
      if (u >= U) break;
      const float c1 = gm * inv[u];
      float* r = st + ((size_t)u * EC + ch) * NST;
      r[ST_C1] = c1;
      r[ST_C2] = c1 * sg[u] / count;
      r[ST_C3] = c1 * sgx[u] / count;
    }
    dgamma[ch] = od + tgx;
    dbeta[ch] = ob + tg;
  }
}

// h = relu(a z + b) -> bf16 (the FC operand), 8 elements per thread.
template <int HW>
// FP8 (fp8 estimator): additionally h8 = e4m3(h * qs[0]) for the fp8 FC GEMM, and amax[0] tracks
// max(h) for the next step's delayed scale (h >= 0 after the ReLU).
__global__ void __launch_bounds__(256) bn_relu_apply_kernel(const uint16_t* __restrict__ z, const float* __restrict__ st,
                                                            uint16_t* __restrict__ h, long n8, int EC, int B,
                                                            uint8_t* __restrict__ h8, const float* __restrict__ qs,
                                                            float* __restrict__ amax) {
  const float q = h8 ? qs[0] : 0.f;
  float mx = 0.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    const long e0 = i * 8;
    const long row = e0 / HW;             // (n, ch)
    const int ch = (int)(row % EC);
    const int n = (int)(row / EC);
    const float* sc = st + ((size_t)(n / B) * EC + ch) * NST;
    const float a = sc[ST_A], b = sc[ST_B];
    float v[8];
    load8(z + e0, v);
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = relu_nan(a * v[j] + b);
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = f32_to_bf16(v[2 * j]) | ((uint32_t)f32_to_bf16(v[2 * j + 1]) << 16);
    *reinterpret_cast<uint4*>(h + e0) = make_uint4(w[0], w[1], w[2], w[3]);
    if (h8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) mx = fmaxf(mx, v[j]);
      const uint32_t p0 = e4m3_pack4(v[0] * q, v[1] * q, v[2] * q, v[3] * q);
      const uint32_t p1 = e4m3_pack4(v[4] * q, v[5] * q, v[6] * q, v[7] * q);
      *reinterpret_cast<uint2*>(h8 + e0) = make_uint2(p0, p1);
    }
  }
  if (h8) amax_block_store(amax, mx);
}

// Layer-3 BN + ReLU apply with the BN tail folded in: one launch instead of two.
// Workgroups [0, U*ach*E), (u, chunk, e): build the (u, e) records from the conv's statistics partials
// (bn_fwd_build, as the conv kernels do for layers 1 / 2; chunk 0 publishes them for the backward), then
// h = relu(a z + b) for spb samples x 32 channels (32*HW contiguous bf16 per sample).  Workgroups
// beyond: every layer's running statistics (+ num_batches_tracked), one (layer, channel) per wave --
// jobs.st[2] is null there, the records of layer 3 come from the apply workgroups only.
template <int HW, int UNR>
__global__ void __launch_bounds__(256) bn_apply_tail_kernel(const uint16_t* __restrict__ z, uint16_t* __restrict__ h,
                                                            BnFwd bnf, FinJobs jobs, int U, int E, int B, int spb,
                                                            int ach, int chunks, int training,
                                                            long long* __restrict__ nbt, int n_nbt, long long nbt_inc,
                                                            uint8_t* __restrict__ h8, const float* __restrict__ qs,
                                                            float* __restrict__ amax) {
  const int EC = E * CO;
  const int napply = U * ach * E;
  if ((int)blockIdx.x >= napply) {
    const int idx = ((int)blockIdx.x - napply) * 4 + (threadIdx.x >> 6);
    if (idx < 3 * EC)
      bn_fin_body(jobs, idx % EC, idx / EC, threadIdx.x & 63, U, chunks, EC, bnf.count, bnf.momentum, bnf.eps,
                  training, nbt, n_nbt, nbt_inc);
    return;
  }
  __shared__ float stl[CO * NST];
  const int e = blockIdx.x % E, rest = blockIdx.x / E, chunk = rest % ach, u = rest / ach;
  const int n0 = u * B + chunk * spb, nend = min((u + 1) * B, n0 + spb);
  constexpr int ITEMS = CO * HW / 8;   // 8-value items per sample
  // UNR items per thread per round, the next round's loads in flight behind this round's math and stores
  // (one load per round trip kept the kernel latency-bound: 16 dependent round trips per thread at spb 8),
  // and the first round's loads issued before the BN records are built (z does not depend on them)
  const int total = (nend - n0) * ITEMS;
  auto off = [&](int t) -> size_t {
    const int n = n0 + t / ITEMS, i = t % ITEMS;
    return ((size_t)n * EC + e * CO) * HW + (size_t)i * 8;
  };
  uint4 raw[UNR];
#pragma unroll
  for (int k = 0; k < UNR; ++k) {
    const int t = threadIdx.x + 256 * k;
    if (t < total) raw[k] = *reinterpret_cast<const uint4*>(z + off(t));
  }
  bn_fwd_build(bnf, stl, u, e, EC, chunk == 0);
  __syncthreads();
  const float q = h8 ? qs[0] : 0.f;
  float mx = 0.f;
  for (int base = 0; base < total; base += 256 * UNR) {
    uint4 nxt[UNR];
#pragma unroll
    for (int k = 0; k < UNR; ++k) {
      const int t = base + 256 * UNR + threadIdx.x + 256 * k;
      if (t < total) nxt[k] = *reinterpret_cast<const uint4*>(z + off(t));
    }
#pragma unroll
    for (int k = 0; k < UNR; ++k) {
      const int t = base + threadIdx.x + 256 * k;
      if (t >= total) continue;
      const size_t e0 = off(t);
      const int c = ((t % ITEMS) * 8) / HW;
      const float a = stl[c * NST + ST_A], b = stl[c * NST + ST_B];
      const uint32_t r4[4] = {raw[k].x, raw[k].y, raw[k].z, raw[k].w};
      float v[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[2 * j] = __uint_as_float(r4[j] << 16);
        v[2 * j + 1] = __uint_as_float(r4[j] & 0xffff0000u);
      }
      uint32_t w[4];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = relu_nan(a * v[j] + b);
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j] = f32_to_bf16(v[2 * j]) | ((uint32_t)f32_to_bf16(v[2 * j + 1]) << 16);
      *reinterpret_cast<uint4*>(h + e0) = make_uint4(w[0], w[1], w[2], w[3]);
      if (h8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) mx = fmaxf(mx, v[j]);
        const uint32_t p0 = e4m3_pack4(v[0] * q, v[1] * q, v[2] * q, v[3] * q);
        const uint32_t p1 = e4m3_pack4(v[4] * q, v[5] * q, v[6] * q, v[7] * q);
        *reinterpret_cast<uint2*>(h8 + e0) = make_uint2(p0, p1);
      }
    }
#pragma unroll
    for (int k = 0; k < UNR; ++k) raw[k] = nxt[k];
  }
  if (h8) amax_block_store(amax, mx);
}

// out[i] += sum_rows slab[g][row][i] for every group g (rows contiguous per group).
// block = 64 columns x 4 row phases; deterministic order (fixed per-thread row sets + fixed combine).
__global__ void __launch_bounds__(256) slab_rows_sum_kernel(const float* __restrict__ slab, float* __restrict__ out,
                                                            int groups, int rows, int width, int accumulate) {
  __shared__ float red[4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + tx;
  const int g = blockIdx.y;
  float t = 0.f;
  if (i < width) {
    const float* s = slab + (size_t)g * rows * width + i;
    for (int r = ty; r < rows; r += 4) t += s[(size_t)r * width];
  }
  red[ty][tx] = t;
  __syncthreads();
  if (ty == 0 && i < width)
    out[(size_t)g * width + i] = (accumulate ? out[(size_t)g * width + i] : 0.f) + (red[0][tx] + red[1][tx]) +
                                 (red[2][tx] + red[3][tx]);
}

// Vector variant (width % 4 == 0, 16-byte aligned rows): 16 column quads x 16 row phases per
// block, float4 loads, unrolled so each thread keeps several independent loads in flight.
// ld: row stride of the slab in floats (>= width; a group spans rows * ld floats).
template <int SR = 8>
__device__ __forceinline__ void slab_rows_sum4_body(const float* __restrict__ slab, float* __restrict__ out, int rows,
                                                    int width, int ld, int g, int bx, int accumulate);
__global__ void __launch_bounds__(256) slab_rows_sum4_kernel(const float* __restrict__ slab, float* __restrict__ out,
                                                             int groups, int rows, int width, int accumulate) {
  slab_rows_sum4_body(slab, out, rows, width, width, blockIdx.y, blockIdx.x, accumulate);
}

// Several independent slab sums in one launch (blockIdx.z = job): every gradient-slab reduction of
// a step phase (conv weight slabs, quantum-layer slab, QSC preprocess slab) at once.  Jobs whose
// width is not a multiple of 4 (or whose buffers are not 16-byte aligned) take a scalar path.
constexpr int kSlabJobs = 16;
struct SlabJobs {
  const float* slab[kSlabJobs];
  float* out[kSlabJobs];
  int groups[kSlabJobs], rows[kSlabJobs], width[kSlabJobs], ld[kSlabJobs], vec[kSlabJobs];
  int accumulate;
};
__device__ __forceinline__ void slab_rows_sum1_body(const float* __restrict__ slab, float* __restrict__ out, int rows,
                                                    int width, int ld, int g, int bx, int accumulate) {
  __shared__ float red1[16][64];
  const int tq = threadIdx.x & 15, ty = threadIdx.x >> 4;
  float t[4] = {0.f, 0.f, 0.f, 0.f};
  const float* s = slab + (size_t)g * rows * ld;
  for (int r = ty; r < rows; r += 16) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = bx * 64 + q * 16 + tq;
      if (i < width) t[q] += s[(size_t)r * ld + i];
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) red1[ty][q * 16 + tq] = t[q];
  __syncthreads();
  if (threadIdx.x < 64) {
    const int i = bx * 64 + threadIdx.x;
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) acc += red1[k][threadIdx.x];
    if (i < width) out[(size_t)g * width + i] = (accumulate ? out[(size_t)g * width + i] : 0.f) + acc;
  }
}
__global__ void __launch_bounds__(256) slab_rows_sum4_multi_kernel(SlabJobs jobs) {
  const int j = blockIdx.z;
  if (blockIdx.y >= jobs.groups[j] || blockIdx.x * 64 >= jobs.width[j]) return;
  if (jobs.vec[j])
    slab_rows_sum4_body(jobs.slab[j], jobs.out[j], jobs.rows[j], jobs.width[j], jobs.ld[j], blockIdx.y, blockIdx.x,
                        jobs.accumulate);
  else
    slab_rows_sum1_body(jobs.slab[j], jobs.out[j], jobs.rows[j], jobs.width[j], jobs.ld[j], blockIdx.y, blockIdx.x,
                        jobs.accumulate);
}

template <int SR>
__device__ __forceinline__ void slab_rows_sum4_body(const float* __restrict__ slab, float* __restrict__ out, int rows,
                                                    int width, int ld, int g, int bx, int accumulate) {
  __shared__ float4 red[16][16];
  const int tq = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int i = (bx * 16 + tq) * 4;
  float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < width) {
    const float* s = slab + (size_t)g * rows * ld + i;
    // rounds of SR rows with every load of a round issued before its adds (same summation order as a
    // row-at-a-time loop: bit-identical sums)
    for (int r0 = ty; r0 < rows; r0 += 16 * SR) {
      // (branch-free: a row past the end re-loads row r0 and is not added -- guarded loads compiled to one
      // round trip each)
      float4 v[SR];
#pragma unroll
      for (int k = 0; k < SR; ++k)
        v[k] = *reinterpret_cast<const float4*>(s + (size_t)(r0 + 16 * k < rows ? r0 + 16 * k : r0) * ld);
#pragma unroll
      for (int k = 0; k < SR; ++k)
        if (r0 + 16 * k < rows) {
          t.x += v[k].x;
          t.y += v[k].y;
          t.z += v[k].z;
          t.w += v[k].w;
        }
    }
  }
  red[ty][tq] = t;
  __syncthreads();
  if (ty == 0 && i < width) {
    float4 acc = red[0][tq];
#pragma unroll
    for (int k = 1; k < 16; ++k) {
      acc.x += red[k][tq].x;
      acc.y += red[k][tq].y;
      acc.z += red[k][tq].z;
      acc.w += red[k][tq].w;
    }
    float4* o = reinterpret_cast<float4*>(out + (size_t)g * width + i);
    float4 cur = accumulate ? *o : make_float4(0.f, 0.f, 0.f, 0.f);
    cur.x += acc.x;
    cur.y += acc.y;
    cur.z += acc.z;
    cur.w += acc.w;
    *o = cur;
  }
}

}  // namespace conv
}  // namespace qd

using namespace qd::conv;

// ---------------------------------------------------------------------------------------------
// C ABI.  Geometry: H=16 and W in {8, 16} (P128 / P256).  All launches on `stream`.
// ---------------------------------------------------------------------------------------------
#define QD_GEOM(W_, ...) \
  if ((H) == 16 && (W) == 8) { constexpr int W_ = 8; __VA_ARGS__; } \
  else if ((H) == 16 && (W) == 16) { constexpr int W_ = 16; __VA_ARGS__; } \
  else return (int)hipErrorInvalidValue;

static size_t fwd_smem(int cin, int H, int W) {
  const int cinp = cin;
  const int ks = (9 * cin + 15) / 16;   // (dgrad: cin = 32 -> 18 = the dgrad pack's k-steps too)
  // 4 wave tiles | B fragments | BN params
  return 4 * (size_t)(H + 2) * (W + 2) * cinp * 2 + (size_t)ks * 64 * 16 + (size_t)cin * NST * sizeof(float);
}

// layer: 1 -> CIN=2 raw f32 input; 2,3 -> CIN=32 bf16 z_prev with BN+ReLU (st_prev).
QD_API int qd_conv_pack_weights(const float* w, uint16_t* out, int E, int cin, int dgrad, void* stream) {
  const int KS = dgrad ? 18 : (9 * cin + 15) / 16;
  hipLaunchKernelGGL(pack_weights_kernel, dim3(KS, E), dim3(64), 0, (hipStream_t)stream, w, out, E, cin, KS, dgrad);
  return (int)hipGetLastError();
}

// n jobs (<= 8): w[j] fp32 (E, 32, cin[j], 3, 3) -> out[j] packed (dgrad[j] selects the dgrad order)
QD_API int qd_conv_pack_weights_multi2(int n, const float* const* w, uint16_t* const* out, const int* cin,
                                       const int* dgrad, int E, int* cursor, int cursor_inc, void* stream);
QD_API int qd_conv_pack_weights_multi(int n, const float* const* w, uint16_t* const* out, const int* cin,
                                      const int* dgrad, int E, void* stream) {
  return qd_conv_pack_weights_multi2(n, w, out, cin, dgrad, E, nullptr, 0, stream);
}
// cursor (nullable): advanced by cursor_inc in the same launch (see PackJobs)
QD_API int qd_conv_pack_weights_multi2(int n, const float* const* w, uint16_t* const* out, const int* cin,
                                       const int* dgrad, int E, int* cursor, int cursor_inc, void* stream) {
  if (n < 1 || n > 8) return (int)hipErrorInvalidValue;
  PackJobs jobs{};
  jobs.cursor = cursor;
  jobs.cursor_inc = cursor_inc;
  int ksmax = 0;
  for (int j = 0; j < n; ++j) {
    jobs.w[j] = w[j];
    jobs.out[j] = out[j];
    jobs.cin[j] = cin[j];
    jobs.dgrad[j] = dgrad[j];
    jobs.ks[j] = dgrad[j] ? 18 : (9 * cin[j] + 15) / 16;
    ksmax = jobs.ks[j] > ksmax ? jobs.ks[j] : ksmax;
  }
  hipLaunchKernelGGL(pack_weights_multi_kernel, dim3(ksmax, E, n), dim3(64), 0, (hipStream_t)stream, jobs);
  return (int)hipGetLastError();
}

// w: packed B fragments from qd_conv_pack_weights(dgrad=0)
// bnf (nullable, layers 2/3): build the input BN records from the previous layer's statistics
// partials in-kernel (fused finalisation; st_prev is then ignored) -- see BnFwd.
QD_API int qd_conv_fwd(int layer, const void* xin, const float* st_prev, const uint16_t* w, uint16_t* z, float* stats,
                       int N, int E, int B, int H, int W, int chunks, int spw, const BnFwd* bnf, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const BnFwd bf = bnf ? *bnf : BnFwd{};
  const BnBwd bb{};
  const int U = N / B;
  dim3 grid(U * chunks, E);
  if (chunks * 4 * spw < B) return (int)hipErrorInvalidValue;
  if (layer == 1) {
    QD_GEOM(WW, hipLaunchKernelGGL((conv3x3_kernel<2, 16, WW, IN_RAW_F32, OUT_Z_STATS, false, float>), grid, dim3(256),
                                    fwd_smem(2, H, W), s, (const float*)xin, nullptr, nullptr, w, z, stats, E, B, chunks,
                                    spw, bf, bb, BnRed{}))
  } else {
    QD_GEOM(WW, hipLaunchKernelGGL((conv3x3_kernel<32, 16, WW, IN_BNRELU, OUT_Z_STATS, false, uint16_t>), grid,
                                    dim3(256), fwd_smem(32, H, W), s, (const uint16_t*)xin, nullptr, st_prev, w, z,
                                    stats, E, B, chunks, spw, bf, bb, BnRed{}))
  }
  return (int)hipGetLastError();
}

// qd_conv_fwd for layers 2 / 3 at P128 on the software-pipelined kernel (conv3x3_fwd_db_kernel): same arguments,
// bit-identical outputs; hipErrorInvalidValue for other geometries (the caller keeps qd_conv_fwd then).
QD_API int qd_conv_fwd_db(const uint16_t* xin, const float* st_prev, const uint16_t* w, uint16_t* z, float* stats,
                          int N, int E, int B, int H, int W, int chunks, int spw, const BnFwd* bnf, void* stream) {
  if (H != 16 || W != 8 || B <= 0 || N % B || chunks * 4 * spw < B) return (int)hipErrorInvalidValue;
  const BnFwd bf = bnf ? *bnf : BnFwd{};
  if (!bnf && !st_prev) return (int)hipErrorInvalidValue;
  constexpr size_t smem = 8 * (size_t)18 * 10 * 32 * 2 + 18 * 64 * 16 + 32 * NST * sizeof(float);
  if (hipError_t e = qd::allow_lds(conv3x3_fwd_db_kernel<8>, smem)) return (int)e;
  hipLaunchKernelGGL(conv3x3_fwd_db_kernel<8>, dim3((N / B) * chunks, E), dim3(256), smem, (hipStream_t)stream, xin,
                     st_prev, w, z, stats, E, B, chunks, spw, bf);
  return (int)hipGetLastError();
}

// qd_conv_fwd on the sample-split kernel (conv3x3_split_kernel): `sps` samples per workgroup, `chunks` = workgroups
// per group (chunks * sps >= B) = the statistics partial rows per group.  Same z as qd_conv_fwd.
static size_t split_smem(int cin, int H, int W) {
  // 2 sample tiles | B fragments | BN records
  return 2 * (size_t)(H + 2) * (W + 2) * cin * 2 + (size_t)((9 * cin + 15) / 16) * 64 * 16 + (size_t)cin * NST * 4;
}
QD_API int qd_conv_fwd_split(int layer, const void* xin, const float* st_prev, const uint16_t* w, uint16_t* z,
                             float* stats, int N, int E, int B, int H, int W, int chunks, int sps, const BnFwd* bnf,
                             void* stream) {
  // (layer 1 also at sps 12 = 4 waves x the per-wave kernel's 3 samples: the same statistics chunking as conv3x3_kernel,
  // so it can replace that layer alone)
  if (B <= 0 || N % B || ((sps < 4 || sps > 6) && !(layer == 1 && sps == 12)) || chunks <= 0 || (long)chunks * sps < B ||
      (layer != 1 && !bnf && !st_prev))
    return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const BnFwd bf = bnf ? *bnf : BnFwd{};
  dim3 grid((N / B) * chunks, E);
  // P128: every sample's loads in flight from the start (D = SPS); P256 (twice the registers per sample): 2 ahead
#define QD_SPLIT(SPS_)                                                                                                \
  if (layer == 1) {                                                                                                   \
    QD_GEOM(WW, hipLaunchKernelGGL((conv3x3_split_kernel<2, WW, IN_RAW_F32, float, SPS_, WW == 8 ? SPS_ : 2>), grid, \
                                    dim3(256), split_smem(2, H, W), s, (const float*)xin, nullptr, w, z, stats, E, B, \
                                    chunks, bf))                                                                      \
  } else {                                                                                                            \
    QD_GEOM(WW, hipLaunchKernelGGL((conv3x3_split_kernel<32, WW, IN_BNRELU, uint16_t, SPS_, WW == 8 ? SPS_ : 2>),    \
                                    grid, dim3(256), split_smem(32, H, W), s, (const uint16_t*)xin, st_prev, w, z,    \
                                    stats, E, B, chunks, bf))                                                         \
  }
  if (sps == 12) {   // (layer 1 only, checked above)
    QD_GEOM(WW, hipLaunchKernelGGL((conv3x3_split_kernel<2, WW, IN_RAW_F32, float, 12, WW == 8 ? 12 : 2>), grid,
                                    dim3(256), split_smem(2, H, W), s, (const float*)xin, nullptr, w, z, stats, E, B,
                                    chunks, bf))
  } else if (sps == 4) { QD_SPLIT(4) } else if (sps == 5) { QD_SPLIT(5) } else { QD_SPLIT(6) }
#undef QD_SPLIT
  return (int)hipGetLastError();
}

// The persistent training forward (conv_fwd_stack_kernel).  sync: (U*E)*2 + E*3 + 1 zero-initialised words --
// the barriers, the per-(expert, layer) arrival counts and the error word (all return to zero after a launch, the
// error word excepted).  Returns hipErrorInvalidValue when the shapes do not fit and hipErrorInvalidConfiguration
// when the grid cannot be resident all at once (the caller keeps the per-layer launches then);
// qd_conv_fwd_stack_fits answers that without launching.
template <int W>
static int stack_fits(int grid) {
  static int cap = -1;   // co-resident workgroups of this kernel on the device (per W)
  if (cap < 0) {
    int nb = 0, dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, conv_fwd_stack_kernel<W>, 256, fwd_smem(32, 16, W)) !=
            hipSuccess)
      return 0;
    cap = nb * cus;
  }
  return grid <= cap;
}
QD_API int qd_conv_fwd_stack_fits(int N, int E, int B, int H, int W, int chunks) {
  if (H != 16 || N % B) return 0;
  const int grid = (N / B) * chunks * E;
  if (W == 8) return stack_fits<8>(grid);
  if (W == 16) return stack_fits<16>(grid);
  return 0;
}
QD_API int qd_conv_fwd_stack(const StackFwd* a, unsigned* sync, int N, int E, int B, int H, int W, int chunks, int spw,
                             void* stream) {
  if (!a || !sync || N % B || chunks * 4 * spw < B || (N / B) > kMaxGroups) return (int)hipErrorInvalidValue;
  if (!qd_conv_fwd_stack_fits(N, E, B, H, W, chunks)) return (int)hipErrorInvalidConfiguration;
  const int U = N / B;
  StackSync sy{sync, sync + 2 * U * E, reinterpret_cast<int*>(sync + 2 * U * E + 3 * E)};
  dim3 grid(U * chunks, E);
  hipStream_t s = (hipStream_t)stream;
  QD_GEOM(WW, hipLaunchKernelGGL((conv_fwd_stack_kernel<WW>), grid, dim3(256), fwd_smem(32, 16, WW), s, *a, sy, E, B,
                                  U, chunks, spw))
  return (int)hipGetLastError();
}

// Diagnostic: the persistent forward with per-workgroup phase stamps (stamps: grid * 8 u64, see
// conv_fwd_stack_kernel).  P128 geometry only.
QD_API int qd_conv_fwd_stack_stamped(const StackFwd* a, unsigned* sync, int N, int E, int B, int chunks, int spw,
                                     unsigned long long* stamps, void* stream) {
  if (!a || !sync || !stamps || N % B || chunks * 4 * spw < B || (N / B) > kMaxGroups) return (int)hipErrorInvalidValue;
  if (!stack_fits<8>((N / B) * chunks * E)) return (int)hipErrorInvalidConfiguration;
  const int U = N / B;
  StackSync sy{sync, sync + 2 * U * E, reinterpret_cast<int*>(sync + 2 * U * E + 3 * E)};
  hipLaunchKernelGGL((conv_fwd_stack_kernel<8, true>), dim3(U * chunks, E), dim3(256), fwd_smem(32, 16, 8),
                     (hipStream_t)stream, *a, sy, E, B, U, chunks, spw, stamps);
  return (int)hipGetLastError();
}

// fp8 forward of a 32->32 layer (see conv3x3_f8_kernel).  w: the layer's fp32 weights (E*32, 32, 3, 3);
// qs / scale: its (activation, weight) pair of quantisation / dequantisation factors; amax_a / amax_w:
// the activation amax partials (indexed by the flat block id) / the weight's (indexed by expert).
QD_API int qd_conv_fwd_f8(const uint16_t* xin, const float* w, uint16_t* z, float* stats, int N, int E, int B, int H,
                          int W, int chunks, int spw, const BnFwd* bnf, const float* qs, const float* scale,
                          float* amax_a, float* amax_w, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (!bnf || chunks * 4 * spw < B || (N / B) * chunks * E > qd::kAmaxParts) return (int)hipErrorInvalidValue;
  const BnFwd bf = *bnf;
  dim3 grid((N / B) * chunks, E);
  QD_GEOM(WW, {
    const size_t sm = 4 * (size_t)(16 + 2) * (WW + 2) * 32 + (size_t)KS8 * 64 * 8 + 32 * NST * sizeof(float);
    hipLaunchKernelGGL((conv3x3_f8_kernel<WW>), grid, dim3(256), sm, s, xin, w, z, stats, E, B, chunks, spw, bf, qs,
                       scale, amax_a, amax_w);
  })
  return (int)hipGetLastError();
}

// data gradient of a 32->32 layer: dx (f32, or bf16 when dx_bf16) from dh (f32 or bf16) of this
// layer, z, st.  w: packed B fragments from qd_conv_pack_weights(dgrad=1)
// bnb (nullable): build this layer's BN backward coefficients from the reduction partials in-kernel.
// bred (nullable; bf16 dx only): also produce the previous layer's BN backward partials (BnRed).
QD_API int qd_conv_dgrad(const void* dh, int dh_bf16, const uint16_t* z, const float* st, const uint16_t* w, void* dx,
                         int dx_bf16, int N, int E, int B, int H, int W, int chunks, int spw, const BnBwd* bnb,
                         const BnRed* bred, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const BnFwd bf{};
  const BnBwd bb = bnb ? *bnb : BnBwd{};
  const BnRed br = bred ? *bred : BnRed{};
  if (br.part && !dx_bf16) return (int)hipErrorInvalidValue;
  dim3 grid((N / B) * chunks, E);
  if (chunks * 4 * spw < B) return (int)hipErrorInvalidValue;
#define QD_DG(OUTM_, TIN_)                                                                                         \
  QD_GEOM(WW, hipLaunchKernelGGL((conv3x3_kernel<32, 16, WW, IN_BNBWD, OUTM_, true, TIN_>), grid, dim3(256),          \
                                  fwd_smem(32, H, W), s, (const TIN_*)dh, z, st, w, dx, nullptr, E, B, chunks, spw, \
                                  bf, bb, br))
  if (dh_bf16) {
    if (dx_bf16) { QD_DG(OUT_BF16, uint16_t) } else { QD_DG(OUT_F32, uint16_t) }
  } else {
    if (dx_bf16) { QD_DG(OUT_BF16, float) } else { QD_DG(OUT_F32, float) }
  }
#undef QD_DG
  return (int)hipGetLastError();
}

// Diagnostic: layer-2/3 forward (dgrad = 0) or bf16 data gradient (dgrad = 1) with per-wave phase
// stamps (stamps: grid * 4 waves * 8 u64; see conv3x3_kernel).  P128 geometry only.
QD_API int qd_conv_stamped(int dgrad, const void* xin, const uint16_t* zaux, const float* st, const uint16_t* w,
                           void* out, float* stats, int N, int E, int B, int chunks, int spw,
                           unsigned long long* stamps, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((N / B) * chunks, E);
  if (dgrad)
    hipLaunchKernelGGL((conv3x3_kernel<32, 16, 8, IN_BNBWD, OUT_BF16, true, uint16_t, true>), grid, dim3(256),
                       fwd_smem(32, 16, 8), s, (const uint16_t*)xin, zaux, st, w, out, nullptr, E, B, chunks, spw,
                       BnFwd{}, BnBwd{}, BnRed{}, stamps);
  else
    hipLaunchKernelGGL((conv3x3_kernel<32, 16, 8, IN_BNRELU, OUT_Z_STATS, false, uint16_t, true>), grid, dim3(256),
                       fwd_smem(32, 16, 8), s, (const uint16_t*)xin, nullptr, st, w, out, stats, E, B, chunks, spw,
                       BnFwd{}, BnBwd{}, BnRed{}, stamps);
  return (int)hipGetLastError();
}

static size_t wgrad_smem(int cin, int H, int W) {
  const size_t stage = (3 * (size_t)cin * ((H + 2) * W + 8) + 32 * (size_t)(H * W + 8)) * 2 + (cin + 32) * NST * 4;
  const size_t red = 2 * 32 * (size_t)(9 * cin + 1) * 4;
  return stage > red ? stage : red;
}

// weight-gradient partials: slab (E, U*chunks, 32*CIN*9).  layer 1: x = raw f32 (CIN=2);
// layers 2,3: x = BN+ReLU(z_prev) (st_prev).  bnb (nullable): this layer's BN backward coefficients
// from the reduction partials in-kernel, and dgamma / dbeta written by one workgroup per expert.
QD_API int qd_conv_wgrad(int layer, const void* xin, const float* st_prev, const void* dh, int dh_bf16,
                         const uint16_t* z, const float* st, float* slab, int N, int E, int B, int H, int W, int chunks,
                         int spb, const BnBwd* bnb, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const BnBwd bb = bnb ? *bnb : BnBwd{};
  dim3 grid((N / B) * chunks, E);
  if (chunks * spb < B) return (int)hipErrorInvalidValue;
#define QD_WG(CIN_, INM_, TIN_, TDH_)                                                                              \
  QD_GEOM(WW, hipLaunchKernelGGL((conv3x3_wgrad_kernel<CIN_, 16, WW, INM_, TIN_, TDH_>), grid, dim3(256),         \
                                  wgrad_smem(CIN_, H, W), s, (const TIN_*)xin, st_prev, (const TDH_*)dh, z, st, slab, \
                                  E, B, chunks, spb, bb))
  if (layer == 1) {
    if (dh_bf16) { QD_WG(2, IN_RAW_F32, float, uint16_t) } else { QD_WG(2, IN_RAW_F32, float, float) }
  } else {
    if (dh_bf16) { QD_WG(32, IN_BNRELU, uint16_t, uint16_t) } else { QD_WG(32, IN_BNRELU, uint16_t, float) }
  }
#undef QD_WG
  return (int)hipGetLastError();
}

// wgrad + dgrad of a 32-channel layer in ONE launch (bf16 dh and dx; see conv3x3_wd_kernel).  Arguments
// as qd_conv_wgrad (layer 2 / 3) and qd_conv_dgrad.
QD_API int qd_conv_wgrad_dgrad(const uint16_t* xin, const float* st_prev, const uint16_t* dh, const uint16_t* z,
                               const float* st, float* slab, int chunks_w, int spb, const uint16_t* w, uint16_t* dx,
                               int chunks_d, int spw, int N, int E, int B, int H, int W, const BnBwd* bnb,
                               const BnRed* bred, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const BnBwd bb = bnb ? *bnb : BnBwd{};
  const BnRed br = bred ? *bred : BnRed{};
  if (chunks_w * spb < B || chunks_d * 4 * spw < B) return (int)hipErrorInvalidValue;
  const int gx_w = (N / B) * chunks_w, gx_d = (N / B) * chunks_d;
  dim3 grid(gx_w + gx_d, E);
  const size_t sm_w = wgrad_smem(32, H, W), sm_d = fwd_smem(32, H, W);
  const size_t sm = sm_w > sm_d ? sm_w : sm_d;
  QD_GEOM(WW, {
    if (hipError_t e = qd::allow_lds(conv3x3_wd_kernel<WW>, sm)) return (int)e;
    hipLaunchKernelGGL((conv3x3_wd_kernel<WW>), grid, dim3(256), sm, s, xin, st_prev, dh, z, st, slab, chunks_w, spb, bb,
                       w, dx, chunks_d, spw, br, E, B, gx_w);
  })
  return (int)hipGetLastError();
}

// wgrad + dgrad + the previous layer's BN backward partials of a 32-channel layer from one staging
// per sample (see conv3x3_bwd_kernel).  zprev / st_prev: the previous layer's pre-BN output and its
// records (x = BN+ReLU(zprev)); wt: dgrad B fragments; part: (U, chunks, 2, EC); slab rows as
// qd_conv_wgrad's with the same chunking.
QD_API int qd_conv_bwd_fused(const uint16_t* zprev, const float* st_prev, const uint16_t* dh, const uint16_t* z,
                             const float* st, float* slab, const uint16_t* w, uint16_t* dx, float* part, int N, int E,
                             int B, int H, int W, int chunks, int spb, const BnBwd* bnb, const qd::LossFinish* lf,
                             void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const BnBwd bb = bnb ? *bnb : BnBwd{};
  const qd::LossFinish lff = lf ? *lf : qd::LossFinish{};
  if (chunks * spb < B || N % B) return (int)hipErrorInvalidValue;
  dim3 grid((N / B) * chunks, E + (lf ? 1 : 0));
  QD_GEOM(WW, {
    const size_t sm = BwdGeo<WW>::SMEM;
    if (hipError_t e = qd::allow_lds(conv3x3_bwd_kernel<WW>, sm)) return (int)e;
    hipLaunchKernelGGL((conv3x3_bwd_kernel<WW>), grid, dim3(256), sm, s, zprev, st_prev, dh, z, st, slab, w, dx, part,
                       E, B, chunks, spb, bb, lff);
  })
  return (int)hipGetLastError();
}

// qd_conv_bwd_fused at P128 on the software-pipelined kernel (conv3x3_bwd_db_kernel): same arguments and outputs
// (bit-identical at the same chunking); hipErrorInvalidValue for other geometries.
QD_API int qd_conv_bwd_db(const uint16_t* zprev, const float* st_prev, const uint16_t* dh, const uint16_t* z,
                          const float* st, float* slab, const uint16_t* w, uint16_t* dx, float* part, int N, int E,
                          int B, int H, int W, int chunks, int spb, const BnBwd* bnb, const qd::LossFinish* lf,
                          void* stream) {
  if (H != 16 || W != 8 || chunks * spb < B || N % B) return (int)hipErrorInvalidValue;
  const BnBwd bb = bnb ? *bnb : BnBwd{};
  const qd::LossFinish lff = lf ? *lf : qd::LossFinish{};
  const size_t sm = BwdDbGeo<8>::SMEM;
  if (sm > 160 * 1024) return (int)hipErrorInvalidValue;
  if (hipError_t e = qd::allow_lds(conv3x3_bwd_db_kernel<8>, sm)) return (int)e;
  hipLaunchKernelGGL(conv3x3_bwd_db_kernel<8>, dim3((N / B) * chunks, E + (lf ? 1 : 0)), dim3(256), sm,
                     (hipStream_t)stream, zprev, st_prev, dh, z, st, slab, w, dx, part, E, B, chunks, spb, bb, lff);
  return (int)hipGetLastError();
}

QD_API int qd_bn_stats_finalize(const float* stats, const float* gamma, const float* beta, float* run_mean,
                                float* run_var, float* st, int U, int chunks, int EC, float count, float momentum,
                                float eps, int training, long long* nbt, int n_nbt, long long nbt_inc,
                                void* stream) {
  if (U < 1 || U > kMaxGroups || n_nbt > 64) return (int)hipErrorInvalidValue;
  FinJobs jobs{};
  jobs.stats[0] = stats;
  jobs.gamma[0] = gamma;
  jobs.beta[0] = beta;
  jobs.run_mean[0] = run_mean;
  jobs.run_var[0] = run_var;
  jobs.st[0] = st;
  hipLaunchKernelGGL(bn_stats_finalize_kernel, dim3(EC, 1), dim3(64), 0, (hipStream_t)stream, jobs, U, chunks, EC,
                     count, momentum, eps, training, nbt, n_nbt, nbt_inc);
  return (int)hipGetLastError();
}

// n (<= 3) layers' finalisations in one launch (arrays of n pointers); nbt as above (layer 0's block).
QD_API int qd_bn_stats_finalize_multi(int n, const float* const* stats, const float* const* gamma,
                                      const float* const* beta, float* const* run_mean, float* const* run_var,
                                      float* const* st, int U, int chunks, int EC, float count, float momentum,
                                      float eps, int training, long long* nbt, int n_nbt, long long nbt_inc,
                                      void* stream) {
  if (n < 1 || n > 3 || U < 1 || U > kMaxGroups || n_nbt > 64) return (int)hipErrorInvalidValue;
  FinJobs jobs{};
  for (int l = 0; l < n; ++l) {
    jobs.stats[l] = stats[l];
    jobs.gamma[l] = gamma[l];
    jobs.beta[l] = beta[l];
    jobs.run_mean[l] = run_mean[l];
    jobs.run_var[l] = run_var[l];
    jobs.st[l] = st[l];
  }
  hipLaunchKernelGGL(bn_stats_finalize_kernel, dim3(EC, n), dim3(64), 0, (hipStream_t)stream, jobs, U, chunks, EC,
                     count, momentum, eps, training, nbt, n_nbt, nbt_inc);
  return (int)hipGetLastError();
}

// lf (nullable): also run this loss finish (see common.h) as one extra workgroup
QD_API int qd_bn_bwd_reduce(const void* dh, int dh_bf16, const uint16_t* z, const float* st, float* slab, int N, int E,
                            int B, int H, int W, int chunks, int spb, const qd::LossFinish* lf_in, void* stream) {
  const qd::LossFinish lf = (lf_in && lf_in->part) ? *lf_in : qd::LossFinish{};
  dim3 grid((N / B) * chunks, E + (lf.part ? 1 : 0));
  hipStream_t s = (hipStream_t)stream;
  if (chunks * spb < B || H * W % 64) return (int)hipErrorInvalidValue;
  if (H * W == 128) {
    if (dh_bf16) hipLaunchKernelGGL((bn_bwd_reduce_kernel<128, uint16_t>), grid, dim3(256), 0, s, (const uint16_t*)dh, z, st, slab, E, B, chunks, spb, lf);
    else hipLaunchKernelGGL((bn_bwd_reduce_kernel<128, float>), grid, dim3(256), 0, s, (const float*)dh, z, st, slab, E, B, chunks, spb, lf);
  } else if (H * W == 256) {
    if (dh_bf16) hipLaunchKernelGGL((bn_bwd_reduce_kernel<256, uint16_t>), grid, dim3(256), 0, s, (const uint16_t*)dh, z, st, slab, E, B, chunks, spb, lf);
    else hipLaunchKernelGGL((bn_bwd_reduce_kernel<256, float>), grid, dim3(256), 0, s, (const float*)dh, z, st, slab, E, B, chunks, spb, lf);
  } else {
    return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

// accumulate = 0: overwrite dgamma/dbeta (no zero_grad needed)
QD_API int qd_bn_bwd_finalize(const float* slab, const float* gamma, float* st, float* dgamma, float* dbeta, int U,
                              int chunks, int EC, float count, int accumulate, void* stream) {
  if (U < 1 || U > kMaxGroups) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(EC), dim3(64), 0, (hipStream_t)stream, slab, gamma, st,
                     dgamma, dbeta, U, chunks, EC, count, accumulate);
  return (int)hipGetLastError();
}

// h8/qs/amax nullable (fp8 estimator only)
QD_API int qd_bn_relu_apply(const uint16_t* z, const float* st, uint16_t* h, int N, int EC, int B, int HW,
                            uint8_t* h8, const float* qs, float* amax, void* stream) {
  const long n8 = (long)N * EC * HW / 8;
  int grid = (int)((n8 + 255) / 256);
  if (grid > 2048) grid = 2048;   // <= kAmaxParts
  if (h8 && (!qs || !amax)) return (int)hipErrorInvalidValue;
  if (HW == 128)
    hipLaunchKernelGGL((bn_relu_apply_kernel<128>), dim3(grid), dim3(256), 0, (hipStream_t)stream, z, st, h, n8, EC, B,
                       h8, qs, amax);
  else if (HW == 256)
    hipLaunchKernelGGL((bn_relu_apply_kernel<256>), dim3(grid), dim3(256), 0, (hipStream_t)stream, z, st, h, n8, EC, B,
                       h8, qs, amax);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

// Layer-3 BN tail + BN/ReLU apply in one launch (bn_apply_tail_kernel).  bnf: layer 3's BnFwd (records
// published to bnf->st_out); stats/gamma/beta/run_mean/run_var/st: the 3 layers' arrays as in
// qd_bn_stats_finalize_multi (st[2] is ignored: layer 3's records come from bnf).  spb: samples per
// apply workgroup (divides B).
QD_API int qd_bn_apply_tail(const uint16_t* z, uint16_t* h, const BnFwd* bnf, const float* const* stats,
                            const float* const* gamma, const float* const* beta, float* const* run_mean,
                            float* const* run_var, float* const* st, int U, int E, int B, int HW, int spb, int chunks,
                            int training, long long* nbt, int n_nbt, long long nbt_inc, uint8_t* h8, const float* qs,
                            float* amax, void* stream) {
  if (!bnf || U < 1 || U > kMaxGroups || n_nbt > 64 || spb < 1 || (h8 && (!qs || !amax)))
    return (int)hipErrorInvalidValue;
  FinJobs jobs{};
  for (int l = 0; l < 3; ++l) {
    jobs.stats[l] = stats[l];
    jobs.gamma[l] = gamma[l];
    jobs.beta[l] = beta[l];
    jobs.run_mean[l] = run_mean[l];
    jobs.run_var[l] = run_var[l];
    jobs.st[l] = l == 2 ? nullptr : st[l];
  }
  // (a group of B samples: ceil(B / spb) apply workgroups, the last one partial -- B need not divide: the test-time
  // BN re-estimation's last chunk of an expert's samples has any size)
  const int ach = (B + spb - 1) / spb, EC = E * CO;
  const int napply = U * ach * E, nfin = (3 * EC + 3) / 4;
  if (h8 && napply > qd::kAmaxParts) return (int)hipErrorInvalidValue;   // (one amax partial per apply workgroup)
  const dim3 grid(napply + nfin);
  hipStream_t s = (hipStream_t)stream;
#define QD_TAIL(HWV, U_)                                                                                          \
  hipLaunchKernelGGL((bn_apply_tail_kernel<HWV, U_>), grid, dim3(256), 0, s, z, h, *bnf, jobs, U, E, B, spb, ach, \
                     chunks, training, nbt, n_nbt, nbt_inc, h8, qs, amax)
  if (HW == 128)
    QD_TAIL(128, 4);
  else if (HW == 256)
    QD_TAIL(256, 4);
#undef QD_TAIL
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

// n <= 16 jobs, each as qd_slab_rows_sum, one launch
// lds (nullable): per-job row strides (default: the width)
QD_API int qd_slab_rows_sum_multi(int n, const float* const* slabs, float* const* outs, const int* groups,
                                  const int* rows, const int* widths, const int* lds, int accumulate, void* stream) {
  if (n < 1 || n > kSlabJobs) return (int)hipErrorInvalidValue;
  SlabJobs jobs{};
  jobs.accumulate = accumulate;
  int gx = 0, gy = 0;
  for (int j = 0; j < n; ++j) {
    jobs.ld[j] = lds ? lds[j] : widths[j];
    if (jobs.ld[j] < widths[j]) return (int)hipErrorInvalidValue;
    jobs.vec[j] = !(widths[j] % 4 || jobs.ld[j] % 4 || ((uintptr_t)slabs[j] & 15) || ((uintptr_t)outs[j] & 15));
    jobs.slab[j] = slabs[j];
    jobs.out[j] = outs[j];
    jobs.groups[j] = groups[j];
    jobs.rows[j] = rows[j];
    jobs.width[j] = widths[j];
    gx = std::max(gx, (widths[j] + 63) / 64);
    gy = std::max(gy, groups[j]);
  }
  hipLaunchKernelGGL(slab_rows_sum4_multi_kernel, dim3(gx, gy, n), dim3(256), 0, (hipStream_t)stream, jobs);
  return (int)hipGetLastError();
}

// accumulate = 1: out += sum; 0: out = sum
QD_API int qd_slab_rows_sum(const float* slab, float* out, int groups, int rows, int width, int accumulate,
                            void* stream) {
  if (width % 4 == 0 && ((uintptr_t)slab & 15) == 0 && ((uintptr_t)out & 15) == 0) {
    hipLaunchKernelGGL(slab_rows_sum4_kernel, dim3((width / 4 + 15) / 16, groups), dim3(256), 0, (hipStream_t)stream,
                       slab, out, groups, rows, width, accumulate);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(slab_rows_sum_kernel, dim3((width + 63) / 64, groups), dim3(256), 0, (hipStream_t)stream, slab,
                     out, groups, rows, width, accumulate);
  return (int)hipGetLastError();
}
