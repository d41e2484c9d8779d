// FC_P128 forward GEMM for gfx950: Y[M, N] = A[M, K] . W[N, K]^T (+ bias), bf16 operands, fp32
// accumulation on MFMA 16x16x32 -- with the HDCE loss fused into the epilogue.
//
// Reference: FC_P128 (Estimators_QuantumNAT_onchipQNN.py:272-279, Linear 4096 -> 2048) followed by
// NMSE_cuda (E:282-286) per (scenario, user) stream (Runner_P128_QuantumNAT_onchipQNN.py:109-113).
//
// Shape: the flagship step has M = 2304 rows (9 streams x 256), N = 2048, K = 4096.  Both operands
// are K-contiguous, so both MFMA fragments are single ds_read_b128s.  Tile 144 x 128 (9 x 8
// fragments): 16 x 16 = 256 tiles = ONE workgroup per CU, no tail wave (hipBLASLt's 128 x 160 /
// 256 x 144 tiles leave a partial second wave).  4 waves side by side along N (144 x 32 each: 18
// accumulators); BK = 64, two LDS stages filled by global_load_lds (16 B), XOR-swizzled 16-B chunks
// (chunk ^ (row & 7)) so every fragment read is bank-conflict-free; one barrier per K step.
// XCD-aware tile order: blocks of one XCD take 4 M-tiles x 8 N-tiles (A and W slabs reused in
// that XCD's L2).
//
// Epilogues:
//   EPI_BIAS  Y = acc + bias -> bf16                                   (inference / eval)
//   EPI_NMSE  the HDCE training loss: per row r (stream s, label row rowoff[r]) with coefficient
//             coef_s = 2 / (S den_s), den_s = sum over the stream's rows of |label|^2 (from the
//             gathered per-row powers rowden): dY = coef_s (Y - L) -> bf16 (Y itself is never
//             stored), per-row partial error sums vs label and perfect channel, and per-tile
//             column sums of dY (the bias gradient); qd_fc_nmse_finish reduces the partials.
#include "common.h"

namespace qd {
namespace fcg {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int BN = 128;        // tile columns (4 waves x 32)
constexpr int BK = 64;         // K step (8 x 16-B chunks per row)
constexpr int NT = 256;        // threads per workgroup
constexpr int ROWB = BK * 2;   // LDS row bytes

enum { EPI_BIAS = 0, EPI_NMSE = 1 };

struct NmseArgs {
  const float* label;      // (rows of the store, N) fp32, row rowoff[r]
  const float* perf;       // same, or null
  const int* rowoff;       // (M,)
  const float2* rowden;    // (M,) per-row (|label|^2, |perf|^2)
  uint16_t* dY;            // (M, N) bf16
  float* rowpart;          // (M, n_tiles_n, 2): row partials (err^2, errperf^2) per N-tile
  float* colpart;          // (n_tiles_m, N): per-M-tile column sums of dY
  int E, U, B;             // row r = (u*B + b)*E + e, stream s = e*U + u
  float loss_scale;
};

// byte offset of (row, 16-B chunk c) in a stage image
__device__ __forceinline__ int lds_off(int row, int c) { return row * ROWB + ((c ^ (row & 7)) << 4); }

template <int MF>
struct Cfg {
  static constexpr int BM = 16 * MF;
  static constexpr int A_BYTES = BM * ROWB;
  static constexpr int B_BYTES = BN * ROWB;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int A_PIECES = A_BYTES / 1024;   // 1-KiB global_load_lds pieces (8 rows each)
  static constexpr int B_PIECES = B_BYTES / 1024;
  static_assert(A_BYTES % 1024 == 0, "BM must be a multiple of 8");
};

// One wave-instruction = 1 KiB = 8 rows x 8 chunks; lane l -> LDS row 8p + l/8, slot l%8, which
// holds global chunk (l%8) ^ (row & 7) (the swizzle lives on the SOURCE address, rule 21).
__device__ __forceinline__ void stage_piece(const uint16_t* __restrict__ g, int ld, int row0, int k0, char* lds_base,
                                            int piece, int lane) {
  const int row = piece * 8 + (lane >> 3);
  const int slot = lane & 7;
  const int c = slot ^ (row & 7);
  const uint16_t* src = g + (size_t)(row0 + row) * ld + k0 + c * 8;
  typedef __attribute__((address_space(3))) void lds_void;
  typedef __attribute__((address_space(1))) void glb_void;
  __builtin_amdgcn_global_load_lds((glb_void*)(src), (lds_void*)(lds_base + piece * 1024), 16, 0, 0);
}

template <int MF>
__device__ __forceinline__ void stage(const uint16_t* __restrict__ A, const uint16_t* __restrict__ W, int K, int m0,
                                      int n0, int k0, char* st, int wave, int lane) {
  using C = Cfg<MF>;
  for (int p = wave; p < C::A_PIECES; p += 4) stage_piece(A, K, m0, k0, st, p, lane);
  for (int p = wave; p < C::B_PIECES; p += 4) stage_piece(W, K, n0, k0, st + C::A_BYTES, p, lane);
}

// s_waitcnt vmcnt(n) needs an immediate: this wave's glds count per tile is 8 or 9 (A pieces
// 18 = 5+5+4+4 over the 4 waves when BM = 144, 16 = 4 x 4 when BM = 128; B pieces 4 each)
template <int NPER>
__device__ __forceinline__ void wait_tiles(int tiles) {   // leave `tiles` (0..2) tiles in flight
  if (tiles >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NPER) : "memory");
  else if (tiles == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPER) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int MF>
__device__ __forceinline__ void wait_tiles_w(int tiles, int wave) {
  using C = Cfg<MF>;
  constexpr int lo = C::A_PIECES / 4 + C::B_PIECES / 4;    // pieces of waves >= A_PIECES % 4
  if constexpr (C::A_PIECES % 4 == 0 && C::B_PIECES % 4 == 0) {
    wait_tiles<lo>(tiles);
  } else {
    static_assert(C::B_PIECES % 4 == 0, "B pieces");
    if (wave < C::A_PIECES % 4) wait_tiles<lo + 1>(tiles);
    else wait_tiles<lo>(tiles);
  }
}

constexpr int NSTAGE = 4;     // LDS stages: 3 tiles in flight while one is consumed
constexpr int CPITCH = BN + 4;  // fp32 epilogue tile row pitch (floats): conflict-free column writes

// DBG (diagnosis builds, scripts/probe_fc_hand.py): 1 = no global loads in the K loop (MFMA + LDS reads
// only), 2 = no MFMAs (loads + LDS reads only)
template <int MF, int EPI, int DBG = 0>
__global__ void __launch_bounds__(NT, 1) fc_gemm_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ W,
                                                        const uint16_t* __restrict__ bias, uint16_t* __restrict__ Y,
                                                        int M, int N, int K, NmseArgs na) {
  using C = Cfg<MF>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_m = M / C::BM, tiles_n = N / BN;
  // XCD-aware tile order: blocks bid, bid+8, ... share an XCD; give each XCD whole 4 x 8 tile groups
  // (falls back to row-major order when the grid does not split that way)
  int tm, tn;
  {
    const int bid = blockIdx.x, nwg = gridDim.x;
    if (nwg % 256 == 0 && tiles_m % 4 == 0 && tiles_n % 8 == 0) {
      const int xcd = bid & 7, loc = bid >> 3;
      const int g = xcd * (nwg / 256) + loc / 32;               // 32-tile group
      const int in = loc & 31;
      const int gm = tiles_m / 4;
      tm = (g % gm) * 4 + (in >> 3);
      tn = (g / gm) * 8 + (in & 7);
    } else {
      tm = bid / tiles_n;
      tn = bid % tiles_n;
    }
  }
  const int m0 = tm * C::BM, n0 = tn * BN;

  f32x4 acc[MF][2];
#pragma unroll
  for (int i = 0; i < MF; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- K loop: NSTAGE-deep glds ring, raw barriers (a __syncthreads() would drain the ring) ----
  const int nk = K / BK;
  for (int t = 0; t < NSTAGE - 1 && t < nk; ++t) stage<MF>(A, W, K, m0, n0, t * BK, smem + t * C::STAGE, wave, lane);
  wait_tiles_w<MF>(nk - 1 < NSTAGE - 2 ? nk - 1 : NSTAGE - 2, wave);
  __builtin_amdgcn_s_barrier();

  const int fr = lane & 15, fq = lane >> 4;
  for (int t = 0; t < nk; ++t) {
    const char* cur = smem + (t % NSTAGE) * C::STAGE;
    if (DBG != 1 && t + NSTAGE - 1 < nk)
      stage<MF>(A, W, K, m0, n0, (t + NSTAGE - 1) * BK, smem + ((t + NSTAGE - 1) % NSTAGE) * C::STAGE, wave, lane);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = 4 * s + fq;
      bf16x8 b[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = wave * 32 + j * 16 + fr;
        b[j] = *reinterpret_cast<const bf16x8*>(cur + C::A_BYTES + lds_off(row, c));
      }
#pragma unroll
      for (int i = 0; i < MF; ++i) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(cur + lds_off(i * 16 + fr, c));
        if constexpr (DBG == 2) {
          asm volatile("" ::"v"(a), "v"(b[0]), "v"(b[1]));
        } else {
          acc[i][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[0], acc[i][0], 0, 0, 0);
          acc[i][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[1], acc[i][1], 0, 0, 0);
        }
      }
    }
    // tile t+1 must have landed for everyone: leave the tiles issued beyond it in flight
    const int issued = (t + NSTAGE - 1 < nk ? t + NSTAGE : nk) - 1;   // last tile index issued
    const int ahead = issued - (t + 1);
    wait_tiles_w<MF>(ahead < 0 ? 0 : (ahead > 2 ? 2 : ahead), wave);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }

  // ---------------------------------------------------------------- epilogue
  // accumulators (+ bias) -> fp32 tile [BM][CPITCH] in LDS (the stage ring is free now), then every
  // wave walks whole rows with coalesced 8-byte accesses.  lane holds C[16i + 4fq + r][16j + fr].
  float* ct = reinterpret_cast<float*>(smem);
  static_assert(C::BM * CPITCH * 4 <= NSTAGE * C::STAGE, "epilogue tile");
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int cl = wave * 32 + j * 16 + fr;
    const float bv = bias ? bf16_to_f32(bias[n0 + cl]) : 0.f;
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) ct[(i * 16 + fq * 4 + r) * CPITCH + cl] = acc[i][j][r] + bv;
  }
  __syncthreads();
  const int c2 = 2 * lane;   // this lane's two columns of the tile
  if constexpr (EPI == EPI_BIAS) {
    for (int row = wave; row < C::BM; row += 4) {
      const float2 v = *reinterpret_cast<const float2*>(ct + row * CPITCH + c2);
      const uint32_t w = (uint32_t)f32_to_bf16(v.x) | ((uint32_t)f32_to_bf16(v.y) << 16);
      *reinterpret_cast<uint32_t*>(Y + (size_t)(m0 + row) * N + n0 + c2) = w;
    }
  } else {
    // per-stream coefficients of the streams this tile touches (den_s summed over the stream's B
    // rows in a fixed order: every block gets bitwise-identical values)
    float* red = ct + C::BM * CPITCH;                        // 64 floats after the tile
    const int E = na.E, B = na.B, U = na.U, S = E * U;
    const int ub = B * E;
    const int u_lo = m0 / ub, u_hi = (m0 + C::BM - 1) / ub;
    const int nst = (u_hi - u_lo + 1) * E;
    for (int q = wave; q < nst; q += 4) {
      const int u = u_lo + q / E, e = q % E;
      float a = 0.f;
      for (int b = lane; b < B; b += 64) a += na.rowden[(u * B + b) * E + e].x;
      a = wave_sum(a);
      if (lane == 0) red[q] = na.loss_scale * 2.f / ((float)S * a);
    }
    __syncthreads();
    float cs0 = 0.f, cs1 = 0.f;
    constexpr int RU = 4;                                    // rows per batch (independent loads)
    static_assert(C::BM % (4 * RU) == 0, "rows per wave");
    for (int r0 = wave * RU; r0 < C::BM; r0 += 4 * RU) {
      float2 l[RU], pv[RU];
      int ro[RU];
#pragma unroll
      for (int q = 0; q < RU; ++q) ro[q] = na.rowoff[m0 + r0 + q];
#pragma unroll
      for (int q = 0; q < RU; ++q) {
        const size_t o = (size_t)ro[q] * N + n0 + c2;
        l[q] = *reinterpret_cast<const float2*>(na.label + o);
        pv[q] = na.perf ? *reinterpret_cast<const float2*>(na.perf + o) : make_float2(0.f, 0.f);
      }
#pragma unroll
      for (int q = 0; q < RU; ++q) {
        const int row = m0 + r0 + q;
        const float2 y = *reinterpret_cast<const float2*>(ct + (r0 + q) * CPITCH + c2);
        const float coef = red[(row / ub - u_lo) * E + row % E];
        const float d0 = y.x - l[q].x, d1 = y.y - l[q].y;
        float se = d0 * d0 + d1 * d1, sp = 0.f;
        if (na.perf) {
          const float p0 = y.x - pv[q].x, p1 = y.y - pv[q].y;
          sp = p0 * p0 + p1 * p1;
        }
        const float g0 = coef * d0, g1 = coef * d1;
        cs0 += g0;
        cs1 += g1;
        *reinterpret_cast<uint32_t*>(na.dY + (size_t)row * N + n0 + c2) =
            (uint32_t)f32_to_bf16(g0) | ((uint32_t)f32_to_bf16(g1) << 16);
        se = wave_sum(se);
        sp = wave_sum(sp);
        if (lane == 0) *reinterpret_cast<float2*>(na.rowpart + ((size_t)row * tiles_n + tn) * 2) = make_float2(se, sp);
      }
    }
    // column sums of dY over the tile: the 4 waves' partials combined in a fixed order
    __syncthreads();
    float2* cpart = reinterpret_cast<float2*>(red + 64);
    cpart[wave * 64 + lane] = make_float2(cs0, cs1);
    __syncthreads();
    if (wave == 0) {
      float2 o = cpart[lane];
#pragma unroll
      for (int w = 1; w < 4; ++w) {
        const float2 v = cpart[w * 64 + lane];
        o.x += v.x;
        o.y += v.y;
      }
      *reinterpret_cast<float2*>(na.colpart + (size_t)tm * N + n0 + c2) = o;
    }
  }
}

// Finish: grid = N/64 + 1 blocks.  Blocks 0 .. N/64-1: bias gradient = column sums of colpart
// (fixed order); the last block: loss = (1/S) sum_s sum_{r in s} err_r / den_s (same for perf),
// skip flag, and the per-stream sums ss (S, 4).
__global__ void __launch_bounds__(256) fc_nmse_finish_kernel(const float* __restrict__ colpart, int tiles_m,
                                                             const float* __restrict__ rowpart, int tiles_n,
                                                             const float2* __restrict__ rowden,
                                                             float* __restrict__ bias_grad, float* __restrict__ ss,
                                                             float* __restrict__ loss, float* __restrict__ skip, int N,
                                                             int E, int U, int B) {
  __shared__ float4 red4[16][16];
  __shared__ float sred[4][4];
  if (blockIdx.x < gridDim.x - 1) {
    const int tq = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int c = blockIdx.x * 64 + tq * 4;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int k = ty; k < tiles_m; k += 16) {
      const float4 v = *reinterpret_cast<const float4*>(colpart + (size_t)k * N + c);
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    red4[ty][tq] = a;
    __syncthreads();
    if (threadIdx.x < 16) {
      float4 o = red4[0][threadIdx.x];
#pragma unroll
      for (int j = 1; j < 16; ++j) {
        const float4 v = red4[j][threadIdx.x];
        o.x += v.x; o.y += v.y; o.z += v.z; o.w += v.w;
      }
      *reinterpret_cast<float4*>(bias_grad + blockIdx.x * 64 + threadIdx.x * 4) = o;
    }
    return;
  }
  const int S = E * U, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float l = 0.f, lp = 0.f;
  for (int s = 0; s < S; ++s) {
    const int e = s / U, u = s % U;
    // 4 waves split the stream's B rows; each row's partials over the N tiles in order
    float n = 0.f, np = 0.f, d = 0.f, dp = 0.f;
    for (int b = wv * 64 + lane; b < B; b += 256) {
      const int r = (u * B + b) * E + e;
      const float* p = rowpart + (size_t)r * tiles_n * 2;
      for (int x = 0; x < tiles_n; ++x) {
        n += p[2 * x];
        np += p[2 * x + 1];
      }
      const float2 rd = rowden[r];
      d += rd.x;
      dp += rd.y;
    }
    n = wave_sum(n);
    np = wave_sum(np);
    d = wave_sum(d);
    dp = wave_sum(dp);
    if (lane == 0) {
      sred[wv][0] = n;
      sred[wv][1] = np;
      sred[wv][2] = d;
      sred[wv][3] = dp;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const float N0 = (sred[0][0] + sred[1][0]) + (sred[2][0] + sred[3][0]);
      const float N1 = (sred[0][1] + sred[1][1]) + (sred[2][1] + sred[3][1]);
      const float D0 = (sred[0][2] + sred[1][2]) + (sred[2][2] + sred[3][2]);
      const float D1 = (sred[0][3] + sred[1][3]) + (sred[2][3] + sred[3][3]);
      ss[s * 4 + 0] = N0;
      ss[s * 4 + 1] = D0;
      ss[s * 4 + 2] = N1;
      ss[s * 4 + 3] = D1;
      l += N0 / D0;
      lp += D1 > 0.f ? N1 / D1 : 0.f;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    loss[0] = l / (float)S;
    loss[1] = lp / (float)S;
    if (skip) *skip = isfinite(loss[0]) ? 0.f : 1.f;
  }
}

template <int MF, int EPI, int DBG = 0>
int launch(const uint16_t* A, const uint16_t* W, const uint16_t* bias, uint16_t* Y, int M, int N, int K,
           const NmseArgs& na, hipStream_t st) {
  using C = Cfg<MF>;
  const int smem = NSTAGE * C::STAGE;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&fc_gemm_kernel<MF, EPI, DBG>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  const int grid = (M / C::BM) * (N / BN);
  hipLaunchKernelGGL((fc_gemm_kernel<MF, EPI, DBG>), dim3(grid), dim3(NT), smem, st, A, W, bias, Y, M, N, K, na);
  return (int)hipGetLastError();
}

}  // namespace fcg
}  // namespace qd

using namespace qd::fcg;

// Which M tile a shape takes: 144 rows (9 fragments) when it divides M, else 128; 0 = unsupported.
QD_API int qd_fc_gemm_tile_m(int M, int N, int K) {
  if (N % BN || K % BK || K < BK) return 0;
  if (M % 144 == 0) return 144;
  if (M % 128 == 0) return 128;
  return 0;
}

// Y = A W^T + bias (bias nullable), bf16 everything.  A (M, K), W (N, K), Y (M, N) row-major.
QD_API int qd_fc_gemm_bias(const uint16_t* A, const uint16_t* W, const uint16_t* bias, uint16_t* Y, int M, int N,
                           int K, void* stream) {
  const int tm = qd_fc_gemm_tile_m(M, N, K);
  NmseArgs na{};
  hipStream_t st = (hipStream_t)stream;
  if (tm == 144) return launch<9, EPI_BIAS>(A, W, bias, Y, M, N, K, na, st);
  if (tm == 128) return launch<8, EPI_BIAS>(A, W, bias, Y, M, N, K, na, st);
  return (int)hipErrorInvalidValue;
}

// diagnosis: the bias GEMM with DBG = 1 (no K-loop loads) or 2 (no MFMAs); M % 144 == 0
QD_API int qd_fc_gemm_diag(const uint16_t* A, const uint16_t* W, uint16_t* Y, int M, int N, int K, int dbg,
                           void* stream) {
  NmseArgs na{};
  hipStream_t st = (hipStream_t)stream;
  if (qd_fc_gemm_tile_m(M, N, K) != 144) return (int)hipErrorInvalidValue;
  if (dbg == 1) return launch<9, EPI_BIAS, 1>(A, W, nullptr, Y, M, N, K, na, st);
  if (dbg == 2) return launch<9, EPI_BIAS, 2>(A, W, nullptr, Y, M, N, K, na, st);
  return launch<9, EPI_BIAS, 0>(A, W, nullptr, Y, M, N, K, na, st);
}

// FC forward with the HDCE loss epilogue + finish (see the header).  rows M = U*B*E in (u, b, e)
// order.  rowpart: (M, N/128, 2); colpart: (M/tile_m, N); ss: (S, 4); loss: (2,); bias_grad (N,).
QD_API int qd_fc_gemm_nmse(const uint16_t* A, const uint16_t* W, const uint16_t* bias, const float* label,
                           const float* perf, const int* rowoff, const float* rowden, uint16_t* dY, float* rowpart,
                           float* colpart, float* bias_grad, float* ss, float* loss, float* skip, int M, int N, int K,
                           int E, int U, int B, float loss_scale, void* stream) {
  const int tm = qd_fc_gemm_tile_m(M, N, K);
  if (!tm || M != U * B * E || E < 1 || E > 4 || (tm / (B * E) + 2) * E > 64 || N % 64) return (int)hipErrorInvalidValue;
  NmseArgs na{label, perf, rowoff, reinterpret_cast<const float2*>(rowden), dY, rowpart, colpart, E, U, B,
              loss_scale};
  hipStream_t st = (hipStream_t)stream;
  int rc = tm == 144 ? launch<9, EPI_NMSE>(A, W, bias, nullptr, M, N, K, na, st)
                     : launch<8, EPI_NMSE>(A, W, bias, nullptr, M, N, K, na, st);
  if (rc) return rc;
  hipLaunchKernelGGL(fc_nmse_finish_kernel, dim3(N / 64 + 1), dim3(256), 0, st, colpart, M / tm, rowpart, N / BN,
                     reinterpret_cast<const float2*>(rowden), bias_grad, ss, loss, skip, N, E, U, B);
  return (int)hipGetLastError();
}
