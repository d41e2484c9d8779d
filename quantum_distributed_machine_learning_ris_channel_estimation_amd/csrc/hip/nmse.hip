// Fused NMSE loss + gradient for the HDCE estimator.
//
// Reference: NMSE_cuda / NMSELoss (Estimators_QuantumNAT_onchipQNN.py:282-295) is a
// batch-GLOBAL ratio sum((x^-x)^2)/sum(x^2); the runner computes it per stream
// (9 calls) against the LS label and against the perfect channel (R:112-113) and sums
// loss/9 (R:195-199).
//
// MI355X design: the 9 streams are one (rows x 2048) activation.  Pass 1 computes
// per-row partial sums (err^2, label^2, errperf^2, perf^2) with one wave per row and
// 16-byte loads; pass 2 (one block) reduces rows by stream in a fixed order
// (deterministic), forms loss, loss_perf and the per-stream gradient coefficients
// 2/(S*den_s), and raises the device `skip` flag if the loss is not finite; pass 3
// writes dY = coef[stream(row)] * (Y - label) directly in the dtype the FC backward
// GEMM consumes (bf16 or fp32).  For data-parallel training the per-stream
// numerators/denominators are all-reduced BEFORE pass 2 (global NMSE, not a mean
// of per-rank ratios) -- see parallel/dp.py.
#include "common.h"

namespace qd {
namespace nmse {

template <typename T>
__device__ __forceinline__ float4 load4(const T* p);
template <>
__device__ __forceinline__ float4 load4<float>(const float* p) {
  return *reinterpret_cast<const float4*>(p);
}
template <>
__device__ __forceinline__ float4 load4<uint16_t>(const uint16_t* p) {
  const ushort4 h = *reinterpret_cast<const ushort4*>(p);
  return make_float4(bf16_to_f32(h.x), bf16_to_f32(h.y), bf16_to_f32(h.z), bf16_to_f32(h.w));
}

// One wave per row; 4 rows per 256-thread block.  out: (rows, 4) fp32.
template <typename TY>
__global__ void __launch_bounds__(256) row_sums_kernel(const TY* __restrict__ Y, const float* __restrict__ Lb,
                                                       const float* __restrict__ Pf, const int* __restrict__ rowoff,
                                                       float* __restrict__ out, int rows, int cols) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const TY* y = Y + (size_t)row * cols;
  const size_t lrow = rowoff ? (size_t)rowoff[row] : (size_t)row;  // labels read in place from the store
  const float* l = Lb + lrow * cols;
  const float* pf = Pf ? Pf + lrow * cols : nullptr;
  float e = 0.f, pw = 0.f, ep = 0.f, pp = 0.f;
  for (int c = lane * 4; c < cols; c += 256) {
    const float4 yv = load4<TY>(y + c);
    const float4 lv = *reinterpret_cast<const float4*>(l + c);
    const float d0 = yv.x - lv.x, d1 = yv.y - lv.y, d2 = yv.z - lv.z, d3 = yv.w - lv.w;
    e += d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
    pw += lv.x * lv.x + lv.y * lv.y + lv.z * lv.z + lv.w * lv.w;
    if (pf) {
      const float4 pv = *reinterpret_cast<const float4*>(pf + c);
      const float q0 = yv.x - pv.x, q1 = yv.y - pv.y, q2 = yv.z - pv.z, q3 = yv.w - pv.w;
      ep += q0 * q0 + q1 * q1 + q2 * q2 + q3 * q3;
      pp += pv.x * pv.x + pv.y * pv.y + pv.z * pv.z + pv.w * pv.w;
    }
  }
  e = wave_sum(e);
  pw = wave_sum(pw);
  ep = wave_sum(ep);
  pp = wave_sum(pp);
  if (lane == 0) {
    float4 o = make_float4(e, pw, ep, pp);
    *reinterpret_cast<float4*>(out + (size_t)row * 4) = o;
  }
}

// Per-stream reduction (rows in index order -> deterministic).  stream_sums: (S,4).
__global__ void __launch_bounds__(1024) stream_sums_kernel(const float* __restrict__ rowsums,
                                                           const int* __restrict__ row_stream, float* __restrict__ ss,
                                                           int rows, int S) {
  const int s = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  for (int r = lane; r < rows; r += 64) {
    if (row_stream[r] != s) continue;
    const float4 v = *reinterpret_cast<const float4*>(rowsums + (size_t)r * 4);
    a0 += v.x;
    a1 += v.y;
    a2 += v.z;
    a3 += v.w;
  }
  a0 = wave_sum(a0);
  a1 = wave_sum(a1);
  a2 = wave_sum(a2);
  a3 = wave_sum(a3);
  if (lane == 0) *reinterpret_cast<float4*>(ss + s * 4) = make_float4(a0, a1, a2, a3);
}

// Fused stream reduction + finalize: wave s sums the partials of stream s's rows, listed by a
// CSR index (order[off[s] .. off[s+1]), built once on the host), in a fixed order
// (deterministic); thread 0 then finalises.  blockDim = 64 * S (S <= 16).
__global__ void __launch_bounds__(1024) stream_reduce_finalize_kernel(const float* __restrict__ rowsums,
                                                                      const int* __restrict__ order,
                                                                      const int* __restrict__ off,
                                                                      float* __restrict__ ss, float* __restrict__ loss,
                                                                      float* __restrict__ coef, float* __restrict__ skip,
                                                                      int S, float loss_scale) {
  const int s = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  const int beg = off[s], end = off[s + 1];
#pragma unroll 4
  for (int j = beg + lane; j < end; j += 64) {
    const float4 v = *reinterpret_cast<const float4*>(rowsums + (size_t)order[j] * 4);
    a0 += v.x;
    a1 += v.y;
    a2 += v.z;
    a3 += v.w;
  }
  a0 = wave_sum(a0);
  a1 = wave_sum(a1);
  a2 = wave_sum(a2);
  a3 = wave_sum(a3);
  if (lane == 0) *reinterpret_cast<float4*>(ss + s * 4) = make_float4(a0, a1, a2, a3);
  __syncthreads();
  if (threadIdx.x == 0) {
    float l = 0.f, lp = 0.f;
    for (int k = 0; k < S; ++k) {
      const float den = ss[k * 4 + 1];
      l += ss[k * 4 + 0] / den;
      const float denp = ss[k * 4 + 3];
      lp += denp > 0.f ? ss[k * 4 + 2] / denp : 0.f;
      coef[k] = loss_scale * 2.f / ((float)S * den);
    }
    loss[0] = l / (float)S;
    loss[1] = lp / (float)S;
    if (skip) *skip = isfinite(loss[0]) ? 0.f : 1.f;
  }
}

// loss = sum_s num_s/den_s / S (same for perf); coef_s = 2/(S den_s); skip if non-finite.
__global__ void finalize_kernel(const float* __restrict__ ss, float* __restrict__ loss, float* __restrict__ coef,
                                float* __restrict__ skip, int S, float loss_scale) {
  if (threadIdx.x != 0) return;
  float l = 0.f, lp = 0.f;
  for (int s = 0; s < S; ++s) {
    const float den = ss[s * 4 + 1];
    l += ss[s * 4 + 0] / den;
    const float denp = ss[s * 4 + 3];
    lp += denp > 0.f ? ss[s * 4 + 2] / denp : 0.f;
    coef[s] = loss_scale * 2.f / ((float)S * den);
  }
  loss[0] = l / (float)S;
  loss[1] = lp / (float)S;
  if (skip) *skip = isfinite(loss[0]) ? 0.f : 1.f;
}

template <typename TY, typename TD>
__global__ void __launch_bounds__(256) grad_kernel(const TY* __restrict__ Y, const float* __restrict__ Lb,
                                                   const float* __restrict__ coef, const int* __restrict__ row_stream,
                                                   const int* __restrict__ rowoff, TD* __restrict__ dY, int rows,
                                                   int cols) {
  const long n4 = (long)rows * cols / 4;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const long e = i * 4;
    const int r = (int)(e / cols);
    const float c = coef[row_stream[r]];
    const float4 yv = load4<TY>(Y + e);
    const size_t le = rowoff ? (size_t)rowoff[r] * cols + (e - (long)r * cols) : (size_t)e;
    const float4 lv = *reinterpret_cast<const float4*>(Lb + le);
    const float g0 = c * (yv.x - lv.x), g1 = c * (yv.y - lv.y), g2 = c * (yv.z - lv.z), g3 = c * (yv.w - lv.w);
    if constexpr (std::is_same<TD, float>::value) {
      *reinterpret_cast<float4*>(dY + e) = make_float4(g0, g1, g2, g3);
    } else {
      ushort4 h;
      h.x = f32_to_bf16(g0);
      h.y = f32_to_bf16(g1);
      h.z = f32_to_bf16(g2);
      h.w = f32_to_bf16(g3);
      *reinterpret_cast<ushort4*>(dY + e) = h;
    }
  }
}

// Same gradient, column-blocked so the FC bias gradient falls out of it: grid (cols / 1024, RB),
// thread = 4 columns x the rows of chunk blockIdx.y; colsum slab (RB, cols) gets each chunk's fp32
// column sums of dY (reduced afterwards by qd_slab_rows_sum: deterministic, no atomics).
template <typename TY, typename TD>
__global__ void __launch_bounds__(256) grad_bias_kernel(const TY* __restrict__ Y, const float* __restrict__ Lb,
                                                        const float* __restrict__ coef,
                                                        const int* __restrict__ row_stream,
                                                        const int* __restrict__ rowoff, TD* __restrict__ dY,
                                                        float* __restrict__ colsum, int rows, int cols, int rpc) {
  const int c0 = (blockIdx.x * 256 + threadIdx.x) * 4;
  const int r0 = blockIdx.y * rpc, r1 = min(rows, r0 + rpc);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c0 < cols) {
    for (int r = r0; r < r1; ++r) {
      const size_t e = (size_t)r * cols + c0;
      const float c = coef[row_stream[r]];
      const float4 yv = load4<TY>(Y + e);
      const size_t le = rowoff ? (size_t)rowoff[r] * cols + c0 : e;
      const float4 lv = *reinterpret_cast<const float4*>(Lb + le);
      const float g0 = c * (yv.x - lv.x), g1 = c * (yv.y - lv.y), g2 = c * (yv.z - lv.z), g3 = c * (yv.w - lv.w);
      acc.x += g0;
      acc.y += g1;
      acc.z += g2;
      acc.w += g3;
      if constexpr (std::is_same<TD, float>::value) {
        *reinterpret_cast<float4*>(dY + e) = make_float4(g0, g1, g2, g3);
      } else {
        ushort4 h;
        h.x = f32_to_bf16(g0);
        h.y = f32_to_bf16(g1);
        h.z = f32_to_bf16(g2);
        h.w = f32_to_bf16(g3);
        *reinterpret_cast<ushort4*>(dY + e) = h;
      }
    }
    *reinterpret_cast<float4*>(colsum + (size_t)blockIdx.y * cols + c0) = acc;
  }
}

// ---------------------------------------------------------------------------------------------
// One-pass loss + gradient for the grouped estimator's row order r = (u*B + b)*E + e (stream
// s = e*U + u), labels read in place through rowoff.  The gradient coefficient 2/(S*den_s) only
// needs den_s = sum |label|^2 over the stream's rows, which is known BEFORE Y: every block sums
// the precomputed per-row label powers (rowpow_l[rowoff[r]], dataset-constant) of its u-block's
// E streams itself, in a fixed order (bitwise identical in every block).  So one pass over
// (Y, label, perf) writes dY, the FC bias-gradient column partials, and the per-stream error
// partials; nmse_finish_kernel then forms loss / loss_perf / skip and sums the bias partials.
//
// block (bx, by): columns 4*(256*bx + t) .. +3, rows [by*rpc, (by+1)*rpc) -- rpc a multiple of E
// dividing B*E, so a chunk lies in one u-block and walks its rows in e-triples (static indices).
// part: (gridDim.y, gridDim.x, E, 2) fp32 = (sum err^2, sum errperf^2) of the block per e.
// dens: (S, 2) = (den, den_perf), written by the blocks with bx == 0 and by at a u-block start.
template <typename TY, typename TD, int E>
__global__ void __launch_bounds__(256) nmse_fused_kernel(const TY* __restrict__ Y, const float* __restrict__ Lb,
                                                         const float* __restrict__ Pf, const int* __restrict__ rowoff,
                                                         const float* __restrict__ rowpow_l,
                                                         const float* __restrict__ rowpow_p, TD* __restrict__ dY,
                                                         float* __restrict__ colsum, float* __restrict__ part,
                                                         float* __restrict__ dens, int cols, int B, int U, int rpc,
                                                         float loss_scale, const float2* __restrict__ rowden) {
  __shared__ float sden[2 * E];
  __shared__ float sred[4][2 * E];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int r0 = blockIdx.y * rpc;
  const int u = r0 / (B * E);
  const int S = E * U;
  const int c0 = (blockIdx.x * 256 + t) * 4;
  const bool act = c0 < cols;
  // The block's rows in batches of RT: a batch's rowoff, Y, label and perf loads are all issued before
  // any of them is used (rowoff -> label is the only dependent pair), and the first batch is issued
  // BEFORE the per-stream label powers below, so the whole block pays ~2 memory round trips instead of
  // one per phase (rowden -> barrier -> rowoff -> label, per batch).
  // (2E rows per round: 4E in one round measured 27.3 vs 16.5 us in the step -- 196 VGPRs halve the occupancy,
  // profiles/r4_25_step_kernel_stats.md)
  constexpr int RT = 2 * E;
  const int r1 = r0 + rpc;
  int ro[RT];
  float4 yv[RT], lv[RT], pv[RT];
  // (branch-free: a row past the block's end re-loads row rb and is never used -- guarded loads compiled to one
  // dependent round trip per rowoff, each behind its own vmcnt(0), before the first label load could issue)
  auto issue = [&](int rb) {
#pragma unroll
    for (int q = 0; q < RT; ++q) ro[q] = rowoff[rb + q < r1 ? rb + q : rb];
#pragma unroll
    for (int q = 0; q < RT; ++q) yv[q] = load4<TY>(Y + (size_t)(rb + q < r1 ? rb + q : rb) * cols + c0);
#pragma unroll
    for (int q = 0; q < RT; ++q) {
      const size_t le = (size_t)ro[q] * cols + c0;
      lv[q] = *reinterpret_cast<const float4*>(Lb + le);
      pv[q] = Pf ? *reinterpret_cast<const float4*>(Pf + le) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  if (act) issue(r0);
  // per-stream label powers of this u-block (wave e: stream e*U + u), fixed order
  for (int e = wv; e < E; e += 4) {
    float a = 0.f, ap = 0.f;
    if (rowden) {   // (gathered per-row powers: independent loads, no rowoff -> rowpow chain)
      // up to 8 rows per lane in flight at once (a loop of guarded loads waited one round trip per row), then
      // the same additions in the same order; rows beyond 512 per stream in the tail loop
      constexpr int NB = 8;
      float2 rv[NB];
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int b = lane + 64 * i < B ? lane + 64 * i : lane < B ? lane : 0;
        rv[i] = rowden[(u * B + b) * E + e];
      }
#pragma unroll
      for (int i = 0; i < NB; ++i)
        if (lane + 64 * i < B) {
          a += rv[i].x;
          ap += Pf ? rv[i].y : 0.f;
        }
      for (int b = lane + 64 * NB; b < B; b += 64) {
        const float2 v = rowden[(u * B + b) * E + e];
        a += v.x;
        ap += Pf ? v.y : 0.f;
      }
    } else {
      for (int b = lane; b < B; b += 64) {
        const int ro = rowoff[(u * B + b) * E + e];
        a += rowpow_l[ro];
        ap += Pf ? rowpow_p[ro] : 0.f;
      }
    }
    a = wave_sum(a);
    ap = wave_sum(ap);
    if (lane == 0) {
      sden[e] = a;
      sden[E + e] = ap;
    }
  }
  __syncthreads();
  if (blockIdx.x == 0 && r0 % (B * E) == 0 && t < E) {
    dens[(t * U + u) * 2 + 0] = sden[t];
    dens[(t * U + u) * 2 + 1] = sden[E + t];
  }
  float coef[E];
#pragma unroll
  for (int e = 0; e < E; ++e) coef[e] = loss_scale * 2.f / ((float)S * sden[e]);
  float num[E], nump[E];
#pragma unroll
  for (int e = 0; e < E; ++e) num[e] = nump[e] = 0.f;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (act) {
    for (int rb = r0; rb < r1; rb += RT) {
      if (rb != r0) issue(rb);
#pragma unroll
      for (int q = 0; q < RT; ++q) {
        if (rb + q >= r1) break;   // (rpc % E == 0: whole e-triples)
        const int e = q % E;
        const size_t ey = (size_t)(rb + q) * cols + c0;
        const float4 y = yv[q], l = lv[q];
        const float d0 = y.x - l.x, d1 = y.y - l.y, d2 = y.z - l.z, d3 = y.w - l.w;
        num[e] += d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
        if (Pf) {
          const float4 p = pv[q];
          const float q0 = y.x - p.x, q1 = y.y - p.y, q2 = y.z - p.z, q3 = y.w - p.w;
          nump[e] += q0 * q0 + q1 * q1 + q2 * q2 + q3 * q3;
        }
        const float c = coef[e];
        const float g0 = c * d0, g1 = c * d1, g2 = c * d2, g3 = c * d3;
        acc.x += g0;
        acc.y += g1;
        acc.z += g2;
        acc.w += g3;
        if constexpr (std::is_same<TD, float>::value) {
          *reinterpret_cast<float4*>(dY + ey) = make_float4(g0, g1, g2, g3);
        } else {
          ushort4 h;
          h.x = f32_to_bf16(g0);
          h.y = f32_to_bf16(g1);
          h.z = f32_to_bf16(g2);
          h.w = f32_to_bf16(g3);
          *reinterpret_cast<ushort4*>(dY + ey) = h;
        }
      }
    }
    *reinterpret_cast<float4*>(colsum + (size_t)blockIdx.y * cols + c0) = acc;
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const float a = wave_sum(num[e]), b = wave_sum(nump[e]);
    if (lane == 0) {
      sred[wv][2 * e] = a;
      sred[wv][2 * e + 1] = b;
    }
  }
  __syncthreads();
  if (t < 2 * E) {
    const float v = sred[0][t] + sred[1][t] + sred[2][t] + sred[3][t];
    part[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 2 * E + t] = v;
  }
}

// blocks 0 .. cols/64-1: 64 bias-gradient columns each (16 threads x float4 per row, 16 row groups,
// fixed-order LDS combine: deterministic); the LAST block's first wave reduces the error partials
// per stream and finalises loss, loss_perf and skip.
template <int E>
__global__ void __launch_bounds__(256) nmse_finish_kernel(const float* __restrict__ colsum,
                                                          const float* __restrict__ part,
                                                          const float* __restrict__ dens, float* __restrict__ bias_grad,
                                                          float* __restrict__ ss, float* __restrict__ loss,
                                                          float* __restrict__ skip, int chunks, int gx, int cols,
                                                          int chunks_per_u, int U) {
  __shared__ float4 red[16][16];
  if (blockIdx.x < gridDim.x - 1) {
    const int tq = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int c = blockIdx.x * 64 + tq * 4;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
    int k = ty;
    for (; k + 16 < chunks; k += 32) {   // two independent loads in flight per thread
      const float4 v = *reinterpret_cast<const float4*>(colsum + (size_t)k * cols + c);
      const float4 w = *reinterpret_cast<const float4*>(colsum + (size_t)(k + 16) * cols + c);
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
      b.x += w.x; b.y += w.y; b.z += w.z; b.w += w.w;
    }
    if (k < chunks) {
      const float4 v = *reinterpret_cast<const float4*>(colsum + (size_t)k * cols + c);
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    red[ty][tq] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
    __syncthreads();
    if (threadIdx.x < 16) {
      float4 o = red[0][threadIdx.x];
#pragma unroll
      for (int j = 1; j < 16; ++j) {
        const float4 v = red[j][threadIdx.x];
        o.x += v.x; o.y += v.y; o.z += v.z; o.w += v.w;
      }
      *reinterpret_cast<float4*>(bias_grad + blockIdx.x * 64 + threadIdx.x * 4) = o;
    }
    return;
  }
  loss_finish_body(LossFinish{part, dens, ss, loss, skip, gx, chunks_per_u, U, E});
}

}  // namespace nmse
}  // namespace qd

using namespace qd::nmse;

// One-pass NMSE + dY + bias gradient (see nmse_fused_kernel).  rows = U*B*E; rpc % E == 0 and
// (B*E) % rpc == 0; cols % 1024 == 0.  colsum: (rows/rpc, cols); part: (rows/rpc, cols/1024, E, 2);
// dens: (S, 2); ss: (S, 4) as qd_nmse_reduce_finalize's.  perf / rowpow_p nullable together.
// finish_bias = 0: the finish launch only forms the loss; the caller reduces colsum -> bias_grad itself
// (e.g. as one job of a later batched slab reduction, off the critical path).  finish_bias = 2: no
// finish launch at all -- the caller runs the loss finish (LossFinish over part / dens / ss / loss /
// skip, gx = cols / 1024, chunks_per_u = B*E / rpc) in a later launch (qd_bn_bwd_reduce's lf).
QD_API int qd_nmse_fused(const void* Y, int y_bf16, const float* label, const float* perf, const int* rowoff,
                         const float* rowpow_l, const float* rowpow_p, void* dY, int dy_bf16, float* colsum,
                         float* part, float* dens, float* bias_grad, float* ss, float* loss, float* skip, int E, int U,
                         int B, int cols, int rpc, float loss_scale, const float* rowden, int finish_bias,
                         void* stream) {
  if (cols % 1024 || rpc < E || rpc % E || (B * E) % rpc || (perf == nullptr) != (rowpow_p == nullptr))
    return (int)hipErrorInvalidValue;
  const int rows = U * B * E;
  dim3 grid(cols / 1024, rows / rpc);
  hipStream_t st = (hipStream_t)stream;
#define QD_F(TY, TD, EE)                                                                                            \
  hipLaunchKernelGGL((nmse_fused_kernel<TY, TD, EE>), grid, dim3(256), 0, st, (const TY*)Y, label, perf, rowoff,     \
                     rowpow_l, rowpow_p, (TD*)dY, colsum, part, dens, cols, B, U, rpc, loss_scale,              \
                     reinterpret_cast<const float2*>(rowden))
#define QD_E(EE)                                          \
  if (y_bf16 && dy_bf16) QD_F(uint16_t, uint16_t, EE);    \
  else if (y_bf16) QD_F(uint16_t, float, EE);             \
  else if (dy_bf16) QD_F(float, uint16_t, EE);            \
  else QD_F(float, float, EE);
  switch (E) {
    case 1: QD_E(1) break;
    case 2: QD_E(2) break;
    case 3: QD_E(3) break;
    case 4: QD_E(4) break;
    default: return (int)hipErrorInvalidValue;
  }
#undef QD_E
#undef QD_F
  if (finish_bias == 2) return (int)hipGetLastError();
  const int chunks = rows / rpc;
#define QD_N(EE)                                                                                                   \
  hipLaunchKernelGGL((nmse_finish_kernel<EE>), dim3(finish_bias ? cols / 64 + 1 : 1),                          \
                     dim3(256), 0, st, colsum, part, dens, bias_grad, ss, \
                     loss, skip, chunks, (int)grid.x, cols, (B * E) / rpc, U)
  switch (E) {
    case 1: QD_N(1); break;
    case 2: QD_N(2); break;
    case 3: QD_N(3); break;
    default: QD_N(4); break;
  }
#undef QD_N
  return (int)hipGetLastError();
}

// dY as qd_nmse_grad, plus colsum (chunks, cols) = per-row-chunk column sums of dY (bias gradient
// partials).  cols % 4 == 0.
QD_API int qd_nmse_grad_bias(const void* Y, int y_bf16, const float* label, const float* coef, const int* row_stream,
                             const int* rowoff, void* dY, int dy_bf16, float* colsum, int chunks, int rows, int cols,
                             void* stream) {
  if (cols % 4 || chunks < 1) return (int)hipErrorInvalidValue;
  const int rpc = (rows + chunks - 1) / chunks;
  dim3 grid((cols / 4 + 255) / 256, chunks);
  hipStream_t st = (hipStream_t)stream;
#define QD_G(TY, TD)                                                                                          \
  hipLaunchKernelGGL((grad_bias_kernel<TY, TD>), grid, dim3(256), 0, st, (const TY*)Y, label, coef, row_stream, \
                     rowoff, (TD*)dY, colsum, rows, cols, rpc)
  if (y_bf16 && dy_bf16) QD_G(uint16_t, uint16_t);
  else if (y_bf16) QD_G(uint16_t, float);
  else if (dy_bf16) QD_G(float, uint16_t);
  else QD_G(float, float);
#undef QD_G
  return (int)hipGetLastError();
}

// y_bf16: 1 if Y is bf16 else fp32.  perf may be null.  rowoff (nullable): label/perf row of
// output row r (labels gathered in place from the dataset store).
QD_API int qd_nmse_row_sums(const void* Y, int y_bf16, const float* label, const float* perf, const int* rowoff,
                            float* rowsums, int rows, int cols, void* stream) {
  if (cols % 4) return (int)hipErrorInvalidValue;
  dim3 grid((rows + 3) / 4);
  if (y_bf16)
    hipLaunchKernelGGL(row_sums_kernel<uint16_t>, grid, dim3(256), 0, (hipStream_t)stream, (const uint16_t*)Y, label,
                       perf, rowoff, rowsums, rows, cols);
  else
    hipLaunchKernelGGL(row_sums_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, (const float*)Y, label, perf,
                       rowoff, rowsums, rows, cols);
  return (int)hipGetLastError();
}

QD_API int qd_nmse_stream_sums(const float* rowsums, const int* row_stream, float* ss, int rows, int S, void* stream) {
  if (S < 1 || S > 16) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(stream_sums_kernel, dim3(1), dim3(64 * S), 0, (hipStream_t)stream, rowsums, row_stream, ss, rows,
                     S);
  return (int)hipGetLastError();
}

// order/off: CSR list of every stream's rows (host-built once).
QD_API int qd_nmse_reduce_finalize(const float* rowsums, const int* order, const int* off, float* ss, float* loss,
                                   float* coef, float* skip, int S, float loss_scale, void* stream) {
  if (S < 1 || S > 16) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(stream_reduce_finalize_kernel, dim3(1), dim3(64 * S), 0, (hipStream_t)stream, rowsums, order, off,
                     ss, loss, coef, skip, S, loss_scale);
  return (int)hipGetLastError();
}

QD_API int qd_nmse_finalize(const float* ss, float* loss, float* coef, float* skip, int S, float loss_scale,
                            void* stream) {
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, ss, loss, coef, skip, S, loss_scale);
  return (int)hipGetLastError();
}

QD_API int qd_nmse_grad(const void* Y, int y_bf16, const float* label, const float* coef, const int* row_stream,
                        const int* rowoff, void* dY, int dy_bf16, int rows, int cols, void* stream) {
  if (cols % 4) return (int)hipErrorInvalidValue;
  long n4 = (long)rows * cols / 4;
  int grid = (int)((n4 + 255) / 256);
  if (grid > 4096) grid = 4096;
  hipStream_t st = (hipStream_t)stream;
#define QD_G(TY, TD) hipLaunchKernelGGL((grad_kernel<TY, TD>), dim3(grid), dim3(256), 0, st, (const TY*)Y, label, coef, \
                                        row_stream, rowoff, (TD*)dY, rows, cols)
  if (y_bf16 && dy_bf16) QD_G(uint16_t, uint16_t);
  else if (y_bf16) QD_G(uint16_t, float);
  else if (dy_bf16) QD_G(float, uint16_t);
  else QD_G(float, float);
#undef QD_G
  return (int)hipGetLastError();
}

// The finish launch alone, for producers other than qd_nmse_fused (csrc/hip/gemm.hip's forward GEMM
// with the loss epilogue): colsum (chunks, cols) -> bias_grad when finish_bias, and the loss finish
// over part (chunks_per_u * U, gx, E, 2) / dens (S, 2).
QD_API int qd_nmse_finish(const float* colsum, int chunks, const float* part, int gx, int chunks_per_u,
                          const float* dens, float* bias_grad, float* ss, float* loss, float* skip, int cols, int U,
                          int E, int finish_bias, void* stream) {
  if (cols % 64 || E < 1 || E > 4) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
#define QD_N(EE)                                                                                               \
  hipLaunchKernelGGL((nmse_finish_kernel<EE>), dim3(finish_bias ? cols / 64 + 1 : 1), dim3(256), 0, st, colsum, \
                     part, dens, bias_grad, ss, loss, skip, chunks, gx, cols, chunks_per_u, U)
  switch (E) {
    case 1: QD_N(1); break;
    case 2: QD_N(2); break;
    case 3: QD_N(3); break;
    default: QD_N(4); break;
  }
#undef QD_N
  return (int)hipGetLastError();
}
