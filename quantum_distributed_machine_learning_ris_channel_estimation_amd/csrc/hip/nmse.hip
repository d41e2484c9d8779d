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

}  // namespace nmse
}  // namespace qd

using namespace qd::nmse;

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
