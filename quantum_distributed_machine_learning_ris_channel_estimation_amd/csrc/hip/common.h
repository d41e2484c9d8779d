// Shared helpers for the CDNA4 (gfx950) kernels of this framework.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp8.h>
#include <stdint.h>
#include <type_traits>

#define QD_API extern "C" __attribute__((visibility("default")))

namespace qd {

constexpr int kWave = 64;  // CDNA wavefront width (never 32)

// Compile-time loop: f(std::integral_constant<int, I>) for I in [B, E).
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// Orders LDS traffic of ONE wave without a workgroup barrier: LDS instructions of a
// wave execute in order, so only the compiler must be kept from reordering.
__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// One element of an Adam step (moments and weight in place; g already scaled / decayed / pruned).  Every
// rounding step is an explicit intrinsic, so no FMA contraction choice of the compiler can differ between
// the kernels that apply it: csrc/hip/optim.hip's update kernel and csrc/hip/gemm.hip's fused
// weight-gradient epilogue give bitwise-identical weights and moments.
__device__ __forceinline__ void adam_elem(float& p, float& m, float& v, float g, float beta1, float beta2, float eps,
                                          float step_size, float rbc2) {
  m = __fmaf_rn(beta1, m, __fmul_rn(1.f - beta1, g));
  v = __fmaf_rn(beta2, v, __fmul_rn(__fmul_rn(1.f - beta2, g), g));
  const float denom = __fmaf_rn(__fsqrt_rn(v), rbc2, eps);
  p = __fmaf_rn(-step_size, __fdiv_rn(m, denom), p);
}

// Diagnostic phase stamp (stamped kernel builds only): s_memtime with its own lgkmcnt wait, fenced
// by scheduling barriers so the compiler keeps each phase's work on its side of the stamp.
__device__ __forceinline__ unsigned long long phase_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

// BatchNorm + ReLU backward pieces with every rounding explicit.  The same quantities are computed in several kernels
// (conv.hip: the dgrad / wgrad / fused-backward stagings, the BN-reduction epilogues and launch; gemm.hip: the FC data
// gradient's BN-reduction epilogue); with plain expressions each kernel's FMA contraction (-ffp-contract=fast) was
// the compiler's choice in that context, so a dz could differ by one bf16 rounding between two kernels computing
// the same thing.  Explicit: bitwise the same values in every kernel.
//   gate  : the ReLU passed, a z + b > 0 (fma)           xhat : (z - mean) * invstd
//   dz    : c1 g - c2 - c3 xhat                           red  : s1 += g, s2 += g xhat (fma)
__device__ __forceinline__ bool bn_gate(float a, float z, float b) { return __fmaf_rn(a, z, b) > 0.f; }
__device__ __forceinline__ float bn_xhat(float z, float mu, float inv) { return __fmul_rn(__fsub_rn(z, mu), inv); }
__device__ __forceinline__ float bn_dz(float g, float xh, float c1, float c2, float c3) {
  return __fsub_rn(__fsub_rn(__fmul_rn(c1, g), c2), __fmul_rn(c3, xh));
}
__device__ __forceinline__ void bn_red(float& s1, float& s2, float g, float xh) {
  s1 = __fadd_rn(s1, g);
  s2 = __fmaf_rn(g, xh, s2);
}

// torch semantics for non-finite inputs: relu / max propagate NaN (v_max_f32 would return the non-NaN
// operand and silently turn a NaN batch into zeros -- and a finite loss the NaN guard never sees)
__device__ __forceinline__ float relu_nan(float v) { return v < 0.f ? 0.f : v; }
// the same as one v_maximum3_f32 (IEEE-754-2019 maximum: NaN in, NaN out; -0 -> +0).  Not the default: in the
// QSC kernels it changed the register allocation (qsc2_fwd 209 -> 222 VGPRs)
__device__ __forceinline__ float relu_max(float v) { return __builtin_elementwise_maximum(v, 0.f); }
__device__ __forceinline__ float max_nan(float a, float b) { return (a > b || a != a) ? a : b; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m));
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64); result valid in every thread.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red /* >= NT/64 floats */) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += red[i];
  __syncthreads();
  return t;
}

__device__ __forceinline__ float bf16_to_f32(uint16_t h) {
  return __uint_as_float(static_cast<uint32_t>(h) << 16);
}
// Round-to-nearest-even f32 -> bf16 (NaN-preserving via the compiler's cvt).
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  __hip_bfloat16 b = __float2bfloat16(f);
  return *reinterpret_cast<uint16_t*>(&b);
}

// Opt a kernel in to more than 64 KiB of dynamic LDS (gfx950 has 160 KiB per CU).
template <class K>
inline hipError_t allow_lds(K kernel, size_t bytes) {
  if (bytes <= 65536) return hipSuccess;
  return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)bytes);
}

// fp32 -> OCP e4m3 (gfx950 native format) with the packed hardware converter; inputs clamped to
// the finite range first (saturating semantics).  pack4 returns 4 bytes (a, b, c, d) little-endian.
constexpr float kE4M3Max = 448.f;
__device__ __forceinline__ uint32_t e4m3_pack4(float a, float b, float c, float d) {
  a = fminf(fmaxf(a, -kE4M3Max), kE4M3Max);
  b = fminf(fmaxf(b, -kE4M3Max), kE4M3Max);
  c = fminf(fmaxf(c, -kE4M3Max), kE4M3Max);
  d = fminf(fmaxf(d, -kE4M3Max), kE4M3Max);
  int p = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  p = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, p, true);
  return (uint32_t)p;
}
__device__ __forceinline__ uint8_t f32_to_e4m3(float v) { return (uint8_t)(e4m3_pack4(v, 0.f, 0.f, 0.f) & 0xffu); }

// Per-workgroup |x| max for delayed fp8 scaling: part[blockIdx.x] = max(part[blockIdx.x], block max).
// No atomics (one contended address per wave serialised ~16k atomics in L2: 8 -> 192 us); the
// scale-update kernel reduces the partials.  Every thread of the block must call it.
__device__ __forceinline__ void amax_block_store(float* part, float local_absmax) {
  __shared__ float wmax[16];
  float m = local_absmax;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float b = 0.f;
    for (int w = 0; w < (int)(blockDim.x + 63) / 64; ++w) b = fmaxf(b, wmax[w]);
    part[blockIdx.x] = fmaxf(part[blockIdx.x], b);
  }
}
constexpr int kAmaxParts = 4096;   // partial slots per scaled tensor (>= any producer grid)

// HDCE loss finish (nmse.hip's one-pass kernel leaves per-block error partials): per-stream sums,
// loss = mean_s err_s / den_s (and the perfect-channel variant), NaN-guard flag.  A block-wide body
// (every thread of a 256-thread block calls it) so that any later launch of the step can host it as
// one extra workgroup -- nmse_finish_kernel, or the BN backward reduction (one launch fewer).
struct LossFinish {
  const float* part;   // (chunks, gx, E, 2)
  const float* dens;   // (S, 2)
  float* ss;           // (S, 4) scratch
  float* loss;         // (2,)
  float* skip;         // (1,) nullable
  int gx, chunks_per_u, U, E;
};
__device__ inline void loss_finish_body(const LossFinish& f) {
  // wave w takes streams w, w + waves, ... (each in a fixed order); then thread 0 forms the loss over
  // the streams in order (deterministic)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int E = f.E, U = f.U, S = E * U;
  for (int s = wv; s < S; s += nw) {
    const int e = s / U, u = s % U;
    float n = 0.f, np = 0.f;
    for (int j = lane; j < f.chunks_per_u * f.gx; j += 64) {
      const int k = u * f.chunks_per_u + j / f.gx, x = j % f.gx;
      const float* p = f.part + ((size_t)k * f.gx + x) * 2 * E + 2 * e;
      n += p[0];
      np += p[1];
    }
    n = wave_sum(n);
    np = wave_sum(np);
    if (lane == 0) {
      f.ss[s * 4 + 0] = n;
      f.ss[s * 4 + 1] = f.dens[s * 2];
      f.ss[s * 4 + 2] = np;
      f.ss[s * 4 + 3] = f.dens[s * 2 + 1];
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float l = 0.f, lp = 0.f;
    for (int s = 0; s < S; ++s) {
      l += f.ss[s * 4 + 0] / f.ss[s * 4 + 1];
      lp += f.ss[s * 4 + 3] > 0.f ? f.ss[s * 4 + 2] / f.ss[s * 4 + 3] : 0.f;
    }
    f.loss[0] = l / (float)S;
    f.loss[1] = lp / (float)S;
    if (f.skip) *f.skip = isfinite(f.loss[0]) ? 0.f : 1.f;
  }
}

}  // namespace qd
