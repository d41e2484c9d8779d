// Fused flat-buffer optimizers (Adam / AdamW / SGD-momentum) for gfx950.
//
// Reference: Y2HRunner.get_optimizer (Runner_P128_QuantumNAT_onchipQNN.py:40-46):
// Adam(lr) for each of the 4 HDCE modules (R:160-163), SGD(lr, momentum 0.9), and
// AdamW(lr, wd=0.01) for the QSC (R:320); on-chip gradient pruning
// g *= (|g| > thr) over all QSC parameters (E:205-228).
//
// MI355X design: every parameter of a model lives in ONE flat fp32 buffer (grads,
// moments likewise), so a whole optimizer step is one launch of a grid-stride
// kernel at HBM rate.  All step-dependent scalars (step count, learning rate) are
// read from DEVICE memory, so the launch can be captured once in a HIP graph and
// replayed every step; `skip` (set by the loss kernel when the loss is not finite)
// turns the step into a no-op without a host sync.  Gradient pruning and the DP
// gradient scale (1/world) are fused into the same pass, and so are
//   * the step-counter increment: the last workgroup to finish (device-wide done counter)
//     bumps it, so a step is one launch, not two;
//   * an optional bf16 "shadow" of a parameter range (the FC weight): the forward GEMM reads
//     the shadow instead of casting 8.4 M fp32 weights every step.
#include <cstdlib>
#include <utility>

#include "common.h"

namespace qd {
namespace optim {

struct AdamArgs {
  float beta1, beta2, eps, weight_decay, grad_scale, prune_thr;
  int decoupled;  // 1 = AdamW
};

struct Shadow {
  uint16_t* out;        // bf16 copy of p[lo, hi) (lo, hi multiples of 4), or null
  long lo, hi;
  uint8_t* out8;        // optional e4m3 copy of the same range, scaled by *qs (fp8 estimator)
  const float* qs;
  float* amax;          // per-workgroup max |p| partials over the range (next step's delayed scale)
};

// Conv weight images written by the update itself: csrc/hip/conv.hip pack_weights_body's B-fragment
// layouts as a scatter (forward image of each layer, dgrad image of layers 2 / 3), so the updated
// weights need no separate pack launch; the step's batch cursor advances with the step tick.
struct PackScatter {
  long lo[3];           // offsets (relative to this launch's p) of the 3 layers' weights (E*32*CIN*9 each)
  int n[3], cin[3];     // n[k] = 0: layer k not in this launch
  uint16_t* fwd[3];     // [e][KS][64][8] bf16, KS = (9*CIN + 15) / 16 (padding written once at init)
  uint16_t* dg[3];      // [e][18][64][8] bf16 (CIN = 32 only), nullable
  int* cursor;          // nullable: *cursor += cursor_inc once per launch (also when the step is skipped)
  int cursor_inc;
};

// Gradients the update sums itself (world 1): job k's gradient over the flat range [off[k], off[k] + groups * width)
// (relative to the stepped part) is the row sum of a workgroup-partial slab -- out[g * width + i] = sum over r < rows
// of slab[(g * rows + r) * ld + i] -- the deterministic slab reduction qd_slab_rows_sum_multi would have written
// into the gradient (conv.hip slab_rows_sum4_body: the same rows per thread in the same order, the same combine, so
// the sums are bit-identical).  The update's workgroups past the regular ones run these jobs, 64 columns each, and
// the regular ones skip the ranges: the slab launch leaves the chain.  Vector jobs only (width, ld, off % 4 == 0).
constexpr int kAdamSlabJobs = 16, kAdamSkips = 4;
struct AdamSlabs {
  const float* slab[kAdamSlabJobs];
  int off[kAdamSlabJobs], groups[kAdamSlabJobs], rows[kAdamSlabJobs], width[kAdamSlabJobs], ld[kAdamSlabJobs];
  int wg0[kAdamSlabJobs + 1];   // first extra workgroup of each job (prefix sums); wg0[n] = extra workgroups
  int n;
  // the regular workgroups skip [skip_lo[k], skip_hi[k]): the jobs' ranges merged across alignment gaps (a gap's
  // elements are padding, never stepped apart from their zero gradient) -- 4 int compares per float4 (the job
  // table itself in the loop cost 25 VGPRs and occupancy 7 -> 5)
  int skip_lo[kAdamSkips], skip_hi[kAdamSkips];
};
__device__ __forceinline__ bool in_slab_job(const AdamSlabs& sj, long i0) {
  bool in = false;
#pragma unroll
  for (int k = 0; k < kAdamSkips; ++k) in |= i0 >= sj.skip_lo[k] && i0 < sj.skip_hi[k];
  return in;
}

__device__ __forceinline__ void pack_scatter(const PackScatter& ps, long i0, const float* v4) {
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (ps.n[k] == 0 || i0 < ps.lo[k] || i0 >= ps.lo[k] + ps.n[k]) continue;
    const int CIN = ps.cin[k], per = 32 * CIN * 9, KS = (9 * CIN + 15) / 16;
    for (int q = 0; q < 4; ++q) {
      const int idx = (int)(i0 - ps.lo[k]) + q;
      const int e = idx / per, r = idx % per, co = r / (CIN * 9), ci = (r % (CIN * 9)) / 9, tap = r % 9;
      const uint16_t b = f32_to_bf16(v4[q]);
      int kk = tap * CIN + ci;   // forward: W[e*32 + col][k % CIN][k / CIN], col = co
      ps.fwd[k][(((size_t)e * KS + kk / 16) * 64 + ((kk % 16) / 8) * 32 + co) * 8 + kk % 8] = b;
      if (ps.dg[k]) {            // dgrad: W[e*32 + k % 32][col][8 - k / 32], col = ci
        kk = (8 - tap) * 32 + co;
        ps.dg[k][(((size_t)e * 18 + kk / 16) * 64 + ((kk % 16) / 8) * 32 + ci) * 8 + kk % 8] = b;
      }
    }
  }
}

// Called by every thread at the end of the kernel: the last workgroup to get here increments the
// step counter and re-arms the done counter.  Every workgroup consumed *step (its value feeds the
// update it already stored) before it arrives, so no workgroup can observe the increment of the
// step it is computing.  Deliberately NO __threadfence(): only the counter itself is shared, and
// on gfx950 an agent-scope release per workgroup writes back the XCD's whole dirty L2 -- measured
// 3x slower for this kernel (47 -> 145 us).  The next kernel sees *step via kernel-boundary ordering.
__device__ __forceinline__ void tick_if_last(float* step, unsigned int* done, int* cursor = nullptr, int inc = 0) {
  __shared__ bool last;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned int prev = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = (prev == gridDim.x - 1);
  }
  __syncthreads();
  if (last && threadIdx.x == 0) {
    *step += 1.f;
    if (cursor) *cursor += inc;
    __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__device__ __forceinline__ float store_shadow(const Shadow& sh, long i0, float4 v) {
  if (sh.out != nullptr && i0 >= sh.lo && i0 < sh.hi) {
    ushort4 h;
    h.x = f32_to_bf16(v.x);
    h.y = f32_to_bf16(v.y);
    h.z = f32_to_bf16(v.z);
    h.w = f32_to_bf16(v.w);
    *reinterpret_cast<ushort4*>(sh.out + (i0 - sh.lo)) = h;
    if (sh.out8 != nullptr) {
      const float q = *sh.qs;
      *reinterpret_cast<uint32_t*>(sh.out8 + (i0 - sh.lo)) = e4m3_pack4(v.x * q, v.y * q, v.z * q, v.w * q);
      return fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
    }
  }
  return 0.f;
}

// NT: streaming (non-temporal) loads / stores for the big parameter ranges (each element is touched
// once per step: keeping it in L2 / MALL only evicts the activations the next kernels re-read)
typedef float f32x4v __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ float4 ldv(const float* a) {
  if constexpr (NT) {
    const f32x4v r = __builtin_nontemporal_load(reinterpret_cast<const f32x4v*>(a));
    return make_float4(r.x, r.y, r.z, r.w);
  } else {
    return *reinterpret_cast<const float4*>(a);
  }
}
template <bool NT>
__device__ __forceinline__ void stv(float* a, float4 v) {
  if constexpr (NT) {
    const f32x4v r = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(r, reinterpret_cast<f32x4v*>(a));
  } else {
    *reinterpret_cast<float4*>(a) = v;
  }
}

template <bool NT, bool SLABS = false>
__global__ void __launch_bounds__(256) adam_kernel(float* __restrict__ p, float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, long n,
                                                   const float* __restrict__ lr_ptr, const float* step_ptr,
                                                   const float* __restrict__ skip, unsigned int* __restrict__ pruned,
                                                   AdamArgs a, float* __restrict__ step_out,
                                                   unsigned int* __restrict__ done, Shadow sh, PackScatter ps,
                                                   long hole_lo, long hole_n, AdamSlabs sj) {
  if (skip != nullptr && *skip != 0.f) {   // uniform across the grid: nobody ticks (the cursor still moves)
    if (ps.cursor && blockIdx.x == 0 && threadIdx.x == 0) *ps.cursor += ps.cursor_inc;
    return;
  }
  // the slab jobs' workgroups come FIRST (dispatched in block order: appended after the 2048 regular ones they ran
  // alone at the end of the launch -- measured no faster than the slab launch they replace)
  const int nsl = SLABS ? sj.wg0[sj.n] : 0, nreg = (int)gridDim.x - nsl, rb = (int)blockIdx.x - nsl;
  const float lr = *lr_ptr;
  const float t = *step_ptr + 1.f;  // step about to be taken
  const float bc1 = 1.f - __powf(a.beta1, t);
  const float bc2 = 1.f - __powf(a.beta2, t);
  const float step_size = lr / bc1;
  const float rbc2 = rsqrtf(bc2);
  unsigned int cnt = 0;
  float wmax = 0.f;
  // one float4 of the update: p, m, v at i0 with gradient gg (already read / summed); returns the updated gg
  auto update4 = [&](long i0, float4 gg) __attribute__((always_inline)) {
    float4 pp = ldv<NT>(p + i0);
    float4 mm = ldv<NT>(m + i0);
    float4 vv = ldv<NT>(v + i0);
    float* pa = &pp.x; float* ga = &gg.x; float* ma = &mm.x; float* va = &vv.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gj = ga[j] * a.grad_scale;
      if (a.prune_thr > 0.f && !(fabsf(gj) > a.prune_thr)) { gj = 0.f; ++cnt; }
      float pj = pa[j];
      if (a.decoupled) pj *= 1.f - lr * a.weight_decay;
      else if (a.weight_decay != 0.f) gj += a.weight_decay * pj;
      adam_elem(pj, ma[j], va[j], gj, a.beta1, a.beta2, a.eps, step_size, rbc2);
      pa[j] = pj;
      ga[j] = gj;
    }
    stv<NT>(p + i0, pp);
    wmax = fmaxf(wmax, store_shadow(sh, i0, pp));
    pack_scatter(ps, i0, &pp.x);
    stv<NT>(m + i0, mm);
    stv<NT>(v + i0, vv);
    return gg;
  };
  if (SLABS && rb < 0) {
    // ---- a slab job's 64 columns: 16 column quads x 16 row phases, rounds of 4 rows with every load in flight
    // (conv.hip slab_rows_sum4_body's order: the same row sequence per thread whatever the round size), then the
    // update of those 64 elements ----
    const int b = (int)blockIdx.x;
    int k = 0;
    while (k + 1 < sj.n && b >= sj.wg0[k + 1]) ++k;
    const int cpg = (sj.width[k] + 63) / 64, lb = b - sj.wg0[k], grp = lb / cpg, bx = lb % cpg;
    const int tq = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int i = (bx * 16 + tq) * 4, rows = sj.rows[k], ld = sj.ld[k];
    __shared__ float4 red[16][16];
    float4 t4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i < sj.width[k]) {
      const float* sp = sj.slab[k] + (size_t)grp * rows * ld + i;
      constexpr int SR = 4;   // (8 raised the kernel to 90 VGPRs: occupancy 5 instead of 7 for the HBM-bound update)
      for (int r0 = ty; r0 < rows; r0 += 16 * SR) {
        float4 vv[SR];
#pragma unroll
        for (int q = 0; q < SR; ++q)
          vv[q] = *reinterpret_cast<const float4*>(sp + (size_t)(r0 + 16 * q < rows ? r0 + 16 * q : r0) * ld);
#pragma unroll
        for (int q = 0; q < SR; ++q)
          if (r0 + 16 * q < rows) {
            t4.x += vv[q].x;
            t4.y += vv[q].y;
            t4.z += vv[q].z;
            t4.w += vv[q].w;
          }
      }
    }
    red[ty][tq] = t4;
    __syncthreads();
    if (ty == 0 && i < sj.width[k]) {
      float4 acc = red[0][tq];
#pragma unroll
      for (int q = 1; q < 16; ++q) {
        acc.x += red[q][tq].x;
        acc.y += red[q][tq].y;
        acc.z += red[q][tq].z;
        acc.w += red[q][tq].w;
      }
      const long i0 = sj.off[k] + (long)grp * sj.width[k] + i;
      *reinterpret_cast<float4*>(g + i0) = update4(i0, acc);   // (the gradient as the update used it)
    }
  } else {
  const long stride = (long)nreg * blockDim.x * 4;
  // [hole_lo, hole_lo + hole_n) (multiples of 4) is skipped: a range another kernel updates (the FC weight,
  // stepped inside its weight-gradient GEMM's epilogue); the loop runs over n - hole_n logical elements
  for (long il = ((long)rb * blockDim.x + threadIdx.x) * 4; il < n - hole_n; il += stride) {
    const long i0 = il < hole_lo ? il : il + hole_n;
    if (SLABS && in_slab_job(sj, i0)) continue;   // (summed and stepped by the slab workgroups)
    if (i0 + 3 < n) {
      const float4 gg = update4(i0, ldv<NT>(g + i0));
      if (a.prune_thr > 0.f || a.grad_scale != 1.f) *reinterpret_cast<float4*>(g + i0) = gg;
    } else {
      for (long i = i0; i < n; ++i) {
        float gj = g[i] * a.grad_scale;
        if (a.prune_thr > 0.f && !(fabsf(gj) > a.prune_thr)) { gj = 0.f; ++cnt; }
        float pj = p[i];
        if (a.decoupled) pj *= 1.f - lr * a.weight_decay;
        else if (a.weight_decay != 0.f) gj += a.weight_decay * pj;
        float mi = m[i], vi = v[i];
        adam_elem(pj, mi, vi, gj, a.beta1, a.beta2, a.eps, step_size, rbc2);
        m[i] = mi;
        v[i] = vi;
        p[i] = pj;
        g[i] = gj;
        if (sh.out != nullptr && i >= sh.lo && i < sh.hi) {
          sh.out[i - sh.lo] = f32_to_bf16(p[i]);
          if (sh.out8 != nullptr) {
            sh.out8[i - sh.lo] = f32_to_e4m3(p[i] * *sh.qs);
            wmax = fmaxf(wmax, fabsf(p[i]));
          }
        }
      }
    }
  }
  }
  if (pruned != nullptr && a.prune_thr > 0.f) {
    // one atomic per wave (the compiler's wave-level atomic coalescing would not sum counts)
    float c = wave_sum((float)cnt);
    if ((threadIdx.x & 63) == 0 && c > 0.f) atomicAdd(pruned, (unsigned int)c);
  }
  if (sh.out8 != nullptr) amax_block_store(sh.amax, wmax);
  tick_if_last(step_out, done, ps.cursor, ps.cursor_inc);
}

__global__ void __launch_bounds__(256) sgd_kernel(float* __restrict__ p, float* __restrict__ g,
                                                  float* __restrict__ buf, long n, const float* __restrict__ lr_ptr,
                                                  const float* step_ptr, const float* __restrict__ skip,
                                                  float momentum, float weight_decay, float grad_scale,
                                                  float* __restrict__ step_out, unsigned int* __restrict__ done) {
  if (skip != nullptr && *skip != 0.f) return;
  const float lr = *lr_ptr;
  const bool first = *step_ptr < 0.5f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float gj = g[i] * grad_scale + weight_decay * p[i];
    float b = first ? gj : momentum * buf[i] + gj;
    buf[i] = b;
    p[i] -= lr * b;
  }
  tick_if_last(step_out, done);
}

// Delayed per-tensor fp8 scaling, one workgroup per tensor: amax = max of the producers'
// per-workgroup partials (then re-armed to 0), scale = amax * 2^margin / fmax (dequantisation
// factor fed to the GEMM), qs = 1 / scale (quantisation factor the producers multiply by).
__global__ void __launch_bounds__(256) fp8_scale_update_kernel(float* amax_parts, float* scale, float* qs, int nparts,
                                                               float fmax, float margin) {
  __shared__ float red[4];
  const int i = blockIdx.x;
  float* part = amax_parts + (size_t)i * nparts;
  float m = 0.f;
  if (nparts == 4096) {   // every load in flight before the re-arming stores (a load / store pair per
    float4* p4 = reinterpret_cast<float4*>(part);   // iteration serialised 16 round trips)
    float4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = p4[threadIdx.x + 256 * q];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      m = fmaxf(m, fmaxf(fmaxf(v[q].x, v[q].y), fmaxf(v[q].z, v[q].w)));
      p4[threadIdx.x + 256 * q] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  } else {
    for (int k = threadIdx.x; k < nparts; k += 256) {
      m = fmaxf(m, part[k]);
      part[k] = 0.f;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float a = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    if (a > 0.f) {   // keep the previous scale if the tensor was not produced since the last update
      const float s = a * exp2f(margin) / fmax;
      scale[i] = s;
      qs[i] = 1.f / s;
    }
  }
}

inline int grid_for(long n, int max_grid = 2048) {
  long b = (n / 4 + 255) / 256;
  if (b < 1) b = 1;
  if (b > max_grid) b = max_grid;
  return (int)b;
}

}  // namespace optim
}  // namespace qd

using namespace qd::optim;

// done: device uint32 counter, zero-initialised once (re-armed by the kernel).
// shadow: optional bf16 copy of p[lo, hi) (lo, hi multiples of 4), written with the update;
// shadow8/qs/amax: optional e4m3 copy of the same range (fp8 estimator).
// nj slab jobs (nullable arrays; see AdamSlabs): job k sums slab[k] (groups[k] x rows[k] rows of ld[k] floats) into
// the gradient of the flat range [off[k], off[k] + groups[k] * width[k]) of this part before updating it
QD_API int qd_adam_step_slabs(float* p, float* g, float* m, float* v, long n, const float* lr, float* step,
                              const float* skip, unsigned int* pruned, float beta1, float beta2, float eps,
                              float weight_decay, int decoupled, float grad_scale, float prune_thr, unsigned int* done,
                              uint16_t* shadow, long shadow_lo, long shadow_hi, uint8_t* shadow8, const float* qs,
                              float* amax, int max_grid, const PackScatter* ps_in, long hole_lo, long hole_n, int nj,
                              const float* const* slab, const long* off, const int* groups, const int* rows,
                              const int* width, const int* ld, void* stream);
QD_API int qd_adam_step(float* p, float* g, float* m, float* v, long n, const float* lr, float* step, const float* skip,
                        unsigned int* pruned, float beta1, float beta2, float eps, float weight_decay, int decoupled,
                        float grad_scale, float prune_thr, unsigned int* done, uint16_t* shadow, long shadow_lo,
                        long shadow_hi, uint8_t* shadow8, const float* qs, float* amax, int max_grid,
                        const PackScatter* ps_in, long hole_lo, long hole_n, void* stream) {
  return qd_adam_step_slabs(p, g, m, v, n, lr, step, skip, pruned, beta1, beta2, eps, weight_decay, decoupled,
                            grad_scale, prune_thr, done, shadow, shadow_lo, shadow_hi, shadow8, qs, amax, max_grid, ps_in,
                            hole_lo, hole_n, 0, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, stream);
}
QD_API int qd_adam_step_slabs(float* p, float* g, float* m, float* v, long n, const float* lr, float* step,
                              const float* skip, unsigned int* pruned, float beta1, float beta2, float eps,
                              float weight_decay, int decoupled, float grad_scale, float prune_thr, unsigned int* done,
                              uint16_t* shadow, long shadow_lo, long shadow_hi, uint8_t* shadow8, const float* qs,
                              float* amax, int max_grid, const PackScatter* ps_in, long hole_lo, long hole_n, int nj,
                              const float* const* slab, const long* off, const int* groups, const int* rows,
                              const int* width, const int* ld, void* stream) {
  const PackScatter ps = ps_in ? *ps_in : PackScatter{};
  if (nj < 0 || nj > kAdamSlabJobs) return (int)hipErrorInvalidValue;
  AdamSlabs sj{};
  sj.n = nj;
  if (nj && n >= (1L << 31)) return (int)hipErrorInvalidValue;
  long lo_k[kAdamSlabJobs], hi_k[kAdamSlabJobs];
  for (int k = 0; k < nj; ++k) {
    if (!slab[k] || off[k] < 0 || groups[k] < 1 || rows[k] < 1 || width[k] < 4 || ld[k] < width[k] ||
        ((off[k] | width[k] | ld[k]) & 3) || off[k] + (long)groups[k] * width[k] > n ||
        (reinterpret_cast<uintptr_t>(slab[k]) & 15))
      return (int)hipErrorInvalidValue;
    // (a job inside the hole -- a range another kernel updates -- would be stepped twice)
    if (hole_n && off[k] < hole_lo + hole_n && hole_lo < off[k] + (long)groups[k] * width[k])
      return (int)hipErrorInvalidValue;
    sj.slab[k] = slab[k];
    sj.off[k] = (int)off[k];
    sj.groups[k] = groups[k];
    sj.rows[k] = rows[k];
    sj.width[k] = width[k];
    sj.ld[k] = ld[k];
    sj.wg0[k + 1] = sj.wg0[k] + groups[k] * ((width[k] + 63) / 64);
    lo_k[k] = off[k];
    hi_k[k] = off[k] + (long)groups[k] * width[k];
  }
  // skip intervals: the job ranges sorted and merged across gaps of < 64 elements (alignment padding)
  for (int a = 0; a < nj; ++a)
    for (int b = a + 1; b < nj; ++b)
      if (lo_k[b] < lo_k[a]) {
        std::swap(lo_k[a], lo_k[b]);
        std::swap(hi_k[a], hi_k[b]);
      }
  int ns = 0;
  for (int k = 0; k < nj; ++k) {
    if (k > 0 && lo_k[k] < hi_k[k - 1]) return (int)hipErrorInvalidValue;   // (overlapping jobs)
    if (ns > 0 && lo_k[k] - sj.skip_hi[ns - 1] < 64 && (hole_n == 0 || !(sj.skip_hi[ns - 1] <= hole_lo && hole_lo < lo_k[k]))) {
      sj.skip_hi[ns - 1] = (int)hi_k[k];
    } else {
      if (ns == kAdamSkips) return (int)hipErrorInvalidValue;
      sj.skip_lo[ns] = (int)lo_k[k];
      sj.skip_hi[ns] = (int)hi_k[k];
      ++ns;
    }
  }
  for (int k = 0; k < 3; ++k)
    if (ps.n[k] && (ps.lo[k] < 0 || ps.lo[k] + ps.n[k] > n || (ps.lo[k] & 3) || (ps.n[k] & 3) || !ps.fwd[k]))
      return (int)hipErrorInvalidValue;
  if (n <= 0 || done == nullptr || (shadow && ((shadow_lo | shadow_hi) & 3))) return (int)hipErrorInvalidValue;
  if (shadow8 && (!shadow || !qs || !amax)) return (int)hipErrorInvalidValue;
  if (hole_n < 0 || hole_lo < 0 || ((hole_lo | hole_n) & 3) || hole_lo + hole_n > n || (hole_n && shadow8))
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  AdamArgs a{beta1, beta2, eps, weight_decay, grad_scale, prune_thr, decoupled};
  Shadow sh{shadow, shadow_lo, shadow_hi, shadow8, qs, amax};
  // max_grid (0 = 2048): fewer workgroups stream the update more slowly but leave most CUs to
  // kernels running beside it (the FC Adam as a side branch of the step graph)
  // streaming loads/stores for large ranges (profiles/r1_17_adam_nt.md)
  const bool nt = n - hole_n >= (1L << 20);
  const dim3 grid(grid_for(n - hole_n, max_grid > 0 ? max_grid : 2048) + sj.wg0[nj]);
#define QD_ADAM(NT_, SL_)                                                                                          \
  hipLaunchKernelGGL((adam_kernel<NT_, SL_>), grid, dim3(256), 0, st, p, g, m, v, n, lr, step, skip, pruned, a, step, \
                     done, sh, ps, hole_lo, hole_n, sj)
  if (nj) {
    if (nt) QD_ADAM(true, true); else QD_ADAM(false, true);
  } else {
    if (nt) QD_ADAM(true, false); else QD_ADAM(false, false);
  }
#undef QD_ADAM
  return (int)hipGetLastError();
}

QD_API int qd_sgd_step(float* p, float* g, float* buf, long n, const float* lr, float* step, const float* skip,
                       float momentum, float weight_decay, float grad_scale, unsigned int* done, void* stream) {
  if (n <= 0 || done == nullptr) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(sgd_kernel, dim3(grid_for(n * 4)), dim3(256), 0, st, p, g, buf, n, lr, step, skip, momentum,
                     weight_decay, grad_scale, step, done);
  return (int)hipGetLastError();
}

// amax_parts: (n, kAmaxParts) floats
QD_API int qd_fp8_scale_update(float* amax_parts, float* scale, float* qs, int n, float fmax, float margin,
                               void* stream) {
  if (n < 1 || n > 64) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(fp8_scale_update_kernel, dim3(n), dim3(256), 0, (hipStream_t)stream, amax_parts, scale, qs,
                     qd::kAmaxParts, fmax, margin);
  return (int)hipGetLastError();
}

QD_API int qd_amax_parts() { return qd::kAmaxParts; }

// ---------------------------------------------------------------------------------------------------------------
// Probe-only (scripts/r4_adam_probe.py): the Adam update with a bf16 shadow, in access-pattern variants, to find what
// limits adam_kernel at ~5 TB/s of its 30 bytes per parameter (6.3 TB/s is the measured float4-copy rate).
//   LNT / SNT: non-temporal loads / stores;  U: parameter quads per thread per round, every load of a round in
//   flight before its math.  Same arithmetic as adam_kernel (Adam, no weight decay / pruning); n % 4 == 0.
namespace qd {
namespace optim {
template <bool LNT, bool SNT, int U>
__global__ void __launch_bounds__(256) adam_probe_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                         float* __restrict__ m, float* __restrict__ v, long n,
                                                         const float* __restrict__ lr_ptr, const float* step_ptr,
                                                         AdamArgs a, uint16_t* __restrict__ shadow) {
  const float lr = *lr_ptr;
  const float t = *step_ptr + 1.f;
  const float step_size = lr / (1.f - __powf(a.beta1, t));
  const float rbc2 = rsqrtf(1.f - __powf(a.beta2, t));
  const long lane0 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const long span = (long)gridDim.x * blockDim.x * 4;   // one quad per thread
  for (long base = lane0; base < n; base += span * U) {
    float4 pp[U], gg[U], mm[U], vv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i0 = base + span * u < n ? base + span * u : lane0;
      pp[u] = ldv<LNT>(p + i0);
      gg[u] = ldv<LNT>(g + i0);
      mm[u] = ldv<LNT>(m + i0);
      vv[u] = ldv<LNT>(v + i0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i0 = base + span * u;
      if (i0 >= n) continue;
      float* pa = &pp[u].x; float* ga = &gg[u].x; float* ma = &mm[u].x; float* va = &vv[u].x;
#pragma unroll
      for (int j = 0; j < 4; ++j) adam_elem(pa[j], ma[j], va[j], ga[j] * a.grad_scale, a.beta1, a.beta2, a.eps,
                                            step_size, rbc2);
      stv<SNT>(p + i0, pp[u]);
      stv<SNT>(m + i0, mm[u]);
      stv<SNT>(v + i0, vv[u]);
      ushort4 h;
      h.x = f32_to_bf16(pp[u].x);
      h.y = f32_to_bf16(pp[u].y);
      h.z = f32_to_bf16(pp[u].z);
      h.w = f32_to_bf16(pp[u].w);
      *reinterpret_cast<ushort4*>(shadow + i0) = h;
    }
  }
}
}  // namespace optim
}  // namespace qd

QD_API int qd_adam_probe(int variant, float* p, const float* g, float* m, float* v, long n, const float* lr,
                         const float* step, float beta1, float beta2, float eps, uint16_t* shadow, int grid,
                         void* stream) {
  if (n <= 0 || (n & 3) || grid <= 0) return (int)hipErrorInvalidValue;
  const AdamArgs a{beta1, beta2, eps, 0.f, 1.f, 0.f, 0};
  hipStream_t st = (hipStream_t)stream;
#define QD_AP(L, S, U) \
  hipLaunchKernelGGL((adam_probe_kernel<L, S, U>), dim3(grid), dim3(256), 0, st, p, g, m, v, n, lr, step, a, shadow)
  switch (variant) {
    case 0: QD_AP(true, true, 1); break;
    case 1: QD_AP(true, true, 2); break;
    case 2: QD_AP(false, true, 1); break;
    case 3: QD_AP(true, false, 1); break;
    case 4: QD_AP(false, false, 1); break;
    case 5: QD_AP(true, true, 4); break;
    case 6: QD_AP(false, false, 2); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef QD_AP
  return (int)hipGetLastError();
}
