// The packed-FP32 WAR hazard probe (round 6; docs/CONCURRENCY.md "the QSC preprocess forward's lanes-48..63
// misread: root cause").  The ONE translation unit built with packed-FP32 instructions enabled (_native.py
// PER_FILE_FLAGS): every other kernel of the library is compiled without them (-packed-fp32-ops), which removes
// the hazard this probe demonstrates from the whole library.
#include "common.h"

// Round 6: root cause of the QSC preprocess forward's lanes-48..63 misread (docs/CONCURRENCY.md).  The pre-fix conv1
// loop (profiles/r6_qsc_conv1_prefix_isa.txt) fed each k's broadcast weights from a ds_read_b128 into packed-FP32
// FMAs (v_pk_fma_f32, op_sel picking the odd register of a pair), and the NEXT k's ds_read_b128 into the same
// registers was issued a few instructions after the last packed FMA that read them.  Packed-FP32 VALU runs at a
// fraction of the plain VALU rate on CDNA; if its operand reads can lag behind a younger LDS return into the same
// registers, the last lanes read the next k's weight -- the observed signature.  This probe reproduces that
// instruction pattern in isolation: probe waves run
//     v_pk_fma_f32 acc, x, w, acc op_sel:[0,1,0] op_sel_hi:[0,0,1]   (w = a broadcast pair from LDS)
//     [pad: 0 / 8 / 24 independent s_nop cycles]
//     ds_read_b64 w, next pair          <- overwrites the registers the FMA just read
//     s_waitcnt lgkmcnt(0)
// and count the (iteration, wave) events where acc is not uniform across the wave (all lanes read the same
// address, so any difference is a lane that read the new w).  Partner waves of the same workgroup (8 waves: two per
// SIMD) optionally issue back-to-back MFMAs, the co-resident matrix work of the graph plans.  mode bits: 1 partner
// MFMAs, 2 plain v_fma_f32 (two of them) instead of the packed FMA, 4/8 pad 8 / 24 cycles.
namespace qd {
namespace rt {
typedef __attribute__((ext_vector_type(2))) float f2v;
typedef __attribute__((ext_vector_type(16))) float f16v;
typedef __attribute__((ext_vector_type(8))) __bf16 bf8v;
template <int PAD, bool PLAIN>
__device__ __forceinline__ void war_step(f2v& acc, f2v& w, f2v x, uint32_t addr) {
  if constexpr (PLAIN) {
    float a0 = acc.x, a1 = acc.y, w0 = w.x, w1 = w.y;
    asm volatile(
        "v_fma_f32 %0, %4, %3, %0\n\t"
        "v_fma_f32 %1, %4, %2, %1\n\t"
        : "+v"(a0), "+v"(a1), "+v"(w0), "+v"(w1)
        : "v"(x.x));
    if constexpr (PAD == 1) asm volatile("s_nop 7" ::: "memory");
    if constexpr (PAD == 2) asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    f2v nw;
    asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(nw) : "v"(addr) : "memory");
    acc = f2v{a0, a1};
    w = nw;
    return;
  }
  // the packed FMA and the reload of ITS source registers in one asm block: the hazard recognizer inserts
  // nothing, the registers are the same by construction (%1 is read by the FMA, then written by the ds_read)
  if constexpr (PAD == 0)
    asm volatile(
        "v_pk_fma_f32 %0, %2, %1, %0 op_sel:[0,1,0] op_sel_hi:[0,0,1]\n\t"
        "ds_read_b64 %1, %3\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "+v"(acc), "+v"(w)
        : "v"(x), "v"(addr)
        : "memory");
  else if constexpr (PAD == 1)
    asm volatile(
        "v_pk_fma_f32 %0, %2, %1, %0 op_sel:[0,1,0] op_sel_hi:[0,0,1]\n\t"
        "s_nop 7\n\t"
        "ds_read_b64 %1, %3\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "+v"(acc), "+v"(w)
        : "v"(x), "v"(addr)
        : "memory");
  else
    asm volatile(
        "v_pk_fma_f32 %0, %2, %1, %0 op_sel:[0,1,0] op_sel_hi:[0,0,1]\n\t"
        "s_nop 7\n\ts_nop 7\n\ts_nop 7\n\t"
        "ds_read_b64 %1, %3\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "+v"(acc), "+v"(w)
        : "v"(x), "v"(addr)
        : "memory");
}

template <int PAD, bool PLAIN>
__global__ void __launch_bounds__(512) pkfma_war_probe_kernel(int mode, int iters, unsigned int* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float wl[2 * 64];
  if (threadIdx.x < 128) wl[threadIdx.x] = 1.0f + 0.0078125f * (float)threadIdx.x;   // 64 distinct pairs
  __syncthreads();
  const int wv = threadIdx.x >> 6;
  if (wv >= 4) {   // partner waves (one per SIMD next to a probe wave): back-to-back MFMAs, or idle
    if (mode & 1) {
      f16v acc = {};
      bf8v a, b;
      for (int j = 0; j < 8; ++j) {
        a[j] = (__bf16)(0.001f * (threadIdx.x + j));
        b[j] = (__bf16)(0.002f * j);
      }
      for (int i = 0; i < iters * 8; ++i) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
      float t = 0.f;
      for (int j = 0; j < 16; ++j) t += acc[j];
      if (t == 12345.f) out[2] = 1;   // (keeps the MFMAs; never true)
    }
    return;
  }
  const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)wl;
  const f2v x = {1.0f, 1.0f};
  unsigned int events = 0;
  for (int it = 0; it < iters; ++it) {
    f2v acc = {0.f, 0.f};
    f2v w;
    asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(w) : "v"(base) : "memory");
#pragma unroll 8
    for (int k = 1; k <= 64; ++k) war_step<PAD, PLAIN>(acc, w, x, base + 8u * (uint32_t)(k & 63));
    // all lanes read the same addresses: acc must be wave-uniform.  (Lane 0's value through ds_bpermute, after a
    // pad: the hazard recognizer does not see the inline asm's last VALU write, and a v_readfirstlane right behind
    // it read a stale value in every mode of the first version of this probe, profiles/r6_01_pkfma_war.txt.)
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
    const float a0 = __shfl(acc.x, 0);
    const float a1 = __shfl(acc.y, 0);
    const bool bad = acc.x != a0 || acc.y != a1;
    if (it == 0 && blockIdx.x == 0 && wv == 0) {   // (diagnostic dump: wave 0's lanes, first iteration)
      out[4 + 2 * (threadIdx.x & 63)] = __builtin_bit_cast(unsigned int, acc.x);
      out[5 + 2 * (threadIdx.x & 63)] = __builtin_bit_cast(unsigned int, acc.y);
    }
    const unsigned long long m = __ballot(bad);
    if (m != 0ull) {
      ++events;
      if ((threadIdx.x & 63) == 0) atomicOr(out + 3, (unsigned int)(m >> 32) | (unsigned int)m);   // which lanes
    }
  }
  if ((threadIdx.x & 63) == 0 && events) atomicAdd(out, events);
  if ((threadIdx.x & 63) == 0) atomicAdd(out + 1, (unsigned int)iters);
}
}  // namespace rt
}  // namespace qd

// out: 132 zero-initialised u32 -- [0] non-uniform (iteration, wave) events, [1] (iteration, wave) pairs run,
// [2] (unused), [3] OR of the lane masks (both halves folded) of the events, [4 + 2 l .. +1] lane l's (acc.x, acc.y)
// of block 0 / wave 0 / iteration 0 (as float bits).  grid workgroups of 8 waves.
extern "C" int qd_pkfma_war_probe(int mode, int iters, int grid, unsigned int* out, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int pad = (mode & 8) ? 2 : (mode & 4) ? 1 : 0;
#define QD_WAR(P, L) hipLaunchKernelGGL((qd::rt::pkfma_war_probe_kernel<P, L>), dim3(grid), dim3(512), 0, s, mode, iters, out)
  if (mode & 2) {
    if (pad == 0) QD_WAR(0, true);
    else if (pad == 1) QD_WAR(1, true);
    else QD_WAR(2, true);
  } else {
    if (pad == 0) QD_WAR(0, false);
    else if (pad == 1) QD_WAR(1, false);
    else QD_WAR(2, false);
  }
#undef QD_WAR
  return (int)hipGetLastError();
}
