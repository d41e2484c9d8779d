// Runtime helpers: CU-masked streams (spatial partitioning of the chip between concurrent branches)
// and a probe kernel that reports which compute units a launch actually ran on.
//
// The training step runs two independent chains at once (HDCE estimator / QSC classifier, see
// train/flagship.py).  Left to the dispatcher, whichever chain's workgroups arrive first take whole
// CUs (the FC GEMM tiles and the QSC preprocess each need most of a CU's 160 KB LDS), so a 256-tile
// GEMM that finds 40 CUs busy runs a second round of tiles.  A CU mask on a stream
// (hipExtStreamCreateWithCUMask) restricts its dispatches to a subset of CUs, so each chain can be
// given a fixed share of the chip instead.
#include "common.h"

namespace qd {
namespace rt {

// one record per workgroup: HW_ID (wave / SIMD / CU / shader-array / shader-engine ids) and XCC_ID
__global__ void __launch_bounds__(64) cu_probe_kernel(unsigned* __restrict__ out, int spin) {
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID, bits [31:0]
  const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);  // HW_REG_XCC_ID, bits [15:0]
  for (int i = 0; i < spin; ++i) __builtin_amdgcn_s_sleep(8);        // keep the CU busy a while
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
  }
}

}  // namespace rt
}  // namespace qd

extern "C" {

// stream restricted to the CUs whose bits are set in mask[0..nwords) (HIP's logical CU numbering)
int qd_stream_create_cu_mask(const uint32_t* mask, int nwords, void** out) {
  hipStream_t s = nullptr;
  hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)nwords, mask);
  *out = (void*)s;
  return (int)e;
}

int qd_stream_get_cu_mask(void* stream, uint32_t* mask, int nwords) {
  return (int)hipExtStreamGetCUMask((hipStream_t)stream, (uint32_t)nwords, mask);
}

int qd_stream_destroy(void* stream) { return (int)hipStreamDestroy((hipStream_t)stream); }

int qd_cu_probe(unsigned* out, int nblocks, int spin, void* stream) {
  hipLaunchKernelGGL(qd::rt::cu_probe_kernel, dim3(nblocks), dim3(64), 0, (hipStream_t)stream, out, spin);
  return (int)hipGetLastError();
}

}  // extern "C"

// ds_read_b64_tr_b8 layout probe: LDS holds bytes b[a] = a & 0xff over 4 KiB (a 256-byte row pitch, 16 rows);
// lane l reads at byte address addr[l] (host-chosen), the 8 returned bytes land in out[8 l .. 8 l + 7]
namespace qd {
namespace rt {
__global__ void __launch_bounds__(64) tr_b8_probe_kernel(const int* __restrict__ addr, uint8_t* __restrict__ out,
                                                         const uint8_t* __restrict__ fill) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[4096];
  for (int i = threadIdx.x; i < 4096; i += 64) lds[i] = fill[i];
  __syncthreads();
  const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)lds;
  typedef __attribute__((ext_vector_type(2))) int v2i;
  v2i r;
  asm volatile("ds_read_b64_tr_b8 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(base + (uint32_t)addr[threadIdx.x]) : "memory");
  *reinterpret_cast<v2i*>(out + 8 * threadIdx.x) = r;
}
}  // namespace rt
}  // namespace qd

extern "C" int qd_tr_b8_probe(const int* addr, uint8_t* out, const uint8_t* fill, void* stream) {
  hipLaunchKernelGGL(qd::rt::tr_b8_probe_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, addr, out, fill);
  return (int)hipGetLastError();
}

// LDS poisoning (sanitizer, _native.set_lds_poison): every workgroup takes the whole 160 KiB of its CU's LDS
// and fills it with `pattern`; 8 workgroups per CU so that every CU of every XCD runs at least one.  A kernel
// that reads LDS it did not write in its own launch then sees the pattern instead of a predecessor's data.
namespace qd {
namespace rt {
constexpr int POISON_LDS = 160 * 1024;
__global__ void __launch_bounds__(256) lds_poison_kernel(uint32_t pattern) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds_all[];
  const uint4 v = make_uint4(pattern, pattern, pattern, pattern);
  uint4* l4 = reinterpret_cast<uint4*>(lds_all);
  for (int i = threadIdx.x; i < POISON_LDS / 16; i += 256) l4[i] = v;
  __syncthreads();
  asm volatile("" ::"v"(l4) : "memory");   // (the stores are the kernel's whole effect: keep them)
}
}  // namespace rt
}  // namespace qd

extern "C" int qd_lds_poison(uint32_t pattern, void* stream) {
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)qd::rt::lds_poison_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, qd::rt::POISON_LDS);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  hipLaunchKernelGGL(qd::rt::lds_poison_kernel, dim3(8 * 256), dim3(256), qd::rt::POISON_LDS, (hipStream_t)stream,
                     pattern);
  return (int)hipGetLastError();
}

// (sanitizer self-test) one wave reads LDS dwords 0..63 it never wrote: after a poison launch, the pattern
namespace qd {
namespace rt {
__global__ void __launch_bounds__(64) lds_peek_kernel(uint32_t* __restrict__ out) {
  __shared__ uint32_t scratch[64];   // (allocates the range; read through asm so the compiler cannot fold it)
  const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)scratch;
  uint32_t v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(base + 4u * threadIdx.x) : "memory");
  out[threadIdx.x] = v;
}
}  // namespace rt
}  // namespace qd

extern "C" int qd_lds_peek(uint32_t* out, void* stream) {
  hipLaunchKernelGGL(qd::rt::lds_peek_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, out);
  return (int)hipGetLastError();
}
