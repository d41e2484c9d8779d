// Runtime helpers: the LDS-poison sanitizer (tests/test_lds_poison_gpu.py) and the ds_read_b64_tr_b8 layout
// probe the e4m3 GEMM's transposed-operand reads were designed from (scripts/probe_tr_b8.py).
// (Round 3's CU-masked streams and CU probe were removed in round 4: every spatial partition of the chip
// measured slower, docs/CONCURRENCY.md.)
#include "common.h"

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

// Phase stamps (FlagshipTrainer.phase_times under the one-graph DP plan, whose phases sit inside ONE graph
// and so have no host-visible boundaries for HIP events): a one-wave kernel, captured as a graph node between
// two phases on the phase's own stream, writes the chip's constant-rate wall clock into out[idx] once the work
// ahead of it on that stream has finished.  The clock is shared by every XCD and queue, so stamps taken on
// different streams of the same step are comparable; qd_wallclock_khz gives its rate.
namespace qd {
namespace rt {
__global__ void __launch_bounds__(64) stamp_kernel(unsigned long long* __restrict__ out, int idx) {
  const unsigned long long t = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) out[idx] = t;   // (a vector store: lane 0 of the wave)
}
}  // namespace rt
}  // namespace qd

extern "C" int qd_stamp(unsigned long long* out, int idx, void* stream) {
  hipLaunchKernelGGL(qd::rt::stamp_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, out, idx);
  return (int)hipGetLastError();
}

extern "C" int qd_wallclock_khz(int device, int* khz) {
  return (int)hipDeviceGetAttribute(khz, hipDeviceAttributeWallClockRate, device);
}
