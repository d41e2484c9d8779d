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

// Cross-queue coherence probe (scripts/probe_coherence.py; docs/CONCURRENCY.md, the stale-read diagnosis).
// A producer grid writes buf[i] = tag * 2^20 + i with tag = *ctr (the step), a consumer grid forked onto
// another stream of the same graph reads buf back and counts the elements that do not hold THIS step's value
// (errs[0]; errs[1] = elements seen holding the PREVIOUS step's value, i.e. a stale cached line), and a tick
// grid advances *ctr at the end of the step.  buf is small (it stays resident in the consumer XCDs' L2 between
// steps), so a consumer that misses an L2 invalidate after the cross-queue edge reads last step's line.
// mode 0: plain loads; 1: an agent-scope acquire fence at consumer entry; 2: system-scope (L2-coherent)
// loads.  Counters are vector atomics.
namespace qd {
namespace rt {
__global__ void __launch_bounds__(256) coh_produce_kernel(int* __restrict__ buf, int n, const int* __restrict__ ctr) {
  const int tag = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // (vector load: the tag
  //                                                                                       itself is not under test)
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) buf[i] = (tag << 20) + i;
}
template <int MODE>
__global__ void __launch_bounds__(256) coh_consume_kernel(const int* buf, int n, const int* __restrict__ ctr,
                                                          unsigned int* __restrict__ errs) {
  if constexpr (MODE == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  const int tag = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned int bad = 0, stale = 0;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    int v;
    if constexpr (MODE == 2) v = __hip_atomic_load(buf + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else v = buf[i];
    bad += v != (tag << 20) + i;
    stale += v == ((tag - 1) << 20) + i;
  }
  if (bad) atomicAdd(errs, bad);
  if (stale) atomicAdd(errs + 1, stale);
}
__global__ void __launch_bounds__(64) coh_tick_kernel(int* __restrict__ ctr) {
  if (threadIdx.x == 0) ctr[0] = ctr[0] + 1;
}
// keeps the producer's queue busy while the consumer runs (so the graph executor gives the branch its own queue)
__global__ void __launch_bounds__(256) coh_busy_kernel(float* __restrict__ x, int n, int iters) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    float v = x[i];
    for (int k = 0; k < iters; ++k) v = v * 0.999f + 0.001f;
    x[i] = v;
  }
}
}  // namespace rt
}  // namespace qd

QD_API int qd_coh_produce(int* buf, int n, const int* ctr, int grid, void* stream) {
  hipLaunchKernelGGL(qd::rt::coh_produce_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, buf, n, ctr);
  return (int)hipGetLastError();
}
QD_API int qd_coh_consume(const int* buf, int n, const int* ctr, unsigned int* errs, int mode, int grid,
                          void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (mode == 0) hipLaunchKernelGGL(qd::rt::coh_consume_kernel<0>, dim3(grid), dim3(256), 0, s, buf, n, ctr, errs);
  else if (mode == 1) hipLaunchKernelGGL(qd::rt::coh_consume_kernel<1>, dim3(grid), dim3(256), 0, s, buf, n, ctr, errs);
  else if (mode == 2) hipLaunchKernelGGL(qd::rt::coh_consume_kernel<2>, dim3(grid), dim3(256), 0, s, buf, n, ctr, errs);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}
QD_API int qd_coh_tick(int* ctr, void* stream) {
  hipLaunchKernelGGL(qd::rt::coh_tick_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, ctr);
  return (int)hipGetLastError();
}
QD_API int qd_coh_busy(float* x, int n, int iters, int grid, void* stream) {
  hipLaunchKernelGGL(qd::rt::coh_busy_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, n, iters);
  return (int)hipGetLastError();
}

// Native crash report (round 6).  A host segfault inside the HIP runtime (round 5: rc 139 in
// hipGraphLaunch under torch.cuda.CUDAGraph.replay, profiles/r5_46_pytest_segfault*.log) showed only the
// Python frames faulthandler prints.  qd_install_crash_handler (called once by _native.hip_lib) puts a
// SIGSEGV / SIGBUS / SIGABRT handler in front of whatever was installed before: it writes the native frames
// (backtrace_symbols_fd: library + offset of every frame) to stderr, restores the previous action and
// returns, so the fault re-raises into the previous handler (Python's faulthandler: the Python frames) and
// finally the default action (exit status 139 / 134).  Async-signal-safe calls only.
// QDML_CRASH_LOG (a file path) also sends the report to that file: under pytest's output capture fd 2 is a
// temporary file that dies with the process (round 6, profiles/r6_11a_pytest_segfault.log: faulthandler's frames only).
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

namespace qd {
namespace rt {
constexpr int kCrashSigs[3] = {SIGSEGV, SIGBUS, SIGABRT};
struct sigaction g_prev[3];
volatile sig_atomic_t g_installed = 0;
int g_logfd = -1;

void crash_write(const char* s) {
  ssize_t r = write(2, s, strlen(s));
  if (g_logfd >= 0) r = write(g_logfd, s, strlen(s));
  (void)r;
}

void crash_handler(int sig, siginfo_t* info, void* uctx) {
  (void)uctx;
  int k = 0;
  while (k < 3 && kCrashSigs[k] != sig) ++k;
  crash_write(sig == SIGSEGV ? "\n[qdml] SIGSEGV" : sig == SIGBUS ? "\n[qdml] SIGBUS" : "\n[qdml] SIGABRT");
  char hex[32];
  uintptr_t a = info ? (uintptr_t)info->si_addr : 0;
  int n = 0;
  hex[n++] = ' ';
  hex[n++] = '@';
  hex[n++] = '0';
  hex[n++] = 'x';
  for (int i = (int)sizeof(a) * 2 - 1; i >= 0; --i) hex[n++] = "0123456789abcdef"[(a >> (4 * i)) & 0xf];
  hex[n++] = '\n';
  hex[n] = 0;
  crash_write(hex);
  crash_write("[qdml] native frames (libqdml_hip crash handler):\n");
  void* frames[64];
  const int nf = backtrace(frames, 64);
  backtrace_symbols_fd(frames, nf, 2);
  if (g_logfd >= 0) backtrace_symbols_fd(frames, nf, g_logfd);
  crash_write("[qdml] end of native frames\n");
  // hand the signal on: the previous action (faulthandler, then the default) runs when the fault re-raises
  if (k < 3) sigaction(sig, &g_prev[k], nullptr);
  if (sig == SIGABRT) raise(sig);   // (abort() re-raises by itself too; a raised SIGABRT is not re-executed)
}
}  // namespace rt
}  // namespace qd

extern "C" int qd_install_crash_handler() {
  using namespace qd::rt;
  if (g_installed) return 0;
  void* warm[2];
  backtrace(warm, 2);   // (loads libgcc's unwinder now: backtrace() may allocate on its first call)
  if (const char* path = getenv("QDML_CRASH_LOG"))
    if (path[0]) g_logfd = open(path, O_WRONLY | O_CREAT | O_APPEND | O_CLOEXEC, 0644);
  for (int k = 0; k < 3; ++k) {
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = crash_handler;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    if (sigaction(kCrashSigs[k], &sa, &g_prev[k]) != 0) return -1;
  }
  g_installed = 1;
  return 0;
}

// (test hook) fault on purpose in native code: tests/test_runtime_crash.py checks the report in a child process
extern "C" void qd_crash_for_test() {
  volatile int* p = nullptr;
  *p = 1;
}
