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
