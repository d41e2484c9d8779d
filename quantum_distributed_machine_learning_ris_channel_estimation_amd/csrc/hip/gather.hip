// Per-step batch assembly from the HBM-resident 9-stream dataset, in ONE launch.
//
// Reference: every step the reference builds its inputs on the host -- DataLoader rows of 9
// streams, complex->real packing, reshape to (B, 2, 16, 8), an H2D copy per stream
// (Runner_P128_QuantumNAT_onchipQNN.py:104-108, R:181-199, R:344-346).  Here the dataset already
// lives in HBM (data/datasets.py DMLStore), and one kernel produces everything a training step
// reads, for a shuffled index vector idx (B):
//   x1     (U*B, E*2, H, W) fp32   grouped-conv input of the HDCE experts: sample (u, b) carries
//                                  the pilots of stream (e, u) in channels [2e, 2e+2)
//   xq     (S*B, 2, H, W)   fp32   scenario-classifier input, stream-major (optional)
//   rowoff (U*B*E)          int32  for every FC output row r = (u*B + b)*E + e, the row of
//                                  stream s = e*U + u, sample idx[b] in the label/perf stores, so
//                                  the NMSE kernels read labels in place (no permuted copies)
// One wave per (stream, sample): the 2*H*W-float plane is copied with float4 loads/stores.
#include "common.h"

namespace qd {
namespace gather {

__global__ void __launch_bounds__(256) gather_step_kernel(const long* __restrict__ idx, const float* __restrict__ Yp,
                                                          long yp_stream_stride, float* __restrict__ x1,
                                                          float* __restrict__ xq, int* __restrict__ rowoff,
                                                          long lab_stream_rows, int E, int U, int B, int plane) {
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int S = E * U;
  if (wid >= S * B) return;
  const int s = wid / B, b = wid % B;
  const int e = s / U, u = s % U;
  const long n = idx[b];
  const float4* src = reinterpret_cast<const float4*>(Yp + s * yp_stream_stride + n * plane);
  float4* d1 = reinterpret_cast<float4*>(x1 + ((size_t)(u * B + b) * E + e) * plane);
  float4* dq = xq ? reinterpret_cast<float4*>(xq + ((size_t)s * B + b) * plane) : nullptr;
  for (int i = lane; i < plane / 4; i += 64) {
    const float4 v = src[i];
    d1[i] = v;
    if (dq) dq[i] = v;
  }
  if (lane == 0) rowoff[(size_t)(u * B + b) * E + e] = (int)(s * lab_stream_rows + n);
}

}  // namespace gather
}  // namespace qd

using namespace qd::gather;

// plane = 2*H*W floats (multiple of 4); strides in elements (Yp) / rows (labels).
QD_API int qd_gather_step(const long* idx, const float* Yp, long yp_stream_stride, float* x1, float* xq, int* rowoff,
                          long lab_stream_rows, int E, int U, int B, int plane, void* stream) {
  if (plane % 4 || E < 1 || U < 1 || B < 1) return (int)hipErrorInvalidValue;
  const int waves = E * U * B;
  hipLaunchKernelGGL(gather_step_kernel, dim3((waves + 3) / 4), dim3(256), 0, (hipStream_t)stream, idx, Yp,
                     yp_stream_stride, x1, xq, rowoff, lab_stream_rows, E, U, B, plane);
  return (int)hipGetLastError();
}
