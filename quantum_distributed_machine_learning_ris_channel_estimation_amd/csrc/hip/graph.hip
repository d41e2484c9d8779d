// Capture-time control of the HIP graph's dependency ORDER (host code only).
//
// The ROCm graph executor maps the captured DAG onto hardware queues: a chain stays on one queue, and a
// node with parents on two queues is placed on ONE of them -- every cross-queue edge becomes a barrier
// packet that costs ~10 us between the producer's end and the consumer's start (profiles/r2_19_*).  In the
// flagship dagq step the next step's gather joins the HDCE chain (Adam) and the QSC branch (AdamW); it
// was placed on the QSC queue, so BOTH the join and the gather -> conv1 edge crossed queues on the
// critical path.  qd_capture_deps reorders the capturing stream's current dependency set (the parents of
// the next captured node) so the executor's choice can be steered.
#include <vector>

#include "common.h"

// mode 1: reverse the order of the current capture dependencies of `stream`; mode 0: only count them.
// Returns the number of dependencies (0 when the stream is not capturing), or -(hipError_t) on failure.
QD_API int qd_capture_deps(void* stream, int mode) {
  hipStream_t st = (hipStream_t)stream;
  hipStreamCaptureStatus status;
  unsigned long long id = 0;
  hipGraph_t graph = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t n = 0;
  hipError_t e = hipStreamGetCaptureInfo_v2(st, &status, &id, &graph, &deps, &n);
  if (e != hipSuccess) return -(int)e;
  if (status != hipStreamCaptureStatusActive) return 0;
  if (mode == 1 && n > 1) {
    std::vector<hipGraphNode_t> rev(deps, deps + n);
    for (size_t i = 0; i < n / 2; ++i) std::swap(rev[i], rev[n - 1 - i]);
    e = hipStreamUpdateCaptureDependencies(st, rev.data(), n, hipStreamSetCaptureDependencies);
    if (e != hipSuccess) return -(int)e;
  }
  return (int)n;
}
