// orbx_scratch.h -- scratch for the per-call host APIs (SearchByBoW, PoseOptimization,
// SearchByProjection, SearchForTriangulation, ComputeDistinctiveDescriptors, UndistortKeyPoints).
//
// The reference calls these once per frame / KeyFrame from the Tracking and LocalMapping threads,
// so each call must not pay a device allocation: hipFree synchronises the whole device (stalling
// every other stream, e.g. the other thread's extraction), and pageable hipMemcpy goes through the
// null stream.  A call instead leases a per-device scratch record -- a grow-only device arena, a
// grow-only pinned host staging block, its own non-blocking stream -- from a pool, and returns it
// when done.  Concurrent callers get different leases (the pool grows to the peak concurrency),
// so calls from different threads still run side by side.  Nothing is freed on the call path;
// the leases live for the process.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace orbx {

struct ScratchLease {
  int device = 0;
  hipStream_t st = nullptr;
  uint8_t* d = nullptr;  // device arena
  size_t dcap = 0;
  uint8_t* h = nullptr;  // pinned host staging
  size_t hcap = 0;
  // grow-only: on growth the old blocks are released first (the lease is idle between calls)
  hipError_t reserve(size_t dbytes, size_t hbytes);
  // wait for the lease's stream (the calls are synchronous, as the reference's are)
  hipError_t sync() { return hipStreamSynchronize(st); }
};

// a lease for the current device (hipSetDevice done by the caller); nullptr on failure
ScratchLease* scratch_acquire(int device);
void scratch_release(ScratchLease* l);

struct ScratchGuard {
  ScratchLease* l;
  explicit ScratchGuard(int device) : l(scratch_acquire(device)) {}
  ~ScratchGuard() {
    if (l) scratch_release(l);
  }
  ScratchGuard(const ScratchGuard&) = delete;
  ScratchGuard& operator=(const ScratchGuard&) = delete;
};

inline size_t scratch_align(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace orbx
