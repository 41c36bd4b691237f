// scratch.hip -- the per-device lease pool of orbx_scratch.h.
#include <mutex>
#include <vector>

#include "orbx_scratch.h"

namespace orbx {

namespace {
struct Pool {
  std::mutex mu;
  std::vector<ScratchLease*> free;
};
constexpr int kMaxDevices = 64;
Pool g_pool[kMaxDevices];
}  // namespace

hipError_t ScratchLease::reserve(size_t dbytes, size_t hbytes) {
  dbytes = dbytes ? dbytes : 256;
  hbytes = hbytes ? hbytes : 256;
  if (dbytes > dcap) {
    if (d) {
      hipError_t e = hipStreamSynchronize(st);  // the previous call's work is done (defensive)
      if (e != hipSuccess) return e;
      (void)hipFree(d);
      d = nullptr;
      dcap = 0;
    }
    const size_t cap = scratch_align(dbytes + dbytes / 4);
    hipError_t e = hipMalloc((void**)&d, cap);
    if (e != hipSuccess) return e;
    dcap = cap;
  }
  if (hbytes > hcap) {
    if (h) {
      (void)hipHostFree(h);
      h = nullptr;
      hcap = 0;
    }
    const size_t cap = scratch_align(hbytes + hbytes / 4);
    hipError_t e = hipHostMalloc((void**)&h, cap, hipHostMallocDefault);
    if (e != hipSuccess) return e;
    hcap = cap;
  }
  return hipSuccess;
}

ScratchLease* scratch_acquire(int device) {
  if (device < 0 || device >= kMaxDevices) return nullptr;
  Pool& p = g_pool[device];
  {
    std::lock_guard<std::mutex> lock(p.mu);
    if (!p.free.empty()) {
      ScratchLease* l = p.free.back();
      p.free.pop_back();
      return l;
    }
  }
  ScratchLease* l = new (std::nothrow) ScratchLease();
  if (!l) return nullptr;
  l->device = device;
  if (hipStreamCreateWithFlags(&l->st, hipStreamNonBlocking) != hipSuccess) {
    delete l;
    return nullptr;
  }
  return l;
}

void scratch_release(ScratchLease* l) {
  if (!l) return;
  Pool& p = g_pool[l->device];
  std::lock_guard<std::mutex> lock(p.mu);
  p.free.push_back(l);
}

}  // namespace orbx
