// orbx_prof.h -- optional per-stage HIP-event timers (orbx_profile_* in orbx.h).
// When enabled, every stage launch is bracketed by two events recorded on the
// stream the kernel runs on; orbx_profile_read() waits for them and folds the
// elapsed times into per-stage totals.
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

namespace orbx {

enum Stage {
  ST_RESIZE = 0, ST_FAST, ST_BLUR, ST_OCTREE, ST_DESCRIBE, ST_STEREO_PREP, ST_STEREO_MATCH, ST_STEREO_FINAL,
  ST_HAMMING, ST_COUNT
};
static const char* const kStageNames[ST_COUNT] = {"k_resize", "k_fast", "k_blur", "k_octree", "k_describe",
                                                  "k_stereo_prep", "k_stereo_match", "k_stereo_finalize",
                                                  "k_hamming"};

struct StageTimer {
  bool enabled = false;
  struct Pending { int stage; hipEvent_t a, b; };
  std::vector<hipEvent_t> pool;
  std::vector<Pending> pending;
  double total_ms[ST_COUNT] = {};
  long long launches[ST_COUNT] = {};
  hipEvent_t cur_a = nullptr;

  hipEvent_t get() {
    if (!pool.empty()) {
      hipEvent_t e = pool.back();
      pool.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
  }
  void begin(hipStream_t st) {
    if (!enabled) return;
    cur_a = get();
    (void)hipEventRecord(cur_a, st);
  }
  void end(int stage, hipStream_t st) {
    if (!enabled) return;
    hipEvent_t b = get();
    (void)hipEventRecord(b, st);
    pending.push_back({stage, cur_a, b});
  }
  void flush() {
    for (auto& p : pending) {
      (void)hipEventSynchronize(p.b);
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
        total_ms[p.stage] += ms;
        launches[p.stage] += 1;
      }
      pool.push_back(p.a);
      pool.push_back(p.b);
    }
    pending.clear();
  }
  void reset() {
    flush();
    for (int i = 0; i < ST_COUNT; i++) {
      total_ms[i] = 0;
      launches[i] = 0;
    }
  }
  ~StageTimer() {
    for (auto& p : pending) {
      (void)hipEventDestroy(p.a);
      (void)hipEventDestroy(p.b);
    }
    for (auto e : pool) (void)hipEventDestroy(e);
  }
};

}  // namespace orbx
