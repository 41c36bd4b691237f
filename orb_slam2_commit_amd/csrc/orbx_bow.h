// orbx_bow.h -- batched SearchByBoW problem descriptor (device pointers).
#pragma once
#include "../../include/orbx.h"

namespace orbx {

constexpr int kMaxBowFeatures = 8192;  // features per side (LDS match table)

// a = KF (KF-F) / KF1 (KF-KF); b = Frame / KF2; mode 0: SearchByBoW(KeyFrame*, Frame&),
// 1: SearchByBoW(KeyFrame*, KeyFrame*); match[b.n] (mode 0) or [a.n] (mode 1).
using BowProblem = orbx_bow_problem;

hipError_t launch_search_by_bow(const BowProblem* d_probs, int n, hipStream_t st);

}  // namespace orbx
