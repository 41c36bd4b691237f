// orbx_proj.h -- batched SearchByProjection problem descriptor (device pointers).
#pragma once
#include "../../include/orbx.h"

namespace orbx {

using ProjProblem = orbx_proj_problem;

hipError_t launch_search_by_projection(const ProjProblem* d_probs, int n, hipStream_t st);

}  // namespace orbx
