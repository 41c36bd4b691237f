/*
 * orbx_debug.h -- introspection of liborbx.so intermediate buffers (test use).
 * Copies one stage buffer of image `image` of the handle's last extraction to
 * host memory so the parity tests can localise a mismatch to a stage.
 */
#ifndef ORBX_DEBUG_H
#define ORBX_DEBUG_H
#include "orbx.h"
#ifdef __cplusplus
extern "C" {
#endif

enum {
  ORBX_DBG_BLUR_LEVEL = 1,  /* arg = level: blurred level image (w*h bytes)                 */
  ORBX_DBG_CELL_COUNTS = 2, /* int32 per FAST cell (all levels, row-major per level)         */
  ORBX_DBG_CELL_TABLE = 3,  /* int32 x8 per cell: level,x0,y0,x1,y1,cand_off,cap,0           */
  ORBX_DBG_CANDIDATES = 4,  /* u32 per candidate slot (score<<24|y<<12|x), cand_total slots   */
  ORBX_DBG_OCT_COUNTS = 5,  /* int32 per level                                                */
  ORBX_DBG_OCT_OUT = 6,     /* u32 per octree output slot, oct_total slots                    */
  ORBX_DBG_LEVEL_INFO = 7   /* int32 x8 per level: w,h,cell_begin,cell_end,oct_off,oct_cap,nfeat,nIni */
};

/* Returns the number of bytes the item occupies (copies min(cap, size)); <0 on error. */
long long orbx_debug_copy(orbx_extractor* h, int what, int image, int arg, void* dst, size_t cap);

/* Solve S x = b (N x N, N a multiple of 6) with the LocalBA reduced-system
 * LDLT kernel; *ms = mean kernel time over reps launches.  ORBX_ERR_STATE on
 * a zero pivot. */
int orbx_debug_ldlt(const double* S, const double* b, int N, double* x, int reps, float* ms);

/* On-box HBM reference: copy `bytes` (multiple of 16) between two device
 * buffers with a streaming 16-B kernel, reps times on the null stream;
 * *ms = mean time per copy (2 * bytes of HBM traffic each). */
int orbx_debug_hbm_copy(void* dst, const void* src, size_t bytes, int reps, float* ms);

#ifdef __cplusplus
}
#endif
#endif
