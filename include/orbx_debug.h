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
/* The same with the kernel chosen as orbx_ba_debug_options.ldlt does; stamps (optional, 64 words):
 * the kernel's s_memtime phase stamps of the last launch, when built with -DORBX_LDLT_TS. */
int orbx_debug_ldlt_ex(const double* S, const double* b, int N, double* x, int reps, float* ms, int kind,
                       unsigned long long* stamps);

/* LocalBA test options of one solver handle (tests and tools only; a production caller never sets
 * them: ldlt = AUTO with nan_trial = raise_stop_after = -1 is the shipped behaviour).  ldlt forces
 * one of the reduced-system kernels the library ships for other sizes (so each is tested at every
 * size it can take); the two hooks reproduce rare events deterministically: nan_trial (the chi2 of
 * that trial of each phase reads NaN, the reference's rho-NaN rejection) and raise_stop_after (the
 * stop flag reads raised after that many trials). */
#define ORBX_BA_LDLT_AUTO 0    /* 8-wide panels (N < 128), column-step (N <= 192), blocked MFMA beyond */
#define ORBX_BA_LDLT_COLUMN 1  /* the column-step kernel wherever it fits */
#define ORBX_BA_LDLT_BLOCKED 2 /* the blocked MFMA kernel */
typedef struct {
  int ldlt;             /* ORBX_BA_LDLT_* */
  int nan_trial;        /* -1 off */
  int raise_stop_after; /* -1 off */
  int trace;            /* one timing line per call on stderr */
  int fused_ctl;        /* 1: a trial's errors and LM verdict in ONE launch (k_ba_errors_ctl: the
                           partials handed to the last block through a release/acquire ticket)
                           instead of the shipped two (k_ba_errors + k_ba_lm_control); tests
                           compare them bit for bit */
} orbx_ba_debug_options;
/* NULL restores the defaults. */
int orbx_debug_ba_options(orbx_ba* h, const orbx_ba_debug_options* options);

/* On-box HBM reference: copy `bytes` (multiple of 16) between two device
 * buffers with a streaming 16-B kernel, reps times on the null stream;
 * *ms = mean time per copy (2 * bytes of HBM traffic each). */
int orbx_debug_hbm_copy(void* dst, const void* src, size_t bytes, int reps, float* ms);

#ifdef __cplusplus
}
#endif
#endif
