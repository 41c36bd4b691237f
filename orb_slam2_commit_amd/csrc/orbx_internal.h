// orbx_internal.h -- geometry "plan" of one (width, height, params) extractor
// configuration, laid out for the device, plus kernel launch entry points.
//
// HBM layout per image (all u8, row-major, stride = level width):
//   level 0            : the caller's input image itself (never copied)
//   pyramid  (levels>=1): pyr  + img*pyr_bytes  + lv[l].off
//   blurred  (all levels): blur + img*blur_bytes + lv[l].boff, 8x16-byte tiles (128 B each),
//                          tile (ty, tx) at (ty * bstride/16 + tx) * 128, row y&7 at 16 * (y & 7)
//   FAST candidates     : cand + img*cand_total + cells[c].cand_off   (u32 score<<24|y<<12|x)
//   octree output       : oct  + img*oct_total  + lv[l].oct_off        (same packing, list order)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/orbx.h"

namespace orbx {

constexpr int kMaxLevelsPlan = 16;
constexpr int kEdgeThresholdHost = 19;  // EDGE_THRESHOLD, src/ORBextractor.cc:74

struct LevelGeom {
  int w, h;
  long long off;    // offset of level in per-image pyramid buffer (levels >= 1)
  long long boff;   // offset of level in per-image blurred buffer (256-B aligned)
  int bstride;      // blurred level width rounded to 16 (tile columns = bstride / 16)
  int minBX, minBY, maxBX, maxBY;  // FAST border box, src/ORBextractor.cc:829-832
  int cell_begin, cell_end;        // range in the cell table (row-major)
  int cand_begin, cand_cap;        // candidate slots of the level in the per-image buffer
  int nfeat;                       // mnFeaturesPerLevel[l]
  int nIni;                        // octree root count, src/ORBextractor.cc:567
  float hX;                        // root width
  int oct_off, oct_cap;            // octree output slots
  float scale;                     // mvScaleFactor[l]
  float kp_size;                   // (float)(int)(PATCH_SIZE * scale)
  int xtab_off, ytab_off;          // resize tables (levels >= 1)
  int tile_begin, tiles_x, tiles_y;  // blur tiles
};

// batches up to this many images run k_octree as one launch over every level (Geometry::og_all)
constexpr int kOctOneLaunch = 2;
// k_octree launch group: levels [l0, l1) as NT-thread blocks with LDS sized for those levels
struct OctGroup {
  int l0, l1, nt;
  int node_cap;  // LDS node capacity (max over the group's levels, multiple of 64)
  int cell_cap;  // max cells of one level
  int kcap;      // candidates of a level kept in LDS (the rest in global scratch)
};

struct Geometry {
  int nlevels, width, height;
  int ini_th, min_th;
  LevelGeom lv[kMaxLevelsPlan];
  long long pyr_bytes, blur_bytes;
  int ncells, cand_total, oct_total, max_kps, ntiles;
  int node_cap;   // octree LDS node capacity (max over levels, multiple of 64)
  int cell_cap;   // max cells in one level
  int oct_kcap;   // octree: candidates of a level kept in LDS (the rest in global scratch)
  OctGroup og[2];  // k_octree launch groups (levels 0..split-1 at 512 threads, the rest at 256)
  int n_og;
  OctGroup og_all;  // every level in one launch (batches of <= kOctOneLaunch images)
  // k_fast launch groups (consecutive cell ranges, one launch each) with their LDS layout, sized by
  // the group's largest cell: row stride s of the window tile and the score map (40, 48 or 80),
  // region rows per compass instruction rp (2 when the group's cells are <= 32 wide)
  struct FastGroup {
    int c0, c1, s, rp, tile_bytes, map_bytes, smem;
  } fg[2];
  int n_fg;
  int rz_rows;    // k_resize: max source rows staged per 128x16 output tile
  int rz_stride;  // k_resize: LDS row stride of the staged footprint (16-B chunks covering the widest span)
  int rz_lc;      // k_resize: log2 of the lanes per footprint row (>= the widest span's 16-B chunks)
};

constexpr int kRzTW = 128, kRzTH = 32;  // k_resize output tile
constexpr int kRzMaxRows = 64;

// A cell's FAST survivors: the first `kin` in its inline slots at cand_off (the cells' inline slots
// packed back to back, so the octree's per-cell reads share 128-B lines), the rest (up to `cap`) in
// its overflow slots at ovf_off.  Both offsets are per image within one cand_total block.
struct CellInfo {
  int16_t level, kin;
  int16_t x0, y0, x1, y1;  // FAST detection region (inclusive, level coordinates)
  int cand_off, cap;
  int lw, loff;  // the level's width and byte offset in an image's pyramid block (level > 0):
                 // k_fast finds its window from this one record, no dependent geometry load
  int ovf_off;
};
// slot p (< cap) of a cell's survivors, relative to the image's candidate block
__host__ __device__ inline int cell_slot(const CellInfo& c, int p) {
  return p < c.kin ? c.cand_off + p : c.ovf_off + (p - c.kin);
}

struct ResizeX {  // horizontal tap of one output column
  int sx0, sx1;
  int16_t a0, a1;
};
struct ResizeY {
  int sy0, sy1;
  int16_t b0, b1;
};

#ifndef ORBX_BLUR_TW  // k_blur output tile (256 threads: TW/4 column groups x 16-row strips)
#define ORBX_BLUR_TW 128
#define ORBX_BLUR_TH 128
#endif
constexpr int kBlurTileW = ORBX_BLUR_TW, kBlurTileH = ORBX_BLUR_TH;
static_assert(kBlurTileW / 4 * (kBlurTileH / 16) == 256, "k_blur: one thread per 4 columns x 16 rows");

// Device pointers for one batch.
struct BatchPtrs {
  const uint8_t* in;
  size_t in_pitch;
  uint8_t* pyr;
  uint8_t* blur;
  uint32_t* cand;
  int* cell_count;
  uint32_t* kpos;   // octree scratch
  int* knode;
  uint32_t* oct;
  int* oct_count;
};

__host__ __device__ inline const uint8_t* level_ptr(const Geometry& G, const BatchPtrs& B, int img, int l) {
  return l == 0 ? B.in + (size_t)img * B.in_pitch : B.pyr + (size_t)img * G.pyr_bytes + G.lv[l].off;
}

}  // namespace orbx
