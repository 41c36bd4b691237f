// capi.hip -- host side of liborbx.so: the C ABI declared in include/orbx.h.
//
// An orbx_extractor owns: one HIP stream, the parameter tables of the
// reference constructor (src/ORBextractor.cc:416-490), a plan per image
// geometry (level sizes, FAST cell table, resize coefficient tables, blur
// tiles; built once on the host and uploaded), and device buffers grown to the
// largest batch seen.  Nothing here computes results on the CPU: every output
// comes from the HIP kernels in extract.hip / stereo.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <new>
#include <utility>
#include <string>
#include <vector>

#include "../../include/orbx.h"
#include "orbx_internal.h"
#include "orbx_scratch.h"
#include "orbx_stereo.h"
#include "orbx_prof.h"
#include "orbx_bow.h"

namespace orbx {
hipError_t upload_constants(const int* umax16, const int* gauss7);
hipError_t launch_blur(const Geometry& Gh, const Geometry* Gd, const int* tile_level, const BatchPtrs& B, int n_img,
                       hipStream_t st);
hipError_t launch_extract_stages(const Geometry& Gh, const Geometry* Gd, const CellInfo* cells, const int* tile_level,
                                 const ResizeX* xt, const ResizeY* yt, const BatchPtrs& B, int n_img,
                                 orbx_keypoint* kps, uint8_t* desc, int32_t* counts, int kp_cap, hipStream_t st,
                                 StageTimer* T);
size_t octree_smem_host(int NC, int cell_cap, int kcap);
hipError_t octree_set_smem_limit(size_t bytes);
}  // namespace orbx

using namespace orbx;

namespace {

inline int round_even(float v) { return (int)std::nearbyintf(v); }

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  hipError_t ensure(size_t count) {
    if (count <= n && p) return hipSuccess;
    release();
    size_t c = std::max<size_t>(count, 1);
    hipError_t e = hipMalloc((void**)&p, c * sizeof(T));
    if (e == hipSuccess) n = c;
    return e;
  }
};

struct Tables {
  std::vector<float> scale, inv_scale, sigma2, inv_sigma2;
  std::vector<int> nfeat;
  int umax[16];
};

// ORBextractor::ORBextractor (src/ORBextractor.cc:416-490): scale factors in
// float from a double member, per-level quotas with cvRound, umax circle.
Tables make_tables(const orbx_extractor_params& p) {
  Tables t;
  const double sf = (double)p.scale_factor;
  const int n = p.nlevels;
  t.scale.assign(n, 1.0f);
  t.sigma2.assign(n, 1.0f);
  for (int i = 1; i < n; i++) {
    t.scale[i] = (float)((double)t.scale[i - 1] * sf);
    t.sigma2[i] = t.scale[i] * t.scale[i];
  }
  t.inv_scale.resize(n);
  t.inv_sigma2.resize(n);
  for (int i = 0; i < n; i++) {
    t.inv_scale[i] = 1.0f / t.scale[i];
    t.inv_sigma2[i] = 1.0f / t.sigma2[i];
  }
  t.nfeat.resize(n);
  const float factor = (float)(1.0f / sf);
  float ndes = (float)p.nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)n));
  int sum = 0;
  for (int l = 0; l < n - 1; l++) {
    t.nfeat[l] = round_even(ndes);
    sum += t.nfeat[l];
    ndes *= factor;
  }
  t.nfeat[n - 1] = std::max(p.nfeatures - sum, 0);
  int vmax = (int)std::floor(15 * std::sqrt(2.f) / 2 + 1);
  int vmin = (int)std::ceil(15 * std::sqrt(2.f) / 2);
  for (int v = 0; v < 16; v++) t.umax[v] = 0;
  for (int v = 0; v <= vmax; ++v) t.umax[v] = (int)std::nearbyint(std::sqrt(225.0 - v * v));
  for (int v = 15, v0 = 0; v >= vmin; --v) {
    while (t.umax[v0] == t.umax[v0 + 1]) ++v0;
    t.umax[v] = v0;
    ++v0;
  }
  return t;
}

// getGaussianKernel(7, 2, CV_32F) -> x256 -> cvRound (OpenCV 3.2 8U separable path).
void gaussian_int_kernel(int k[7]) {
  float cf[7];
  double sum = 0;
  const double scale2X = -0.5 / (2.0 * 2.0);
  for (int i = 0; i < 7; i++) {
    double x = i - 3.0;
    cf[i] = (float)std::exp(scale2X * x * x);
    sum += cf[i];
  }
  sum = 1. / sum;
  for (int i = 0; i < 7; i++) {
    cf[i] = (float)(cf[i] * sum);
    k[i] = round_even(cf[i] * 256.0f);
  }
}

struct Plan {
  Geometry G{};
  std::vector<CellInfo> cells;
  std::vector<int> tile_level;
  std::vector<ResizeX> xt;
  std::vector<ResizeY> yt;
  DevBuf<Geometry> dG;
  DevBuf<CellInfo> dcells;
  DevBuf<int> dtiles;
  DevBuf<ResizeX> dxt;
  DevBuf<ResizeY> dyt;
};

// Builds the per-geometry plan.  Level sizes: ComputePyramid
// (src/ORBextractor.cc:1219-1221); FAST cells: ComputeKeyPointsOctTree
// (:826-880); octree roots: DistributeOctTree (:567-570); resize tables:
// OpenCV 3.2 resizeGeneric_ coefficient setup.
orbx_status build_plan(const orbx_extractor_params& p, const Tables& t, int W, int H, Plan& P) {
  Geometry& G = P.G;
  std::memset(&G, 0, sizeof(G));
  G.nlevels = p.nlevels;
  G.width = W;
  G.height = H;
  G.ini_th = p.ini_th_fast;
  G.min_th = p.min_th_fast;
  long long pyr = 0, blur = 0;
  int cand = 0, oct = 0, ntiles = 0, node_cap = 64, cell_cap = 1;
  int lv_wmax[kMaxLevelsPlan] = {}, lv_hmax[kMaxLevelsPlan] = {};  // k_fast: largest cell per level
  P.cells.clear();
  P.tile_level.clear();
  P.xt.clear();
  P.yt.clear();
  for (int l = 0; l < p.nlevels; l++) {
    LevelGeom& L = G.lv[l];
    L.w = round_even((float)W * t.inv_scale[l]);
    L.h = round_even((float)H * t.inv_scale[l]);
    if (L.w < 1 || L.h < 1 || L.w > 4095 || L.h > 4095) return ORBX_ERR_SIZE;
    L.off = l == 0 ? 0 : pyr;
    if (l > 0) pyr += (long long)L.w * L.h;
    // blurred level: tiles of 8 rows x 16 bytes (128 B), tile (ty, tx) at (ty * bstride/16 + tx) * 128,
    // row y of a tile at 16 * (y & 7): a 37x37 patch k_describe gathers covers 5-6 x 3-4 such
    // 128-B tiles (~20) against ~48 128-B lines in a row-major layout
    L.bstride = (L.w + 15) & ~15;
    L.boff = blur;
    blur += ((long long)L.bstride * ((L.h + 7) & ~7) + 255) & ~255LL;
    L.minBX = L.minBY = kEdgeThresholdHost - 3;
    L.maxBX = L.w - kEdgeThresholdHost + 3;
    L.maxBY = L.h - kEdgeThresholdHost + 3;
    L.scale = t.scale[l];
    L.kp_size = (float)(int)(31 * t.scale[l]);
    L.nfeat = t.nfeat[l];
    // FAST cells
    L.cell_begin = (int)P.cells.size();
    L.cand_begin = cand;
    const float width = (float)(L.maxBX - L.minBX), height = (float)(L.maxBY - L.minBY);
    const int nCols = (int)(width / 30), nRows = (int)(height / 30);
    if (width > 0 && height > 0 && nCols > 0 && nRows > 0) {
      const int wCell = (int)std::ceil(width / nCols), hCell = (int)std::ceil(height / nRows);
      for (int i = 0; i < nRows; i++) {
        const float iniY = (float)(L.minBY + i * hCell);
        float maxY = iniY + hCell + 6;
        if (iniY >= L.maxBY - 3) continue;
        if (maxY > L.maxBY) maxY = (float)L.maxBY;
        for (int j = 0; j < nCols; j++) {
          const float iniX = (float)(L.minBX + j * wCell);
          float maxX = iniX + wCell + 6;
          if (iniX >= L.maxBX - 6) continue;
          if (maxX > L.maxBX) maxX = (float)L.maxBX;
          CellInfo c{};
          c.level = (int16_t)l;
          c.x0 = (int16_t)((int)iniX + 3);
          c.y0 = (int16_t)((int)iniY + 3);
          c.x1 = (int16_t)((int)maxX - 4);
          c.y1 = (int16_t)((int)maxY - 4);
          if (c.x1 < c.x0 || c.y1 < c.y0) continue;
          const int cw = c.x1 - c.x0 + 1, ch = c.y1 - c.y0 + 1;
          if (cw > 60 || ch > 60) return ORBX_ERR_SIZE;  // k_fast LDS tile bound
          lv_wmax[l] = std::max(lv_wmax[l], cw);
          lv_hmax[l] = std::max(lv_hmax[l], ch);
          c.cap = ((cw + 1) / 2) * ((ch + 1) / 2);
          c.lw = L.w;
          c.loff = (int)L.off;
          // inline slots: a level-dependent share of the cap (cells cover more of the scene, and
          // keep more survivors, at the coarser levels: ~5 at level 0 to ~28 at level 7 on KITTI)
          c.kin = (int16_t)std::min(c.cap, 4 * (int)std::ceil(2.0 * std::pow(1.25, (double)l)));
          cand += c.cap;
          P.cells.push_back(c);
        }
      }
    }
    L.cell_end = (int)P.cells.size();
    L.cand_cap = cand - L.cand_begin;
    cell_cap = std::max(cell_cap, L.cell_end - L.cell_begin);
    // octree roots
    int nIni = 1;
    if (L.maxBY - L.minBY > 0) nIni = (int)std::round((float)(L.maxBX - L.minBX) / (L.maxBY - L.minBY));
    if (nIni < 1) nIni = 1;
    L.nIni = nIni;
    L.hX = (float)(L.maxBX - L.minBX) / nIni;
    L.oct_cap = std::max(L.nfeat + 3, 4 * nIni);
    L.oct_off = oct;
    oct += L.oct_cap;
    node_cap = std::max(node_cap, (L.oct_cap + 63) / 64 * 64);
    // blur tiles
    L.tiles_x = (L.w + kBlurTileW - 1) / kBlurTileW;
    L.tiles_y = (L.h + kBlurTileH - 1) / kBlurTileH;
    L.tile_begin = ntiles;
    ntiles += L.tiles_x * L.tiles_y;
    for (int q = 0; q < L.tiles_x * L.tiles_y; q++) P.tile_level.push_back(l);
    // resize tables (source = level l-1)
    if (l > 0) {
      const LevelGeom& S = G.lv[l - 1];
      const int sw = S.w, sh = S.h, dw = L.w, dh = L.h;
      const double scale_x = 1. / ((double)dw / sw), scale_y = 1. / ((double)dh / sh);
      L.xtab_off = (int)P.xt.size();
      for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = (int)std::floor(fx);
        fx -= sx;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx + 1 >= sw && sx >= sw - 1) { fx = 0; sx = sw - 1; }
        ResizeX X;
        X.sx0 = sx;
        X.sx1 = std::min(sx + 1, sw - 1);
        X.a0 = (int16_t)round_even((1.f - fx) * 2048);
        X.a1 = (int16_t)round_even(fx * 2048);
        if (sx + 1 >= sw) {  // xmax region: D = S[sx]*2048
          X.a0 = 2048;
          X.a1 = 0;
        }
        P.xt.push_back(X);
      }
      L.ytab_off = (int)P.yt.size();
      for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = (int)std::floor(fy);
        fy -= sy;
        ResizeY Y;
        Y.sy0 = std::min(std::max(sy, 0), sh - 1);
        Y.sy1 = std::min(std::max(sy + 1, 0), sh - 1);
        Y.b0 = (int16_t)round_even((1.f - fy) * 2048);
        Y.b1 = (int16_t)round_even(fy * 2048);
        P.yt.push_back(Y);
      }
    }
  }
  // k_fast LDS layout of a launch group, sized by its largest cell: window tile of H+6 rows at
  // stride S, score map (H+2) x S (one zero row/column each side), compass list W*H u16.  The
  // compass reads up to 6 rows past the tile for lanes below the region (masked): they land in the
  // map or list, or past the allocation (reads as 0).  One-wave blocks per CU are LDS-bound and
  // k_fast is latency-bound (+1 / +2 KB of LDS per block measured +8 / +15 % time), so the stride
  // is the smallest the kernel is built for (40 for 31-32 px cells), and the levels whose cells fit
  // 5 KB (32 blocks per CU) get their own launch when taller cells of the other levels would not
  // (KITTI: levels 0-3 at 5.0 KB, levels 4-7 with their 38-40-row cells at 6.0 KB).
  {
    auto layout = [&](int wmax, int hmax, Geometry::FastGroup& g) {
      g.s = wmax + 6 <= 40 ? 40 : wmax + 6 <= 48 ? 48 : 80;
      g.rp = wmax <= 32 ? 2 : 1;
      g.tile_bytes = ((hmax + 6) * g.s + 15) & ~15;
      g.map_bytes = ((hmax + 2) * g.s + 15) & ~15;
      g.smem = g.tile_bytes + g.map_bytes + 2 * wmax * hmax;
    };
    constexpr int kFastLdsFit = 5 * 1024;
    int split = 0, wa = 1, ha = 1;  // levels [0, split) fit kFastLdsFit together
    for (int l = 0; l < p.nlevels; l++) {
      Geometry::FastGroup g{};
      layout(std::max(wa, lv_wmax[l]), std::max(ha, lv_hmax[l]), g);
      if (g.smem > kFastLdsFit) break;
      wa = std::max(wa, lv_wmax[l]);
      ha = std::max(ha, lv_hmax[l]);
      split = l + 1;
    }
    if (split == 0 || split == p.nlevels) split = p.nlevels;  // one launch
    int wb = 1, hb = 1;
    for (int l = split; l < p.nlevels; l++) {
      wb = std::max(wb, lv_wmax[l]);
      hb = std::max(hb, lv_hmax[l]);
    }
    G.n_fg = 0;
    if (split == p.nlevels) {
      int w = 1, h = 1;
      for (int l = 0; l < p.nlevels; l++) {
        w = std::max(w, lv_wmax[l]);
        h = std::max(h, lv_hmax[l]);
      }
      layout(w, h, G.fg[0]);
      G.fg[0].c0 = 0;
      G.fg[0].c1 = (int)P.cells.size();
      G.n_fg = 1;
    } else {
      layout(wa, ha, G.fg[0]);
      G.fg[0].c0 = 0;
      G.fg[0].c1 = G.lv[split].cell_begin;
      layout(wb, hb, G.fg[1]);
      G.fg[1].c0 = G.lv[split].cell_begin;
      G.fg[1].c1 = (int)P.cells.size();
      G.n_fg = 2;
    }
  }
  // k_resize staging bound: source footprint of every 128x16 output tile
  G.rz_rows = 1;
  G.rz_stride = 16;
  for (int l = 1; l < G.nlevels; l++) {
    const LevelGeom& L = G.lv[l];
    for (int oy = 0; oy < L.h; oy += kRzTH) {
      const int rows = P.yt[L.ytab_off + std::min(oy + kRzTH, L.h) - 1].sy1 - P.yt[L.ytab_off + oy].sy0 + 1;
      G.rz_rows = std::max(G.rz_rows, rows);
    }
    for (int ox = 0; ox < L.w; ox += kRzTW) {
      const int span = P.xt[L.xtab_off + std::min(ox + kRzTW, L.w) - 1].sx1 - P.xt[L.xtab_off + ox].sx0 + 1;
      G.rz_stride = std::max(G.rz_stride, (span + 15) / 16 * 16);
    }
  }
  if (G.rz_rows > kRzMaxRows || (size_t)G.rz_rows * (G.rz_stride + 2 * kRzTW) > 64 * 1024) return ORBX_ERR_SIZE;
  G.rz_lc = 0;
  while ((1 << G.rz_lc) < G.rz_stride / 16) G.rz_lc++;
  // every footprint row must be loaded: rows per thread = ceil(rz_rows / (256 >> rz_lc)) <= the kernel's 4
  if (G.rz_lc > 8 || (G.rz_rows + (256 >> G.rz_lc) - 1) / (256 >> G.rz_lc) > (kRzMaxRows + 15) / 16) return ORBX_ERR_SIZE;
  G.pyr_bytes = (pyr + 255) & ~255LL;
  G.blur_bytes = (blur + 255) & ~255LL;
  G.ncells = (int)P.cells.size();
  G.cand_total = std::max(cand, 1);
  {  // the cells' inline slots back to back, then their overflow slots (cand_total slots in all)
    int in_off = 0, ov_off = 0;
    for (const CellInfo& c : P.cells) in_off += c.kin;
    const int n_in = in_off;
    in_off = 0;
    for (CellInfo& c : P.cells) {
      c.cand_off = in_off;
      c.ovf_off = n_in + ov_off;
      in_off += c.kin;
      ov_off += c.cap - c.kin;
    }
  }
  G.oct_total = oct;
  G.max_kps = oct;
  G.ntiles = ntiles;
  G.node_cap = node_cap;
  G.cell_cap = cell_cap;
  if (node_cap > 8192) return ORBX_ERR_SIZE;
  if (octree_smem_host(node_cap, cell_cap, 0) > 160 * 1024 - 1024) return ORBX_ERR_SIZE;
  // octree candidate slots in LDS: fill the block up to 50 KB with the kernel's static LDS (three
  // 512-thread blocks must fit the CU's 160 KB -- the VGPR limit allows three; at 53 KB the
  // allocation granularity left two and the kernel ran 15 % slower), at least 1024, never more
  // than a level can hold
  {
    int max_lv_cand = 1;
    for (int l = 0; l < p.nlevels; l++) max_lv_cand = std::max(max_lv_cand, G.lv[l].cand_cap);
    const long long base = (long long)octree_smem_host(node_cap, cell_cap, 0);
    long long kc = (50 * 1024 - 512 - base) / 6;
    kc = std::max(kc, 1024LL) & ~63LL;
    kc = std::min(kc, (long long)(max_lv_cand + 63) / 64 * 64);
    while (kc > 64 && (long long)octree_smem_host(node_cap, cell_cap, (int)kc) > 160 * 1024 - 1024) kc -= 64;
    G.oct_kcap = (int)kc;
  }
  // k_octree launch groups: the levels with more than 0.4 x level 0's pixels as 512-thread blocks
  // with the 50 KB budget above (three per CU), the smaller ones as 256-thread blocks in <= 24 KB
  // (six per CU: their blocks are short and barrier-bound, so more of them in flight is what pays;
  // 0.231 -> 0.212 ms per step; 128-thread blocks, other budgets and splits measured no better,
  // profiles/r04/ab_octree_groups.txt)
  {
    const long long P0 = (long long)G.lv[0].w * G.lv[0].h;
    int split = 1;
    while (split < p.nlevels && (long long)G.lv[split].w * G.lv[split].h * 10 > 4 * P0) split++;
    auto group = [&](int l0, int l1, int nt, long long budget, OctGroup& g) {
      g.l0 = l0;
      g.l1 = l1;
      g.nt = nt;
      g.node_cap = 64;
      g.cell_cap = 1;
      int mc = 1;
      for (int l = l0; l < l1; l++) {
        g.node_cap = std::max(g.node_cap, (G.lv[l].oct_cap + 63) / 64 * 64);
        g.cell_cap = std::max(g.cell_cap, G.lv[l].cell_end - G.lv[l].cell_begin);
        mc = std::max(mc, G.lv[l].cand_cap);
      }
      const long long base = (long long)octree_smem_host(g.node_cap, g.cell_cap, 0);
      long long kc = (budget - 512 - base) / 6;
      kc = std::max(kc, 1024LL) & ~63LL;
      kc = std::min(kc, (long long)(mc + 63) / 64 * 64);
      while (kc > 64 && (long long)octree_smem_host(g.node_cap, g.cell_cap, (int)kc) > 160 * 1024 - 1024) kc -= 64;
      g.kcap = (int)kc;
    };
    G.n_og = 0;
    group(0, split, 512, 50 * 1024, G.og[G.n_og++]);
    if (split < p.nlevels) group(split, p.nlevels, 256, 24 * 1024, G.og[G.n_og++]);
    // one or two images (the host-API calls): every level in ONE launch of 512-thread blocks with
    // the CU's LDS to spend -- a handful of blocks, so the groups' two launches would only run one
    // after the other
    group(0, p.nlevels, 512, 150 * 1024, G.og_all);
  }
  return ORBX_OK;
}

}  // namespace

struct orbx_extractor {
  orbx_extractor_params params{};
  int device = 0;
  hipStream_t stream = nullptr;
  Tables tables;
  std::map<std::pair<int, int>, std::unique_ptr<Plan>> plans;
  // batch buffers
  int batch_cap = 0;
  long long bytes_pyr = 0, bytes_blur = 0, n_cand = 0, n_oct = 0, n_cells = 0;
  DevBuf<uint8_t> pyr, blur;
  DevBuf<uint32_t> cand, kpos, oct;
  DevBuf<int> cell_count, knode, oct_count;
  // host-API staging: the input image, and ONE output block [count | keypoints | descriptors]
  // (orbx_extract reads it back with one copy; orbx_stereo_match reads it in place)
  DevBuf<uint8_t> in, out;
  size_t out_kps = 0, out_desc = 0, out_bytes = 0;
  uint8_t* hstage = nullptr;  // pinned: the input image on the way in, the output block on the way out
  size_t hstage_cap = 0;
  // stereo scratch
  DevBuf<uint64_t> rkeys;
  DevBuf<int2> rxi;
  DevBuf<uint4> rdesc;
  DevBuf<uint32_t> rtab;
  DevBuf<uint4> lrange;
  DevBuf<int> oct_start, sad;
  DevBuf<float> sres;  // orbx_stereo_match: uRight | depth, adjacent (one copy back)
  DevBuf<int32_t> nmatch;
  StageTimer timer;
  // last batch (mvImagePyramid)
  Plan* last_plan = nullptr;
  const uint8_t* last_in = nullptr;
  size_t last_pitch = 0;
  int last_n = 0;
  // fingerprint of the keypoints the last host-API orbx_extract returned: orbx_stereo_match only
  // reads this handle's pyramid for exactly those keypoints (a batch extraction clears it)
  bool last_host = false;
  int last_fp_n = 0;
  uint64_t last_fp = 0;
  // mvImagePyramid readback (orbx_extractor_set_pyramid_readback): level 0 (the packed input) then
  // levels 1.. exactly as packed on the device, in pinned memory; valid for the last orbx_extract
  bool pyr_readback = false;
  bool hpyr_valid = false;
  uint8_t* hpyr = nullptr;
  size_t hpyr_cap = 0, hpyr_l0 = 0;
  ~orbx_extractor() {
    if (hstage) (void)hipHostFree(hstage);
    if (hpyr) (void)hipHostFree(hpyr);
  }
  hipError_t ensure_hpyr(size_t bytes) {
    if (bytes <= hpyr_cap && hpyr) return hipSuccess;
    if (hpyr) (void)hipHostFree(hpyr);
    hpyr = nullptr;
    hpyr_cap = 0;
    const size_t cap = (bytes + 4095) & ~(size_t)4095;
    hipError_t e = hipHostMalloc((void**)&hpyr, cap, hipHostMallocDefault);
    if (e == hipSuccess) hpyr_cap = cap;
    return e;
  }
  hipError_t ensure_stage(size_t bytes) {
    if (bytes <= hstage_cap && hstage) return hipSuccess;
    if (hstage) (void)hipHostFree(hstage);
    hstage = nullptr;
    hstage_cap = 0;
    const size_t cap = (bytes + 4095) & ~(size_t)4095;
    hipError_t e = hipHostMalloc((void**)&hstage, cap, hipHostMallocDefault);
    if (e == hipSuccess) hstage_cap = cap;
    return e;
  }
};

namespace {

orbx_status hip_status(hipError_t e) { return e == hipSuccess ? ORBX_OK : ORBX_ERR_HIP; }

orbx_status get_plan(orbx_extractor* h, int W, int H, Plan** out) {
  auto key = std::make_pair(W, H);
  auto it = h->plans.find(key);
  if (it != h->plans.end()) {
    *out = it->second.get();
    return ORBX_OK;
  }
  std::unique_ptr<Plan> P(new (std::nothrow) Plan());
  if (!P) return ORBX_ERR_HIP;
  orbx_status s = build_plan(h->params, h->tables, W, H, *P);
  if (s != ORBX_OK) return s;
  hipError_t e;
  if ((e = P->dG.ensure(1)) != hipSuccess) return ORBX_ERR_HIP;
  if ((e = P->dcells.ensure(P->cells.size())) != hipSuccess) return ORBX_ERR_HIP;
  if ((e = P->dtiles.ensure(P->tile_level.size())) != hipSuccess) return ORBX_ERR_HIP;
  if ((e = P->dxt.ensure(P->xt.size())) != hipSuccess) return ORBX_ERR_HIP;
  if ((e = P->dyt.ensure(P->yt.size())) != hipSuccess) return ORBX_ERR_HIP;
  e = hipMemcpy(P->dG.p, &P->G, sizeof(Geometry), hipMemcpyHostToDevice);
  if (e == hipSuccess && !P->cells.empty())
    e = hipMemcpy(P->dcells.p, P->cells.data(), P->cells.size() * sizeof(CellInfo), hipMemcpyHostToDevice);
  if (e == hipSuccess && !P->tile_level.empty())
    e = hipMemcpy(P->dtiles.p, P->tile_level.data(), P->tile_level.size() * sizeof(int), hipMemcpyHostToDevice);
  if (e == hipSuccess && !P->xt.empty())
    e = hipMemcpy(P->dxt.p, P->xt.data(), P->xt.size() * sizeof(ResizeX), hipMemcpyHostToDevice);
  if (e == hipSuccess && !P->yt.empty())
    e = hipMemcpy(P->dyt.p, P->yt.data(), P->yt.size() * sizeof(ResizeY), hipMemcpyHostToDevice);
  if (e != hipSuccess) return ORBX_ERR_HIP;
  {
    size_t mx = 0;
    for (int g = 0; g < P->G.n_og; g++)
      mx = std::max(mx, octree_smem_host(P->G.og[g].node_cap, P->G.og[g].cell_cap, P->G.og[g].kcap));
    mx = std::max(mx, octree_smem_host(P->G.og_all.node_cap, P->G.og_all.cell_cap, P->G.og_all.kcap));
    e = octree_set_smem_limit(mx);
  }
  if (e != hipSuccess) return ORBX_ERR_HIP;
  *out = P.get();
  h->plans[key] = std::move(P);
  return ORBX_OK;
}

orbx_status ensure_batch(orbx_extractor* h, const Plan& P, int n) {
  const Geometry& G = P.G;
  hipError_t e = hipSuccess;
  auto chk = [&](hipError_t x) { if (x != hipSuccess) e = x; };
  chk(h->pyr.ensure((size_t)G.pyr_bytes * n + 256));
  chk(h->blur.ensure((size_t)G.blur_bytes * n + 256));
  chk(h->cand.ensure((size_t)G.cand_total * n));
  chk(h->kpos.ensure((size_t)G.cand_total * n));
  chk(h->knode.ensure((size_t)G.cand_total * n));
  chk(h->cell_count.ensure((size_t)std::max(G.ncells, 1) * n));
  chk(h->oct.ensure((size_t)G.oct_total * n));
  chk(h->oct_count.ensure((size_t)G.nlevels * n));
  return hip_status(e);
}

BatchPtrs batch_ptrs(orbx_extractor* h, const uint8_t* in, size_t pitch) {
  BatchPtrs B;
  B.in = in;
  B.in_pitch = pitch;
  B.pyr = h->pyr.p;
  B.blur = h->blur.p;
  B.cand = h->cand.p;
  B.cell_count = h->cell_count.p;
  B.kpos = h->kpos.p;
  B.knode = h->knode.p;
  B.oct = h->oct.p;
  B.oct_count = h->oct_count.p;
  return B;
}

orbx_status run_extract(orbx_extractor* h, Plan* P, int n, const uint8_t* d_in, size_t pitch, orbx_keypoint* d_kps,
                        uint8_t* d_desc, int32_t* d_counts, int kp_cap, hipStream_t st) {
  if (kp_cap < P->G.max_kps) return ORBX_ERR_CAPACITY;
  orbx_status s = ensure_batch(h, *P, n);
  if (s != ORBX_OK) return s;
  BatchPtrs B = batch_ptrs(h, d_in, pitch);
  hipError_t e = launch_extract_stages(P->G, P->dG.p, P->dcells.p, P->dtiles.p, P->dxt.p, P->dyt.p, B, n, d_kps,
                                       d_desc, d_counts, kp_cap, st, &h->timer);
  if (e != hipSuccess) return ORBX_ERR_HIP;
  h->last_plan = P;
  h->last_in = d_in;
  h->last_pitch = pitch;
  h->last_n = n;
  h->last_host = false;  // orbx_extract sets it again after its readback
  h->hpyr_valid = false;
  return ORBX_OK;
}

hipStream_t pick_stream(orbx_extractor* h, void* s) {
  return s == ORBX_STREAM_NULL ? (hipStream_t)0 : s ? (hipStream_t)s : h->stream;
}

// 64-bit fingerprint of n keypoint records and their descriptors (multiply-xorshift over 32-bit
// words, a few microseconds for 2,000 keypoints): orbx_stereo_match uses the device copies of the
// extraction only when the caller hands back exactly what that extraction returned
uint64_t fingerprint_words(const void* p, size_t nw, uint64_t h) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(p);
  for (size_t i = 0; i < nw; i++) {
    h = (h ^ w[i]) * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
  }
  return h;
}
uint64_t keypoint_fingerprint(const orbx_keypoint* k, const uint8_t* desc, int n) {
  uint64_t h = 1469598103934665603ull ^ (uint64_t)n;
  h = fingerprint_words(k, (size_t)n * (sizeof(orbx_keypoint) / 4), h);
  if (desc) h = fingerprint_words(desc, (size_t)n * 8, h ^ 0xD6E8FEB86659FD93ull);
  return h;
}

bool params_ok(const orbx_extractor_params* p) {
  return p && p->nlevels >= 1 && p->nlevels <= kMaxLevelsPlan && p->scale_factor > 0.f && p->nfeatures >= 0;
}

}  // namespace

extern "C" {

const char* orbx_version(void) { return "orbx 0.1.0 (gfx950)"; }

long long orbx_sizeof(const char* type) {
  if (!type) return -1;
  const std::string t(type);
#define ORBX_SIZEOF(T) \
  if (t == #T) return (long long)sizeof(T);
  ORBX_SIZEOF(orbx_keypoint) ORBX_SIZEOF(orbx_extractor_params) ORBX_SIZEOF(orbx_bow_side)
  ORBX_SIZEOF(orbx_bow_problem) ORBX_SIZEOF(orbx_ba_problem) ORBX_SIZEOF(orbx_ba_result)
  ORBX_SIZEOF(orbx_pnp_problem) ORBX_SIZEOF(orbx_pnp_params) ORBX_SIZEOF(orbx_pnp_result)
  ORBX_SIZEOF(orbx_rand_state) ORBX_SIZEOF(orbx_proj_frame) ORBX_SIZEOF(orbx_proj_problem)
  ORBX_SIZEOF(orbx_tri_kf) ORBX_SIZEOF(orbx_tri_problem) ORBX_SIZEOF(orbx_pose_problem)
  ORBX_SIZEOF(orbx_track_gather) ORBX_SIZEOF(orbx_frame_points) ORBX_SIZEOF(orbx_track_step)
  ORBX_SIZEOF(orbx_camera) ORBX_SIZEOF(orbx_sim3_problem) ORBX_SIZEOF(orbx_init_problem)
#undef ORBX_SIZEOF
  return -1;
}

int orbx_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

orbx_status orbx_extractor_create(const orbx_extractor_params* params, int device, orbx_extractor** out) {
  if (!out || !params_ok(params)) return ORBX_ERR_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return ORBX_ERR_NODEV;
  if (device < 0 || device >= n) return ORBX_ERR_ARG;
  if (hipSetDevice(device) != hipSuccess) return ORBX_ERR_HIP;
  orbx_extractor* h = new (std::nothrow) orbx_extractor();
  if (!h) return ORBX_ERR_HIP;
  h->params = *params;
  h->device = device;
  h->tables = make_tables(*params);
  int gauss[7];
  gaussian_int_kernel(gauss);
  if (upload_constants(h->tables.umax, gauss) != hipSuccess ||
      hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
    delete h;
    return ORBX_ERR_HIP;
  }
  *out = h;
  return ORBX_OK;
}

void orbx_extractor_destroy(orbx_extractor* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  if (h->stream) {
    (void)hipStreamSynchronize(h->stream);
    (void)hipStreamDestroy(h->stream);
  }
  delete h;
}

int orbx_extractor_get_levels(const orbx_extractor* h) { return h ? h->params.nlevels : ORBX_ERR_ARG; }

orbx_status orbx_extractor_scale_tables(const orbx_extractor* h, float* scale, float* inv_scale, float* sigma2,
                                        float* inv_sigma2) {
  if (!h) return ORBX_ERR_ARG;
  const int n = h->params.nlevels;
  for (int i = 0; i < n; i++) {
    if (scale) scale[i] = h->tables.scale[i];
    if (inv_scale) inv_scale[i] = h->tables.inv_scale[i];
    if (sigma2) sigma2[i] = h->tables.sigma2[i];
    if (inv_sigma2) inv_sigma2[i] = h->tables.inv_sigma2[i];
  }
  return ORBX_OK;
}

orbx_status orbx_extractor_tables(const orbx_extractor* h, int* features_per_level, int* umax, int* pattern) {
  if (!h) return ORBX_ERR_ARG;
  static const int8_t kPattern[512 * 2] = {
#include "brief_pattern_31.inc"
  };
  for (int i = 0; i < h->params.nlevels; i++)
    if (features_per_level) features_per_level[i] = h->tables.nfeat[i];
  for (int v = 0; v < 16; v++)
    if (umax) umax[v] = h->tables.umax[v];
  for (int i = 0; i < 1024; i++)
    if (pattern) pattern[i] = kPattern[i];
  return ORBX_OK;
}

orbx_status orbx_extractor_set_pyramid_readback(orbx_extractor* h, int on) {
  if (!h) return ORBX_ERR_ARG;
  h->pyr_readback = on != 0;
  if (!h->pyr_readback) h->hpyr_valid = false;
  return ORBX_OK;
}

int orbx_extractor_max_keypoints(orbx_extractor* h, int width, int height) {
  if (!h) return ORBX_ERR_ARG;
  Plan* P = nullptr;
  orbx_status s = get_plan(h, width, height, &P);
  return s == ORBX_OK ? P->G.max_kps : s;
}

orbx_status orbx_extract(orbx_extractor* h, const uint8_t* img, int width, int height, size_t stride,
                         orbx_keypoint* kps, int cap, uint8_t* desc, int* n) {
  if (!h || !n) return ORBX_ERR_ARG;
  *n = 0;
  if (!img || width <= 0 || height <= 0) return ORBX_OK;  // src/ORBextractor.cc:1141
  if (stride < (size_t)width) return ORBX_ERR_ARG;
  if (hipSetDevice(h->device) != hipSuccess) return ORBX_ERR_HIP;
  Plan* P = nullptr;
  orbx_status s = get_plan(h, width, height, &P);
  if (s != ORBX_OK) return s;
  const int kcap = P->G.max_kps;
  hipError_t e = hipSuccess;
  auto chk = [&](hipError_t x) { if (x != hipSuccess) e = x; };
  const size_t npx = (size_t)width * height;
  h->out_kps = 256;
  h->out_desc = h->out_kps + (((size_t)kcap * sizeof(orbx_keypoint) + 255) & ~(size_t)255);
  h->out_bytes = h->out_desc + (size_t)kcap * 32;
  chk(h->in.ensure(npx));
  chk(h->out.ensure(h->out_bytes));
  chk(h->ensure_stage(std::max(npx, h->out_bytes)));
  if (e != hipSuccess) return ORBX_ERR_HIP;
  hipStream_t st = h->stream;
  // the image through pinned staging (a pageable copy is staged by the runtime, synchronously)
  for (int y = 0; y < height; y++) std::memcpy(h->hstage + (size_t)y * width, img + (size_t)y * stride, width);
  if (hipMemcpyAsync(h->in.p, h->hstage, npx, hipMemcpyHostToDevice, st) != hipSuccess) return ORBX_ERR_HIP;
  int32_t* d_count = (int32_t*)h->out.p;
  orbx_keypoint* d_kps = (orbx_keypoint*)(h->out.p + h->out_kps);
  uint8_t* d_desc = h->out.p + h->out_desc;
  s = run_extract(h, P, 1, h->in.p, npx, d_kps, d_desc, d_count, kcap, st);
  if (s != ORBX_OK) return s;
  const bool pyr = h->pyr_readback;
  if (pyr) {
    // mvImagePyramid (src/ORBextractor.cc:1215-1250 rebuilds it on every call): levels 1.. leave in
    // one more D2H behind the output block; level 0 is the staged input, copied on the host while
    // the kernels run
    h->hpyr_l0 = (npx + 255) & ~(size_t)255;
    if (h->ensure_hpyr(h->hpyr_l0 + (size_t)P->G.pyr_bytes) != hipSuccess) return ORBX_ERR_HIP;
  }
  // count, keypoints and descriptors in ONE copy, then the stream's only synchronisation
  chk(hipMemcpyAsync(h->hstage, h->out.p, h->out_bytes, hipMemcpyDeviceToHost, st));
  if (pyr && P->G.nlevels > 1)
    chk(hipMemcpyAsync(h->hpyr + h->hpyr_l0, h->pyr.p, (size_t)P->G.pyr_bytes, hipMemcpyDeviceToHost, st));
  if (pyr)  // from the caller's image (hstage is the output's destination by now)
    for (int y = 0; y < height; y++) std::memcpy(h->hpyr + (size_t)y * width, img + (size_t)y * stride, width);
  chk(hipStreamSynchronize(st));
  if (e != hipSuccess) return ORBX_ERR_HIP;
  const int32_t cnt = *(const int32_t*)h->hstage;
  *n = cnt;
  if (cnt > cap) return ORBX_ERR_CAPACITY;
  const orbx_keypoint* hk = (const orbx_keypoint*)(h->hstage + h->out_kps);
  if (cnt > 0) {
    if (kps) std::memcpy(kps, hk, sizeof(orbx_keypoint) * cnt);
    if (desc) std::memcpy(desc, h->hstage + h->out_desc, (size_t)32 * cnt);
  }
  h->last_host = true;
  h->hpyr_valid = pyr;
  h->last_fp_n = cnt;
  h->last_fp = keypoint_fingerprint(hk, h->hstage + h->out_desc, cnt);
  return ORBX_OK;
}

orbx_status orbx_pyramid_level(orbx_extractor* h, int image, int level, uint8_t* dst, size_t dst_stride,
                               int* width, int* height) {
  if (!h) return ORBX_ERR_ARG;
  if (!h->last_plan) return ORBX_ERR_STATE;
  const Geometry& G = h->last_plan->G;
  if (level < 0 || level >= G.nlevels || image < 0 || image >= h->last_n) return ORBX_ERR_ARG;
  const int w = G.lv[level].w, hh = G.lv[level].h;
  if (width) *width = w;
  if (height) *height = hh;
  if (!dst) return ORBX_OK;
  if (dst_stride < (size_t)w) return ORBX_ERR_ARG;
  if (h->hpyr_valid && image == 0) {
    // staged by the last orbx_extract: a host copy, no device call
    const uint8_t* src = level == 0 ? h->hpyr : h->hpyr + h->hpyr_l0 + G.lv[level].off;
    for (int y = 0; y < hh; y++) std::memcpy(dst + (size_t)y * dst_stride, src + (size_t)y * w, w);
    return ORBX_OK;
  }
  if (hipSetDevice(h->device) != hipSuccess) return ORBX_ERR_HIP;
  BatchPtrs B = batch_ptrs(h, h->last_in, h->last_pitch);
  const uint8_t* src = level_ptr(G, B, image, level);
  hipError_t e = hipMemcpy2DAsync(dst, dst_stride, src, w, w, hh, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  return hip_status(e);
}

orbx_status orbx_extract_batch_device(orbx_extractor* h, int n_images, const uint8_t* d_images, int width,
                                      int height, size_t image_pitch, orbx_keypoint* d_kps, uint8_t* d_desc,
                                      int32_t* d_counts, int kp_capacity, void* stream) {
  if (!h || n_images < 0 || !d_kps || !d_desc || !d_counts) return ORBX_ERR_ARG;
  if (n_images == 0) return ORBX_OK;
  if (!d_images || width <= 0 || height <= 0 || image_pitch < (size_t)width * height) return ORBX_ERR_ARG;
  if (hipSetDevice(h->device) != hipSuccess) return ORBX_ERR_HIP;
  Plan* P = nullptr;
  orbx_status s = get_plan(h, width, height, &P);
  if (s != ORBX_OK) return s;
  return run_extract(h, P, n_images, d_images, image_pitch, d_kps, d_desc, d_counts, kp_capacity,
                     pick_stream(h, stream));
}

static orbx_status run_stereo(orbx_extractor* hl, orbx_extractor* hr, int n_frames, const orbx_keypoint* kL,
                              const uint8_t* dL, const int32_t* nL, long long kL_stride, long long nL_stride,
                              const orbx_keypoint* kR, const uint8_t* dR, const int32_t* nR, long long kR_stride,
                              long long nR_stride, int l_step, int l_off, int r_step, int r_off, int maxL,
                              float bf, float baseline, float* uR, float* depth, long long out_stride,
                              int32_t* nmatches, hipStream_t st) {
  orbx_extractor* h = hl;
  Plan* P = hl->last_plan;
  hipError_t e = hipSuccess;
  auto chk = [&](hipError_t x) { if (x != hipSuccess) e = x; };
  chk(h->rkeys.ensure((size_t)n_frames * kMaxStereoKps));
  chk(h->oct_start.ensure((size_t)n_frames * (kMaxLevelsPlan + 1)));
  chk(h->rxi.ensure((size_t)n_frames * kMaxStereoKps));
  chk(h->rdesc.ensure((size_t)n_frames * kMaxStereoKps * 2));
  chk(h->rtab.ensure((size_t)n_frames * P->G.nlevels * std::max(P->G.height, 1)));
  chk(h->lrange.ensure((size_t)n_frames * std::max(maxL, 1)));
  chk(h->sad.ensure((size_t)n_frames * out_stride));
  if (e != hipSuccess) return ORBX_ERR_HIP;
  StereoArgs A;
  std::memset(&A, 0, sizeof(A));
  A.kpL = kL;
  A.dL = dL;
  A.nL = nL;
  A.kL_stride = kL_stride;
  A.n_stride_L = nL_stride;
  A.kpR = kR;
  A.dR = dR;
  A.nR = nR;
  A.kR_stride = kR_stride;
  A.n_stride_R = nR_stride;
  A.BL = batch_ptrs(hl, hl->last_in, hl->last_pitch);
  A.BR = batch_ptrs(hr, hr->last_in, hr->last_pitch);
  A.l_step = l_step;
  A.l_off = l_off;
  A.r_step = r_step;
  A.r_off = r_off;
  A.nlevels = P->G.nlevels;
  A.maxL = maxL;
  for (int l = 0; l < P->G.nlevels; l++) A.inv_scale[l] = hl->tables.inv_scale[l];
  A.bf = bf;
  A.minZ = baseline;
  A.minD = 0.f;
  A.maxD = bf / baseline;  // mbf/minZ, src/Frame.cc:595-597
  A.uR = uR;
  A.depth = depth;
  A.sad = h->sad.p;
  A.out_stride = out_stride;
  A.rkeys = h->rkeys.p;
  A.oct_start = h->oct_start.p;
  A.rxi = h->rxi.p;
  A.rdesc = h->rdesc.p;
  A.rtab = h->rtab.p;
  A.lrange = h->lrange.p;
  A.rows = std::max(P->G.height, 1);
  A.nmatches = nmatches;
  return hip_status(launch_stereo(A, P->dG.p, n_frames, maxL, st, &h->timer));
}

orbx_status orbx_stereo_match(orbx_extractor* left, orbx_extractor* right, const orbx_keypoint* kpsL,
                              const uint8_t* descL, int nL, const orbx_keypoint* kpsR, const uint8_t* descR,
                              int nR, float bf, float baseline, float* uRight, float* depth) {
  if (!left || !right || !uRight || !depth || nL < 0 || nR < 0) return ORBX_ERR_ARG;
  if ((nL > 0 && (!kpsL || !descL)) || (nR > 0 && (!kpsR || !descR))) return ORBX_ERR_ARG;
  if (!left->last_plan || !right->last_plan) return ORBX_ERR_STATE;
  // the pyramids must belong to the supplied keypoints: each handle's last call was orbx_extract and
  // returned exactly these keypoints (src/Frame.cc:556,681 read mpORBextractorLeft/Right->mvImagePyramid
  // of the extraction that produced mvKeys/mvKeysRight)
  if (!left->last_host || !right->last_host || nL != left->last_fp_n || nR != right->last_fp_n ||
      (nL > 0 && keypoint_fingerprint(kpsL, descL, nL) != left->last_fp) ||
      (nR > 0 && keypoint_fingerprint(kpsR, descR, nR) != right->last_fp))
    return ORBX_ERR_STATE;
  if (left->last_plan->G.width != right->last_plan->G.width ||
      left->last_plan->G.height != right->last_plan->G.height || left->device != right->device)
    return ORBX_ERR_ARG;
  if (nR > kMaxStereoKps) return ORBX_ERR_CAPACITY;
  if (nL == 0) return ORBX_OK;
  orbx_extractor* h = left;
  if (hipSetDevice(h->device) != hipSuccess) return ORBX_ERR_HIP;
  hipError_t e = hipSuccess;
  auto chk = [&](hipError_t x) { if (x != hipSuccess) e = x; };
  chk(h->sres.ensure(2 * (size_t)nL));
  chk(h->nmatch.ensure(1));
  chk(h->ensure_stage(std::max(h->hstage_cap, (size_t)8 * nL)));
  if (e != hipSuccess) return ORBX_ERR_HIP;
  hipStream_t st = h->stream;
  // The keypoints and descriptors are the ones each handle's last orbx_extract left on the device
  // (the fingerprints above prove it): no upload.  orbx_extract synchronised both streams before
  // returning them, so the right handle's block and pyramid are complete.
  const int32_t* cL = (const int32_t*)left->out.p;
  const int32_t* cR = (const int32_t*)right->out.p;
  orbx_status s = run_stereo(left, right, 1, (const orbx_keypoint*)(left->out.p + left->out_kps),
                             left->out.p + left->out_desc, cL, 0, 0,
                             (const orbx_keypoint*)(right->out.p + right->out_kps), right->out.p + right->out_desc,
                             cR, 0, 0, 0, 0, 0, 0, nL, bf, baseline, h->sres.p, h->sres.p + nL, nL, h->nmatch.p, st);
  if (s != ORBX_OK) return s;
  chk(hipMemcpyAsync(h->hstage, h->sres.p, sizeof(float) * 2 * nL, hipMemcpyDeviceToHost, st));
  chk(hipStreamSynchronize(st));
  if (e != hipSuccess) return ORBX_ERR_HIP;
  std::memcpy(uRight, h->hstage, sizeof(float) * nL);
  std::memcpy(depth, h->hstage + sizeof(float) * nL, sizeof(float) * nL);
  return ORBX_OK;
}

orbx_status orbx_frame_stereo(orbx_extractor* h, const uint8_t* imL, size_t strideL, const uint8_t* imR,
                              size_t strideR, int width, int height, float bf, float baseline, orbx_keypoint* kpsL,
                              uint8_t* descL, int capL, int* nL, orbx_keypoint* kpsR, uint8_t* descR, int capR,
                              int* nR, float* uRight, float* depth) {
  if (!h || !nL || !nR) return ORBX_ERR_ARG;
  *nL = *nR = 0;
  if (!imL || !imR || width <= 0 || height <= 0) return ORBX_ERR_ARG;
  if (strideL < (size_t)width || strideR < (size_t)width) return ORBX_ERR_ARG;
  if (hipSetDevice(h->device) != hipSuccess) return ORBX_ERR_HIP;
  Plan* P = nullptr;
  orbx_status s = get_plan(h, width, height, &P);
  if (s != ORBX_OK) return s;
  const int kc = P->G.max_kps;
  if (kc > kMaxStereoKps) return ORBX_ERR_CAPACITY;
  // device output block: counts (L, R) and the match count | keypoints (L | R, kc each) |
  // descriptors (L | R) | uRight | depth -- one copy back; the images go in as a batch of two
  const size_t npx = (size_t)width * height;
  const size_t o_kps = 256, o_desc = o_kps + (((size_t)2 * kc * sizeof(orbx_keypoint) + 255) & ~(size_t)255),
               o_ur = o_desc + (size_t)2 * kc * 32, o_dep = o_ur + (size_t)kc * 4, o_end = o_dep + (size_t)kc * 4;
  hipError_t e = hipSuccess;
  auto chk = [&](hipError_t x) { if (x != hipSuccess) e = x; };
  chk(h->in.ensure(2 * npx));
  chk(h->out.ensure(o_end));
  chk(h->ensure_stage(std::max(2 * npx, o_end)));
  if (e != hipSuccess) return ORBX_ERR_HIP;
  hipStream_t st = h->stream;
  // the left image's copy runs while the right one is staged
  uint8_t* hs = h->hstage;
  for (int y = 0; y < height; y++) std::memcpy(hs + (size_t)y * width, imL + (size_t)y * strideL, width);
  chk(hipMemcpyAsync(h->in.p, hs, npx, hipMemcpyHostToDevice, st));
  for (int y = 0; y < height; y++) std::memcpy(hs + npx + (size_t)y * width, imR + (size_t)y * strideR, width);
  chk(hipMemcpyAsync(h->in.p + npx, hs + npx, npx, hipMemcpyHostToDevice, st));
  if (e != hipSuccess) return ORBX_ERR_HIP;
  int32_t* d_counts = (int32_t*)h->out.p;
  orbx_keypoint* d_kps = (orbx_keypoint*)(h->out.p + o_kps);
  uint8_t* d_desc = h->out.p + o_desc;
  float* d_ur = (float*)(h->out.p + o_ur);
  float* d_dep = (float*)(h->out.p + o_dep);
  s = run_extract(h, P, 2, h->in.p, npx, d_kps, d_desc, d_counts, kc, st);
  if (s != ORBX_OK) return s;
  // images 0 (left) and 1 (right) of the batch: strides 1 frame apart, as orbx_stereo_frames_device
  s = run_stereo(h, h, 1, d_kps, d_desc, d_counts, 2 * (long long)kc, 2, d_kps + kc, d_desc + (size_t)kc * 32,
                 d_counts + 1, 2 * (long long)kc, 2, 2, 0, 2, 1, kc, bf, baseline, d_ur, d_dep, kc, d_counts + 2, st);
  if (s != ORBX_OK) return s;
  chk(hipMemcpyAsync(hs, h->out.p, o_end, hipMemcpyDeviceToHost, st));
  chk(hipStreamSynchronize(st));
  if (e != hipSuccess) return ORBX_ERR_HIP;
  // this handle's block no longer holds a single orbx_extract result (orbx_stereo_match refuses it);
  // orbx_pyramid_level serves images 0 / 1 of this batch from the device
  h->last_host = false;
  h->hpyr_valid = false;
  const int cl = ((const int32_t*)hs)[0], cr = ((const int32_t*)hs)[1];
  *nL = cl;
  *nR = cr;
  if (cl > capL || cr > capR) return ORBX_ERR_CAPACITY;
  const orbx_keypoint* hk = (const orbx_keypoint*)(hs + o_kps);
  if (cl > 0) {
    if (kpsL) std::memcpy(kpsL, hk, sizeof(orbx_keypoint) * cl);
    if (descL) std::memcpy(descL, hs + o_desc, (size_t)32 * cl);
    if (uRight) std::memcpy(uRight, hs + o_ur, sizeof(float) * cl);
    if (depth) std::memcpy(depth, hs + o_dep, sizeof(float) * cl);
  }
  if (cr > 0) {
    if (kpsR) std::memcpy(kpsR, hk + kc, sizeof(orbx_keypoint) * cr);
    if (descR) std::memcpy(descR, hs + o_desc + (size_t)kc * 32, (size_t)32 * cr);
  }
  return ORBX_OK;
}

orbx_status orbx_stereo_frames_device(orbx_extractor* h, int n_frames, const uint8_t* d_images, int width,
                                      int height, size_t image_pitch, orbx_keypoint* d_kps, uint8_t* d_desc,
                                      int32_t* d_counts, int kp_capacity, float bf, float baseline,
                                      float* d_uright, float* d_depth, int32_t* d_nmatches, void* stream) {
  if (!h || n_frames < 0 || !d_uright || !d_depth || !d_nmatches) return ORBX_ERR_ARG;
  if (n_frames == 0) return ORBX_OK;
  orbx_status s = orbx_extract_batch_device(h, 2 * n_frames, d_images, width, height, image_pitch, d_kps, d_desc,
                                            d_counts, kp_capacity, stream);
  if (s != ORBX_OK) return s;
  if (h->last_plan->G.max_kps > kMaxStereoKps) return ORBX_ERR_CAPACITY;
  const long long kc = kp_capacity;
  return run_stereo(h, h, n_frames, d_kps, d_desc, d_counts, 2 * kc, 2, d_kps + kc, d_desc + kc * 32, d_counts + 1,
                    2 * kc, 2, 2, 0, 2, 1, h->last_plan->G.max_kps, bf, baseline, d_uright, d_depth, kc,
                    d_nmatches, pick_stream(h, stream));
}

static orbx_status bow_host(const orbx_bow_side* A, const orbx_bow_side* B, float nnratio, int check_ori, int mode,
                            int32_t* match, int* nmatches, int device) {
  if (!A || !B || !match || !nmatches) return ORBX_ERR_ARG;
  const int nout = mode ? A->n : B->n;
  *nmatches = 0;
  if (A->n > kMaxBowFeatures || B->n > kMaxBowFeatures || A->n < 0 || B->n < 0) return ORBX_ERR_CAPACITY;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return ORBX_ERR_NODEV;
  if (device < 0 || device >= ndev || hipSetDevice(device) != hipSuccess) return ORBX_ERR_ARG;
  // one arena: both sides' arrays + outputs + the problem descriptor
  auto side_bytes = [](const orbx_bow_side* s) {
    return (size_t)s->n * 32 + (size_t)s->n * 4 + (size_t)s->n + (size_t)s->n_nodes * 4 +
           (size_t)(s->n_nodes + 1) * 4 + (size_t)(s->n_nodes ? s->node_off[s->n_nodes] : 0) * 4 + 64;
  };
  const size_t bytes = side_bytes(A) + side_bytes(B) + (size_t)nout * 4 + 64 + sizeof(BowProblem) + 64;
  // a pooled lease (orbx_scratch.h): no allocation, no device-wide synchronisation per call
  ScratchGuard g(device);
  if (!g.l || g.l->reserve(bytes, bytes) != hipSuccess) return ORBX_ERR_HIP;
  uint8_t* host = g.l->h;
  uint8_t* dbase = g.l->d;
  size_t off = 0;
  auto put = [&](const void* src, size_t nbytes) -> void* {
    off = (off + 15) & ~(size_t)15;
    if (src && nbytes) std::memcpy(host + off, src, nbytes);
    void* d = dbase + off;
    off += nbytes;
    return d;
  };
  auto side = [&](const orbx_bow_side* s) {
    orbx_bow_side d = *s;
    const int nf = s->n_nodes ? s->node_off[s->n_nodes] : 0;
    d.desc = (const uint8_t*)put(s->desc, (size_t)s->n * 32);
    d.angle = (const float*)put(s->angle, (size_t)s->n * 4);
    d.valid = s->valid ? (const uint8_t*)put(s->valid, (size_t)s->n) : nullptr;
    d.node_id = (const uint32_t*)put(s->node_id, (size_t)s->n_nodes * 4);
    d.node_off = (const int32_t*)put(s->node_off, (size_t)(s->n_nodes + 1) * 4);
    d.feat = (const int32_t*)put(s->feat, (size_t)nf * 4);
    return d;
  };
  BowProblem P;
  std::memset(&P, 0, sizeof(P));  // no device-count overrides on the host path
  P.a = side(A);
  P.b = side(B);
  P.nnratio = nnratio;
  P.check_ori = check_ori;
  P.mode = mode;
  const size_t o_out = (off + 15) & ~(size_t)15;
  P.match = (int32_t*)put(nullptr, (size_t)nout * 4);
  P.nmatches = (int32_t*)put(nullptr, 4);
  const size_t o_end = off;
  BowProblem* dP = (BowProblem*)put(&P, sizeof(P));
  hipStream_t st = g.l->st;
  // outputs [o_out, o_end) come back in one copy: matches then the count
  hipError_t e = hipMemcpyAsync(dbase, host, off, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = launch_search_by_bow(dP, 1, st);
  if (e == hipSuccess) e = hipMemcpyAsync(host + o_out, dbase + o_out, o_end - o_out, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = g.l->sync();
  if (e != hipSuccess) return ORBX_ERR_HIP;
  if (nout) std::memcpy(match, host + o_out, (size_t)nout * 4);
  std::memcpy(nmatches, host + ((uint8_t*)P.nmatches - dbase), 4);
  return ORBX_OK;
}

orbx_status orbx_search_by_bow_kf_f(const orbx_bow_side* kf, const orbx_bow_side* f, float nnratio, int check_ori,
                                    int32_t* match_f, int* nmatches, int device) {
  return bow_host(kf, f, nnratio, check_ori, 0, match_f, nmatches, device);
}

orbx_status orbx_search_by_bow_kf_kf(const orbx_bow_side* kf1, const orbx_bow_side* kf2, float nnratio,
                                     int check_ori, int32_t* match12, int* nmatches, int device) {
  return bow_host(kf1, kf2, nnratio, check_ori, 1, match12, nmatches, device);
}

orbx_status orbx_search_by_bow_device(const orbx_bow_problem* problems, int n, void* stream) {
  if (n < 0 || (n > 0 && !problems)) return ORBX_ERR_ARG;
  if (n == 0) return ORBX_OK;
  for (int i = 0; i < n; i++)
    if (problems[i].a.n > kMaxBowFeatures || problems[i].b.n > kMaxBowFeatures) return ORBX_ERR_CAPACITY;
  hipStream_t st = (hipStream_t)stream;
  BowProblem* dP = nullptr;
  if (hipMallocAsync((void**)&dP, sizeof(BowProblem) * n, st) != hipSuccess) return ORBX_ERR_HIP;
  hipError_t e = hipMemcpyAsync(dP, problems, sizeof(BowProblem) * n, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = launch_search_by_bow(dP, n, st);
  hipError_t e2 = hipFreeAsync(dP, st);
  return hip_status(e != hipSuccess ? e : e2);
}

orbx_status orbx_profile_enable(orbx_extractor* h, int enable) {
  if (!h) return ORBX_ERR_ARG;
  h->timer.flush();
  h->timer.enabled = enable != 0;
  return ORBX_OK;
}

orbx_status orbx_profile_reset(orbx_extractor* h) {
  if (!h) return ORBX_ERR_ARG;
  (void)hipSetDevice(h->device);
  h->timer.reset();
  return ORBX_OK;
}

int orbx_profile_read(orbx_extractor* h, int stage, double* total_ms, long long* launches, const char** name) {
  if (!h) return ORBX_ERR_ARG;
  if (stage < 0) return ST_COUNT;
  if (stage >= ST_COUNT) return ORBX_ERR_ARG;
  (void)hipSetDevice(h->device);
  h->timer.flush();
  if (total_ms) *total_ms = h->timer.total_ms[stage];
  if (launches) *launches = h->timer.launches[stage];
  if (name) *name = kStageNames[stage];
  return ORBX_OK;
}

orbx_status orbx_descriptor_distance_device(const uint8_t* d_a, const uint8_t* d_b, int n, int32_t* d_out,
                                            void* stream) {
  if (n < 0 || (n > 0 && (!d_a || !d_b || !d_out))) return ORBX_ERR_ARG;
  return hip_status(launch_hamming(d_a, d_b, n, d_out, (hipStream_t)stream));
}

}  // extern "C"

#include "../../include/orbx_debug.h"

extern "C" long long orbx_debug_copy(orbx_extractor* h, int what, int image, int arg, void* dst, size_t cap) {
  if (!h) return ORBX_ERR_ARG;
  if (!h->last_plan) return ORBX_ERR_STATE;
  const Plan& P = *h->last_plan;
  const Geometry& G = P.G;
  if (image < 0 || image >= h->last_n) return ORBX_ERR_ARG;
  if (hipSetDevice(h->device) != hipSuccess) return ORBX_ERR_HIP;
  if (hipStreamSynchronize(h->stream) != hipSuccess) return ORBX_ERR_HIP;
  std::vector<int> host;
  const void* src = nullptr;
  size_t bytes = 0;
  bool device_src = true;
  switch (what) {
    case ORBX_DBG_BLUR_LEVEL: {
      if (arg < 0 || arg >= G.nlevels) return ORBX_ERR_ARG;
      const LevelGeom& L = G.lv[arg];
      bytes = (size_t)L.w * L.h;
      if (dst && cap >= bytes) {
        // the blurred levels of the last batch, re-blurred from its pyramid (the same bytes k_blur
        // wrote; the batch that follows may have reused the buffer)
        if (h->blur.ensure((size_t)G.blur_bytes * h->last_n + 256) != hipSuccess) return ORBX_ERR_HIP;
        const BatchPtrs B = batch_ptrs(h, h->last_in, h->last_pitch);
        if (launch_blur(G, P.dG.p, P.dtiles.p, B, h->last_n, h->stream) != hipSuccess ||
            hipStreamSynchronize(h->stream) != hipSuccess)
          return ORBX_ERR_HIP;
        const uint8_t* b = h->blur.p + (size_t)image * G.blur_bytes + L.boff;
        std::vector<uint8_t> tiles((size_t)L.bstride * ((L.h + 7) & ~7));
        if (hipMemcpy(tiles.data(), b, tiles.size(), hipMemcpyDeviceToHost) != hipSuccess) return ORBX_ERR_HIP;
        uint8_t* o = static_cast<uint8_t*>(dst);
        for (int yy = 0; yy < L.h; yy++)
          for (int xx = 0; xx < L.w; xx++)
            o[(size_t)yy * L.w + xx] = tiles[((size_t)(yy >> 3) * (L.bstride >> 4) + (xx >> 4)) * 128 + (yy & 7) * 16 + (xx & 15)];
      }
      return (long long)bytes;
    }
    case ORBX_DBG_CELL_COUNTS:
      src = h->cell_count.p + (size_t)image * G.ncells;
      bytes = sizeof(int) * G.ncells;
      break;
    case ORBX_DBG_CELL_TABLE: {  // cand_off: the cell's slot range in ORBX_DBG_CANDIDATES' view
      int loff = 0;
      for (const CellInfo& c : P.cells) {
        int v[8] = {c.level, c.x0, c.y0, c.x1, c.y1, loff, c.cap, 0};
        host.insert(host.end(), v, v + 8);
        loff += c.cap;
      }
      device_src = false;
      break;
    }
    case ORBX_DBG_CANDIDATES: {  // every cell's slots contiguous (inline then overflow), cells in order
      std::vector<uint32_t> raw((size_t)G.cand_total);
      if (hipMemcpy(raw.data(), h->cand.p + (size_t)image * G.cand_total, raw.size() * 4, hipMemcpyDeviceToHost) !=
          hipSuccess)
        return ORBX_ERR_HIP;
      std::vector<uint32_t> logical;
      logical.reserve(raw.size());
      for (const CellInfo& c : P.cells)
        for (int q = 0; q < c.cap; q++) logical.push_back(raw[cell_slot(c, q)]);
      static_assert(sizeof(uint32_t) == sizeof(int), "host staging is int words");
      host.resize(logical.size());
      std::memcpy(host.data(), logical.data(), logical.size() * 4);
      device_src = false;
      break;
    }
    case ORBX_DBG_OCT_COUNTS:
      src = h->oct_count.p + (size_t)image * G.nlevels;
      bytes = sizeof(int) * G.nlevels;
      break;
    case ORBX_DBG_OCT_OUT:
      src = h->oct.p + (size_t)image * G.oct_total;
      bytes = sizeof(uint32_t) * G.oct_total;
      break;
    case ORBX_DBG_LEVEL_INFO:
      for (int l = 0; l < G.nlevels; l++) {
        const LevelGeom& L = G.lv[l];
        int v[8] = {L.w, L.h, L.cell_begin, L.cell_end, L.oct_off, L.oct_cap, L.nfeat, L.nIni};
        host.insert(host.end(), v, v + 8);
      }
      device_src = false;
      break;
    default:
      return ORBX_ERR_ARG;
  }
  if (!device_src) {
    bytes = host.size() * sizeof(int);
    if (dst) std::memcpy(dst, host.data(), std::min(bytes, cap));
    return (long long)bytes;
  }
  if (dst && cap) {
    if (hipMemcpy(dst, src, std::min(bytes, cap), hipMemcpyDeviceToHost) != hipSuccess) return ORBX_ERR_HIP;
  }
  return (long long)bytes;
}

// On-box HBM reference for the roofline: a streaming device-to-device copy,
// one 16-B non-temporal load + store per thread over the whole buffer (the
// fastest of the forms measured: 6.52 TB/s against 6.21 with default-policy
// accesses and 4.7-5.0 with grid-stride loops).  *ms = mean time per copy.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_hbm_copy(u32x4* __restrict__ dst, const u32x4* __restrict__ src, size_t n) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

extern "C" int orbx_debug_hbm_copy(void* dst, const void* src, size_t bytes, int reps, float* ms) {
  if (!dst || !src || (bytes & 15) || reps < 1 || bytes / 16 / 256 >= (size_t)1 << 31) return ORBX_ERR_ARG;
  const size_t n = bytes / 16;
  const int grid = (int)((n + 255) / 256);
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess) return ORBX_ERR_HIP;
  if (hipEventCreate(&e1) != hipSuccess) {
    (void)hipEventDestroy(e0);
    return ORBX_ERR_HIP;
  }
  hipLaunchKernelGGL(k_hbm_copy, dim3(grid), dim3(256), 0, 0, (u32x4*)dst, (const u32x4*)src, n);  // warm-up
  (void)hipEventRecord(e0, 0);
  for (int r = 0; r < reps; r++)
    hipLaunchKernelGGL(k_hbm_copy, dim3(grid), dim3(256), 0, 0, (u32x4*)dst, (const u32x4*)src, n);
  (void)hipEventRecord(e1, 0);
  hipError_t e = hipEventSynchronize(e1);
  float t = 0;
  if (e == hipSuccess) e = hipEventElapsedTime(&t, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (e != hipSuccess) return ORBX_ERR_HIP;
  if (ms) *ms = t / reps;
  return ORBX_OK;
}
