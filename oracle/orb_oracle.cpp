// orb_oracle.cpp -- CPU ORACLE: restatement of the reference hot path.
//
// TEST INFRASTRUCTURE ONLY (see orb_oracle.h).  Compiled with
// -O2 -ffp-contract=off so float expressions round exactly as written.
// Each function cites the reference file:line it restates.  Where the
// reference defers to OpenCV 3.2 (absent here) the OpenCV generic/SSE2
// arithmetic is restated and the choice documented in DESIGN.md §Parity.
#include "orb_oracle.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <list>
#include <utility>
#include <vector>

namespace {

const int kPatchSize = 31;      // src/ORBextractor.cc:72
const int kHalfPatch = 15;      // src/ORBextractor.cc:73
const int kEdgeThreshold = 19;  // src/ORBextractor.cc:74

const signed char kPattern[1024] = {
#include "brief_pattern_31.inc"
};

// ---------------------------------------------------------------- numerics
// cvRound: SSE2 cvtss2si / cvtsd2si, round-half-even.
inline int round_even(float v) { return (int)std::nearbyintf(v); }
inline int round_even_d(double v) { return (int)std::nearbyint(v); }

// fastAtan2, OpenCV 3.2 core/mathfuncs: 7th order polynomial in degrees.
const float kAtanP1 = 0.9997878412794807f * (float)(180 / M_PI);
const float kAtanP3 = -0.3258083974640975f * (float)(180 / M_PI);
const float kAtanP5 = 0.1555786518463281f * (float)(180 / M_PI);
const float kAtanP7 = -0.04432655554792128f * (float)(180 / M_PI);

float fast_atan2(float y, float x) {
  float ax = std::fabs(x), ay = std::fabs(y);
  float a, c, c2;
  if (ax >= ay) {
    c = ay / (ax + (float)DBL_EPSILON);
    c2 = c * c;
    a = (((kAtanP7 * c2 + kAtanP5) * c2 + kAtanP3) * c2 + kAtanP1) * c;
  } else {
    c = ax / (ay + (float)DBL_EPSILON);
    c2 = c * c;
    a = 90.f - (((kAtanP7 * c2 + kAtanP5) * c2 + kAtanP3) * c2 + kAtanP1) * c;
  }
  if (x < 0) a = 180.f - a;
  if (y < 0) a = 360.f - a;
  return a;
}

// Deterministic float cos/sin (src/ORBextractor.cc:117 calls std::cos/sin on
// float).  Evaluated in double with a fixed operation sequence (Cody-Waite
// reduction by pi/2 + Taylor polynomials) and rounded once to float, so the
// HIP kernels reproduce it bit for bit; agrees with a correctly rounded cosf
// except in astronomically rare near-tie cases.
void sincos_det(float xf, float* s_out, float* c_out) {
  const double x = (double)xf;
  const double kInvPio2 = 6.36619772367581382433e-01;
  const double kPio2Hi = 1.57079632673412561417e+00;
  const double kPio2Lo = 6.07710050650619224932e-11;
  double kd = std::nearbyint(x * kInvPio2);
  int q = (int)kd;
  double r = (x - kd * kPio2Hi) - kd * kPio2Lo;
  double r2 = r * r;
  // sin(r) = r - r^3/3! + ... up to r^21 ; cos(r) = 1 - r^2/2! ... up to r^20
  double ps = 1.0 / 51090942171709440000.0;  // 1/21!
  ps = ps * r2 - 1.0 / 121645100408832000.0;  // 1/19!
  ps = ps * r2 + 1.0 / 355687428096000.0;     // 1/17!
  ps = ps * r2 - 1.0 / 1307674368000.0;       // 1/15!
  ps = ps * r2 + 1.0 / 6227020800.0;          // 1/13!
  ps = ps * r2 - 1.0 / 39916800.0;            // 1/11!
  ps = ps * r2 + 1.0 / 362880.0;              // 1/9!
  ps = ps * r2 - 1.0 / 5040.0;                // 1/7!
  ps = ps * r2 + 1.0 / 120.0;                 // 1/5!
  ps = ps * r2 - 1.0 / 6.0;                   // 1/3!
  double sr = r + r * (r2 * ps);
  double pc = 1.0 / 2432902008176640000.0;    // 1/20!
  pc = pc * r2 - 1.0 / 6402373705728000.0;    // 1/18!
  pc = pc * r2 + 1.0 / 20922789888000.0;      // 1/16!
  pc = pc * r2 - 1.0 / 87178291200.0;         // 1/14!
  pc = pc * r2 + 1.0 / 479001600.0;           // 1/12!
  pc = pc * r2 - 1.0 / 3628800.0;             // 1/10!
  pc = pc * r2 + 1.0 / 40320.0;               // 1/8!
  pc = pc * r2 - 1.0 / 720.0;                 // 1/6!
  pc = pc * r2 + 1.0 / 24.0;                  // 1/4!
  pc = pc * r2 - 0.5;                         // 1/2!
  double cr = 1.0 + r2 * pc;
  double s, c;
  switch (q & 3) {
    case 0: s = sr; c = cr; break;
    case 1: s = cr; c = -sr; break;
    case 2: s = -sr; c = -cr; break;
    default: s = -cr; c = sr; break;
  }
  *s_out = (float)s;
  *c_out = (float)c;
}

// ------------------------------------------------------------ scale tables
struct Tables {
  int nlevels;
  std::vector<float> scale, inv_scale, sigma2, inv_sigma2;
  std::vector<int> nfeat;
  std::vector<int> umax;
};

// ORBextractor::ORBextractor, src/ORBextractor.cc:416-490.
Tables make_tables(const oracle_params& p) {
  Tables t;
  t.nlevels = p.nlevels;
  const double sf = (double)p.scale_factor;  // member is double (include/ORBextractor.h:134)
  t.scale.resize(p.nlevels);
  t.sigma2.resize(p.nlevels);
  t.scale[0] = 1.0f;
  t.sigma2[0] = 1.0f;
  for (int i = 1; i < p.nlevels; i++) {
    t.scale[i] = (float)((double)t.scale[i - 1] * sf);
    t.sigma2[i] = t.scale[i] * t.scale[i];
  }
  t.inv_scale.resize(p.nlevels);
  t.inv_sigma2.resize(p.nlevels);
  for (int i = 0; i < p.nlevels; i++) {
    t.inv_scale[i] = 1.0f / t.scale[i];
    t.inv_sigma2[i] = 1.0f / t.sigma2[i];
  }
  t.nfeat.resize(p.nlevels);
  float factor = (float)(1.0f / sf);
  float ndes = (float)p.nfeatures * (1 - factor) /
               (1 - (float)std::pow((double)factor, (double)p.nlevels));
  int sum = 0;
  for (int l = 0; l < p.nlevels - 1; l++) {
    t.nfeat[l] = round_even(ndes);
    sum += t.nfeat[l];
    ndes *= factor;
  }
  t.nfeat[p.nlevels - 1] = std::max(p.nfeatures - sum, 0);

  t.umax.assign(kHalfPatch + 1, 0);
  int vmax = (int)std::floor(kHalfPatch * std::sqrt(2.f) / 2 + 1);
  int vmin = (int)std::ceil(kHalfPatch * std::sqrt(2.f) / 2);
  const double hp2 = kHalfPatch * kHalfPatch;
  for (int v = 0; v <= vmax; ++v) t.umax[v] = round_even_d(std::sqrt(hp2 - v * v));
  for (int v = kHalfPatch, v0 = 0; v >= vmin; --v) {
    while (t.umax[v0] == t.umax[v0 + 1]) ++v0;
    t.umax[v] = v0;
    ++v0;
  }
  return t;
}

struct Img {
  int w = 0, h = 0;
  std::vector<uint8_t> px;
  uint8_t at(int y, int x) const { return px[(size_t)y * w + x]; }
};

// ------------------------------------------------------------------ resize
// cv::resize(INTER_LINEAR, CV_8U) as called at src/ORBextractor.cc:1236
// (OpenCV 3.2 imgproc/resize.cpp resizeGeneric_ with HResizeLinear<uchar,int,
// short,2048> and the VResizeLinear<uchar,int,short,FixedPtCast<..,22>>
// specialisation, whose scalar body and SSE2 VResizeLinearVec_32s8u both
// compute ((b0*(S0>>4))>>16 + (b1*(S1>>4))>>16 + 2)>>2).
void resize_linear(const Img& src, Img& dst, int dw, int dh) {
  dst.w = dw;
  dst.h = dh;
  dst.px.assign((size_t)dw * dh, 0);
  const int sw = src.w, sh = src.h;
  const double scale_x = 1. / ((double)dw / sw);
  const double scale_y = 1. / ((double)dh / sh);
  std::vector<int> xofs(dw);
  std::vector<short> ialpha(2 * dw);
  int xmax = dw;
  for (int dx = 0; dx < dw; dx++) {
    float fx = (float)((dx + 0.5) * scale_x - 0.5);
    int sx = (int)std::floor(fx);
    fx -= sx;
    if (sx < 0) { fx = 0; sx = 0; }
    if (sx + 1 >= sw) {
      xmax = std::min(xmax, dx);
      if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
    }
    xofs[dx] = sx;
    float c0 = 1.f - fx, c1 = fx;
    ialpha[2 * dx] = (short)round_even(c0 * 2048);
    ialpha[2 * dx + 1] = (short)round_even(c1 * 2048);
  }
  std::vector<int> r0(dw), r1(dw);
  auto hresize = [&](const uint8_t* S, int* D) {
    int dx = 0;
    for (; dx < xmax; dx++) {
      int sx = xofs[dx];
      D[dx] = S[sx] * ialpha[2 * dx] + S[sx + 1] * ialpha[2 * dx + 1];
    }
    for (; dx < dw; dx++) D[dx] = S[xofs[dx]] * 2048;
  };
  for (int dy = 0; dy < dh; dy++) {
    float fy = (float)((dy + 0.5) * scale_y - 0.5);
    int sy = (int)std::floor(fy);
    fy -= sy;
    short b0 = (short)round_even((1.f - fy) * 2048);
    short b1 = (short)round_even(fy * 2048);
    int y0 = std::min(std::max(sy, 0), sh - 1);
    int y1 = std::min(std::max(sy + 1, 0), sh - 1);
    hresize(&src.px[(size_t)y0 * sw], r0.data());
    hresize(&src.px[(size_t)y1 * sw], r1.data());
    uint8_t* out = &dst.px[(size_t)dy * dw];
    for (int x = 0; x < dw; x++)
      out[x] = (uint8_t)((((b0 * (r0[x] >> 4)) >> 16) + ((b1 * (r1[x] >> 4)) >> 16) + 2) >> 2);
  }
}

// ---------------------------------------------------------------- Gaussian
// GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101) at src/ORBextractor.cc:1190.
// OpenCV 3.2: getGaussianKernel(7,2,CV_32F), converted to int32 x256 (cvRound)
// for the 8U fixed-point separable path; row pass exact int; column pass:
// SSE2 SymmColumnVec_32s8u on 4-column groups computes
// rint(acc * 2^-16) in float (round-half-even), the scalar tail
// FixedPtCastEx computes (acc + 2^15) >> 16.  Both saturate to u8.
void gaussian_int_kernel(int k[7]) {
  float cf[7];
  double sum = 0;
  const double sigma = 2.0;
  const double scale2X = -0.5 / (sigma * sigma);
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

inline int reflect101(int p, int n) {
  if (n == 1) return 0;
  while (p < 0 || p >= n) {
    if (p < 0) p = -p;
    if (p >= n) p = 2 * n - 2 - p;
  }
  return p;
}

void gaussian_blur7(const Img& src, Img& dst) {
  int k[7];
  gaussian_int_kernel(k);
  const int w = src.w, h = src.h;
  dst.w = w;
  dst.h = h;
  dst.px.assign((size_t)w * h, 0);
  std::vector<int> rows((size_t)w * h);
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      int s = 0;
      for (int t = -3; t <= 3; t++) s += k[t + 3] * src.at(y, reflect101(x + t, w));
      rows[(size_t)y * w + x] = s;
    }
  const int simd_w = w & ~3;
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      int acc = 0;
      for (int t = -3; t <= 3; t++) acc += k[t + 3] * rows[(size_t)reflect101(y + t, h) * w + x];
      int v;
      if (x < simd_w)
        v = (int)std::nearbyintf((float)acc * (1.0f / 65536.0f));
      else
        v = (acc + (1 << 15)) >> 16;
      dst.px[(size_t)y * w + x] = (uint8_t)std::min(std::max(v, 0), 255);
    }
}

// -------------------------------------------------------------------- FAST
// cv::FAST(img, kps, th, nonmax=true) -> FAST_t<16> + cornerScore<16>
// (OpenCV 3.2 features2d/fast.cpp), called per cell at
// src/ORBextractor.cc:892-900.
const int kRing[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},  {3, 0},  {3, -1},
                          {2, -2}, {1, -3},  {0, -3},  {-1, -3}, {-2, -2}, {-3, -1},
                          {-3, 0}, {-3, 1},  {-2, 2},  {-1, 3}};

// cornerScore<16>: max over the 16 cyclic arcs of 9 of max(min d, -max d),
// minus one, with d = centre - ring.
int corner_score(const uint8_t* p, size_t stride) {
  int v = p[0];
  int d[25];
  for (int k = 0; k < 16; k++) d[k] = v - p[kRing[k][1] * (ptrdiff_t)stride + kRing[k][0]];
  for (int k = 16; k < 25; k++) d[k] = d[k - 16];
  int a0 = -1000, b0 = 1000;
  for (int k = 0; k < 16; k++) {
    int mn = d[k], mx = d[k];
    for (int j = 1; j < 9; j++) {
      mn = std::min(mn, d[k + j]);
      mx = std::max(mx, d[k + j]);
    }
    a0 = std::max(a0, mn);
    b0 = std::min(b0, mx);
  }
  return std::max(a0, -b0) - 1;
}

// Segment test: >= 9 contiguous ring pixels all > v+t or all < v-t.
bool is_corner(const uint8_t* p, size_t stride, int t) {
  int v = p[0];
  int dark = 0, bright = 0;
  int cd = 0, cb = 0;
  for (int k = 0; k < 25; k++) {
    int x = p[kRing[k & 15][1] * (ptrdiff_t)stride + kRing[k & 15][0]];
    if (x < v - t) { if (++cd > 8) dark = 1; } else cd = 0;
    if (x > v + t) { if (++cb > 8) bright = 1; } else cb = 0;
  }
  return dark || bright;
}

struct Kp {
  float x, y, size, angle, response;
  int octave;
};

// FAST on a w x h window: detection rows [3,h-4], cols [3,w-4]; 3x3 strict
// non-max suppression against the window-local score map (0 elsewhere);
// emission row-major.
void fast_window(const uint8_t* img, int w, int h, size_t stride, int threshold, std::vector<Kp>& out) {
  out.clear();
  threshold = std::min(std::max(threshold, 0), 255);
  if (w < 7 || h < 7) return;
  std::vector<int> score((size_t)w * h, 0);
  std::vector<char> corner((size_t)w * h, 0);
  for (int y = 3; y <= h - 4; y++)
    for (int x = 3; x <= w - 4; x++) {
      const uint8_t* p = img + (size_t)y * stride + x;
      if (is_corner(p, stride, threshold)) {
        corner[(size_t)y * w + x] = 1;
        score[(size_t)y * w + x] = corner_score(p, stride);
      }
    }
  for (int y = 3; y <= h - 4; y++)
    for (int x = 3; x <= w - 4; x++) {
      if (!corner[(size_t)y * w + x]) continue;
      int s = score[(size_t)y * w + x];
      bool keep = true;
      for (int dy = -1; dy <= 1 && keep; dy++)
        for (int dx = -1; dx <= 1; dx++) {
          if (!dx && !dy) continue;
          if (!(s > score[(size_t)(y + dy) * w + x + dx])) { keep = false; break; }
        }
      if (keep) out.push_back({(float)x, (float)y, 7.f, -1.f, (float)s, 0});
    }
}

// ----------------------------------------------------------------- octree
// ExtractorNode::DivideNode (src/ORBextractor.cc:501-560) and
// ORBextractor::DistributeOctTree (:562-815).  std::sort over
// (size, ExtractorNode*) at :733 orders equal sizes by heap address; the
// oracle (and the GPU) use the node's creation sequence number instead.
struct Node {
  int x0, y0, x1, y1;  // UL=(x0,y0), UR=(x1,y0), BL=(x0,y1), BR=(x1,y1)
  std::vector<int> keys;  // indices into the candidate vector, in order
  long seq;
  std::list<Node>::iterator self;
};

void divide(const Node& n, const std::vector<Kp>& kp, Node c[4]) {
  const int hx = (int)std::ceil((float)(n.x1 - n.x0) / 2);
  const int hy = (int)std::ceil((float)(n.y1 - n.y0) / 2);
  c[0].x0 = n.x0;      c[0].y0 = n.y0;      c[0].x1 = n.x0 + hx; c[0].y1 = n.y0 + hy;
  c[1].x0 = n.x0 + hx; c[1].y0 = n.y0;      c[1].x1 = n.x1;      c[1].y1 = n.y0 + hy;
  c[2].x0 = n.x0;      c[2].y0 = n.y0 + hy; c[2].x1 = n.x0 + hx; c[2].y1 = n.y1;
  c[3].x0 = n.x0 + hx; c[3].y0 = n.y0 + hy; c[3].x1 = n.x1;      c[3].y1 = n.y1;
  for (int q = 0; q < 4; q++) c[q].keys.clear();
  for (int i : n.keys) {
    const Kp& k = kp[i];
    int q = (k.x < (float)(n.x0 + hx) ? 0 : 1) + (k.y < (float)(n.y0 + hy) ? 0 : 2);
    c[q].keys.push_back(i);
  }
}

std::vector<Kp> distribute_octree(const std::vector<Kp>& kp, int minX, int maxX, int minY, int maxY, int N) {
  std::vector<Kp> result;
  if (kp.empty()) return result;
  int nIni = (int)std::round((float)(maxX - minX) / (maxY - minY));
  if (nIni < 1) nIni = 1;  // reference indexes out of bounds here (tall images): UB guard
  const float hX = (float)(maxX - minX) / nIni;
  std::list<Node> nodes;
  long seq = 0;
  std::vector<Node*> ini(nIni);
  for (int i = 0; i < nIni; i++) {
    Node n;
    n.x0 = (int)(hX * (float)i);
    n.x1 = (int)(hX * (float)(i + 1));
    n.y0 = 0;
    n.y1 = maxY - minY;
    n.seq = seq++;
    nodes.push_back(n);
    ini[i] = &nodes.back();
  }
  for (size_t i = 0; i < kp.size(); i++) ini[(size_t)(kp[i].x / hX)]->keys.push_back((int)i);
  for (auto it = nodes.begin(); it != nodes.end();) {
    if (it->keys.empty()) it = nodes.erase(it); else ++it;
  }
  typedef std::pair<std::pair<int, long>, Node*> Entry;
  std::vector<Entry> expand;
  bool finish = false;
  while (!finish) {
    int prev = (int)nodes.size();
    int nToExpand = 0;
    expand.clear();
    for (auto it = nodes.begin(); it != nodes.end();) {
      if (it->keys.size() == 1) { ++it; continue; }
      Node c[4];
      divide(*it, kp, c);
      for (int q = 0; q < 4; q++) {
        if (c[q].keys.empty()) continue;
        c[q].seq = seq++;
        nodes.push_front(c[q]);
        nodes.front().self = nodes.begin();
        if (c[q].keys.size() > 1) {
          nToExpand++;
          expand.push_back({{(int)nodes.front().keys.size(), nodes.front().seq}, &nodes.front()});
        }
      }
      it = nodes.erase(it);
    }
    if ((int)nodes.size() >= N || (int)nodes.size() == prev) {
      finish = true;
    } else if ((int)nodes.size() + nToExpand * 3 > N) {
      while (!finish) {
        prev = (int)nodes.size();
        std::vector<Entry> prevExpand = expand;
        expand.clear();
        std::sort(prevExpand.begin(), prevExpand.end(),
                  [](const Entry& a, const Entry& b) { return a.first < b.first; });
        for (int j = (int)prevExpand.size() - 1; j >= 0; j--) {
          Node c[4];
          Node* parent = prevExpand[j].second;
          divide(*parent, kp, c);
          for (int q = 0; q < 4; q++) {
            if (c[q].keys.empty()) continue;
            c[q].seq = seq++;
            nodes.push_front(c[q]);
            nodes.front().self = nodes.begin();
            if (c[q].keys.size() > 1)
              expand.push_back({{(int)nodes.front().keys.size(), nodes.front().seq}, &nodes.front()});
          }
          nodes.erase(parent->self);
          if ((int)nodes.size() >= N) break;
        }
        if ((int)nodes.size() >= N || (int)nodes.size() == prev) finish = true;
      }
    }
  }
  // Keep the first maximum-response keypoint of every node (:796-812).
  for (auto& n : nodes) {
    int best = n.keys[0];
    for (size_t k = 1; k < n.keys.size(); k++)
      if (kp[n.keys[k]].response > kp[best].response) best = n.keys[k];
    result.push_back(kp[best]);
  }
  return result;
}

// ------------------------------------------------------------ orientation
// IC_Angle, src/ORBextractor.cc:77-105.
float ic_angle(const Img& im, float px, float py, const std::vector<int>& umax) {
  int m01 = 0, m10 = 0;
  const int cy = round_even(py), cx = round_even(px);
  for (int u = -kHalfPatch; u <= kHalfPatch; ++u) m10 += u * im.at(cy, cx + u);
  for (int v = 1; v <= kHalfPatch; ++v) {
    int vsum = 0;
    int d = umax[v];
    for (int u = -d; u <= d; ++u) {
      int vp = im.at(cy + v, cx + u), vm = im.at(cy - v, cx + u);
      vsum += vp - vm;
      m10 += u * (vp + vm);
    }
    m01 += v * vsum;
  }
  return fast_atan2((float)m01, (float)m10);
}

// Trig used for the keypoint rotation.  0 (default, shared with the GPU): sincos_det.
// 1: the host libm's float cos/sin, literally what src/ORBextractor.cc:117 calls
// (`(float)cos(angle)` with `using namespace std` on a float -> std::cos(float) -> cosf).
// Only the libm-divergence census test (tests/test_oracle_kat.py) sets 1.
static int g_trig_mode = 0;

// computeOrbDescriptor, src/ORBextractor.cc:110-152.
void orb_descriptor(const Img& blurred, const Kp& kp, uint8_t* desc) {
  const float factorPI = (float)(M_PI / 180.f);
  float angle = kp.angle * factorPI;
  float a, b;
  if (g_trig_mode == 1) {
    a = std::cos(angle);
    b = std::sin(angle);
  } else {
    float s, c;
    sincos_det(angle, &s, &c);
    a = c;
    b = s;
  }
  const int cy = round_even(kp.y), cx = round_even(kp.x);
  for (int i = 0; i < 32; ++i) {
    int val = 0;
    for (int k = 0; k < 8; k++) {
      int t[2];
      for (int e = 0; e < 2; e++) {
        const int idx = 32 * i + 4 * k + 2 * e;
        const float x = (float)kPattern[idx], y = (float)kPattern[idx + 1];
        const int r = round_even(x * b + y * a);
        const int c = round_even(x * a - y * b);
        t[e] = blurred.at(cy + r, cx + c);
      }
      val |= (t[0] < t[1]) << k;
    }
    desc[i] = (uint8_t)val;
  }
}

struct Extraction {
  std::vector<Img> pyr;
  std::vector<Kp> kps;
  std::vector<uint8_t> desc;
};

// ORBextractor::operator() (src/ORBextractor.cc:1138-1211) with
// ComputePyramid (:1215-1250) and ComputeKeyPointsOctTree (:818-946).
void extract(const oracle_params& p, const Tables& t, const Img& image, Extraction& ex) {
  ex.pyr.assign(p.nlevels, Img());
  ex.kps.clear();
  ex.desc.clear();
  for (int l = 0; l < p.nlevels; l++) {
    const float s = t.inv_scale[l];
    const int w = round_even((float)image.w * s), h = round_even((float)image.h * s);
    if (l == 0) ex.pyr[0] = image;
    else resize_linear(ex.pyr[l - 1], ex.pyr[l], w, h);
  }
  std::vector<std::vector<Kp>> all(p.nlevels);
  const float W = 30;
  for (int l = 0; l < p.nlevels; l++) {
    const Img& im = ex.pyr[l];
    const int minBX = kEdgeThreshold - 3, minBY = minBX;
    const int maxBX = im.w - kEdgeThreshold + 3, maxBY = im.h - kEdgeThreshold + 3;
    std::vector<Kp> cand;
    const float width = (float)(maxBX - minBX), height = (float)(maxBY - minBY);
    const int nCols = (int)(width / W), nRows = (int)(height / W);
    if (nCols > 0 && nRows > 0) {
      const int wCell = (int)std::ceil(width / nCols), hCell = (int)std::ceil(height / nRows);
      std::vector<Kp> cell;
      for (int i = 0; i < nRows; i++) {
        const float iniY = (float)(minBY + i * hCell);
        float maxY = iniY + hCell + 6;
        if (iniY >= maxBY - 3) continue;
        if (maxY > maxBY) maxY = (float)maxBY;
        for (int j = 0; j < nCols; j++) {
          const float iniX = (float)(minBX + j * wCell);
          float maxX = iniX + wCell + 6;
          if (iniX >= maxBX - 6) continue;
          if (maxX > maxBX) maxX = (float)maxBX;
          const int x0 = (int)iniX, y0 = (int)iniY, ww = (int)maxX - x0, hh = (int)maxY - y0;
          const uint8_t* win = &im.px[(size_t)y0 * im.w + x0];
          fast_window(win, ww, hh, im.w, p.ini_th_fast, cell);
          if (cell.empty()) fast_window(win, ww, hh, im.w, p.min_th_fast, cell);
          for (auto& k : cell) {
            k.x += j * wCell;
            k.y += i * hCell;
            cand.push_back(k);
          }
        }
      }
    }
    std::vector<Kp>& kps = all[l];
    kps = distribute_octree(cand, minBX, maxBX, minBY, maxBY, t.nfeat[l]);
    const int scaledPatch = (int)(kPatchSize * t.scale[l]);
    for (auto& k : kps) {
      k.x += minBX;
      k.y += minBY;
      k.octave = l;
      k.size = (float)scaledPatch;
    }
    for (auto& k : kps) k.angle = ic_angle(im, k.x, k.y, t.umax);
  }
  for (int l = 0; l < p.nlevels; l++) {
    std::vector<Kp>& kps = all[l];
    if (kps.empty()) continue;
    Img blurred;
    gaussian_blur7(ex.pyr[l], blurred);
    size_t off = ex.desc.size();
    ex.desc.resize(off + 32 * kps.size());
    for (size_t i = 0; i < kps.size(); i++) orb_descriptor(blurred, kps[i], &ex.desc[off + 32 * i]);
    if (l != 0) {
      const float sc = t.scale[l];
      for (auto& k : kps) {
        k.x *= sc;
        k.y *= sc;
      }
    }
    ex.kps.insert(ex.kps.end(), kps.begin(), kps.end());
  }
}

// ORBmatcher::DescriptorDistance, src/ORBmatcher.cc:1844-1860 (SWAR popcount
// over 8 int32 words).
int descriptor_distance(const uint8_t* a, const uint8_t* b) {
  int dist = 0;
  for (int i = 0; i < 8; i++) {
    uint32_t wa, wb;
    std::memcpy(&wa, a + 4 * i, 4);
    std::memcpy(&wb, b + 4 * i, 4);
    uint32_t v = wa ^ wb;
    v = v - ((v >> 1) & 0x55555555u);
    v = (v & 0x33333333u) + ((v >> 2) & 0x33333333u);
    dist += (int)((((v + (v >> 4)) & 0xF0F0F0Fu) * 0x1010101u) >> 24);
  }
  return dist;
}

}  // namespace

extern "C" {

int oracle_scale_tables(const oracle_params* p, float* scale, float* inv_scale, float* sigma2,
                        float* inv_sigma2, int* fpl) {
  if (!p || p->nlevels < 1) return -1;
  Tables t = make_tables(*p);
  for (int i = 0; i < p->nlevels; i++) {
    if (scale) scale[i] = t.scale[i];
    if (inv_scale) inv_scale[i] = t.inv_scale[i];
    if (sigma2) sigma2[i] = t.sigma2[i];
    if (inv_sigma2) inv_sigma2[i] = t.inv_sigma2[i];
    if (fpl) fpl[i] = t.nfeat[i];
  }
  return 0;
}

int oracle_extract(const oracle_params* p, const uint8_t* img, int w, int h, size_t stride,
                   oracle_keypoint* kps, int cap, uint8_t* desc, uint8_t* pyramid_out,
                   size_t pyramid_cap, int* level_wh) {
  if (!p || !img || w <= 0 || h <= 0) return 0;  // empty image: silent return (:1141)
  Tables t = make_tables(*p);
  Img im;
  im.w = w;
  im.h = h;
  im.px.resize((size_t)w * h);
  for (int y = 0; y < h; y++) std::memcpy(&im.px[(size_t)y * w], img + (size_t)y * stride, w);
  Extraction ex;
  extract(*p, t, im, ex);
  const int n = (int)ex.kps.size();
  if (n > cap) return -2;
  for (int i = 0; i < n; i++) {
    const Kp& k = ex.kps[i];
    kps[i] = {k.x, k.y, k.size, k.angle, k.response, k.octave, -1};
  }
  if (desc && n) std::memcpy(desc, ex.desc.data(), (size_t)32 * n);
  size_t off = 0;
  for (int l = 0; l < p->nlevels; l++) {
    const Img& L = ex.pyr[l];
    if (level_wh) {
      level_wh[2 * l] = L.w;
      level_wh[2 * l + 1] = L.h;
    }
    if (pyramid_out) {
      if (off + L.px.size() > pyramid_cap) return -3;
      std::memcpy(pyramid_out + off, L.px.data(), L.px.size());
    }
    off += L.px.size();
  }
  return n;
}

int oracle_resize_linear(const uint8_t* src, int sw, int sh, uint8_t* dst, int dw, int dh) {
  Img s, d;
  s.w = sw;
  s.h = sh;
  s.px.assign(src, src + (size_t)sw * sh);
  resize_linear(s, d, dw, dh);
  std::memcpy(dst, d.px.data(), d.px.size());
  return 0;
}

int oracle_gaussian_blur7(const uint8_t* src, int w, int h, uint8_t* dst) {
  Img s, d;
  s.w = w;
  s.h = h;
  s.px.assign(src, src + (size_t)w * h);
  gaussian_blur7(s, d);
  std::memcpy(dst, d.px.data(), d.px.size());
  return 0;
}

int oracle_fast_window(const uint8_t* img, int w, int h, size_t stride, int threshold, uint32_t* out, int cap) {
  std::vector<Kp> kp;
  fast_window(img, w, h, stride, threshold, kp);
  int n = std::min((int)kp.size(), cap);
  for (int i = 0; i < n; i++)
    out[i] = ((uint32_t)kp[i].response << 24) | ((uint32_t)kp[i].y << 12) | (uint32_t)kp[i].x;
  return (int)kp.size();
}

int oracle_fast_score(const uint8_t* img, size_t stride, int x, int y) {
  return corner_score(img + (size_t)y * stride + x, stride);
}

float oracle_fast_atan2(float y, float x) { return fast_atan2(y, x); }
float oracle_cosf(float x) { float s, c; sincos_det(x, &s, &c); return c; }
float oracle_sinf(float x) { float s, c; sincos_det(x, &s, &c); return s; }

void oracle_set_trig_mode(int mode) { g_trig_mode = mode; }

// Census over every float in [lo, hi] with bit pattern index step `step`: how many inputs
// give libm cosf/sinf != sincos_det (out[0] cos, out[1] sin, out[2] floats visited).
void oracle_trig_census(float lo, float hi, int step, long long* out) {
  uint32_t a, b;
  std::memcpy(&a, &lo, 4);
  std::memcpy(&b, &hi, 4);
  long long dc = 0, ds = 0, n = 0;
  for (uint64_t u = a; u <= b; u += (uint64_t)step) {
    uint32_t w = (uint32_t)u;
    float x;
    std::memcpy(&x, &w, 4);
    float s, c;
    sincos_det(x, &s, &c);
    float lc = std::cos(x), ls = std::sin(x);
    dc += std::memcmp(&lc, &c, 4) != 0;
    ds += std::memcmp(&ls, &s, 4) != 0;
    n++;
  }
  out[0] = dc;
  out[1] = ds;
  out[2] = n;
}

// For every float angle (radians) in [lo, hi] with index step `step` whose libm cosf/sinf differ from
// sincos_det, whether any of the 512 rotated pattern offsets cvRound(x*b + y*a), cvRound(x*a - y*b)
// (src/ORBextractor.cc:119-125) changes.  out[0] angles with a trig difference, out[1] angles whose
// rotated pattern differs, out[2] floats visited.
void oracle_trig_pattern_census(float lo, float hi, int step, long long* out, float* angles, int cap) {
  uint32_t a0, b0;
  std::memcpy(&a0, &lo, 4);
  std::memcpy(&b0, &hi, 4);
  long long nt = 0, np = 0, n = 0;
  for (uint64_t u = a0; u <= b0; u += (uint64_t)step) {
    uint32_t w = (uint32_t)u;
    float ang;
    std::memcpy(&ang, &w, 4);
    n++;
    float s, c;
    sincos_det(ang, &s, &c);
    const float la = std::cos(ang), lb = std::sin(ang);
    if (la == c && lb == s) continue;
    nt++;
    bool diff = false;
    for (int idx = 0; idx < 1024 && !diff; idx += 2) {
      const float x = (float)kPattern[idx], y = (float)kPattern[idx + 1];
      diff = round_even(x * s + y * c) != round_even(x * lb + y * la) ||
             round_even(x * c - y * s) != round_even(x * la - y * lb);
    }
    if (diff && angles && np < cap) angles[np] = ang;
    np += diff;
  }
  out[0] = nt;
  out[1] = np;
  out[2] = n;
}

int oracle_descriptor_distance(const uint8_t* a, const uint8_t* b) { return descriptor_distance(a, b); }

void oracle_hamming_pairs(const uint8_t* a, const uint8_t* b, int n, int32_t* d) {
  for (int i = 0; i < n; i++) d[i] = descriptor_distance(a + 32 * (size_t)i, b + 32 * (size_t)i);
}

// Frame::ComputeStereoMatches, src/Frame.cc:547-788.
int oracle_stereo_match(const oracle_params* p, const oracle_keypoint* kL, const uint8_t* dL, int nL,
                        const oracle_keypoint* kR, const uint8_t* dR, int nR, const uint8_t* pyrL,
                        const uint8_t* pyrR, const int* level_wh, float bf, float b, float* uRight,
                        float* depth) {
  Tables t = make_tables(*p);
  for (int i = 0; i < nL; i++) uRight[i] = depth[i] = -1.0f;
  std::vector<size_t> lvl_off(p->nlevels);
  size_t off = 0;
  for (int l = 0; l < p->nlevels; l++) {
    lvl_off[l] = off;
    off += (size_t)level_wh[2 * l] * level_wh[2 * l + 1];
  }
  const int thOrbDist = (100 + 50) / 2;  // (TH_HIGH+TH_LOW)/2, src/ORBmatcher.cc:37-38
  const int nRows = level_wh[1];
  std::vector<std::vector<int>> rowIdx(nRows);
  for (int iR = 0; iR < nR; iR++) {
    const float kpY = kR[iR].y;
    const float r = 2.0f * t.scale[kR[iR].octave];
    const int maxr = (int)std::ceil(kpY + r);
    const int minr = (int)std::floor(kpY - r);
    for (int yi = std::max(minr, 0); yi <= std::min(maxr, nRows - 1); yi++) rowIdx[yi].push_back(iR);
  }
  const float minZ = b, minD = 0, maxD = bf / minZ;
  std::vector<std::pair<int, int>> distIdx;
  for (int iL = 0; iL < nL; iL++) {
    const oracle_keypoint& kpL = kL[iL];
    const int levelL = kpL.octave;
    const float vL = kpL.y, uL = kpL.x;
    const std::vector<int>& cands = rowIdx[(size_t)vL];
    if (cands.empty()) continue;
    const float minU = uL - maxD, maxU = uL - minD;
    if (maxU < 0) continue;
    int bestDist = 100;  // TH_HIGH
    int bestIdxR = 0;
    for (int iR : cands) {
      const oracle_keypoint& kpR = kR[iR];
      if (kpR.octave < levelL - 1 || kpR.octave > levelL + 1) continue;
      const float uR = kpR.x;
      if (uR >= minU && uR <= maxU) {
        const int dist = descriptor_distance(dL + 32 * (size_t)iL, dR + 32 * (size_t)iR);
        if (dist < bestDist) {
          bestDist = dist;
          bestIdxR = iR;
        }
      }
    }
    if (bestDist >= thOrbDist) continue;
    const float uR0 = kR[bestIdxR].x;
    const float sf = t.inv_scale[levelL];
    const float scaleduL = std::round(kpL.x * sf);
    const float scaledvL = std::round(kpL.y * sf);
    const float scaleduR0 = std::round(uR0 * sf);
    const int w = 5, L = 5;
    const int lw = level_wh[2 * levelL];
    const uint8_t* imL = pyrL + lvl_off[levelL];
    const uint8_t* imR = pyrR + lvl_off[levelL];
    const float iniu = scaleduR0 + L - w;
    const float endu = scaleduR0 + L + w + 1;
    if (iniu < 0 || endu >= lw) continue;
    // the reference asserts in cv::Mat::colRange/rowRange if a patch leaves the
    // level; unreachable for keypoints >= 16 px inside their level
    const int lh = level_wh[2 * levelL + 1];
    if (scaleduR0 - 2 * w < 0 || scaledvL - w < 0 || scaledvL + w >= lh || scaleduL - w < 0 ||
        scaleduL + w >= lw)
      continue;
    const int cyL = (int)scaledvL, cxL = (int)scaleduL, cxR0 = (int)scaleduR0;
    const int cL = imL[(size_t)cyL * lw + cxL];
    int sadBest = INT32_MAX;
    int bestinc = 0;
    float dists[2 * L + 1];
    for (int inc = -L; inc <= L; inc++) {
      const int cx = cxR0 + inc;
      const int cR = imR[(size_t)cyL * lw + cx];
      int sad = 0;
      for (int dy = -w; dy <= w; dy++)
        for (int dx = -w; dx <= w; dx++) {
          int a = (int)imL[(size_t)(cyL + dy) * lw + cxL + dx] - cL;
          int c = (int)imR[(size_t)(cyL + dy) * lw + cx + dx] - cR;
          sad += std::abs(a - c);
        }
      const float dist = (float)sad;
      if (dist < (float)sadBest) {
        sadBest = sad;
        bestinc = inc;
      }
      dists[L + inc] = dist;
    }
    if (bestinc == -L || bestinc == L) continue;
    const float d1 = dists[L + bestinc - 1], d2 = dists[L + bestinc], d3 = dists[L + bestinc + 1];
    const float deltaR = (d1 - d3) / (2.0f * (d1 + d3 - 2.0f * d2));
    if (deltaR < -1 || deltaR > 1) continue;
    float bestuR = t.scale[levelL] * ((float)scaleduR0 + (float)bestinc + deltaR);
    float disparity = uL - bestuR;
    if (disparity >= minD && disparity < maxD) {
      if (disparity <= 0) {
        disparity = 0.01f;
        bestuR = uL - 0.01f;
      }
      depth[iL] = bf / disparity;
      uRight[iL] = bestuR;
      distIdx.push_back({sadBest, iL});
    }
  }
  if (distIdx.empty()) return 0;  // reference reads v[0] of an empty vector here (UB)
  std::sort(distIdx.begin(), distIdx.end());
  const float median = (float)distIdx[distIdx.size() / 2].first;
  const float thDist = 1.5f * 1.4f * median;
  int kept = (int)distIdx.size();
  for (int i = (int)distIdx.size() - 1; i >= 0; i--) {
    if ((float)distIdx[i].first < thDist) break;
    uRight[distIdx[i].second] = -1;
    depth[distIdx[i].second] = -1;
    kept--;
  }
  return kept;
}

}  // extern "C"

// ------------------------------------------------------------ SearchByBoW
namespace {

const int kThLow = 50, kHistoLength = 30;  // src/ORBmatcher.cc:37-39

// ORBmatcher::ComputeThreeMaxima, src/ORBmatcher.cc:1797-1839.
void three_maxima(const int* h, int L, int& ind1, int& ind2, int& ind3) {
  int max1 = 0, max2 = 0, max3 = 0;
  for (int i = 0; i < L; i++) {
    const int s = h[i];
    if (s > max1) {
      max3 = max2; max2 = max1; max1 = s;
      ind3 = ind2; ind2 = ind1; ind1 = i;
    } else if (s > max2) {
      max3 = max2; max2 = s;
      ind3 = ind2; ind2 = i;
    } else if (s > max3) {
      max3 = s;
      ind3 = i;
    }
  }
  if (max2 < 0.1f * (float)max1) {
    ind2 = -1;
    ind3 = -1;
  } else if (max3 < 0.1f * (float)max1) {
    ind3 = -1;
  }
}

int rot_bin(float angA, float angB) {
  const float factor = 1.0f / kHistoLength;
  float rot = angA - angB;
  if (rot < 0.0) rot += 360.0f;
  int bin = (int)std::round(rot * factor);
  if (bin == kHistoLength) bin = 0;
  return bin;
}

// Merge-walk of two FeatureVectors (std::map iteration with lower_bound jumps
// visits exactly the common node ids in ascending order).
template <class F>
void for_common_nodes(const oracle_bow_side& a, const oracle_bow_side& b, F fn) {
  int i = 0, j = 0;
  while (i < a.n_nodes && j < b.n_nodes) {
    if (a.node_id[i] == b.node_id[j]) {
      fn(i, j);
      i++;
      j++;
    } else if (a.node_id[i] < b.node_id[j]) {
      i++;
    } else {
      j++;
    }
  }
}

int search_by_bow(const oracle_bow_side& A, const oracle_bow_side& B, float nnratio, bool checkOri, bool kfkf,
                  int32_t* match, int nmatch_out) {
  // match indexed by B feature (KF-F) or by A feature (KF-KF)
  for (int i = 0; i < nmatch_out; i++) match[i] = -1;
  std::vector<char> matchedB(B.n, 0);
  std::vector<int> rotHist[kHistoLength];
  int nmatches = 0;
  for_common_nodes(A, B, [&](int ia, int jb) {
    for (int pa = A.node_off[ia]; pa < A.node_off[ia + 1]; pa++) {
      const int idxA = A.feat[pa];
      if (A.valid && !A.valid[idxA]) continue;
      int best1 = 256, bestIdx = -1, best2 = 256;
      for (int pb = B.node_off[jb]; pb < B.node_off[jb + 1]; pb++) {
        const int idxB = B.feat[pb];
        if (matchedB[idxB]) continue;
        if (kfkf && B.valid && !B.valid[idxB]) continue;
        const int dist = descriptor_distance(A.desc + 32 * (size_t)idxA, B.desc + 32 * (size_t)idxB);
        if (dist < best1) {
          best2 = best1;
          best1 = dist;
          bestIdx = idxB;
        } else if (dist < best2) {
          best2 = dist;
        }
      }
      const bool pass = kfkf ? best1 < kThLow : best1 <= kThLow;
      if (!pass) continue;
      if (!((float)best1 < nnratio * (float)best2)) continue;
      matchedB[bestIdx] = 1;
      const int out = kfkf ? idxA : bestIdx;
      match[out] = kfkf ? bestIdx : idxA;
      if (checkOri) rotHist[rot_bin(A.angle[idxA], B.angle[bestIdx])].push_back(out);
      nmatches++;
    }
  });
  if (checkOri) {
    int counts[kHistoLength];
    for (int i = 0; i < kHistoLength; i++) counts[i] = (int)rotHist[i].size();
    int ind1 = -1, ind2 = -1, ind3 = -1;
    three_maxima(counts, kHistoLength, ind1, ind2, ind3);
    for (int i = 0; i < kHistoLength; i++) {
      if (i == ind1 || i == ind2 || i == ind3) continue;
      for (int o : rotHist[i]) {
        match[o] = -1;
        nmatches--;
      }
    }
  }
  return nmatches;
}

}  // namespace

extern "C" {

int oracle_search_by_bow_kf_f(const oracle_bow_side* kf, const oracle_bow_side* f, float nnratio, int check_ori,
                              int32_t* match_f) {
  return search_by_bow(*kf, *f, nnratio, check_ori != 0, false, match_f, f->n);
}

int oracle_search_by_bow_kf_kf(const oracle_bow_side* kf1, const oracle_bow_side* kf2, float nnratio, int check_ori,
                               int32_t* match12) {
  return search_by_bow(*kf1, *kf2, nnratio, check_ori != 0, true, match12, kf1->n);
}

void oracle_three_maxima(const int* counts, int L, int* ind1, int* ind2, int* ind3) {
  *ind1 = *ind2 = *ind3 = -1;
  three_maxima(counts, L, *ind1, *ind2, *ind3);
}

}  // extern "C"
