// test_shim.cpp -- drives the C++ shim (shim/include/*.h, the reference class signatures) the way
// ORB-SLAM2 calls it.  Modes:
//   abi                 no GPU needed: layouts, cv::Mat semantics, DescriptorDistance, and that every
//                       GPU-backed constructor/call fails loudly (std::runtime_error) without a device
//   stereo  IN OUT      Frame stereo ctor (two extraction threads + ComputeStereoMatches)
//   bow     IN OUT      ORBmatcher::SearchByBoW(KeyFrame*, Frame&, ...) / (KeyFrame*, KeyFrame*, ...)
//   ba      IN OUT      Optimizer::LocalBundleAdjustment on an explicit problem
//   bagraph IN OUT      Optimizer::LocalBundleAdjustment(KeyFrame*, bool*, Map*) on an object graph
//   pnp     IN OUT      PnPsolver(Frame, matches) + SetRansacParameters + iterate(5) in
//                       Tracking::Relocalization's candidate loop
// IN/OUT are little-endian binary files written/read by tests/test_shim.py, which compares the
// outputs with the CPU oracle.  Exit status 0 = ok.
#include <cassert>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <list>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "ORBextractor.h"
#include "ORBmatcher.h"
#include "Objects.h"
#include "Optimizer.h"
#include "PnPsolver.h"
#include "orbx.h"

using namespace ORB_SLAM2;

#define REQUIRE(c)                                                    \
  do {                                                                \
    if (!(c)) {                                                       \
      std::fprintf(stderr, "REQUIRE failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                   \
    }                                                                 \
  } while (0)

struct Reader {
  FILE* f;
  explicit Reader(const char* p) : f(std::fopen(p, "rb")) { REQUIRE(f); }
  ~Reader() { std::fclose(f); }
  template <class T> T get() {
    T v;
    REQUIRE(std::fread(&v, sizeof(T), 1, f) == 1);
    return v;
  }
  template <class T> std::vector<T> vec(size_t n) {
    std::vector<T> v(n);
    if (n) REQUIRE(std::fread(v.data(), sizeof(T), n, f) == n);
    return v;
  }
};

struct Writer {
  FILE* f;
  explicit Writer(const char* p) : f(std::fopen(p, "wb")) { REQUIRE(f); }
  ~Writer() { std::fclose(f); }
  template <class T> void put(T v) { REQUIRE(std::fwrite(&v, sizeof(T), 1, f) == 1); }
  void raw(const void* p, size_t n) {
    if (n) REQUIRE(std::fwrite(p, 1, n, f) == n);
  }
};

template <class F> static bool throws_runtime(F f) {
  try {
    f();
  } catch (const std::runtime_error&) {
    return true;
  }
  return false;
}

static int mode_abi() {
  // cv::KeyPoint is orbx_keypoint (include/orbx.h) byte for byte
  REQUIRE(sizeof(cv::KeyPoint) == 28);
  cv::KeyPoint kp(1.5f, 2.5f, 31.f, 90.f, 7.f, 3);
  orbx_keypoint ok;
  std::memcpy(&ok, &kp, sizeof(ok));
  REQUIRE(ok.x == 1.5f && ok.y == 2.5f && ok.size == 31.f && ok.angle == 90.f && ok.response == 7.f &&
          ok.octave == 3 && ok.class_id == -1);
  // cv::Mat: shallow copies share, clone/copyTo deep-copy, row views alias
  cv::Mat a(4, 32, CV_8U);
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 32; c++) a.at<uint8_t>(r, c) = (uint8_t)(r * 32 + c);
  cv::Mat b = a, c = a.clone(), d;
  a.copyTo(d);
  a.at<uint8_t>(0, 0) = 255;
  REQUIRE(b.at<uint8_t>(0, 0) == 255 && c.at<uint8_t>(0, 0) == 0 && d.at<uint8_t>(0, 0) == 0);
  REQUIRE(a.row(2).data == a.data + 64 && a.rowRange(1, 3).rows == 2 && a.isContinuous());
  cv::Mat e;
  REQUIRE(e.empty() && !a.empty());
  // DescriptorDistance (src/ORBmatcher.cc:1844-1860)
  cv::Mat z(1, 32, CV_8U), o(1, 32, CV_8U);
  std::memset(z.data, 0, 32);
  std::memset(o.data, 0xFF, 32);
  REQUIRE(ORBmatcher::DescriptorDistance(z, o) == 256 && ORBmatcher::DescriptorDistance(o, o) == 0);
  REQUIRE(ORBmatcher::DescriptorDistance(a.row(1), a.row(3)) == ORBmatcher::DescriptorDistance(a.row(3), a.row(1)));
  int manual = 0;
  for (int i = 0; i < 32; i++) manual += __builtin_popcount((unsigned)(a.at<uint8_t>(1, i) ^ a.at<uint8_t>(3, i)));
  REQUIRE(ORBmatcher::DescriptorDistance(a.row(1), a.row(3)) == manual);
  REQUIRE(ORBmatcher::TH_LOW == 50 && ORBmatcher::TH_HIGH == 100 && ORBmatcher::HISTO_LENGTH == 30);
  // GPU-backed members fail loudly without a device (never a silent CPU path)
  if (orbx_device_count() <= 0) {
    REQUIRE(throws_runtime([] { ORBextractor ex(1000, 1.2f, 8, 20, 7); }));
    LocalBAProblem P;
    LocalBAResult R;
    REQUIRE(throws_runtime([&] { Optimizer::LocalBundleAdjustment(P, nullptr, R); }));
    KeyFrame kf;
    Frame F;
    std::vector<MapPoint*> m;
    ORBmatcher matcher(0.75f, true);
    REQUIRE(throws_runtime([&] { matcher.SearchByBoW(&kf, F, m); }));
    // PnPsolver: gathering needs no device, iterate() does
    PnPsolver solver(F, m);
    bool bNoMore = false;
    std::vector<bool> inl;
    int ni = 0;
    REQUIRE(throws_runtime([&] { solver.iterate(5, bNoMore, inl, ni); }));
    // the reference-signature LocalBA gathers from the graph, then needs the device
    Map map;
    KeyFrame k1;
    cv::Mat I4(4, 4, CV_32F);
    std::memset(I4.data, 0, 64);
    for (int i = 0; i < 4; i++) I4.at<float>(i, i) = 1.f;
    k1.SetPose(I4);
    REQUIRE(throws_runtime([&] { Optimizer::LocalBundleAdjustment(&k1, nullptr, &map); }));
    std::printf("abi ok (no device: GPU members throw)\n");
  } else {
    std::printf("abi ok (device present)\n");
  }
  return 0;
}

static int mode_stereo(const char* in, const char* out) {
  Reader r(in);
  const int w = r.get<int32_t>(), h = r.get<int32_t>(), nf = r.get<int32_t>();
  const float sf = r.get<float>();
  const int nl = r.get<int32_t>(), ini = r.get<int32_t>(), mn = r.get<int32_t>();
  const float bf = r.get<float>(), fx = r.get<float>();
  std::vector<uint8_t> L = r.vec<uint8_t>((size_t)w * h), R = r.vec<uint8_t>((size_t)w * h);
  ORBextractor exL(nf, sf, nl, ini, mn), exR(nf, sf, nl, ini, mn);
  REQUIRE(!exL.mbDownloadPyramid);  // off by default: the stereo matcher reads the device copy
  exL.mbDownloadPyramid = true;     // this test also checks the host copy
  cv::Mat imL(h, w, CV_8U, L.data()), imR(h, w, CV_8U, R.data());
  cv::Mat K(3, 3, CV_32F), dist(4, 1, CV_32F);
  std::memset(K.data, 0, 36);
  std::memset(dist.data, 0, 16);
  K.at<float>(0, 0) = fx;
  K.at<float>(1, 1) = fx;
  K.at<float>(0, 2) = w / 2.f;
  K.at<float>(1, 2) = h / 2.f;
  K.at<float>(2, 2) = 1.f;
  Frame F(imL, imR, &exL, &exR, K, dist, bf, 35.f * bf / fx);
  REQUIRE(F.N == (int)F.mvKeys.size() && (int)F.mvuRight.size() == F.N && (int)F.mvDepth.size() == F.N);
  REQUIRE(F.mvKeysUn.size() == F.mvKeys.size());
  Writer o(out);
  o.put<int32_t>(F.N);
  o.put<int32_t>((int32_t)F.mvKeysRight.size());
  o.raw(F.mvKeys.data(), F.mvKeys.size() * 28);
  for (int i = 0; i < F.N; i++) o.raw(F.mDescriptors.ptr<uint8_t>(i), 32);
  o.raw(F.mvKeysRight.data(), F.mvKeysRight.size() * 28);
  for (size_t i = 0; i < F.mvKeysRight.size(); i++) o.raw(F.mDescriptorsRight.ptr<uint8_t>((int)i), 32);
  o.raw(F.mvuRight.data(), F.mvuRight.size() * 4);
  o.raw(F.mvDepth.data(), F.mvDepth.size() * 4);
  // the host copy of the left pyramid (mvImagePyramid)
  for (int l = 0; l < nl; l++) {
    const cv::Mat& m = exL.mvImagePyramid[l];
    o.put<int32_t>(m.cols);
    o.put<int32_t>(m.rows);
    for (int y = 0; y < m.rows; y++) o.raw(m.ptr<uint8_t>(y), m.cols);
  }
  // the free-function form gives the same answer on the same extraction
  std::vector<float> uR2, d2;
  ComputeStereoMatches(exL, exR, F.mvKeys, F.mDescriptors, F.mvKeysRight, F.mDescriptorsRight, F.mbf, F.mb, uR2, d2);
  REQUIRE(uR2.size() == F.mvuRight.size() &&
          std::memcmp(uR2.data(), F.mvuRight.data(), uR2.size() * 4) == 0 &&
          std::memcmp(d2.data(), F.mvDepth.data(), d2.size() * 4) == 0);
  // an empty image: silent return, no keypoints (src/ORBextractor.cc:1141)
  std::vector<cv::KeyPoint> k0;
  cv::Mat d0;
  exL(cv::Mat(), cv::Mat(), k0, d0);
  REQUIRE(k0.empty());
  std::printf("stereo ok: %d / %d keypoints\n", F.N, (int)F.mvKeysRight.size());
  return 0;
}

struct SideIn {
  int n = 0;
  std::vector<uint8_t> desc, valid;
  std::vector<float> angle;
  std::vector<uint32_t> ids;
  std::vector<int32_t> off, feat;
};

static SideIn read_side(Reader& r) {
  SideIn s;
  s.n = r.get<int32_t>();
  s.desc = r.vec<uint8_t>((size_t)s.n * 32);
  s.angle = r.vec<float>(s.n);
  s.valid = r.vec<uint8_t>(s.n);
  const int nn = r.get<int32_t>();
  s.ids = r.vec<uint32_t>(nn);
  s.off = r.vec<int32_t>(nn + 1);
  s.feat = r.vec<int32_t>(s.off.empty() ? 0 : s.off.back());
  return s;
}

static DBoW2::FeatureVector to_fv(const SideIn& s) {
  DBoW2::FeatureVector fv;
  for (size_t j = 0; j < s.ids.size(); j++)
    for (int k = s.off[j]; k < s.off[j + 1]; k++) fv[s.ids[j]].push_back((unsigned)s.feat[k]);
  return fv;
}

static int mode_bow(const char* in, const char* out) {
  Reader r(in);
  const int kfkf = r.get<int32_t>();
  const float nn = r.get<float>();
  const int check = r.get<int32_t>();
  SideIn A = read_side(r), B = read_side(r);
  // one MapPoint per feature; invalid ones alternate between NULL and isBad() (both skip, :211-219)
  std::vector<MapPoint> mpA(A.n), mpB(B.n);
  auto make_kf = [](KeyFrame& kf, const SideIn& s, std::vector<MapPoint>& mps) {
    kf.N = s.n;
    kf.mvKeysUn.resize(s.n);
    for (int i = 0; i < s.n; i++) kf.mvKeysUn[i].angle = s.angle[i];
    kf.mDescriptors = cv::Mat(s.n, 32, CV_8U);
    if (s.n) std::memcpy(kf.mDescriptors.data, s.desc.data(), (size_t)s.n * 32);
    kf.mFeatVec = to_fv(s);
    kf.mvpMapPoints.assign(s.n, nullptr);
    for (int i = 0; i < s.n; i++) {
      if (s.valid[i]) {
        kf.mvpMapPoints[i] = &mps[i];
      } else if (i % 2) {
        mps[i].mbBad = true;
        kf.mvpMapPoints[i] = &mps[i];
      }
    }
  };
  ORBmatcher matcher(nn, check != 0);
  Writer o(out);
  if (!kfkf) {
    KeyFrame kf;
    make_kf(kf, A, mpA);
    Frame F;
    F.N = B.n;
    F.mvKeys.resize(B.n);
    for (int i = 0; i < B.n; i++) F.mvKeys[i].angle = B.angle[i];
    F.mDescriptors = cv::Mat(B.n, 32, CV_8U);
    if (B.n) std::memcpy(F.mDescriptors.data, B.desc.data(), (size_t)B.n * 32);
    F.mFeatVec = to_fv(B);
    std::vector<MapPoint*> m;
    const int n = matcher.SearchByBoW(&kf, F, m);
    REQUIRE((int)m.size() == F.N);
    o.put<int32_t>(n);
    for (int i = 0; i < F.N; i++) o.put<int32_t>(m[i] ? (int32_t)(m[i] - mpA.data()) : -1);
  } else {
    KeyFrame kf1, kf2;
    make_kf(kf1, A, mpA);
    make_kf(kf2, B, mpB);
    std::vector<MapPoint*> m;
    const int n = matcher.SearchByBoW(&kf1, &kf2, m);
    REQUIRE((int)m.size() == A.n);
    o.put<int32_t>(n);
    for (int i = 0; i < A.n; i++) o.put<int32_t>(m[i] ? (int32_t)(m[i] - mpB.data()) : -1);
  }
  std::printf("bow ok\n");
  return 0;
}

static int mode_ba(const char* in, const char* out) {
  Reader r(in);
  const int nc = r.get<int32_t>(), np = r.get<int32_t>(), ne = r.get<int32_t>();
  const std::vector<float> T = r.vec<float>(12 * (size_t)nc);
  const std::vector<uint8_t> fixed = r.vec<uint8_t>(nc);
  const std::vector<float> intr = r.vec<float>(5 * (size_t)nc), X = r.vec<float>(3 * (size_t)np);
  const std::vector<int32_t> ep = r.vec<int32_t>(ne), ec = r.vec<int32_t>(ne);
  const std::vector<float> obs = r.vec<float>(3 * (size_t)ne), isig = r.vec<float>(ne);
  bool stop = r.get<int32_t>() != 0;
  LocalBAProblem P;
  P.cameras.resize(nc);
  for (int c = 0; c < nc; c++) {
    cv::Mat Tc(4, 4, CV_32F);
    for (int i = 0; i < 12; i++) Tc.at<float>(i / 4, i % 4) = T[12 * c + i];
    Tc.at<float>(3, 0) = Tc.at<float>(3, 1) = Tc.at<float>(3, 2) = 0.f;
    Tc.at<float>(3, 3) = 1.f;
    P.cameras[c].Tcw = Tc;
    P.cameras[c].fixed = fixed[c] != 0;
    P.cameras[c].fx = intr[5 * c];
    P.cameras[c].fy = intr[5 * c + 1];
    P.cameras[c].cx = intr[5 * c + 2];
    P.cameras[c].cy = intr[5 * c + 3];
    P.cameras[c].bf = intr[5 * c + 4];
  }
  P.points.resize(np);
  for (int p = 0; p < np; p++) {
    cv::Mat Xp(3, 1, CV_32F);
    for (int k = 0; k < 3; k++) Xp.at<float>(k, 0) = X[3 * p + k];
    P.points[p] = Xp;
  }
  P.observations.resize(ne);
  for (int e = 0; e < ne; e++) {
    LocalBAProblem::Observation& ob = P.observations[e];
    ob.point = ep[e];
    ob.camera = ec[e];
    ob.u = obs[3 * e];
    ob.v = obs[3 * e + 1];
    ob.ur = obs[3 * e + 2];
    ob.invSigma2 = isig[e];
  }
  LocalBAResult R;
  Optimizer::LocalBundleAdjustment(P, &stop, R);
  Writer o(out);
  for (int c = 0; c < nc; c++)
    for (int i = 0; i < 12; i++) o.put<float>(R.Tcw[c].at<float>(i / 4, i % 4));
  for (int p = 0; p < np; p++)
    for (int k = 0; k < 3; k++) o.put<float>(R.points[p].at<float>(k, 0));
  for (int e = 0; e < ne; e++) o.put<uint8_t>(R.erase[e] ? 1 : 0);
  o.put<int32_t>(R.iterations[0]);
  o.put<int32_t>(R.iterations[1]);
  o.put<int32_t>(R.trials);
  std::printf("ba ok: iterations %d %d trials %d\n", R.iterations[0], R.iterations[1], R.trials);
  return 0;
}

// ---------------------------------------------------------------- LocalBA on an object graph
// Input: the synthetic problem (cameras, points, edges grouped by point) with per-edge octaves into
// a level table.  The graph: one KeyFrame per camera (addresses ascending, so GetObservations()
// walks cameras in index order), local KeyFrames = the non-fixed cameras (pKF = the first) plus
// fixed camera 0 as a covisible KeyFrame with mnId 0 (a local vertex fixed by the mnId == 0 rule);
// the other fixed cameras are reached only through the points' observations (lFixedCameras).
// Distractors the gather must skip: a bad covisible KeyFrame that observes the first points, a bad
// MapPoint and empty feature slots in every KeyFrame.
static LocalBAProblem g_gathered;
static std::vector<KeyFrame*> g_gathered_cams;
static bool* g_raise_after_gather = nullptr;  // stop == 2: the flag goes up after the shim's own check
static void gathered_hook(const LocalBAProblem& P, const std::vector<KeyFrame*>& cams) {
  g_gathered = P;
  g_gathered_cams = cams;
  if (g_raise_after_gather) {
    // another thread (LoopClosing) moves pKF meanwhile, then LocalMapping::InterruptBA raises the flag:
    // the library sees it before optimize(5), and the stale gathered copy must not be written back
    cv::Mat T = cams[0]->GetPose();
    T.at<float>(0, 3) += 1.0f;
    cams[0]->SetPose(T);
    *g_raise_after_gather = true;
  }
}

static int mode_bagraph(const char* in, const char* out) {
  Reader r(in);
  const int nc = r.get<int32_t>(), np = r.get<int32_t>(), ne = r.get<int32_t>(), nl = r.get<int32_t>();
  const std::vector<float> T = r.vec<float>(12 * (size_t)nc);
  const std::vector<uint8_t> fixed = r.vec<uint8_t>(nc);
  const std::vector<float> intr = r.vec<float>(5 * (size_t)nc), X = r.vec<float>(3 * (size_t)np);
  const std::vector<int32_t> ep = r.vec<int32_t>(ne), ec = r.vec<int32_t>(ne);
  const std::vector<float> obs = r.vec<float>(3 * (size_t)ne);
  const std::vector<float> levels = r.vec<float>(nl);
  const std::vector<int32_t> octave = r.vec<int32_t>(ne);
  const int stop = r.get<int32_t>();
  Map map;
  std::vector<KeyFrame> kfs(nc + 1);  // + the bad covisible KeyFrame
  std::vector<MapPoint> mps(np + 1);  // + a bad MapPoint
  std::vector<int> nfeat(nc + 1, 0);
  for (int e = 0; e < ne; e++) nfeat[ec[e]]++;
  int first_fixed = -1;
  for (int c = 0; c < nc; c++)
    if (fixed[c] && first_fixed < 0) first_fixed = c;
  for (int c = 0; c <= nc; c++) {
    KeyFrame& K = kfs[c];
    const int cc = c < nc ? c : 0;
    K.mnId = (c == first_fixed) ? 0 : (unsigned long)(c + 1);
    K.fx = intr[5 * cc];
    K.fy = intr[5 * cc + 1];
    K.cx = intr[5 * cc + 2];
    K.cy = intr[5 * cc + 3];
    K.mbf = intr[5 * cc + 4];
    K.mnScaleLevels = 8;
    for (int l = 0; l < 8; l++) K.mvScaleFactors.push_back(std::pow(1.2f, (float)l));
    K.mvInvLevelSigma2 = levels;
    cv::Mat Tc(4, 4, CV_32F);
    for (int i = 0; i < 12; i++) Tc.at<float>(i / 4, i % 4) = T[12 * cc + i];
    Tc.at<float>(3, 0) = Tc.at<float>(3, 1) = Tc.at<float>(3, 2) = 0.f;
    Tc.at<float>(3, 3) = 1.f;
    K.SetPose(Tc);
    const int nf = nfeat[c] + 10 + (c == 0 ? 1 : 0) + (c == nc ? 50 : 0);
    K.N = nf;
    K.mvKeysUn.resize(nf);
    K.mvuRight.assign(nf, -1.f);
    K.mvpMapPoints.assign(nf, nullptr);
  }
  kfs[nc].mbBad = true;
  for (int p = 0; p < np; p++) {
    cv::Mat Xp(3, 1, CV_32F);
    for (int k = 0; k < 3; k++) Xp.at<float>(k, 0) = X[3 * p + k];
    mps[p].SetWorldPos(Xp);
    mps[p].mnId = (unsigned long)(p + 1);
    mps[p].mpMap = &map;
    map.mspMapPoints.insert(&mps[p]);
  }
  std::vector<int> slot(nc + 1, 0);
  std::vector<int> edge_slot(ne);
  for (int e = 0; e < ne; e++) {
    KeyFrame& K = kfs[ec[e]];
    const int idx = slot[ec[e]]++;
    edge_slot[e] = idx;
    K.mvKeysUn[idx] = cv::KeyPoint(obs[3 * e], obs[3 * e + 1], 31.f, -1.f, 0.f, octave[e]);
    K.mvuRight[idx] = obs[3 * e + 2];
    K.mvpMapPoints[idx] = &mps[ep[e]];
    mps[ep[e]].AddObservation(&K, idx);
    if (!mps[ep[e]].mpRefKF) mps[ep[e]].mpRefKF = &K;
  }
  // the bad KeyFrame observes the first 50 points (monocular): its edges must not enter the window
  KeyFrame& Kb = kfs[nc];
  for (int p = 0; p < 50 && p < np; p++) {
    const int idx = slot[nc]++;
    Kb.mvKeysUn[idx] = cv::KeyPoint(100.f, 100.f, 31.f, -1.f, 0.f, 0);
    Kb.mvpMapPoints[idx] = &mps[p];
    mps[p].AddObservation(&Kb, idx);
  }
  // a bad MapPoint in pKF's matches
  mps[np].mbBad = true;
  int local0 = -1;
  for (int c = 0; c < nc; c++)
    if (!fixed[c]) {
      local0 = c;
      break;
    }
  REQUIRE(local0 >= 0);
  KeyFrame* pKF = &kfs[local0];
  pKF->mvpMapPoints[slot[local0]] = &mps[np];
  for (int c = 0; c < nc; c++)
    if (c != local0 && !fixed[c]) pKF->mvpOrderedConnectedKeyFrames.push_back(&kfs[c]);
  pKF->mvpOrderedConnectedKeyFrames.push_back(&kfs[nc]);
  if (first_fixed >= 0) pKF->mvpOrderedConnectedKeyFrames.push_back(&kfs[first_fixed]);
  std::vector<int> nobs0(np);
  for (int p = 0; p < np; p++) nobs0[p] = mps[p].Observations();
  Optimizer::mpfnGatheredHook = gathered_hook;
  bool bStop = stop == 1;
  g_raise_after_gather = stop == 2 ? &bStop : nullptr;
  Optimizer::LocalBundleAdjustment(pKF, &bStop, &map);
  Optimizer::mpfnGatheredHook = nullptr;
  g_raise_after_gather = nullptr;
  // output: the gathered window (as orbx_ba_problem arrays), then the graph after the call
  const LocalBAProblem& G = g_gathered;
  const int gnc = (int)G.cameras.size(), gnp = (int)G.points.size(), gne = (int)G.observations.size();
  Writer o(out);
  o.put<int32_t>(gnc);
  o.put<int32_t>(gnp);
  o.put<int32_t>(gne);
  for (int c = 0; c < gnc; c++)
    for (int i = 0; i < 12; i++) o.put<float>(G.cameras[c].Tcw.at<float>(i / 4, i % 4));
  for (int c = 0; c < gnc; c++) o.put<uint8_t>(G.cameras[c].fixed ? 1 : 0);
  for (int c = 0; c < gnc; c++) {
    const float in5[5] = {G.cameras[c].fx, G.cameras[c].fy, G.cameras[c].cx, G.cameras[c].cy, G.cameras[c].bf};
    o.raw(in5, sizeof(in5));
  }
  for (int p = 0; p < gnp; p++)
    for (int k = 0; k < 3; k++) o.put<float>(G.points[p].at<float>(k, 0));
  for (int e = 0; e < gne; e++) o.put<int32_t>(G.observations[e].point);
  for (int e = 0; e < gne; e++) o.put<int32_t>(G.observations[e].camera);
  for (int e = 0; e < gne; e++) {
    o.put<float>(G.observations[e].u);
    o.put<float>(G.observations[e].v);
    o.put<float>(G.observations[e].ur);
  }
  for (int e = 0; e < gne; e++) o.put<float>(G.observations[e].invSigma2);
  // camera -> input index, point -> input index (the Python side maps the oracle's answer back)
  for (int c = 0; c < gnc; c++) o.put<int32_t>((int32_t)(g_gathered_cams[c] - kfs.data()));
  // poses after the call (all KeyFrames, gathered order), points (gathered order by id), edge state
  for (int c = 0; c < gnc; c++) {
    const cv::Mat Tc = g_gathered_cams[c]->GetPose();
    for (int i = 0; i < 12; i++) o.put<float>(Tc.at<float>(i / 4, i % 4));
  }
  for (int p = 0; p < np; p++) {
    const cv::Mat Xp = mps[p].GetWorldPos();
    for (int k = 0; k < 3; k++) o.put<float>(Xp.at<float>(k, 0));
  }
  for (int p = 0; p < np; p++) o.put<uint8_t>(mps[p].isBad() ? 1 : 0);
  for (int p = 0; p < np; p++) o.put<int32_t>(nobs0[p]);
  for (int e = 0; e < ne; e++) {  // per INPUT edge: observation and KeyFrame match still present
    const int pidx = mps[ep[e]].GetIndexInKeyFrame(&kfs[ec[e]]);
    const bool kf_has = kfs[ec[e]].mvpMapPoints[edge_slot[e]] == &mps[ep[e]];
    o.put<uint8_t>(pidx == edge_slot[e] ? 1 : 0);
    o.put<uint8_t>(kf_has ? 1 : 0);
  }
  std::printf("bagraph ok: window %d cams / %d points / %d edges\n", gnc, gnp, gne);
  return 0;
}

// ---------------------------------------------------------------- PnPsolver in Relocalization's loop
// Input: C candidates, each with n correspondences (p3d, p2d, octave into its level table) and
// intrinsics.  Every candidate's Frame interleaves features without a MapPoint and features whose
// MapPoint is bad (the gather skips both), so vbInliers must come back in feature indices.
static int mode_pnp(const char* in, const char* out) {
  Reader r(in);
  const int C = r.get<int32_t>();
  const double prob = r.get<double>();
  const int minInl = r.get<int32_t>(), maxIt = r.get<int32_t>(), minSet = r.get<int32_t>();
  const float eps = r.get<float>(), th2 = r.get<float>();
  const int max_rounds = r.get<int32_t>();
  struct Cand {
    Frame F;
    std::unique_ptr<MapPoint[]> mps;
    std::vector<int> feat_of;  // correspondence -> feature index
    std::unique_ptr<PnPsolver> solver;
  };
  std::vector<std::unique_ptr<Cand>> cs;
  for (int c = 0; c < C; c++) {
    std::unique_ptr<Cand> cd(new Cand());
    const int n = r.get<int32_t>();
    const float fx = r.get<float>(), fy = r.get<float>(), cx = r.get<float>(), cy = r.get<float>();
    const int nl = r.get<int32_t>();
    const std::vector<float> levels = r.vec<float>(nl);
    const std::vector<float> p3 = r.vec<float>(3 * (size_t)n), p2 = r.vec<float>(2 * (size_t)n);
    const std::vector<int32_t> oc = r.vec<int32_t>(n);
    Frame& F = cd->F;
    F.mvLevelSigma2 = levels;
    cd->mps.reset(new MapPoint[n + n / 5 + 1]);
    int bad = n;
    std::vector<MapPoint*> matches;
    for (int i = 0; i < n; i++) {
      if (i % 3 == 0) {  // a feature without a MapPoint
        F.mvKeysUn.push_back(cv::KeyPoint(1.f, 1.f, 31.f));
        matches.push_back(nullptr);
      }
      if (i % 5 == 0) {  // a feature whose MapPoint is bad
        MapPoint& b = cd->mps[bad++];
        b.mbBad = true;
        F.mvKeysUn.push_back(cv::KeyPoint(2.f, 2.f, 31.f));
        matches.push_back(&b);
      }
      MapPoint& m = cd->mps[i];
      cv::Mat Xp(3, 1, CV_32F);
      for (int k = 0; k < 3; k++) Xp.at<float>(k, 0) = p3[3 * i + k];
      m.SetWorldPos(Xp);
      cd->feat_of.push_back((int)F.mvKeysUn.size());
      F.mvKeysUn.push_back(cv::KeyPoint(p2[2 * i], p2[2 * i + 1], 31.f, -1.f, 0.f, oc[i]));
      matches.push_back(&m);
    }
    F.N = (int)F.mvKeysUn.size();
    Frame::fx = fx;  // static, as in the reference (one camera)
    Frame::fy = fy;
    Frame::cx = cx;
    Frame::cy = cy;
    cd->solver.reset(new PnPsolver(F, matches));
    cd->solver->SetRansacParameters(prob, minInl, maxIt, minSet, eps, th2);  // src/Tracking.cc:1720
    cs.push_back(std::move(cd));
  }
  // src/Tracking.cc:1738-1757 (a returned pose counts as the match)
  Writer o(out);
  std::vector<bool> discarded(C, false);
  int ncand = C;
  bool match = false;
  int calls = 0;
  for (int round = 0; round < max_rounds && ncand > 0 && !match; round++) {
    for (int i = 0; i < C; i++) {
      if (discarded[i]) continue;
      bool bNoMore = false;
      std::vector<bool> vbInliers;
      int nInliers = 0;
      const cv::Mat Tcw = cs[i]->solver->iterate(5, bNoMore, vbInliers, nInliers);
      calls++;
      o.put<int32_t>(i);
      o.put<int32_t>(Tcw.empty() ? 0 : 1);
      o.put<int32_t>(bNoMore ? 1 : 0);
      o.put<int32_t>(nInliers);
      for (int k = 0; k < 16; k++) o.put<float>(Tcw.empty() ? 0.f : Tcw.at<float>(k / 4, k % 4));
      const int n = (int)cs[i]->feat_of.size();
      REQUIRE(Tcw.empty() || (int)vbInliers.size() == cs[i]->F.N);
      for (int k = 0; k < n; k++) o.put<uint8_t>(!Tcw.empty() && vbInliers[cs[i]->feat_of[k]] ? 1 : 0);
      if (!Tcw.empty()) {  // features without a correspondence are never inliers
        int cnt = 0;
        for (bool b : vbInliers) cnt += b;
        REQUIRE(cnt == nInliers);
      }
      if (bNoMore) {
        discarded[i] = true;
        ncand--;
      }
      if (!Tcw.empty()) {
        match = true;
        break;
      }
    }
  }
  bool threw = false;  // parameters are fixed once RANSAC has started
  try {
    cs[0]->solver->SetRansacParameters();
  } catch (const std::logic_error&) {
    threw = true;
  }
  REQUIRE(threw);
  std::printf("pnp ok: %d iterate() calls, match %d\n", calls, (int)match);
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: test_shim abi | stereo IN OUT | bow IN OUT | ba IN OUT | bagraph IN OUT | pnp IN OUT\n");
    return 2;
  }
  const std::string m = argv[1];
  try {
    if (m == "abi") return mode_abi();
    if (argc < 4) return 2;
    if (m == "stereo") return mode_stereo(argv[2], argv[3]);
    if (m == "bow") return mode_bow(argv[2], argv[3]);
    if (m == "ba") return mode_ba(argv[2], argv[3]);
    if (m == "bagraph") return mode_bagraph(argv[2], argv[3]);
    if (m == "pnp") return mode_pnp(argv[2], argv[3]);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "exception: %s\n", e.what());
    return 3;
  }
  return 2;
}
