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
//   proj    IN OUT      ORBmatcher::SearchByProjection x3 (local map / last frame / KeyFrame)
//   fuse    IN OUT      ORBmatcher::Fuse(KeyFrame*, vector<MapPoint*>, th) incl. Replace / AddObservation
//   sim3    IN OUT      ORBmatcher::SearchByProjection(KeyFrame*, Scw, vpPoints, vpMatched, th)
//   fusesim3 IN OUT     ORBmatcher::Fuse(KeyFrame*, Scw, vpPoints, th, vpReplacePoint)
//   bysim3  IN OUT      ORBmatcher::SearchBySim3(KeyFrame*, KeyFrame*, vpMatches12, s12, R12, t12, th)
//   init    IN OUT      ORBmatcher::SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize)
//   tri     IN OUT      ORBmatcher::SearchForTriangulation(KeyFrame*, KeyFrame*, F12, pairs, bOnlyStereo)
//   pose    IN OUT      Optimizer::PoseOptimization(Frame*)
//   distinct IN OUT     MapPoint::ComputeDistinctiveDescriptors
//   voc     IN OUT      ORBVocabulary::loadFromTextFile + Frame::ComputeBoW / KeyFrame::ComputeBoW
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

#include "ORBVocabulary.h"
#include "ORBextractor.h"
#include "ORBmatcher.h"
#include "Objects.h"
#include "Optimizer.h"
#include "PnPsolver.h"
#include "orbx.h"
#include "orbx_shim.h"

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
  // the reference's layouts: ORBmatcher holds {float mfNNratio; bool mbCheckOrientation;}
  // (include/ORBmatcher.h:175-177); cv::Point is Point_<int>
  REQUIRE(sizeof(ORBmatcher) == 8 && sizeof(cv::Point) == 8 && sizeof(cv::Point2f) == 8);
  {
    ORBmatcher dflt;  // ORBmatcher(float nnratio=0.6, bool checkOri=true), include/ORBmatcher.h:47
    (void)dflt;
  }
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
  cv::Mat imL(h, w, CV_8U, L.data()), imR(h, w, CV_8U, R.data());
  cv::Mat K(3, 3, CV_32F), dist(4, 1, CV_32F);
  std::memset(K.data, 0, 36);
  std::memset(dist.data, 0, 16);
  K.at<float>(0, 0) = fx;
  K.at<float>(1, 1) = fx;
  K.at<float>(0, 2) = w / 2.f;
  K.at<float>(1, 2) = h / 2.f;
  K.at<float>(2, 2) = 1.f;
  Frame F(imL, imR, &exL, &exR, K, dist, bf, 35.f * bf / fx);  // one orbx_frame_stereo call (gOrbxFrameStereoFused)
  REQUIRE(F.N == (int)F.mvKeys.size() && (int)F.mvuRight.size() == F.N && (int)F.mvDepth.size() == F.N);
  REQUIRE(F.mvKeysUn.size() == F.mvKeys.size());
  {  // the reference's form -- two extraction threads, then ComputeStereoMatches -- gives the same frame
    gOrbxFrameStereoFused = false;
    Frame F2(imL, imR, &exL, &exR, K, dist, bf, 35.f * bf / fx);
    gOrbxFrameStereoFused = true;
    REQUIRE(F2.N == F.N && F2.mvKeysRight.size() == F.mvKeysRight.size());
    REQUIRE(std::memcmp(F2.mvKeys.data(), F.mvKeys.data(), (size_t)F.N * 28) == 0);
    REQUIRE(std::memcmp(F2.mvKeysRight.data(), F.mvKeysRight.data(), F.mvKeysRight.size() * 28) == 0);
    REQUIRE(F2.mDescriptors.rows == F.mDescriptors.rows && F2.mDescriptorsRight.rows == F.mDescriptorsRight.rows);
    for (int i = 0; i < F.N; i++) REQUIRE(std::memcmp(F2.mDescriptors.ptr<uint8_t>(i), F.mDescriptors.ptr<uint8_t>(i), 32) == 0);
    for (int i = 0; i < F.mDescriptorsRight.rows; i++)
      REQUIRE(std::memcmp(F2.mDescriptorsRight.ptr<uint8_t>(i), F.mDescriptorsRight.ptr<uint8_t>(i), 32) == 0);
    REQUIRE(std::memcmp(F2.mvuRight.data(), F.mvuRight.data(), (size_t)F.N * 4) == 0);
    REQUIRE(std::memcmp(F2.mvDepth.data(), F.mvDepth.data(), (size_t)F.N * 4) == 0);
    REQUIRE(F2.mb == F.mb && F2.mvKeysUn.size() == F.mvKeysUn.size());
  }
  Writer o(out);
  o.put<int32_t>(F.N);
  o.put<int32_t>((int32_t)F.mvKeysRight.size());
  o.raw(F.mvKeys.data(), F.mvKeys.size() * 28);
  for (int i = 0; i < F.N; i++) o.raw(F.mDescriptors.ptr<uint8_t>(i), 32);
  o.raw(F.mvKeysRight.data(), F.mvKeysRight.size() * 28);
  for (size_t i = 0; i < F.mvKeysRight.size(); i++) o.raw(F.mDescriptorsRight.ptr<uint8_t>((int)i), 32);
  o.raw(F.mvuRight.data(), F.mvuRight.size() * 4);
  o.raw(F.mvDepth.data(), F.mvDepth.size() * 4);
  // Frame reads the device pyramids, so its extractions leave mvImagePyramid empty (never stale)
  for (int l = 0; l < nl; l++) REQUIRE(exL.mvImagePyramid[l].empty());
  // operator() itself refreshes mvImagePyramid on every call (src/ORBextractor.cc:1215-1250): first
  // on the right image, then on the left one, whose levels must be the left image's
  {
    std::vector<cv::KeyPoint> kr, kl;
    cv::Mat dr, dl;
    exL(imR, cv::Mat(), kr, dr);
    REQUIRE((int)exL.mvImagePyramid.size() == nl && exL.mvImagePyramid[0].cols == w && exL.mvImagePyramid[0].rows == h);
    REQUIRE(std::memcmp(exL.mvImagePyramid[0].data, R.data(), (size_t)w * h) == 0);
    const cv::Mat keep = exL.mvImagePyramid[1];  // a level a caller kept survives the next call
    std::vector<uint8_t> keep_bytes(keep.data, keep.data + (size_t)keep.rows * keep.step);
    exL(imL, cv::Mat(), kl, dl);
    REQUIRE(kl.size() == F.mvKeys.size() && std::memcmp(kl.data(), F.mvKeys.data(), kl.size() * 28) == 0);
    REQUIRE(keep.data != exL.mvImagePyramid[1].data &&
            std::memcmp(keep.data, keep_bytes.data(), keep_bytes.size()) == 0);
  }
  // the host copy of the left pyramid (mvImagePyramid)
  for (int l = 0; l < nl; l++) {
    const cv::Mat& m = exL.mvImagePyramid[l];
    o.put<int32_t>(m.cols);
    o.put<int32_t>(m.rows);
    for (int y = 0; y < m.rows; y++) o.raw(m.ptr<uint8_t>(y), m.cols);
  }
  // the free-function form gives the same answer on each extractor's last extraction (the left one
  // just re-extracted imLeft above; the right one extracts imRight here)
  {
    std::vector<cv::KeyPoint> kr;
    cv::Mat dr;
    exR(imR, cv::Mat(), kr, dr);
    REQUIRE(kr.size() == F.mvKeysRight.size() && std::memcmp(kr.data(), F.mvKeysRight.data(), kr.size() * 28) == 0);
  }
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
  // as in the reference, SetRansacParameters may be called after iterate() (in place)
  cs[0]->solver->SetRansacParameters(prob, minInl, maxIt, minSet, eps, th2);
  std::printf("pnp ok: %d iterate() calls, match %d\n", calls, (int)match);
  return 0;
}

// ---------------------------------------------------------------------------- §8(f) members
// A current Frame from the payload: N, keypoints (cv::KeyPoint bytes), descriptors, mvuRight (or
// none), the entry occupancy (0 NULL, 1 a MapPoint with no observation, 2 one with observations),
// the static bounds / grid, scale tables, intrinsics and pose.
struct FramePayload {
  Frame F;
  std::vector<std::unique_ptr<MapPoint>> occupants;  // the entry MapPoints of F.mvpMapPoints
  std::vector<int8_t> occ;
};

static void read_frame(Reader& r, FramePayload& fp) {
  Frame& F = fp.F;
  const int n = r.get<int32_t>();
  F.N = n;
  F.mvKeysUn.resize(n);
  if (n) REQUIRE(std::fread(F.mvKeysUn.data(), 28, n, r.f) == (size_t)n);
  F.mvKeys = F.mvKeysUn;
  F.mDescriptors.create(n > 0 ? n : 1, 32, CV_8U);
  if (n) REQUIRE(std::fread(F.mDescriptors.data, 32, n, r.f) == (size_t)n);
  if (n == 0) F.mDescriptors.release();
  const int has_ur = r.get<int32_t>();
  F.mvuRight = has_ur ? r.vec<float>(n) : std::vector<float>(n, -1.f);
  fp.occ = r.vec<int8_t>(n);
  F.mvpMapPoints.assign(n, nullptr);
  F.mvbOutlier.assign(n, false);
  for (int i = 0; i < n; i++) {
    if (!fp.occ[i]) continue;
    fp.occupants.emplace_back(new MapPoint());
    fp.occupants.back()->nObs = fp.occ[i] == 2 ? 2 : 0;
    F.mvpMapPoints[i] = fp.occupants.back().get();
  }
  const float b[6] = {r.get<float>(), r.get<float>(), r.get<float>(), r.get<float>(), r.get<float>(), r.get<float>()};
  Frame::mnMinX = b[0];
  Frame::mnMaxX = b[1];
  Frame::mnMinY = b[2];
  Frame::mnMaxY = b[3];
  Frame::mfGridElementWidthInv = b[4];
  Frame::mfGridElementHeightInv = b[5];
  F.mnScaleLevels = r.get<int32_t>();
  F.mvScaleFactors = r.vec<float>(F.mnScaleLevels);
  F.mvInvLevelSigma2 = r.vec<float>(F.mnScaleLevels);
  F.mvLevelSigma2.resize(F.mnScaleLevels);
  for (int l = 0; l < F.mnScaleLevels; l++) F.mvLevelSigma2[l] = F.mvScaleFactors[l] * F.mvScaleFactors[l];
  F.mfLogScaleFactor = r.get<float>();
  Frame::fx = r.get<float>();
  Frame::fy = r.get<float>();
  Frame::cx = r.get<float>();
  Frame::cy = r.get<float>();
  F.mbf = r.get<float>();
  F.mb = r.get<float>();
  cv::Mat T(4, 4, CV_32F);
  for (int i = 0; i < 16; i++) T.at<float>(i / 4, i % 4) = r.get<float>();
  F.SetPose(T);
}

struct PointPayload {
  int n = 0;
  std::vector<uint8_t> desc, flags;
  std::vector<float> pos, normal, dist, angle, track;
  std::vector<int32_t> octave, level;
};

static void read_points(Reader& r, PointPayload& P) {
  P.n = r.get<int32_t>();
  const size_t n = P.n;
  P.desc = r.vec<uint8_t>(32 * n);
  P.flags = r.vec<uint8_t>(n);
  P.pos = r.vec<float>(3 * n);
  P.normal = r.vec<float>(3 * n);
  P.dist = r.vec<float>(2 * n);
  P.angle = r.vec<float>(n);
  P.octave = r.vec<int32_t>(n);
  P.track = r.vec<float>(4 * n);
  P.level = r.vec<int32_t>(n);
}

static void make_point(MapPoint& m, const PointPayload& P, int k) {
  cv::Mat X(3, 1, CV_32F), N(3, 1, CV_32F), D(1, 32, CV_8U);
  for (int c = 0; c < 3; c++) {
    X.at<float>(c, 0) = P.pos[3 * k + c];
    N.at<float>(c, 0) = P.normal[3 * k + c];
  }
  std::memcpy(D.data, &P.desc[32 * (size_t)k], 32);
  m.SetWorldPos(X);
  m.mNormalVector = N;
  m.mDescriptor = D;
  m.mfMinDistance = P.dist[2 * k];
  m.mfMaxDistance = P.dist[2 * k + 1];
  m.nObs = (P.flags[k] & 2) ? 2 : 0;
  m.mnId = (unsigned long)(k + 1);
}

// the Frame's mvpMapPoints after the call: point index k, -1 NULL, -10 - occ for an entry occupant
static void write_frame_state(Writer& o, const FramePayload& fp, const std::vector<MapPoint*>& pts) {
  std::map<const MapPoint*, int> index;
  for (size_t k = 0; k < pts.size(); k++)
    if (pts[k]) index[pts[k]] = (int)k;
  for (int i = 0; i < fp.F.N; i++) {
    MapPoint* m = fp.F.mvpMapPoints[i];
    int v = -1;
    if (m) {
      auto it = index.find(m);
      if (it != index.end())
        v = it->second;
      else
        v = -10 - (m->nObs > 0 ? 2 : 1);
    }
    o.put<int32_t>(v);
  }
}

// SearchByProjection x3 through the reference signatures
static int mode_proj(const char* in, const char* out) {
  Reader r(in);
  const int kind = r.get<int32_t>();
  const float th = r.get<float>(), nnratio = r.get<float>();
  const int check_ori = r.get<int32_t>(), mono = r.get<int32_t>(), orb_dist = r.get<int32_t>();
  cv::Mat lastT(4, 4, CV_32F);
  for (int i = 0; i < 16; i++) lastT.at<float>(i / 4, i % 4) = r.get<float>();
  FramePayload fp;
  read_frame(r, fp);
  PointPayload P;
  read_points(r, P);
  const int n = P.n;
  std::vector<std::unique_ptr<MapPoint>> store;
  std::vector<MapPoint*> pts(n, nullptr);
  ORBmatcher matcher(nnratio, check_ori != 0);
  int nm = 0;
  if (kind == 0) {  // Tracking::SearchLocalPoints' list: every point non-NULL, in view by bit0
    for (int k = 0; k < n; k++) {
      store.emplace_back(new MapPoint());
      MapPoint& m = *store.back();
      make_point(m, P, k);
      m.mbTrackInView = (P.flags[k] & 1) != 0;
      m.mTrackProjX = P.track[4 * k];
      m.mTrackProjY = P.track[4 * k + 1];
      m.mTrackProjXR = P.track[4 * k + 2];
      m.mTrackViewCos = P.track[4 * k + 3];
      m.mnTrackScaleLevel = P.level[k];
      pts[k] = &m;
    }
    nm = matcher.SearchByProjection(fp.F, pts, th);
  } else if (kind == 1) {  // LastFrame: bit0 = pMP && !mvbOutlier -- NULL or outlier otherwise
    Frame Last;
    Last.N = n;
    Last.mvpMapPoints.assign(n, nullptr);
    Last.mvbOutlier.assign(n, false);
    Last.mvKeys.resize(n);
    Last.mvKeysUn.resize(n);
    for (int k = 0; k < n; k++) {
      Last.mvKeys[k].octave = P.octave[k];
      Last.mvKeysUn[k].octave = P.octave[k];
      Last.mvKeysUn[k].angle = P.angle[k];
      if (!(P.flags[k] & 1) && k % 2 == 0) continue;  // no MapPoint
      store.emplace_back(new MapPoint());
      make_point(*store.back(), P, k);
      Last.mvpMapPoints[k] = pts[k] = store.back().get();
      Last.mvbOutlier[k] = !(P.flags[k] & 1);
    }
    Last.SetPose(lastT);
    nm = matcher.SearchByProjection(fp.F, Last, th, mono != 0);
  } else {  // KeyFrame: bit0 = pMP && !isBad() && !sAlreadyFound.count(pMP)
    KeyFrame K;
    K.N = n;
    K.mvKeysUn.resize(n);
    K.mvpMapPoints.assign(n, nullptr);
    std::set<MapPoint*> found;
    for (int k = 0; k < n; k++) {
      K.mvKeysUn[k].angle = P.angle[k];
      K.mvKeysUn[k].octave = P.octave[k];
      if (!(P.flags[k] & 1) && k % 3 == 0) continue;  // no MapPoint
      store.emplace_back(new MapPoint());
      MapPoint& m = *store.back();
      make_point(m, P, k);
      if (!(P.flags[k] & 1)) {
        if (k % 3 == 1)
          m.mbBad = true;
        else
          found.insert(&m);
      }
      K.mvpMapPoints[k] = pts[k] = &m;
    }
    nm = matcher.SearchByProjection(fp.F, &K, found, th, orb_dist);
  }
  Writer o(out);
  o.put<int32_t>(nm);
  write_frame_state(o, fp, pts);
  std::printf("proj ok: kind %d, %d matches\n", kind, nm);
  return 0;
}

// Fuse(KeyFrame*, const vector<MapPoint*>&, th) with its Replace / AddObservation block.  pKF is the
// payload frame (its features' MapPoints: the entry occupants, each observed by pKF and by some of
// `nother` extra KeyFrames); every fuse candidate is observed by some extra KeyFrames.
static int mode_fuse(const char* in, const char* out) {
  Reader r(in);
  const float th = r.get<float>();
  FramePayload fp;
  read_frame(r, fp);
  PointPayload P;
  read_points(r, P);
  const int nother = r.get<int32_t>();
  const int nocc = (int)fp.occupants.size();
  // observation sets: per candidate / per occupant, a bitmask over the extra KeyFrames
  const std::vector<uint32_t> cand_obs = r.vec<uint32_t>(P.n), occ_obs = r.vec<uint32_t>(nocc);
  const int ikf = r.get<int32_t>();  // bounds of pKF as its integer copies
  (void)ikf;
  Map map;
  const Frame& F = fp.F;
  KeyFrame K;
  K.mnId = 1000;
  K.N = F.N;
  K.mvKeysUn = F.mvKeysUn;
  K.mDescriptors = F.mDescriptors;
  K.mvuRight = F.mvuRight;
  K.mvpMapPoints.assign(F.N, nullptr);
  K.mnMinX = (int)Frame::mnMinX;
  K.mnMaxX = (int)Frame::mnMaxX;
  K.mnMinY = (int)Frame::mnMinY;
  K.mnMaxY = (int)Frame::mnMaxY;
  K.mfGridElementWidthInv = Frame::mfGridElementWidthInv;
  K.mfGridElementHeightInv = Frame::mfGridElementHeightInv;
  K.mnScaleLevels = F.mnScaleLevels;
  K.mvScaleFactors = F.mvScaleFactors;
  K.mvLevelSigma2 = F.mvLevelSigma2;
  K.mvInvLevelSigma2 = F.mvInvLevelSigma2;
  K.mfLogScaleFactor = F.mfLogScaleFactor;
  K.fx = Frame::fx;
  K.fy = Frame::fy;
  K.cx = Frame::cx;
  K.cy = Frame::cy;
  K.mbf = F.mbf;
  K.mb = F.mb;
  K.SetPose(F.mTcw);
  // extra KeyFrames: one monocular feature slot per MapPoint that observes them, random descriptors
  const int nmp = P.n + nocc;
  std::vector<std::unique_ptr<KeyFrame>> others;
  for (int j = 0; j < nother; j++) {
    others.emplace_back(new KeyFrame());
    KeyFrame& O = *others.back();
    O.mnId = (unsigned long)(2000 + j);
    O.N = nmp;
    O.mvKeysUn.resize(nmp);
    O.mvuRight.assign(nmp, -1.f);
    O.mvpMapPoints.assign(nmp, nullptr);
    O.mDescriptors.create(nmp, 32, CV_8U);
    for (int q = 0; q < nmp; q++)
      for (int b = 0; b < 32; b++) O.mDescriptors.at<uint8_t>(q, b) = (uint8_t)((q * 131 + j * 71 + b * 29) & 0xFF);
  }
  std::vector<std::unique_ptr<MapPoint>> cands;
  std::vector<MapPoint*> pts(P.n, nullptr);
  auto observe_others = [&](MapPoint* m, uint32_t mask, int slot) {
    for (int j = 0; j < nother; j++)
      if (mask >> j & 1) {
        others[j]->mvpMapPoints[slot] = m;
        m->AddObservation(others[j].get(), slot);
      }
  };
  for (int k = 0; k < P.n; k++) {
    cands.emplace_back(new MapPoint());
    MapPoint& m = *cands.back();
    make_point(m, P, k);
    m.nObs = 0;
    m.mpMap = &map;
    map.mspMapPoints.insert(&m);
    observe_others(&m, cand_obs[k], k);
    if (!(P.flags[k] & 1)) m.mbBad = (k % 2 == 0);  // bit0 off: bad, or already in pKF (below)
    pts[k] = &m;
  }
  // the entry occupants become pKF's own MapPoints (observed by pKF at their feature)
  std::vector<MapPoint*> occs;
  int oi = 0;
  for (int i = 0; i < F.N; i++) {
    MapPoint* m = F.mvpMapPoints[i];
    if (!m) continue;
    m->nObs = 0;
    m->mnId = (unsigned long)(100000 + oi);
    m->mpMap = &map;
    map.mspMapPoints.insert(m);
    cv::Mat D(1, 32, CV_8U);
    std::memcpy(D.data, F.mDescriptors.ptr<uint8_t>(i), 32);
    m->mDescriptor = D;
    K.mvpMapPoints[i] = m;
    m->AddObservation(&K, i);
    observe_others(m, occ_obs[oi], P.n + oi);
    occs.push_back(m);
    oi++;
  }
  // candidates with bit0 off and odd index: already observed by pKF at a free feature of theirs
  for (int k = 0; k < P.n; k++)
    if (!(P.flags[k] & 1) && k % 2 == 1) {
      for (int i = 0; i < F.N; i++)
        if (!K.mvpMapPoints[i]) {
          K.mvpMapPoints[i] = pts[k];
          pts[k]->AddObservation(&K, i);
          break;
        }
    }
  ORBmatcher matcher;
  const int nf = matcher.Fuse(&K, pts, th);
  Writer o(out);
  o.put<int32_t>(nf);
  // pKF's features: candidate k, or -100 - occupant index, -1 NULL
  for (int i = 0; i < K.N; i++) {
    MapPoint* m = K.mvpMapPoints[i];
    int v = -1;
    for (int k = 0; k < P.n && v == -1; k++)
      if (pts[k] == m) v = k;
    for (int q = 0; q < nocc && v == -1; q++)
      if (occs[q] == m) v = -100 - q;
    o.put<int32_t>(m ? v : -1);
  }
  // every MapPoint (candidates, then occupants): bad, nObs, mDescriptor
  auto put_mp = [&](MapPoint* m) {
    o.put<uint8_t>(m->isBad() ? 1 : 0);
    o.put<int32_t>(m->Observations());
    const cv::Mat d = m->GetDescriptor();
    o.raw(d.data, 32);
  };
  for (MapPoint* m : pts) put_mp(m);
  for (MapPoint* m : occs) put_mp(m);
  std::printf("fuse ok: %d fused\n", nf);
  return 0;
}

// SearchByProjection(KeyFrame*, Scw, vpPoints, vpMatched, th).  pKF is the payload frame.  vpMatched
// on entry holds its occupied features: the first of them take the odd-index candidates with bit0
// off (so those are in spAlreadyFound), the rest their own entry MapPoints; even-index candidates
// with bit0 off are bad.
static void keyframe_from_frame(const Frame& F, KeyFrame& K) {
  K.mnId = 1000;
  K.N = F.N;
  K.mvKeysUn = F.mvKeysUn;
  K.mDescriptors = F.mDescriptors;
  K.mvuRight = F.mvuRight;
  K.mvpMapPoints.assign(F.N, nullptr);
  K.mnMinX = (int)Frame::mnMinX;
  K.mnMaxX = (int)Frame::mnMaxX;
  K.mnMinY = (int)Frame::mnMinY;
  K.mnMaxY = (int)Frame::mnMaxY;
  K.mfGridElementWidthInv = Frame::mfGridElementWidthInv;
  K.mfGridElementHeightInv = Frame::mfGridElementHeightInv;
  K.mnScaleLevels = F.mnScaleLevels;
  K.mvScaleFactors = F.mvScaleFactors;
  K.mvLevelSigma2 = F.mvLevelSigma2;
  K.mvInvLevelSigma2 = F.mvInvLevelSigma2;
  K.mfLogScaleFactor = F.mfLogScaleFactor;
  K.fx = Frame::fx;
  K.fy = Frame::fy;
  K.cx = Frame::cx;
  K.cy = Frame::cy;
  K.mbf = F.mbf;
  K.mb = F.mb;
  K.SetPose(F.mTcw);
}

// The candidates of a Sim3 mode, and the entry MapPoints of the KeyFrame's occupied features: the first
// occupied features take the odd-index candidates with bit0 off, the rest their own entry MapPoints.
// Every other candidate with bit0 off is bad, so bit0 is exactly "!isBad() && not already there".
static void sim3_points(const FramePayload& fp, const PointPayload& P, std::vector<std::unique_ptr<MapPoint>>& cands,
                        std::vector<MapPoint*>& pts, std::vector<MapPoint*>& entry) {
  const Frame& F = fp.F;
  pts.assign(P.n, nullptr);
  for (int k = 0; k < P.n; k++) {
    cands.emplace_back(new MapPoint());
    MapPoint& m = *cands.back();
    make_point(m, P, k);
    m.mbBad = !(P.flags[k] & 1);  // cleared below for the candidates that become entry MapPoints
    pts[k] = &m;
  }
  entry.assign(F.N, nullptr);
  int kk = 1;
  for (int i = 0; i < F.N; i++) {
    if (!F.mvpMapPoints[i]) continue;
    while (kk < P.n && (P.flags[kk] & 1)) kk += 2;
    if (kk < P.n) {
      entry[i] = pts[kk];
      pts[kk]->mbBad = false;
      kk += 2;
    } else {
      entry[i] = F.mvpMapPoints[i];
    }
  }
}

// MapPoint -> code: candidate k, -1000 - i for the entry MapPoint of feature i, -1 NULL
static int sim3_code(const MapPoint* m, const std::vector<MapPoint*>& pts, const std::vector<MapPoint*>& entry) {
  if (!m) return -1;
  for (size_t k = 0; k < pts.size(); k++)
    if (pts[k] == m) return (int)k;
  for (size_t i = 0; i < entry.size(); i++)
    if (entry[i] == m) return -1000 - (int)i;
  return -2;
}

static int mode_sim3(const char* in, const char* out) {
  Reader r(in);
  const int th = r.get<int32_t>();
  cv::Mat Scw(4, 4, CV_32F);
  for (int i = 0; i < 16; i++) Scw.at<float>(i / 4, i % 4) = r.get<float>();
  FramePayload fp;
  read_frame(r, fp);
  PointPayload P;
  read_points(r, P);
  const Frame& F = fp.F;
  KeyFrame K;
  keyframe_from_frame(F, K);
  std::vector<std::unique_ptr<MapPoint>> cands;
  std::vector<MapPoint*> pts, vpMatched;
  sim3_points(fp, P, cands, pts, vpMatched);
  const std::vector<MapPoint*> entry(vpMatched);
  ORBmatcher matcher;
  const int nm = matcher.SearchByProjection(&K, Scw, pts, vpMatched, th);
  Writer o(out);
  o.put<int32_t>(nm);
  // vpMatched afterwards: candidate k, -1000 - i the entry MapPoint of feature i, -1 NULL
  for (int i = 0; i < F.N; i++) o.put<int32_t>(sim3_code(vpMatched[i], pts, entry));
  std::printf("sim3 ok: %d matches\n", nm);
  return 0;
}

// Fuse(KeyFrame*, Scw, vpPoints, th, vpReplacePoint): pKF's MapPoints are the entry MapPoints of
// sim3_points (those of features i with i % 3 == 0 that are not candidates are bad).  Out: nFused,
// vpReplacePoint per point and pKF's MapPoints per feature afterwards, as sim3_code codes.
static int mode_fusesim3(const char* in, const char* out) {
  Reader r(in);
  const float th = r.get<float>();
  cv::Mat Scw(4, 4, CV_32F);
  for (int i = 0; i < 16; i++) Scw.at<float>(i / 4, i % 4) = r.get<float>();
  FramePayload fp;
  read_frame(r, fp);
  PointPayload P;
  read_points(r, P);
  const Frame& F = fp.F;
  KeyFrame K;
  keyframe_from_frame(F, K);
  std::vector<std::unique_ptr<MapPoint>> cands;
  std::vector<MapPoint*> pts, entry;
  sim3_points(fp, P, cands, pts, entry);
  for (int i = 0; i < F.N; i++) {
    K.mvpMapPoints[i] = entry[i];
    if (entry[i] && i % 3 == 0 && sim3_code(entry[i], pts, entry) < -1) entry[i]->mbBad = true;
  }
  std::vector<MapPoint*> rep(P.n, nullptr);
  ORBmatcher matcher;
  const int nf = matcher.Fuse(&K, Scw, pts, th, rep);
  Writer o(out);
  o.put<int32_t>(nf);
  for (int k = 0; k < P.n; k++) o.put<int32_t>(sim3_code(rep[k], pts, entry));
  for (int i = 0; i < F.N; i++) o.put<int32_t>(sim3_code(K.mvpMapPoints[i], pts, entry));
  std::printf("fusesim3 ok: %d fused\n", nf);
  return 0;
}

// SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th): both KeyFrames are the payload frame (two
// frame records), feature i of KeyFrame j holds point i of points payload j.  Points with bit0 off:
// i % 3 == 0 NULL, == 1 bad, == 2 "already matched" -- KF1's such features take vpMatches12 entries
// pointing at KF2's such MapPoints in order (observed by KF2 there; KF2's left over are bad, KF1's left
// over point at a MapPoint outside KF2).  Out: nFound, vpMatches12 per KF1 feature (KF2 feature
// index of the MapPoint, -2 one outside KF2, -1 NULL).
static int mode_bysim3(const char* in, const char* out) {
  Reader r(in);
  const float th = r.get<float>(), s12 = r.get<float>();
  cv::Mat R12(3, 3, CV_32F), t12(3, 1, CV_32F);
  for (int i = 0; i < 9; i++) R12.at<float>(i / 3, i % 3) = r.get<float>();
  for (int i = 0; i < 3; i++) t12.at<float>(i, 0) = r.get<float>();
  FramePayload fp1, fp2;
  read_frame(r, fp1);
  read_frame(r, fp2);
  PointPayload P1, P2;
  read_points(r, P1);
  read_points(r, P2);
  KeyFrame K1, K2;
  keyframe_from_frame(fp1.F, K1);
  keyframe_from_frame(fp2.F, K2);
  K2.mnId = 1001;
  std::vector<std::unique_ptr<MapPoint>> own;
  auto fill = [&](KeyFrame& K, const PointPayload& P, std::vector<MapPoint*>& mp) {
    mp.assign(K.N, nullptr);
    for (int i = 0; i < K.N && i < P.n; i++) {
      if (!(P.flags[i] & 1) && i % 3 == 0) continue;  // NULL
      own.emplace_back(new MapPoint());
      MapPoint& m = *own.back();
      make_point(m, P, i);
      m.mbBad = !(P.flags[i] & 1) && i % 3 == 1;
      mp[i] = &m;
      K.mvpMapPoints[i] = &m;
    }
  };
  std::vector<MapPoint*> mp1, mp2;
  fill(K1, P1, mp1);
  fill(K2, P2, mp2);
  std::vector<int> targets;  // KF2's "already matched" features
  for (int j = 0; j < K2.N && j < P2.n; j++)
    if (!(P2.flags[j] & 1) && j % 3 == 2) targets.push_back(j);
  std::vector<MapPoint*> vpMatches12(K1.N, nullptr);
  own.emplace_back(new MapPoint());
  MapPoint* outside = own.back().get();
  size_t t = 0;
  for (int i = 0; i < K1.N && i < P1.n; i++) {
    if ((P1.flags[i] & 1) || i % 3 != 2) continue;
    if (t < targets.size()) {
      MapPoint* m = mp2[targets[t]];
      m->AddObservation(&K2, targets[t]);
      vpMatches12[i] = m;
      t++;
    } else {
      vpMatches12[i] = outside;
    }
  }
  for (; t < targets.size(); t++) mp2[targets[t]]->mbBad = true;
  ORBmatcher matcher;
  const int nf = matcher.SearchBySim3(&K1, &K2, vpMatches12, s12, R12, t12, th);
  Writer o(out);
  o.put<int32_t>(nf);
  for (int i = 0; i < K1.N; i++) {
    int v = vpMatches12[i] ? -2 : -1;
    for (int j = 0; j < K2.N && v == -2; j++)
      if (mp2[j] == vpMatches12[i]) v = j;
    o.put<int32_t>(v);
  }
  std::printf("bysim3 ok: %d found\n", nf);
  return 0;
}

// SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize) with ORBmatcher(nnratio, check).
// Out: nmatches, vnMatches12, vbPrevMatched (x, y floats).
static int mode_init(const char* in, const char* out) {
  Reader r(in);
  const int window = r.get<int32_t>();
  const float nn = r.get<float>();
  const int check = r.get<int32_t>();
  FramePayload fp1, fp2;
  read_frame(r, fp1);
  read_frame(r, fp2);
  std::vector<cv::Point2f> prev(fp1.F.N);
  for (int i = 0; i < fp1.F.N; i++) {
    const float x = r.get<float>();
    prev[i] = cv::Point2f(x, r.get<float>());
  }
  std::vector<int> m12;
  ORBmatcher matcher(nn, check != 0);
  const int nm = matcher.SearchForInitialization(fp1.F, fp2.F, prev, m12, window);
  Writer o(out);
  o.put<int32_t>(nm);
  for (int i = 0; i < fp1.F.N; i++) o.put<int32_t>(m12[i]);
  for (int i = 0; i < fp1.F.N; i++) {
    o.put<float>(prev[i].x);
    o.put<float>(prev[i].y);
  }
  std::printf("init ok: %d matches\n", nm);
  return 0;
}

// SearchForTriangulation(KeyFrame*, KeyFrame*, F12, vMatchedPairs, bOnlyStereo)
static void read_tri_kf(Reader& r, KeyFrame& K) {
  K.N = r.get<int32_t>();
  const int n = K.N;
  K.mvKeysUn.resize(n);
  if (n) REQUIRE(std::fread(K.mvKeysUn.data(), 28, n, r.f) == (size_t)n);
  K.mDescriptors.create(n > 0 ? n : 1, 32, CV_8U);
  if (n) REQUIRE(std::fread(K.mDescriptors.data, 32, n, r.f) == (size_t)n);
  const int has_ur = r.get<int32_t>();
  K.mvuRight = has_ur ? r.vec<float>(n) : std::vector<float>(n, -1.f);
  const std::vector<uint8_t> has_mp = r.vec<uint8_t>(n);
  K.mvpMapPoints.assign(n, nullptr);
  static MapPoint dummy;
  for (int i = 0; i < n; i++)
    if (has_mp[i]) K.mvpMapPoints[i] = &dummy;
  const int nn = r.get<int32_t>();
  const std::vector<uint32_t> ids = r.vec<uint32_t>(nn);
  const std::vector<int32_t> off = r.vec<int32_t>(nn + 1);
  const std::vector<int32_t> feat = r.vec<int32_t>(nn ? off[nn] : 0);
  for (int j = 0; j < nn; j++)
    for (int q = off[j]; q < off[j + 1]; q++) K.mFeatVec[ids[j]].push_back((unsigned)feat[q]);
}

static int mode_tri(const char* in, const char* out) {
  Reader r(in);
  const int only_stereo = r.get<int32_t>(), check_ori = r.get<int32_t>();
  KeyFrame K1, K2;
  read_tri_kf(r, K1);
  read_tri_kf(r, K2);
  cv::Mat F12(3, 3, CV_32F);
  for (int i = 0; i < 9; i++) F12.at<float>(i / 3, i % 3) = r.get<float>();
  // pKF1's camera centre through a pose whose Ow is exactly C1w: Tcw = [I | -C1w]
  cv::Mat T1(4, 4, CV_32F);
  for (int i = 0; i < 16; i++) T1.at<float>(i / 4, i % 4) = (i % 5 == 0) ? 1.f : 0.f;
  for (int k = 0; k < 3; k++) T1.at<float>(k, 3) = -r.get<float>();
  K1.SetPose(T1);
  cv::Mat T2(4, 4, CV_32F);
  for (int i = 0; i < 16; i++) T2.at<float>(i / 4, i % 4) = r.get<float>();
  K2.SetPose(T2);
  K2.fx = r.get<float>();
  K2.fy = r.get<float>();
  K2.cx = r.get<float>();
  K2.cy = r.get<float>();
  K2.mnScaleLevels = r.get<int32_t>();
  K2.mvScaleFactors = r.vec<float>(K2.mnScaleLevels);
  K2.mvLevelSigma2 = r.vec<float>(K2.mnScaleLevels);
  ORBmatcher matcher(0.6f, check_ori != 0);
  std::vector<std::pair<size_t, size_t>> pairs;
  const int nm = matcher.SearchForTriangulation(&K1, &K2, F12, pairs, only_stereo != 0);
  REQUIRE(nm == (int)pairs.size());
  Writer o(out);
  o.put<int32_t>(nm);
  for (const auto& pr : pairs) {
    o.put<int32_t>((int32_t)pr.first);
    o.put<int32_t>((int32_t)pr.second);
  }
  std::printf("tri ok: %d pairs\n", nm);
  return 0;
}

// Optimizer::PoseOptimization(Frame*): edges from the Frame's MapPoints (every third feature
// without one), mvbOutlier and the pose written back
static int mode_pose(const char* in, const char* out) {
  Reader r(in);
  const int n = r.get<int32_t>();
  const std::vector<float> obs = r.vec<float>(3 * (size_t)n), X = r.vec<float>(3 * (size_t)n),
                           isig = r.vec<float>(n);
  Frame::fx = r.get<float>();
  Frame::fy = r.get<float>();
  Frame::cx = r.get<float>();
  Frame::cy = r.get<float>();
  const float bf = r.get<float>();
  cv::Mat T(4, 4, CV_32F);
  for (int i = 0; i < 16; i++) T.at<float>(i / 4, i % 4) = r.get<float>();
  Frame F;
  F.mbf = bf;
  std::vector<std::unique_ptr<MapPoint>> mps;
  std::vector<int> feat_of;
  // the information of each edge comes from mvInvLevelSigma2[octave]: one level per distinct value
  std::vector<float> levels;
  for (int k = 0; k < n; k++) {
    if (k % 3 == 0) {  // a feature without a MapPoint (no edge), flagged outlier before the call
      F.mvKeysUn.push_back(cv::KeyPoint(5.f, 5.f, 31.f, -1.f, 0.f, 0));
      F.mvuRight.push_back(-1.f);
      F.mvpMapPoints.push_back(nullptr);
    }
    int lv = -1;
    for (size_t l = 0; l < levels.size(); l++)
      if (levels[l] == isig[k]) lv = (int)l;
    if (lv < 0) {
      lv = (int)levels.size();
      levels.push_back(isig[k]);
    }
    mps.emplace_back(new MapPoint());
    cv::Mat Xp(3, 1, CV_32F);
    for (int c = 0; c < 3; c++) Xp.at<float>(c, 0) = X[3 * k + c];
    mps.back()->SetWorldPos(Xp);
    feat_of.push_back((int)F.mvKeysUn.size());
    F.mvKeysUn.push_back(cv::KeyPoint(obs[3 * k], obs[3 * k + 1], 31.f, -1.f, 0.f, lv));
    F.mvuRight.push_back(obs[3 * k + 2]);
    F.mvpMapPoints.push_back(mps.back().get());
  }
  F.N = (int)F.mvKeysUn.size();
  F.mvInvLevelSigma2 = levels;
  F.mvbOutlier.assign(F.N, true);
  F.SetPose(T);
  const int ngood = Optimizer::PoseOptimization(&F);
  Writer o(out);
  o.put<int32_t>(ngood);
  for (int i = 0; i < 16; i++) o.put<float>(F.mTcw.at<float>(i / 4, i % 4));
  for (int k = 0; k < n; k++) o.put<uint8_t>(F.mvbOutlier[feat_of[k]] ? 1 : 0);
  // features without a MapPoint keep their flag
  for (int i = 0; i < F.N; i++)
    if (!F.mvpMapPoints[i]) REQUIRE(F.mvbOutlier[i]);
  std::printf("pose ok: %d good\n", ngood);
  return 0;
}

// MapPoint::ComputeDistinctiveDescriptors on points observed by several KeyFrames (some bad)
static int mode_distinct(const char* in, const char* out) {
  Reader r(in);
  const int np = r.get<int32_t>(), nkf = r.get<int32_t>();
  // one array: ascending addresses, so mObservations (a map keyed by KeyFrame*) iterates in j order
  std::unique_ptr<KeyFrame[]> kfs(new KeyFrame[nkf > 0 ? nkf : 1]);
  for (int j = 0; j < nkf; j++) {
    KeyFrame& K = kfs[j];
    K.mnId = (unsigned long)j;
    K.N = np;
    K.mvuRight.assign(np, -1.f);
    K.mvKeysUn.resize(np);
    K.mvpMapPoints.assign(np, nullptr);
    K.mDescriptors.create(np > 0 ? np : 1, 32, CV_8U);
    if (np) REQUIRE(std::fread(K.mDescriptors.data, 32, np, r.f) == (size_t)np);
    K.mbBad = r.get<uint8_t>() != 0;
  }
  Writer o(out);
  for (int p = 0; p < np; p++) {
    MapPoint m;
    const uint32_t mask = r.get<uint32_t>();
    for (int j = 0; j < nkf; j++)
      if (mask >> j & 1) m.AddObservation(&kfs[j], p);
    m.mDescriptor = cv::Mat(1, 32, CV_8U);
    std::memset(m.mDescriptor.data, 0xAB, 32);  // kept when nothing is observed
    m.ComputeDistinctiveDescriptors();
    o.raw(m.GetDescriptor().data, 32);
  }
  std::printf("distinct ok\n");
  return 0;
}

// ORBVocabulary::loadFromTextFile + Frame::ComputeBoW / KeyFrame::ComputeBoW
static int mode_voc(const char* in, const char* out) {
  Reader r(in);
  const int len = r.get<int32_t>();
  const std::vector<char> text = r.vec<char>(len);
  const std::string path = std::string(out) + ".voc.txt";
  {
    FILE* f = std::fopen(path.c_str(), "wb");
    REQUIRE(f);
    REQUIRE(std::fwrite(text.data(), 1, text.size(), f) == text.size());
    std::fclose(f);
  }
  ORBVocabulary voc;
  REQUIRE(!voc.loadFromTextFile(path + ".missing"));
  REQUIRE(voc.loadFromTextFile(path));
  const int n = r.get<int32_t>();
  Frame F;
  F.mpORBvocabulary = &voc;
  F.N = n;
  F.mDescriptors.create(n > 0 ? n : 1, 32, CV_8U);
  if (n) REQUIRE(std::fread(F.mDescriptors.data, 32, n, r.f) == (size_t)n);
  F.ComputeBoW();
  KeyFrame K;
  K.mpORBvocabulary = &voc;
  K.mDescriptors = F.mDescriptors;
  K.ComputeBoW();
  REQUIRE(K.mBowVec.size() == F.mBowVec.size() && K.mFeatVec.size() == F.mFeatVec.size());
  Writer o(out);
  o.put<int32_t>((int32_t)F.mBowVec.size());
  for (const auto& w : F.mBowVec) {
    o.put<uint32_t>(w.first);
    o.put<double>(w.second);
  }
  o.put<int32_t>((int32_t)F.mFeatVec.size());
  for (const auto& node : F.mFeatVec) {
    o.put<uint32_t>(node.first);
    o.put<int32_t>((int32_t)node.second.size());
    for (unsigned int f : node.second) o.put<int32_t>((int32_t)f);
  }
  std::remove(path.c_str());
  std::printf("voc ok: %zu words\n", F.mBowVec.size());
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
    if (m == "proj") return mode_proj(argv[2], argv[3]);
    if (m == "fuse") return mode_fuse(argv[2], argv[3]);
    if (m == "sim3") return mode_sim3(argv[2], argv[3]);
    if (m == "fusesim3") return mode_fusesim3(argv[2], argv[3]);
    if (m == "bysim3") return mode_bysim3(argv[2], argv[3]);
    if (m == "init") return mode_init(argv[2], argv[3]);
    if (m == "tri") return mode_tri(argv[2], argv[3]);
    if (m == "pose") return mode_pose(argv[2], argv[3]);
    if (m == "distinct") return mode_distinct(argv[2], argv[3]);
    if (m == "voc") return mode_voc(argv[2], argv[3]);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "exception: %s\n", e.what());
    return 3;
  }
  return 2;
}
