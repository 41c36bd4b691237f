// test_shim.cpp -- drives the C++ shim (shim/include/*.h, the reference class signatures) the way
// ORB-SLAM2 calls it.  Modes:
//   abi                 no GPU needed: layouts, cv::Mat semantics, DescriptorDistance, and that every
//                       GPU-backed constructor/call fails loudly (std::runtime_error) without a device
//   stereo  IN OUT      Frame stereo ctor (two extraction threads + ComputeStereoMatches)
//   bow     IN OUT      ORBmatcher::SearchByBoW(KeyFrame*, Frame&, ...) / (KeyFrame*, KeyFrame*, ...)
//   ba      IN OUT      Optimizer::LocalBundleAdjustment on an explicit problem
// IN/OUT are little-endian binary files written/read by tests/test_shim.py, which compares the
// outputs with the CPU oracle.  Exit status 0 = ok.
#include <cassert>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "ORBextractor.h"
#include "ORBmatcher.h"
#include "Objects.h"
#include "Optimizer.h"
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

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: test_shim abi | stereo IN OUT | bow IN OUT | ba IN OUT\n");
    return 2;
  }
  const std::string m = argv[1];
  try {
    if (m == "abi") return mode_abi();
    if (argc < 4) return 2;
    if (m == "stereo") return mode_stereo(argv[2], argv[3]);
    if (m == "bow") return mode_bow(argv[2], argv[3]);
    if (m == "ba") return mode_ba(argv[2], argv[3]);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "exception: %s\n", e.what());
    return 3;
  }
  return 2;
}
