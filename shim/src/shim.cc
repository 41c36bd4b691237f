// shim.cc -- the reference's hot-path classes (ORBextractor, Frame's ORB/stereo part, ORBmatcher's
// SearchByBoW / DescriptorDistance, Optimizer::LocalBundleAdjustment) as thin C++ over the C ABI of
// liborbx.so (include/orbx.h).  Argument meaning and error behaviour follow the reference; a
// library error (no device, bad geometry) throws std::runtime_error where the reference would
// assert or crash.  No computation happens here beyond marshalling.
#include <cstddef>
#include <cstdio>
#include <exception>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

#include "ORBextractor.h"
#include "ORBmatcher.h"
#include "Objects.h"
#include "Optimizer.h"
#include "orbx.h"

static_assert(sizeof(cv::KeyPoint) == sizeof(orbx_keypoint), "cv::KeyPoint layout");
static_assert(offsetof(cv::KeyPoint, octave) == offsetof(orbx_keypoint, octave), "cv::KeyPoint layout");
static_assert(offsetof(cv::KeyPoint, response) == offsetof(orbx_keypoint, response), "cv::KeyPoint layout");

namespace ORB_SLAM2 {

static void check(orbx_status s, const char* what) {
  if (s != ORBX_OK) throw std::runtime_error(std::string(what) + " failed: orbx_status " + std::to_string(s));
}

// rows of 32 bytes back to back (cv::Mat descriptors are continuous unless they are views)
static cv::Mat continuous(const cv::Mat& m) { return m.isContinuous() ? m : m.clone(); }

// ------------------------------------------------------------------ ORBextractor
ORBextractor::ORBextractor(int nfeatures_, float scaleFactor_, int nlevels_, int iniThFAST_, int minThFAST_,
                           int device)
    : nfeatures(nfeatures_), scaleFactor(scaleFactor_), nlevels(nlevels_), iniThFAST(iniThFAST_),
      minThFAST(minThFAST_) {
  orbx_extractor_params p{nfeatures, scaleFactor_, nlevels, iniThFAST, minThFAST};
  check(orbx_extractor_create(&p, device, &mpGpu), "orbx_extractor_create");
  mvScaleFactor.resize(nlevels);
  mvInvScaleFactor.resize(nlevels);
  mvLevelSigma2.resize(nlevels);
  mvInvLevelSigma2.resize(nlevels);
  check(orbx_extractor_scale_tables(mpGpu, mvScaleFactor.data(), mvInvScaleFactor.data(), mvLevelSigma2.data(),
                                    mvInvLevelSigma2.data()),
        "orbx_extractor_scale_tables");
  mvImagePyramid.resize(nlevels);
}

ORBextractor::~ORBextractor() {
  if (mpGpu) orbx_extractor_destroy(mpGpu);
}

void ORBextractor::operator()(cv::InputArray _image, cv::InputArray, std::vector<cv::KeyPoint>& _keypoints,
                              cv::OutputArray _descriptors) {
  if (_image.empty()) return;  // src/ORBextractor.cc:1141
  cv::Mat image = _image.getMat();
  if (image.type() != CV_8UC1) throw std::invalid_argument("ORBextractor: image must be CV_8UC1");  // :1145
  const int cap = orbx_extractor_max_keypoints(mpGpu, image.cols, image.rows);
  if (cap < 0) check(cap, "orbx_extractor_max_keypoints");
  _keypoints.resize(cap);
  cv::Mat desc(cap > 0 ? cap : 1, 32, CV_8U);
  int n = 0;
  check(orbx_extract(mpGpu, image.data, image.cols, image.rows, image.step,
                     reinterpret_cast<orbx_keypoint*>(_keypoints.data()), cap, desc.data, &n),
        "orbx_extract");
  _keypoints.resize(n);
  if (n == 0) {
    _descriptors.release();  // :1173
  } else {
    _descriptors.create(n, 32, CV_8U);
    cv::Mat& out = _descriptors.getMatRef();
    for (int i = 0; i < n; i++) std::memcpy(out.ptr<uint8_t>(i), desc.ptr<uint8_t>(i), 32);
  }
  if (mbDownloadPyramid) {
    for (int l = 0; l < nlevels; l++) {
      int w = 0, h = 0;
      check(orbx_pyramid_level(mpGpu, 0, l, nullptr, 0, &w, &h), "orbx_pyramid_level");
      mvImagePyramid[l].create(h, w, CV_8U);
      check(orbx_pyramid_level(mpGpu, 0, l, mvImagePyramid[l].data, mvImagePyramid[l].step, &w, &h),
            "orbx_pyramid_level");
    }
  }
}

// ------------------------------------------------------------------ Frame (stereo ORB part)
Frame::Frame(const cv::Mat& imLeft, const cv::Mat& imRight, ORBextractor* extractorLeft,
             ORBextractor* extractorRight, const cv::Mat& K, const cv::Mat& distCoef, float bf, float thDepth)
    : mpORBextractorLeft(extractorLeft), mpORBextractorRight(extractorRight), mbf(bf), mThDepth(thDepth) {
  mK = K.clone();
  mDistCoef = distCoef.clone();
  // two extraction threads, each on its own extractor handle / HIP stream (src/Frame.cc:80-84)
  std::exception_ptr errL, errR;
  std::thread threadLeft([&] {
    try { ExtractORB(0, imLeft); } catch (...) { errL = std::current_exception(); }
  });
  std::thread threadRight([&] {
    try { ExtractORB(1, imRight); } catch (...) { errR = std::current_exception(); }
  });
  threadLeft.join();
  threadRight.join();
  if (errL) std::rethrow_exception(errL);
  if (errR) std::rethrow_exception(errR);
  N = (int)mvKeys.size();
  if (mvKeys.empty()) return;
  mb = mbf / mK.at<float>(0, 0);  // :133-134
  UndistortKeyPoints();
  ComputeStereoMatches();
  mvpMapPoints.assign(N, nullptr);
  mvbOutlier.assign(N, false);
}

void Frame::ExtractORB(int flag, const cv::Mat& im) {
  if (flag == 0)
    (*mpORBextractorLeft)(im, cv::Mat(), mvKeys, mDescriptors);
  else
    (*mpORBextractorRight)(im, cv::Mat(), mvKeysRight, mDescriptorsRight);
}

void Frame::UndistortKeyPoints() {
  // src/Frame.cc:471-506: no distortion -> copy; otherwise cv::undistortPoints with P = K on the GPU
  if (mDistCoef.empty() || mDistCoef.at<float>(0, 0) == 0.0f) {
    mvKeysUn = mvKeys;
    return;
  }
  orbx_camera cam;
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) cam.K[3 * r + c] = mK.at<float>(r, c);
  const int nd = mDistCoef.rows * mDistCoef.cols;
  cam.n_dist = nd;
  for (int i = 0; i < 5; i++) cam.dist[i] = i < nd ? mDistCoef.ptr<float>(0)[i] : 0.f;
  mvKeysUn.resize(N);
  check(orbx_undistort_keypoints(reinterpret_cast<const orbx_keypoint*>(mvKeys.data()), N, &cam,
                                 reinterpret_cast<orbx_keypoint*>(mvKeysUn.data()), 0),
        "orbx_undistort_keypoints");
}

void Frame::ComputeStereoMatches() {
  ORB_SLAM2::ComputeStereoMatches(*mpORBextractorLeft, *mpORBextractorRight, mvKeys, mDescriptors, mvKeysRight,
                                  mDescriptorsRight, mbf, mb, mvuRight, mvDepth);
}

void ComputeStereoMatches(ORBextractor& left, ORBextractor& right, const std::vector<cv::KeyPoint>& kpsL,
                          const cv::Mat& descL, const std::vector<cv::KeyPoint>& kpsR, const cv::Mat& descR,
                          float mbf, float mb, std::vector<float>& mvuRight, std::vector<float>& mvDepth) {
  const int N = (int)kpsL.size();
  mvuRight.assign(N, -1.0f);  // src/Frame.cc:549-550
  mvDepth.assign(N, -1.0f);
  if (N == 0) return;
  const cv::Mat dL = continuous(descL), dR = continuous(descR);
  check(orbx_stereo_match(left.gpu(), right.gpu(), reinterpret_cast<const orbx_keypoint*>(kpsL.data()), dL.data, N,
                          reinterpret_cast<const orbx_keypoint*>(kpsR.data()), kpsR.empty() ? nullptr : dR.data,
                          (int)kpsR.size(), mbf, mb, mvuRight.data(), mvDepth.data()),
        "orbx_stereo_match");
}

// ------------------------------------------------------------------ ORBmatcher
const int ORBmatcher::TH_HIGH = 100;
const int ORBmatcher::TH_LOW = 50;
const int ORBmatcher::HISTO_LENGTH = 30;

ORBmatcher::ORBmatcher(float nnratio, bool checkOri, int device)
    : mfNNratio(nnratio), mbCheckOrientation(checkOri), mDevice(device) {}

int ORBmatcher::DescriptorDistance(const cv::Mat& a, const cv::Mat& b) {
  // src/ORBmatcher.cc:1844-1860: popcount of the 256-bit XOR (the bit-trick sum there is a popcount)
  const uint32_t* pa = a.ptr<uint32_t>();
  const uint32_t* pb = b.ptr<uint32_t>();
  int dist = 0;
  for (int i = 0; i < 8; i++) dist += __builtin_popcount(pa[i] ^ pb[i]);
  return dist;
}

namespace {
// One side of SearchByBoW with the FeatureVector flattened to CSR (ascending node ids = map order).
struct BowSide {
  std::vector<float> angle;
  std::vector<uint8_t> valid;
  std::vector<uint32_t> ids;
  std::vector<int32_t> off, feat;
  cv::Mat desc;
  orbx_bow_side side(int n, bool with_valid) const {
    return orbx_bow_side{n, n ? desc.data : nullptr, angle.data(), with_valid ? valid.data() : nullptr,
                         (int)ids.size(), ids.data(), off.data(), feat.data()};
  }
};

void fill_fv(BowSide& s, const DBoW2::FeatureVector& fv) {
  s.off.push_back(0);
  for (const auto& node : fv) {
    s.ids.push_back(node.first);
    for (unsigned int f : node.second) s.feat.push_back((int32_t)f);
    s.off.push_back((int32_t)s.feat.size());
  }
}

void fill_keyframe(BowSide& s, const KeyFrame* kf, const std::vector<MapPoint*>& mps) {
  const int n = (int)kf->mvKeysUn.size();
  for (int i = 0; i < n; i++) {
    s.angle.push_back(kf->mvKeysUn[i].angle);
    s.valid.push_back(i < (int)mps.size() && mps[i] && !mps[i]->isBad());
  }
  s.desc = continuous(kf->mDescriptors);
  fill_fv(s, kf->mFeatVec);
}
}  // namespace

int ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, std::vector<MapPoint*>& vpMapPointMatches) {
  const std::vector<MapPoint*> vpMapPointsKF = pKF->GetMapPointMatches();
  vpMapPointMatches.assign(F.N, nullptr);
  BowSide a, b;
  fill_keyframe(a, pKF, vpMapPointsKF);
  for (int i = 0; i < F.N; i++) b.angle.push_back(F.mvKeys[i].angle);  // rot uses F.mvKeys (:272)
  b.desc = continuous(F.mDescriptors);
  fill_fv(b, F.mFeatVec);
  const orbx_bow_side sa = a.side((int)pKF->mvKeysUn.size(), true), sb = b.side(F.N, false);
  std::vector<int32_t> match(F.N > 0 ? F.N : 1, -1);
  int n = 0;
  check(orbx_search_by_bow_kf_f(&sa, &sb, mfNNratio, mbCheckOrientation, match.data(), &n, mDevice),
        "orbx_search_by_bow_kf_f");
  for (int i = 0; i < F.N; i++)
    if (match[i] >= 0) vpMapPointMatches[i] = vpMapPointsKF[match[i]];
  return n;
}

int ORBmatcher::SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12) {
  const std::vector<MapPoint*> vpMapPoints1 = pKF1->GetMapPointMatches();
  const std::vector<MapPoint*> vpMapPoints2 = pKF2->GetMapPointMatches();
  const int n1 = (int)pKF1->mvKeysUn.size(), n2 = (int)pKF2->mvKeysUn.size();
  vpMatches12.assign(vpMapPoints1.size(), nullptr);  // :603
  BowSide a, b;
  fill_keyframe(a, pKF1, vpMapPoints1);
  fill_keyframe(b, pKF2, vpMapPoints2);
  const orbx_bow_side sa = a.side(n1, true), sb = b.side(n2, true);
  std::vector<int32_t> match(n1 > 0 ? n1 : 1, -1);
  int n = 0;
  check(orbx_search_by_bow_kf_kf(&sa, &sb, mfNNratio, mbCheckOrientation, match.data(), &n, mDevice),
        "orbx_search_by_bow_kf_kf");
  for (int i = 0; i < n1 && i < (int)vpMatches12.size(); i++)
    if (match[i] >= 0) vpMatches12[i] = vpMapPoints2[match[i]];
  return n;
}

// ------------------------------------------------------------------ Optimizer
void Optimizer::LocalBundleAdjustment(const LocalBAProblem& P, bool* pbStopFlag, LocalBAResult& R, int device) {
  const int nc = (int)P.cameras.size(), np = (int)P.points.size(), ne = (int)P.observations.size();
  std::vector<float> Tcw(12 * (size_t)nc), intr(5 * (size_t)nc), Xw(3 * (size_t)np), obs(3 * (size_t)ne),
      isig(ne);
  std::vector<uint8_t> fixed(nc);
  std::vector<int32_t> ep(ne), ec(ne);
  for (int c = 0; c < nc; c++) {
    const LocalBAProblem::Camera& C = P.cameras[c];
    for (int r = 0; r < 3; r++)
      for (int k = 0; k < 4; k++) Tcw[12 * c + 4 * r + k] = C.Tcw.at<float>(r, k);
    fixed[c] = C.fixed;
    const float in[5] = {C.fx, C.fy, C.cx, C.cy, C.bf};
    std::memcpy(&intr[5 * c], in, sizeof(in));
  }
  for (int p = 0; p < np; p++)
    for (int k = 0; k < 3; k++) Xw[3 * p + k] = P.points[p].at<float>(k, 0);
  for (int e = 0; e < ne; e++) {
    const LocalBAProblem::Observation& o = P.observations[e];
    ep[e] = o.point;
    ec[e] = o.camera;
    obs[3 * e] = o.u;
    obs[3 * e + 1] = o.v;
    obs[3 * e + 2] = o.ur;
    isig[e] = o.invSigma2;
  }
  orbx_ba_problem prob{nc, Tcw.data(), fixed.data(), intr.data(), np, Xw.data(),
                       ne, ep.data(), ec.data(), obs.data(), isig.data()};
  std::vector<float> Tout(12 * (size_t)nc), Xout(3 * (size_t)np);
  std::vector<uint8_t> erase(ne > 0 ? ne : 1);
  orbx_ba_result res;
  std::memset(&res, 0, sizeof(res));
  res.Tcw = Tout.data();
  res.Xw = Xout.data();
  res.edge_outlier = erase.data();
  // the LocalMapping thread keeps one solver (device buffers and stream reused across calls)
  static thread_local orbx_ba* ba = nullptr;
  static thread_local int ba_device = -1;
  if (ba && ba_device != device) {
    orbx_ba_destroy(ba);
    ba = nullptr;
  }
  if (!ba) {
    check(orbx_ba_create(device, &ba), "orbx_ba_create");
    ba_device = device;
  }
  check(orbx_ba_run_bool(ba, &prob, &res, pbStopFlag), "orbx_ba_run");
  R.Tcw.resize(nc);
  for (int c = 0; c < nc; c++) {
    cv::Mat T(4, 4, CV_32F);
    for (int r = 0; r < 3; r++)
      for (int k = 0; k < 4; k++) T.at<float>(r, k) = Tout[12 * c + 4 * r + k];
    T.at<float>(3, 0) = T.at<float>(3, 1) = T.at<float>(3, 2) = 0.f;
    T.at<float>(3, 3) = 1.f;
    R.Tcw[c] = T;
  }
  R.points.resize(np);
  for (int p = 0; p < np; p++) {
    cv::Mat X(3, 1, CV_32F);
    for (int k = 0; k < 3; k++) X.at<float>(k, 0) = Xout[3 * p + k];
    R.points[p] = X;
  }
  R.erase.assign(ne, false);
  for (int e = 0; e < ne; e++) R.erase[e] = erase[e] != 0;
  R.iterations[0] = res.iterations[0];
  R.iterations[1] = res.iterations[1];
  R.trials = res.trials;
}

}  // namespace ORB_SLAM2
