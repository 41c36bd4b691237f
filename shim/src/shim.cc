// shim.cc -- the reference's hot-path classes (ORBextractor, Frame's ORB/stereo part and ComputeBoW,
// ORBmatcher's SearchByBoW x2 / SearchByProjection x3 / SearchForTriangulation / Fuse /
// DescriptorDistance, PnPsolver, Optimizer::PoseOptimization / LocalBundleAdjustment,
// MapPoint::ComputeDistinctiveDescriptors, ORBVocabulary) as thin C++ over the C ABI of liborbx.so
// (include/orbx.h).  Argument meaning and error behaviour follow the
// reference; a library error (no device, bad geometry) throws std::runtime_error where the
// reference would assert or crash.  No computation happens here beyond marshalling: gathering the
// inputs from the object graph and applying the results to it, as the reference's own members do.
#include <cstddef>
#include <cstdio>
#include <exception>
#include <cstring>
#include <list>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>

#include <algorithm>
#include <cmath>
#include <fstream>
#include <iterator>
#include <set>
#include <sstream>

#include "ORBVocabulary.h"
#include "ORBextractor.h"
#include "ORBmatcher.h"
#include "Objects.h"
#include "Optimizer.h"
#include "PnPsolver.h"
#include "orbx.h"
#include "orbx_shim.h"

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
ORBextractor::ORBextractor(int nfeatures_, float scaleFactor_, int nlevels_, int iniThFAST_, int minThFAST_)
    : nfeatures(nfeatures_), scaleFactor(scaleFactor_), nlevels(nlevels_), iniThFAST(iniThFAST_),
      minThFAST(minThFAST_) {
  orbx_extractor_params p{nfeatures, scaleFactor_, nlevels, iniThFAST, minThFAST};
  check(orbx_extractor_create(&p, gOrbxDevice, &mpGpu), "orbx_extractor_create");
  mvScaleFactor.resize(nlevels);
  mvInvScaleFactor.resize(nlevels);
  mvLevelSigma2.resize(nlevels);
  mvInvLevelSigma2.resize(nlevels);
  check(orbx_extractor_scale_tables(mpGpu, mvScaleFactor.data(), mvInvScaleFactor.data(), mvLevelSigma2.data(),
                                    mvInvLevelSigma2.data()),
        "orbx_extractor_scale_tables");
  // the constructor's other tables (src/ORBextractor.cc:433-490): quotas, the IC_Angle circle, pattern
  mnFeaturesPerLevel.resize(nlevels);
  umax.resize(16);  // HALF_PATCH_SIZE + 1
  std::vector<int> pts(1024);
  check(orbx_extractor_tables(mpGpu, mnFeaturesPerLevel.data(), umax.data(), pts.data()), "orbx_extractor_tables");
  pattern.resize(512);
  for (int i = 0; i < 512; i++) pattern[i] = cv::Point(pts[2 * i], pts[2 * i + 1]);
  check(orbx_extractor_set_pyramid_readback(mpGpu, 1), "orbx_extractor_set_pyramid_readback");
  mvImagePyramid.resize(nlevels);
}

ORBextractor::~ORBextractor() {
  if (mpGpu) orbx_extractor_destroy(mpGpu);
}

void ORBextractor::operator()(cv::InputArray _image, cv::InputArray, std::vector<cv::KeyPoint>& _keypoints,
                              cv::OutputArray _descriptors) {
  Extract(_image, _keypoints, _descriptors, true);
}

void ORBextractor::ExtractForFrame(const cv::Mat& image, std::vector<cv::KeyPoint>& keypoints, cv::Mat& descriptors) {
  Extract(image, keypoints, descriptors, false);
}

void ORBextractor::Extract(cv::InputArray _image, std::vector<cv::KeyPoint>& _keypoints,
                           cv::OutputArray _descriptors, bool pyramid) {
  if (_image.empty()) return;  // src/ORBextractor.cc:1141
  cv::Mat image = _image.getMat();
  if (image.type() != CV_8UC1) throw std::invalid_argument("ORBextractor: image must be CV_8UC1");  // :1145
  const int cap = orbx_extractor_max_keypoints(mpGpu, image.cols, image.rows);
  if (cap < 0) check(cap, "orbx_extractor_max_keypoints");
  _keypoints.resize(cap);
  cv::Mat desc(cap > 0 ? cap : 1, 32, CV_8U);
  int n = 0;
  check(orbx_extractor_set_pyramid_readback(mpGpu, pyramid ? 1 : 0), "orbx_extractor_set_pyramid_readback");
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
  for (int l = 0; l < nlevels; l++) {
    if (!pyramid) {
      mvImagePyramid[l].release();
      continue;
    }
    // new Mats every call, as ComputePyramid assigns fresh ones (an older level a caller kept stays
    // intact); the copy comes from the pinned readback orbx_extract already waited for
    int w = 0, h = 0;
    check(orbx_pyramid_level(mpGpu, 0, l, nullptr, 0, &w, &h), "orbx_pyramid_level");
    cv::Mat m(h, w, CV_8U);
    check(orbx_pyramid_level(mpGpu, 0, l, m.data, m.step, &w, &h), "orbx_pyramid_level");
    mvImagePyramid[l] = m;
  }
}

// ------------------------------------------------------------------ Frame (stereo ORB part)
float Frame::fx = 0.f, Frame::fy = 0.f, Frame::cx = 0.f, Frame::cy = 0.f, Frame::invfx = 0.f, Frame::invfy = 0.f;

Frame::Frame(const cv::Mat& imLeft, const cv::Mat& imRight, ORBextractor* extractorLeft,
             ORBextractor* extractorRight, const cv::Mat& K, const cv::Mat& distCoef, float bf, float thDepth)
    : mpORBextractorLeft(extractorLeft), mpORBextractorRight(extractorRight), mbf(bf), mThDepth(thDepth) {
  mK = K.clone();
  mDistCoef = distCoef.clone();
  ORBextractor* eL = extractorLeft;
  ORBextractor* eR = extractorRight;
  // Tracking builds both extractors with the same parameters (src/Tracking.cc:113-126): then the two
  // ExtractORB calls and ComputeStereoMatches run as one library call on the left handle (both
  // images one batch, the matcher on the device right behind them, one copy back)
  if (gOrbxFrameStereoFused && eL && eR && eL != eR && eL->nfeatures == eR->nfeatures &&
      eL->scaleFactor == eR->scaleFactor && eL->nlevels == eR->nlevels && eL->iniThFAST == eR->iniThFAST && eL->minThFAST == eR->minThFAST &&
      !imLeft.empty() && !imRight.empty() && imLeft.type() == CV_8UC1 && imRight.type() == CV_8UC1 &&
      imLeft.rows == imRight.rows && imLeft.cols == imRight.cols && K.at<float>(0, 0) != 0.f) {
    const int cap = orbx_extractor_max_keypoints(eL->gpu(), imLeft.cols, imLeft.rows);
    if (cap < 0) check(cap, "orbx_extractor_max_keypoints");
    mvKeys.resize(cap);
    mvKeysRight.resize(cap);
    cv::Mat dL(cap > 0 ? cap : 1, 32, CV_8U), dR(cap > 0 ? cap : 1, 32, CV_8U);
    std::vector<float> uR(cap > 0 ? cap : 1), dep(cap > 0 ? cap : 1);
    int nL = 0, nR = 0;
    const float fx0 = K.at<float>(0, 0);
    check(orbx_frame_stereo(eL->gpu(), imLeft.data, imLeft.step, imRight.data, imRight.step, imLeft.cols,
                            imLeft.rows, bf, bf / fx0, reinterpret_cast<orbx_keypoint*>(mvKeys.data()), dL.data, cap,
                            &nL, reinterpret_cast<orbx_keypoint*>(mvKeysRight.data()), dR.data, cap, &nR, uR.data(),
                            dep.data()),
          "orbx_frame_stereo");
    mvKeys.resize(nL);
    mvKeysRight.resize(nR);
    // ExtractForFrame's outputs: exactly n descriptor rows (none for an empty side), no pyramid kept
    if (nL) {
      mDescriptors.create(nL, 32, CV_8U);
      std::memcpy(mDescriptors.data, dL.data, (size_t)32 * nL);
    }
    if (nR) {
      mDescriptorsRight.create(nR, 32, CV_8U);
      std::memcpy(mDescriptorsRight.data, dR.data, (size_t)32 * nR);
    }
    for (int l = 0; l < eL->nlevels; l++) {
      eL->mvImagePyramid[l].release();
      eR->mvImagePyramid[l].release();
    }
    finish_stereo_frame(&uR, &dep);
    return;
  }
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
  finish_stereo_frame(nullptr, nullptr);
}

// The rest of the stereo constructor after ExtractORB (src/Frame.cc:86-123); uR / dep: the stereo
// matches orbx_frame_stereo already computed (else ComputeStereoMatches runs here)
void Frame::finish_stereo_frame(const std::vector<float>* uR, const std::vector<float>* dep) {
  N = (int)mvKeys.size();
  // scale tables (src/Frame.cc:66-73) and the static intrinsics (:111-126)
  mnScaleLevels = mpORBextractorLeft->GetLevels();
  mfScaleFactor = mpORBextractorLeft->GetScaleFactor();
  mfLogScaleFactor = std::log(mfScaleFactor);
  mvScaleFactors = mpORBextractorLeft->GetScaleFactors();
  mvInvScaleFactors = mpORBextractorLeft->GetInverseScaleFactors();
  mvLevelSigma2 = mpORBextractorLeft->GetScaleSigmaSquares();
  mvInvLevelSigma2 = mpORBextractorLeft->GetInverseScaleSigmaSquares();
  fx = mK.at<float>(0, 0);
  fy = mK.at<float>(1, 1);
  cx = mK.at<float>(0, 2);
  cy = mK.at<float>(1, 2);
  invfx = 1.0f / fx;
  invfy = 1.0f / fy;
  if (mvKeys.empty()) return;
  mb = mbf / fx;  // :133-134
  UndistortKeyPoints();
  if (uR && dep) {  // ComputeStereoMatches' results (mvKeys, mvKeysRight, mb: the same inputs)
    mvuRight.assign(uR->begin(), uR->begin() + N);
    mvDepth.assign(dep->begin(), dep->begin() + N);
  } else {
    ComputeStereoMatches();
  }
  mvpMapPoints.assign(N, nullptr);
  mvbOutlier.assign(N, false);
}

long unsigned int Frame::nNextId = 0;
float Frame::mnMinX = 0.f, Frame::mnMaxX = 0.f, Frame::mnMinY = 0.f, Frame::mnMaxY = 0.f;
float Frame::mfGridElementWidthInv = 0.f, Frame::mfGridElementHeightInv = 0.f;
bool Frame::mbInitialComputations = true;
int gOrbxDevice = 0;
bool gOrbxFrameStereoFused = true;

Frame::Frame(const cv::Mat& imLeft, const cv::Mat& imRight, const double& timeStamp, ORBextractor* extractorLeft,
             ORBextractor* extractorRight, ORBVocabulary* voc, cv::Mat& K, cv::Mat& distCoef, const float& bf,
             const float& thDepth)
    : Frame(imLeft, imRight, extractorLeft, extractorRight, K, distCoef, bf, thDepth) {
  mnId = nNextId++;
  mTimeStamp = timeStamp;
  mpORBvocabulary = voc;
  if (mvKeys.empty()) return;  // src/Frame.cc:87-88
  // :100-120 on the first frame: image bounds and the grid's cell inverses (FRAME_GRID_COLS/ROWS)
  if (mbInitialComputations) {
    ComputeImageBounds(imLeft);
    mfGridElementWidthInv = static_cast<float>(ORBX_GRID_COLS) / (mnMaxX - mnMinX);
    mfGridElementHeightInv = static_cast<float>(ORBX_GRID_ROWS) / (mnMaxY - mnMinY);
    mbInitialComputations = false;
  }
  // AssignFeaturesToGrid (:131): the matchers build the 64x48 grid on the device per call
}

void Frame::ComputeImageBounds(const cv::Mat& imLeft) {
  // src/Frame.cc:508-537: the undistorted image corners (cv::undistortPoints with P = K on the GPU)
  if (!mDistCoef.empty() && mDistCoef.at<float>(0, 0) != 0.0f) {
    const float cols = (float)imLeft.cols, rows = (float)imLeft.rows;
    std::vector<cv::KeyPoint> corners = {cv::KeyPoint(0.f, 0.f, 1.f), cv::KeyPoint(cols, 0.f, 1.f),
                                         cv::KeyPoint(0.f, rows, 1.f), cv::KeyPoint(cols, rows, 1.f)};
    std::vector<cv::KeyPoint> un(4);
    orbx_camera cam;
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) cam.K[3 * r + c] = mK.at<float>(r, c);
    const int nd = mDistCoef.rows * mDistCoef.cols;
    cam.n_dist = nd;
    for (int i = 0; i < 5; i++) cam.dist[i] = i < nd ? mDistCoef.ptr<float>(0)[i] : 0.f;
    check(orbx_undistort_keypoints(reinterpret_cast<const orbx_keypoint*>(corners.data()), 4, &cam,
                                   reinterpret_cast<orbx_keypoint*>(un.data()), gOrbxDevice),
          "orbx_undistort_keypoints");
    mnMinX = std::min(un[0].pt.x, un[2].pt.x);
    mnMaxX = std::max(un[1].pt.x, un[3].pt.x);
    mnMinY = std::min(un[0].pt.y, un[1].pt.y);
    mnMaxY = std::max(un[2].pt.y, un[3].pt.y);
  } else {
    mnMinX = 0.0f;
    mnMaxX = (float)imLeft.cols;
    mnMinY = 0.0f;
    mnMaxY = (float)imLeft.rows;
  }
}

void Frame::SetPose(const cv::Mat& Tcw) {  // src/Frame.cc:287-291
  mTcw = Tcw.clone();
  UpdatePoseMatrices();
}

void Frame::UpdatePoseMatrices() {  // src/Frame.cc:294-304
  mRcw.create(3, 3, CV_32F);
  mRwc.create(3, 3, CV_32F);
  mtcw.create(3, 1, CV_32F);
  mOw.create(3, 1, CV_32F);
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) {
      mRcw.at<float>(r, c) = mTcw.at<float>(r, c);
      mRwc.at<float>(c, r) = mTcw.at<float>(r, c);
    }
    mtcw.at<float>(r, 0) = mTcw.at<float>(r, 3);
  }
  // mOw = -mRcw.t()*mtcw: one float gemm with alpha = -1, accumulated in double, rounded once
  for (int r = 0; r < 3; r++) {
    double acc = 0.0;
    for (int k = 0; k < 3; k++) acc += (double)mRcw.at<float>(k, r) * (double)mtcw.at<float>(k, 0);
    mOw.at<float>(r, 0) = (float)(-acc);
  }
}

void Frame::ComputeBoW() {  // src/Frame.cc:462-469
  if (mBowVec.empty()) {
    if (!mpORBvocabulary) throw std::runtime_error("Frame::ComputeBoW: no vocabulary");
    mpORBvocabulary->transform(mDescriptors, mBowVec, mFeatVec, 4);
  }
}

void KeyFrame::ComputeBoW() {  // src/KeyFrame.cc:65-80
  if (mBowVec.empty() || mFeatVec.empty()) {
    if (!mpORBvocabulary) throw std::runtime_error("KeyFrame::ComputeBoW: no vocabulary");
    mpORBvocabulary->transform(mDescriptors, mBowVec, mFeatVec, 4);
  }
}

void Frame::ExtractORB(int flag, const cv::Mat& im) {
  if (flag == 0)
    mpORBextractorLeft->ExtractForFrame(im, mvKeys, mDescriptors);
  else
    mpORBextractorRight->ExtractForFrame(im, mvKeysRight, mDescriptorsRight);
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
                                 reinterpret_cast<orbx_keypoint*>(mvKeysUn.data()), gOrbxDevice),
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

ORBmatcher::ORBmatcher(float nnratio, bool checkOri) : mfNNratio(nnratio), mbCheckOrientation(checkOri) {}

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
  check(orbx_search_by_bow_kf_f(&sa, &sb, mfNNratio, mbCheckOrientation, match.data(), &n, gOrbxDevice),
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
  check(orbx_search_by_bow_kf_kf(&sa, &sb, mfNNratio, mbCheckOrientation, match.data(), &n, gOrbxDevice),
        "orbx_search_by_bow_kf_kf");
  for (int i = 0; i < n1 && i < (int)vpMatches12.size(); i++)
    if (match[i] >= 0) vpMatches12[i] = vpMapPoints2[match[i]];
  return n;
}

// ------------------------------------------------------------------ SearchByProjection / Fuse
namespace {
// mvpMapPoints on entry, as the kernel reads it: 0 NULL, 1 a MapPoint with Observations() == 0,
// 2 a MapPoint with Observations() > 0 (the reference's "F.mvpMapPoints[idx]->Observations() > 0")
int8_t occupancy(MapPoint* p) { return !p ? 0 : (p->Observations() > 0 ? 2 : 1); }

void copy_desc(MapPoint* p, uint8_t* dst) {
  const cv::Mat d = p->GetDescriptor();
  if (d.empty())
    std::memset(dst, 0, 32);
  else
    std::memcpy(dst, d.ptr<uint8_t>(0), 32);
}

void copy_pos(MapPoint* p, float* dst) {
  const cv::Mat X = p->GetWorldPos();
  for (int k = 0; k < 3; k++) dst[k] = X.at<float>(k, 0);
}

void copy_dist(MapPoint* p, float* dst) {  // mfMinDistance, mfMaxDistance (the kernel applies 0.8 / 1.2)
  std::unique_lock<std::mutex> lock(p->mMutexPos);
  dst[0] = p->mfMinDistance;
  dst[1] = p->mfMaxDistance;
}

void copy_mat44(const cv::Mat& T, float* dst) {
  for (int i = 0; i < 16; i++) dst[i] = (i < 12 || T.rows == 4) ? T.at<float>(i / 4, i % 4) : (i == 15 ? 1.f : 0.f);
}

void set_levels(orbx_proj_frame& f, int nlevels, const std::vector<float>& sf, const std::vector<float>& isig) {
  if (nlevels < 1 || nlevels > 16 || (int)sf.size() < nlevels) throw std::invalid_argument("orbx shim: nlevels");
  f.nlevels = nlevels;
  for (int l = 0; l < 16; l++) {
    f.scale_factors[l] = l < nlevels ? sf[l] : 0.f;
    f.inv_level_sigma2[l] = l < nlevels && l < (int)isig.size() ? isig[l] : 0.f;
  }
}

// The current Frame as orbx_proj_frame (pointers into F and into the caller's occ / desc buffers)
orbx_proj_frame proj_frame(Frame& F, std::vector<int8_t>& occ, cv::Mat& desc) {
  orbx_proj_frame f;
  std::memset(&f, 0, sizeof(f));
  f.n = F.N;
  occ.resize(F.N > 0 ? F.N : 1);
  for (int i = 0; i < F.N; i++) occ[i] = occupancy(F.mvpMapPoints[i]);
  desc = continuous(F.mDescriptors);
  f.keys_un = reinterpret_cast<const orbx_keypoint*>(F.mvKeysUn.data());
  f.desc = F.N > 0 ? desc.data : nullptr;
  f.u_right = F.mvuRight.empty() ? nullptr : F.mvuRight.data();
  f.occ = occ.data();
  f.min_x = Frame::mnMinX;
  f.max_x = Frame::mnMaxX;
  f.min_y = Frame::mnMinY;
  f.max_y = Frame::mnMaxY;
  f.grid_inv_w = Frame::mfGridElementWidthInv;
  f.grid_inv_h = Frame::mfGridElementHeightInv;
  set_levels(f, F.mnScaleLevels, F.mvScaleFactors, F.mvInvLevelSigma2);
  f.log_scale_factor = F.mfLogScaleFactor;
  f.fx = Frame::fx;
  f.fy = Frame::fy;
  f.cx = Frame::cx;
  f.cy = Frame::cy;
  f.bf = F.mbf;
  f.b = F.mb;
  copy_mat44(F.mTcw, f.Tcw);
  return f;
}

// The projected MapPoints of one call, SoA
struct ProjPoints {
  std::vector<uint8_t> desc, flags;
  std::vector<float> pos, normal, dist, angle, track;
  std::vector<int32_t> octave, level, point_match;
  explicit ProjPoints(size_t n)
      : desc(32 * std::max<size_t>(n, 1), 0), flags(std::max<size_t>(n, 1), 0), pos(3 * std::max<size_t>(n, 1), 0.f),
        normal(3 * std::max<size_t>(n, 1), 0.f), dist(2 * std::max<size_t>(n, 1), 0.f),
        angle(std::max<size_t>(n, 1), 0.f), track(4 * std::max<size_t>(n, 1), 0.f),
        octave(std::max<size_t>(n, 1), 0), level(std::max<size_t>(n, 1), 0), point_match(std::max<size_t>(n, 1), -1) {}
  void fill(orbx_proj_problem& p, int n) {
    p.n_points = n;
    p.desc = desc.data();
    p.flags = flags.data();
    p.pos = pos.data();
    p.normal = normal.data();
    p.dist_minmax = dist.data();
    p.angle = angle.data();
    p.octave = octave.data();
    p.track = track.data();
    p.track_level = level.data();
    p.point_match = point_match.data();
  }
};

orbx_proj_problem proj_problem(int kind, float th, const ORBmatcher& m) {
  orbx_proj_problem p;
  std::memset(&p, 0, sizeof(p));
  p.kind = kind;
  p.th = th;
  p.view_cos_limit = 0.5f;
  (void)m;
  return p;
}

// frame_out -> the Frame's mvpMapPoints, as the reference's assignments leave them
void apply_frame_out(Frame& F, const std::vector<int32_t>& frame_out, const std::vector<MapPoint*>& pts) {
  for (int i = 0; i < F.N; i++) {
    const int k = frame_out[i];
    if (k >= 0)
      F.mvpMapPoints[i] = pts[k];
    else if (k == -2)
      F.mvpMapPoints[i] = nullptr;
  }
}
}  // namespace

int ORBmatcher::SearchByProjection(Frame& F, const std::vector<MapPoint*>& vpMapPoints, const float th) {
  // src/ORBmatcher.cc:46-142.  The MapPoints carry Tracking::SearchLocalPoints' frustum results
  // (mbTrackInView, mTrackProjX/Y/XR, mnTrackScaleLevel, mTrackViewCos).
  const int n = (int)vpMapPoints.size();
  std::vector<int8_t> occ;
  cv::Mat desc;
  orbx_proj_problem p = proj_problem(ORBX_PROJ_LOCAL, th, *this);
  p.f = proj_frame(F, occ, desc);
  ProjPoints P(n);
  for (int k = 0; k < n; k++) {
    MapPoint* pMP = vpMapPoints[k];
    if (!pMP) continue;
    const bool take = pMP->mbTrackInView && !pMP->isBad();
    P.flags[k] = (uint8_t)((take ? 1 : 0) | (pMP->Observations() > 0 ? 2 : 0));
    if (!take) continue;
    copy_desc(pMP, &P.desc[32 * (size_t)k]);
    P.track[4 * k] = pMP->mTrackProjX;
    P.track[4 * k + 1] = pMP->mTrackProjY;
    P.track[4 * k + 2] = pMP->mTrackProjXR;
    P.track[4 * k + 3] = pMP->mTrackViewCos;
    P.level[k] = pMP->mnTrackScaleLevel;
  }
  P.fill(p, n);
  p.frustum = 0;
  p.nnratio = mfNNratio;
  p.check_ori = mbCheckOrientation;
  std::vector<int32_t> frame_out(F.N > 0 ? F.N : 1, -1);
  int32_t nm = 0;
  p.frame_out = frame_out.data();
  p.nmatches = &nm;
  check(orbx_search_by_projection(&p, gOrbxDevice), "orbx_search_by_projection");
  apply_frame_out(F, frame_out, vpMapPoints);
  return nm;
}

int ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, const float th, const bool bMono) {
  // src/ORBmatcher.cc:1489-1646: the last frame's non-outlier MapPoints
  const int n = LastFrame.N;
  std::vector<int8_t> occ;
  cv::Mat desc;
  orbx_proj_problem p = proj_problem(ORBX_PROJ_LAST_FRAME, th, *this);
  p.f = proj_frame(CurrentFrame, occ, desc);
  ProjPoints P(n);
  for (int i = 0; i < n; i++) {
    MapPoint* pMP = LastFrame.mvpMapPoints[i];
    if (!pMP) continue;
    const bool take = !LastFrame.mvbOutlier[i];
    P.flags[i] = (uint8_t)((take ? 1 : 0) | (pMP->Observations() > 0 ? 2 : 0));
    if (!take) continue;
    copy_desc(pMP, &P.desc[32 * (size_t)i]);
    copy_pos(pMP, &P.pos[3 * (size_t)i]);
    P.angle[i] = LastFrame.mvKeysUn[i].angle;
    P.octave[i] = LastFrame.mvKeys[i].octave;
  }
  P.fill(p, n);
  p.check_ori = mbCheckOrientation;
  p.mono = bMono;
  copy_mat44(LastFrame.mTcw, p.last_Tcw);
  std::vector<int32_t> frame_out(CurrentFrame.N > 0 ? CurrentFrame.N : 1, -1);
  int32_t nm = 0;
  p.frame_out = frame_out.data();
  p.nmatches = &nm;
  check(orbx_search_by_projection(&p, gOrbxDevice), "orbx_search_by_projection");
  apply_frame_out(CurrentFrame, frame_out, LastFrame.mvpMapPoints);
  return nm;
}

int ORBmatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const std::set<MapPoint*>& sAlreadyFound,
                                   const float th, const int ORBdist) {
  // src/ORBmatcher.cc:1648-1795: the KeyFrame's MapPoints not found yet
  const std::vector<MapPoint*> vpMPs = pKF->GetMapPointMatches();
  const int n = (int)vpMPs.size();
  std::vector<int8_t> occ;
  cv::Mat desc;
  orbx_proj_problem p = proj_problem(ORBX_PROJ_KEYFRAME, th, *this);
  p.f = proj_frame(CurrentFrame, occ, desc);
  ProjPoints P(n);
  for (int i = 0; i < n; i++) {
    MapPoint* pMP = vpMPs[i];
    if (!pMP) continue;
    const bool take = !pMP->isBad() && !sAlreadyFound.count(pMP);
    P.flags[i] = (uint8_t)((take ? 1 : 0) | (pMP->Observations() > 0 ? 2 : 0));
    if (!take) continue;
    copy_desc(pMP, &P.desc[32 * (size_t)i]);
    copy_pos(pMP, &P.pos[3 * (size_t)i]);
    copy_dist(pMP, &P.dist[2 * (size_t)i]);
    P.angle[i] = pKF->mvKeysUn[i].angle;
  }
  P.fill(p, n);
  p.check_ori = mbCheckOrientation;
  p.orb_dist = ORBdist;
  std::vector<int32_t> frame_out(CurrentFrame.N > 0 ? CurrentFrame.N : 1, -1);
  int32_t nm = 0;
  p.frame_out = frame_out.data();
  p.nmatches = &nm;
  check(orbx_search_by_projection(&p, gOrbxDevice), "orbx_search_by_projection");
  apply_frame_out(CurrentFrame, frame_out, vpMPs);
  return nm;
}

namespace {
// pKF as the frame of a Fuse problem: its keypoints, descriptors, mvuRight, its own (integer) image
// bounds and grid, scale tables and pose (src/ORBmatcher.cc:918-1054 reads exactly these)
orbx_proj_frame fuse_frame(KeyFrame* pKF, cv::Mat& desc) {
  orbx_proj_frame f;
  std::memset(&f, 0, sizeof(f));
  f.n = pKF->N;
  desc = continuous(pKF->mDescriptors);
  f.keys_un = reinterpret_cast<const orbx_keypoint*>(pKF->mvKeysUn.data());
  f.desc = pKF->N > 0 ? desc.data : nullptr;
  f.u_right = pKF->mvuRight.empty() ? nullptr : pKF->mvuRight.data();
  f.occ = nullptr;
  f.min_x = (float)pKF->mnMinX;
  f.max_x = (float)pKF->mnMaxX;
  f.min_y = (float)pKF->mnMinY;
  f.max_y = (float)pKF->mnMaxY;
  f.grid_inv_w = pKF->mfGridElementWidthInv;
  f.grid_inv_h = pKF->mfGridElementHeightInv;
  // mGrid came from the Frame (KeyFrame.cc constructor), built with the float Frame::mnMinX/mnMinY;
  // the KeyFrame's own (integer) copies above give GetFeaturesInArea's cell range and IsInImage
  f.grid_min_x = Frame::mnMinX;
  f.grid_min_y = Frame::mnMinY;
  f.grid_min_set = 1;
  set_levels(f, pKF->mnScaleLevels, pKF->mvScaleFactors, pKF->mvInvLevelSigma2);
  f.log_scale_factor = pKF->mfLogScaleFactor;
  f.fx = pKF->fx;
  f.fy = pKF->fy;
  f.cx = pKF->cx;
  f.cy = pKF->cy;
  f.bf = pKF->mbf;
  f.b = pKF->mb;
  copy_mat44(pKF->GetPose(), f.Tcw);
  return f;
}

// The matching half of Fuse for the points `which` (indices into vpMapPoints) in their current state:
// best[k] = pKF feature for which[k], or -1
void fuse_match(KeyFrame* pKF, const std::vector<MapPoint*>& vpMapPoints, const std::vector<int>& which, float th,
                int device, std::vector<int32_t>& best) {
  const int n = (int)which.size();
  cv::Mat desc;
  orbx_proj_problem p;
  std::memset(&p, 0, sizeof(p));
  p.kind = ORBX_PROJ_FUSE;
  p.th = th;
  p.f = fuse_frame(pKF, desc);
  ProjPoints P(n);
  for (int k = 0; k < n; k++) {
    MapPoint* pMP = vpMapPoints[which[k]];
    if (!pMP) continue;
    const bool take = !pMP->isBad() && !pMP->IsInKeyFrame(pKF);
    P.flags[k] = (uint8_t)((take ? 1 : 0) | (pMP->Observations() > 0 ? 2 : 0));
    if (!take) continue;
    copy_desc(pMP, &P.desc[32 * (size_t)k]);
    copy_pos(pMP, &P.pos[3 * (size_t)k]);
    const cv::Mat nrm = pMP->GetNormal();
    for (int c = 0; c < 3; c++) P.normal[3 * (size_t)k + c] = nrm.empty() ? 0.f : nrm.at<float>(c, 0);
    copy_dist(pMP, &P.dist[2 * (size_t)k]);
  }
  P.fill(p, n);
  std::vector<int32_t> frame_out(pKF->N > 0 ? pKF->N : 1, -1);
  int32_t nm = 0;
  p.frame_out = frame_out.data();
  p.nmatches = &nm;
  check(orbx_search_by_projection(&p, device), "orbx_search_by_projection (Fuse)");
  best.assign(P.point_match.begin(), P.point_match.begin() + n);
}
}  // namespace

int ORBmatcher::Fuse(KeyFrame* pKF, const std::vector<MapPoint*>& vpMapPoints, const float th) {
  // src/ORBmatcher.cc:918-1092.  Point i's match depends only on point i and pKF's keypoints, so all
  // points are matched in one launch on their entry state; the Replace / AddObservation block then
  // runs here in point order, as the reference's loop does.  A later point whose own state an
  // earlier Replace changed (it received observations and a new descriptor, or became bad) is
  // matched again in its current state before it is applied.
  const int n = (int)vpMapPoints.size();
  std::vector<int> all(n);
  for (int i = 0; i < n; i++) all[i] = i;
  std::vector<int32_t> best;
  fuse_match(pKF, vpMapPoints, all, th, gOrbxDevice, best);
  std::set<MapPoint*> touched;  // MapPoints an earlier Replace modified
  int nFused = 0;
  for (int i = 0; i < n; i++) {
    MapPoint* pMP = vpMapPoints[i];
    if (!pMP) continue;
    int bestIdx = best[i];
    if (touched.count(pMP)) {
      std::vector<int32_t> b1;
      fuse_match(pKF, vpMapPoints, std::vector<int>{i}, th, gOrbxDevice, b1);
      bestIdx = b1[0];
    }
    if (bestIdx < 0) continue;
    if (pMP->isBad() || pMP->IsInKeyFrame(pKF)) continue;  // the reference's check, at this point's turn
    MapPoint* pMPinKF = pKF->GetMapPoint(bestIdx);
    if (pMPinKF) {
      if (!pMPinKF->isBad()) {
        if (pMPinKF->Observations() > pMP->Observations()) {
          pMP->Replace(pMPinKF);
          touched.insert(pMPinKF);
        } else {
          pMPinKF->Replace(pMP);
          touched.insert(pMP);
        }
        touched.insert(pMP);
        touched.insert(pMPinKF);
      }
    } else {
      pMP->AddObservation(pKF, bestIdx);
      pKF->AddMapPoint(pMP, bestIdx);
      touched.insert(pMP);
    }
    nFused++;
  }
  return nFused;
}

int ORBmatcher::SearchByProjection(KeyFrame* pKF, cv::Mat Scw, const std::vector<MapPoint*>& vpPoints,
                                   std::vector<MapPoint*>& vpMatched, int th) {
  // src/ORBmatcher.cc:327-440 (caller LoopClosing::ComputeSim3, src/LoopClosing.cc:504): one
  // ORBX_PROJ_SIM3 problem; vpMatched on entry blocks its features (occ) and its MapPoints
  // (spAlreadyFound), the kernel's sweeps reproduce the in-order "vpMatched[idx]" skips
  const int n = (int)vpPoints.size();
  cv::Mat desc;
  orbx_proj_problem p;
  std::memset(&p, 0, sizeof(p));
  p.kind = ORBX_PROJ_SIM3;
  p.th = (float)th;
  p.f = fuse_frame(pKF, desc);
  copy_mat44(Scw, p.f.Tcw);
  std::vector<int8_t> occ(pKF->N > 0 ? pKF->N : 1, 0);
  std::set<MapPoint*> found;
  for (int i = 0; i < pKF->N && i < (int)vpMatched.size(); i++)
    if (vpMatched[i]) {
      occ[i] = 1;
      found.insert(vpMatched[i]);
    }
  p.f.occ = occ.data();
  ProjPoints P(n);
  for (int k = 0; k < n; k++) {
    MapPoint* pMP = vpPoints[k];
    if (!pMP || pMP->isBad() || found.count(pMP)) continue;
    P.flags[k] = 1;
    copy_desc(pMP, &P.desc[32 * (size_t)k]);
    copy_pos(pMP, &P.pos[3 * (size_t)k]);
    const cv::Mat nrm = pMP->GetNormal();
    for (int c = 0; c < 3; c++) P.normal[3 * (size_t)k + c] = nrm.empty() ? 0.f : nrm.at<float>(c, 0);
    copy_dist(pMP, &P.dist[2 * (size_t)k]);
  }
  P.fill(p, n);
  std::vector<int32_t> frame_out(pKF->N > 0 ? pKF->N : 1, -1);
  int32_t nm = 0;
  p.frame_out = frame_out.data();
  p.nmatches = &nm;
  check(orbx_search_by_projection(&p, gOrbxDevice), "orbx_search_by_projection (Sim3)");
  for (int i = 0; i < pKF->N && i < (int)vpMatched.size(); i++)
    if (frame_out[i] >= 0) vpMatched[i] = vpPoints[frame_out[i]];
  return nm;
}

int ORBmatcher::SearchForInitialization(Frame& F1, Frame& F2, std::vector<cv::Point2f>& vbPrevMatched,
                                        std::vector<int>& vnMatches12, int windowSize) {
  // src/ORBmatcher.cc:442-587 (caller Tracking::MonocularInitialization, src/Tracking.cc:711)
  std::vector<int8_t> occ1, occ2;
  cv::Mat d1, d2;
  orbx_init_problem p;
  std::memset(&p, 0, sizeof(p));
  p.f1 = proj_frame(F1, occ1, d1);
  p.f2 = proj_frame(F2, occ2, d2);
  const int n1 = F1.N;
  std::vector<float> prev(2 * (size_t)(n1 > 0 ? n1 : 1), 0.f);
  for (int i = 0; i < n1 && i < (int)vbPrevMatched.size(); i++) {
    prev[2 * i] = vbPrevMatched[i].x;
    prev[2 * i + 1] = vbPrevMatched[i].y;
  }
  std::vector<int32_t> m(n1 > 0 ? n1 : 1, -1);
  int32_t nm = 0;
  p.prev_matched = prev.data();
  p.window = windowSize;
  p.nnratio = mfNNratio;
  p.check_ori = mbCheckOrientation ? 1 : 0;
  p.match12 = m.data();
  p.nmatches = &nm;
  check(orbx_search_for_initialization(&p, gOrbxDevice), "orbx_search_for_initialization");
  vnMatches12.assign(m.begin(), m.begin() + n1);
  for (int i = 0; i < n1 && i < (int)vbPrevMatched.size(); i++)
    if (m[i] >= 0) vbPrevMatched[i] = cv::Point2f(prev[2 * i], prev[2 * i + 1]);
  return nm;
}

int ORBmatcher::SearchBySim3(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12, const float& s12,
                             const cv::Mat& R12, const cv::Mat& t12, const float th) {
  // src/ORBmatcher.cc:1238-1487 (caller LoopClosing::ComputeSim3, src/LoopClosing.cc:422): both
  // directions on the GPU (orbx_search_by_sim3), vbAlreadyMatched1/2 from vpMatches12 here (:1262-1273)
  const std::vector<MapPoint*> vp1 = pKF1->GetMapPointMatches(), vp2 = pKF2->GetMapPointMatches();
  const int N1 = (int)vp1.size(), N2 = (int)vp2.size();
  std::vector<char> am1(N1, 0), am2(N2, 0);
  for (int i = 0; i < N1 && i < (int)vpMatches12.size(); i++) {
    MapPoint* pMP = vpMatches12[i];
    if (!pMP) continue;
    am1[i] = 1;
    const int idx2 = pMP->GetIndexInKeyFrame(pKF2);
    if (idx2 >= 0 && idx2 < N2) am2[idx2] = 1;
  }
  orbx_sim3_problem p;
  std::memset(&p, 0, sizeof(p));
  cv::Mat d1, d2;
  p.kf1 = fuse_frame(pKF1, d1);
  p.kf2 = fuse_frame(pKF2, d2);
  ProjPoints P1(N1), P2(N2);
  auto side = [](const std::vector<MapPoint*>& vp, const std::vector<char>& am, ProjPoints& P) {
    for (size_t i = 0; i < vp.size(); i++) {
      MapPoint* pMP = vp[i];
      if (!pMP || am[i] || pMP->isBad()) continue;
      P.flags[i] = 1;
      copy_desc(pMP, &P.desc[32 * i]);
      copy_pos(pMP, &P.pos[3 * i]);
      copy_dist(pMP, &P.dist[2 * i]);
    }
  };
  side(vp1, am1, P1);
  side(vp2, am2, P2);
  p.desc1 = P1.desc.data();
  p.pos1 = P1.pos.data();
  p.dist_minmax1 = P1.dist.data();
  p.flags1 = P1.flags.data();
  p.desc2 = P2.desc.data();
  p.pos2 = P2.pos.data();
  p.dist_minmax2 = P2.dist.data();
  p.flags2 = P2.flags.data();
  p.s12 = s12;
  for (int i = 0; i < 9; i++) p.R12[i] = R12.at<float>(i / 3, i % 3);
  for (int i = 0; i < 3; i++) p.t12[i] = t12.at<float>(i, 0);
  p.th = th;
  std::vector<int32_t> m12(N1 > 0 ? N1 : 1, -1);
  int32_t nf = 0;
  p.match12 = m12.data();
  p.nfound = &nf;
  check(orbx_search_by_sim3(&p, gOrbxDevice), "orbx_search_by_sim3");
  for (int i1 = 0; i1 < N1 && i1 < (int)vpMatches12.size(); i1++)
    if (m12[i1] >= 0) vpMatches12[i1] = vp2[m12[i1]];
  return nf;
}

std::set<MapPoint*> KeyFrame::GetMapPoints() {
  std::unique_lock<std::mutex> lock(mMutexFeatures);
  std::set<MapPoint*> s;
  for (MapPoint* pMP : mvpMapPoints)
    if (pMP && !pMP->isBad()) s.insert(pMP);
  return s;
}

int ORBmatcher::Fuse(KeyFrame* pKF, cv::Mat Scw, const std::vector<MapPoint*>& vpPoints, float th,
                     std::vector<MapPoint*>& vpReplacePoint) {
  // src/ORBmatcher.cc:1094-1236 (caller LoopClosing::SearchAndFuse, src/LoopClosing.cc:837).  The
  // candidate loop reads no state the loop writes, so every point is matched in one launch
  // (ORBX_PROJ_FUSE_SIM3); the replace / AddMapPoint block then runs here in point order.
  const std::set<MapPoint*> found = pKF->GetMapPoints();
  const int n = (int)vpPoints.size();
  cv::Mat desc;
  orbx_proj_problem p;
  std::memset(&p, 0, sizeof(p));
  p.kind = ORBX_PROJ_FUSE_SIM3;
  p.th = th;
  p.f = fuse_frame(pKF, desc);
  copy_mat44(Scw, p.f.Tcw);
  ProjPoints P(n);
  for (int k = 0; k < n; k++) {
    MapPoint* pMP = vpPoints[k];
    if (!pMP || pMP->isBad() || found.count(pMP)) continue;
    P.flags[k] = 1;
    copy_desc(pMP, &P.desc[32 * (size_t)k]);
    copy_pos(pMP, &P.pos[3 * (size_t)k]);
    const cv::Mat nrm = pMP->GetNormal();
    for (int c = 0; c < 3; c++) P.normal[3 * (size_t)k + c] = nrm.empty() ? 0.f : nrm.at<float>(c, 0);
    copy_dist(pMP, &P.dist[2 * (size_t)k]);
  }
  P.fill(p, n);
  std::vector<int32_t> frame_out(pKF->N > 0 ? pKF->N : 1, -1);
  int32_t nm = 0;
  p.frame_out = frame_out.data();
  p.nmatches = &nm;
  check(orbx_search_by_projection(&p, gOrbxDevice), "orbx_search_by_projection (Fuse Sim3)");
  int nFused = 0;
  for (int i = 0; i < n; i++) {
    const int bestIdx = P.point_match[i];
    if (bestIdx < 0) continue;
    MapPoint* pMP = vpPoints[i];
    MapPoint* pMPinKF = pKF->GetMapPoint(bestIdx);
    if (pMPinKF) {
      if (!pMPinKF->isBad() && i < (int)vpReplacePoint.size()) vpReplacePoint[i] = pMPinKF;
    } else {
      pMP->AddObservation(pKF, bestIdx);
      pKF->AddMapPoint(pMP, bestIdx);
    }
    nFused++;
  }
  return nFused;
}

int ORBmatcher::SearchForTriangulation(KeyFrame* pKF1, KeyFrame* pKF2, cv::Mat F12,
                                       std::vector<std::pair<size_t, size_t>>& vMatchedPairs, const bool bOnlyStereo) {
  // src/ORBmatcher.cc:738-925 (caller LocalMapping::CreateNewMapPoints, src/LocalMapping.cc:363)
  struct Side {
    std::vector<uint8_t> has_mp;
    std::vector<uint32_t> ids;
    std::vector<int32_t> off, feat;
    cv::Mat desc;
    orbx_tri_kf kf(KeyFrame* K) {
      const int n = K->N;
      has_mp.assign(n > 0 ? n : 1, 0);
      for (int i = 0; i < n; i++) has_mp[i] = K->GetMapPoint(i) != nullptr;
      off.push_back(0);
      for (const auto& node : K->mFeatVec) {
        ids.push_back(node.first);
        for (unsigned int f : node.second) feat.push_back((int32_t)f);
        off.push_back((int32_t)feat.size());
      }
      desc = continuous(K->mDescriptors);
      return orbx_tri_kf{n, reinterpret_cast<const orbx_keypoint*>(K->mvKeysUn.data()), n > 0 ? desc.data : nullptr,
                         K->mvuRight.empty() ? nullptr : K->mvuRight.data(), has_mp.data(), (int)ids.size(),
                         ids.data(), off.data(), feat.data()};
    }
  } s1, s2;
  orbx_tri_problem p;
  std::memset(&p, 0, sizeof(p));
  p.kf1 = s1.kf(pKF1);
  p.kf2 = s2.kf(pKF2);
  for (int i = 0; i < 9; i++) p.F12[i] = F12.at<float>(i / 3, i % 3);
  const cv::Mat C1 = pKF1->GetCameraCenter();
  for (int k = 0; k < 3; k++) p.C1w[k] = C1.at<float>(k, 0);
  copy_mat44(pKF2->GetPose(), p.T2w);
  p.fx = pKF2->fx;
  p.fy = pKF2->fy;
  p.cx = pKF2->cx;
  p.cy = pKF2->cy;
  const int nl = pKF2->mnScaleLevels;
  if (nl < 1 || nl > 16) throw std::invalid_argument("SearchForTriangulation: nlevels");
  for (int l = 0; l < 16; l++) {
    p.scale_factors2[l] = l < nl ? pKF2->mvScaleFactors[l] : 0.f;
    p.level_sigma2_2[l] = l < nl ? pKF2->mvLevelSigma2[l] : 0.f;
  }
  p.only_stereo = bOnlyStereo;
  p.check_ori = mbCheckOrientation;
  std::vector<int32_t> m12(pKF1->N > 0 ? pKF1->N : 1, -1);
  int32_t nm = 0;
  p.match12 = m12.data();
  p.nmatches = &nm;
  check(orbx_search_for_triangulation(&p, gOrbxDevice), "orbx_search_for_triangulation");
  vMatchedPairs.clear();
  vMatchedPairs.reserve(nm);
  for (int i = 0; i < pKF1->N; i++)
    if (m12[i] >= 0) vMatchedPairs.push_back(std::make_pair((size_t)i, (size_t)m12[i]));
  return nm;
}

// ------------------------------------------------------------------ MapPoint / ORBVocabulary
void MapPoint::ComputeDistinctiveDescriptors() {
  // src/MapPoint.cc:249-320: the observed descriptors of non-bad KeyFrames in observation (map)
  // order; the one with the least median distance to the others becomes mDescriptor
  std::map<KeyFrame*, size_t> observations;
  {
    std::unique_lock<std::mutex> lock1(mMutexFeatures);
    if (mbBad) return;
    observations = mObservations;
  }
  if (observations.empty()) return;
  std::vector<uint8_t> desc;
  desc.reserve(32 * observations.size());
  for (const auto& o : observations) {
    KeyFrame* pKF = o.first;
    if (pKF->isBad()) continue;
    const uint8_t* row = pKF->mDescriptors.ptr<uint8_t>((int)o.second);
    desc.insert(desc.end(), row, row + 32);
  }
  if (desc.empty()) return;
  const int32_t off[2] = {0, (int32_t)(desc.size() / 32)};
  int32_t best = -1;
  check(orbx_distinctive_descriptors(desc.data(), off, 1, &best, nullptr, gOrbxDevice), "orbx_distinctive_descriptors");
  if (best < 0) return;
  cv::Mat d(1, 32, CV_8U);
  std::memcpy(d.data, &desc[32 * (size_t)best], 32);
  std::unique_lock<std::mutex> lock(mMutexFeatures);
  mDescriptor = d;
}

ORBVocabulary::~ORBVocabulary() {
  if (mpGpu) orbx_voc_destroy(mpGpu);
}

bool ORBVocabulary::loadFromText(const std::string& text) {
  if (mpGpu) {
    orbx_voc_destroy(mpGpu);
    mpGpu = nullptr;
  }
  check(orbx_voc_load_text(text.data(), text.size(), gOrbxDevice, &mpGpu), "orbx_voc_load_text");
  check(orbx_voc_info(mpGpu, mInfo), "orbx_voc_info");
  return true;
}

bool ORBVocabulary::loadFromTextFile(const std::string& filename) {
  std::ifstream f(filename.c_str(), std::ios::binary);
  if (!f.is_open()) return false;  // TemplatedVocabulary.h:1343-1347
  std::string text((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  return loadFromText(text);
}

void ORBVocabulary::transform(const cv::Mat& descriptors, DBoW2::BowVector& v, DBoW2::FeatureVector& fv,
                              int levelsup) const {
  // TemplatedVocabulary.h:1125-1196 on the device: every row descends the tree there
  v.clear();
  fv.clear();
  if (!mpGpu) throw std::runtime_error("ORBVocabulary::transform: no vocabulary loaded");
  const int n = descriptors.empty() ? 0 : descriptors.rows;
  if (n == 0) return;
  const cv::Mat d = continuous(descriptors);
  const int32_t set_off[2] = {0, n};
  std::vector<uint32_t> words(n), nodes(n);
  std::vector<double> values(n);
  std::vector<int32_t> fv_off(n + 1), fv_feat(n);
  int32_t nb = 0, nf = 0;
  check(orbx_voc_transform(mpGpu, d.data, set_off, 1, levelsup, words.data(), values.data(), &nb, nodes.data(),
                           fv_off.data(), fv_feat.data(), &nf),
        "orbx_voc_transform");
  for (int k = 0; k < nb; k++) v.emplace_hint(v.end(), words[k], values[k]);
  for (int j = 0; j < nf; j++) {
    std::vector<unsigned int>& feats = fv[nodes[j]];
    for (int q = fv_off[j]; q < fv_off[j + 1]; q++) feats.push_back((unsigned int)fv_feat[q]);
  }
}

void ORBVocabulary::transform(const std::vector<cv::Mat>& features, DBoW2::BowVector& v, DBoW2::FeatureVector& fv,
                              int levelsup) const {
  cv::Mat d((int)features.size(), 32, CV_8U);
  for (size_t i = 0; i < features.size(); i++) std::memcpy(d.ptr<uint8_t>((int)i), features[i].ptr<uint8_t>(0), 32);
  if (features.empty()) d.release();
  transform(d, v, fv, levelsup);
}

// ------------------------------------------------------------------ PnPsolver

namespace {
// the process-wide stream DUtils::Random::RandomInt draws from (glibc rand(), seed 1)
std::mutex g_rand_mu;
orbx_rand_state g_rand = [] {
  orbx_rand_state s;
  orbx_rand_seed(&s, 1);
  return s;
}();
}  // namespace

void PnPsolver::SeedRandom(unsigned int seed) {
  std::lock_guard<std::mutex> lock(g_rand_mu);
  orbx_rand_seed(&g_rand, seed);
}

PnPsolver::PnPsolver(const Frame& F, const std::vector<MapPoint*>& vpMapPointMatches)
    : mvpMapPointMatches(vpMapPointMatches) {
  // src/PnPsolver.cc:67-125: one correspondence per matched, non-bad MapPoint, in feature order
  for (size_t i = 0; i < vpMapPointMatches.size(); i++) {
    MapPoint* pMP = vpMapPointMatches[i];
    if (!pMP || pMP->isBad()) continue;
    const cv::KeyPoint& kp = F.mvKeysUn[i];
    mvP2D.push_back(kp.pt.x);
    mvP2D.push_back(kp.pt.y);
    mvSigma2.push_back(F.mvLevelSigma2[kp.octave]);
    const cv::Mat Pos = pMP->GetWorldPos();
    for (int k = 0; k < 3; k++) mvP3Dw.push_back(Pos.at<float>(k, 0));
    mvKeyPointIndices.push_back(i);
  }
  fu = F.fx;
  fv = F.fy;
  uc = F.cx;
  vc = F.cy;
  SetRansacParameters();
}

PnPsolver::~PnPsolver() {
  if (mpGpu) orbx_pnp_destroy(mpGpu);
}

void PnPsolver::SetRansacParameters(double probability, int minInliers, int maxIterations, int minSet, float epsilon,
                                    float th2) {
  mParams = orbx_pnp_params{probability, minInliers, maxIterations, minSet, epsilon, th2};
  if (mpGpu) {  // a live solver keeps mnIterations and its best set
    check(orbx_pnp_set_ransac_parameters(mpGpu, mvSigma2.data(), &mParams), "orbx_pnp_set_ransac_parameters");
    int mi = 0;
    float eps = 0;
    check(orbx_pnp_get_params(mpGpu, &mi, &mRansacMaxIts, &eps), "orbx_pnp_get_params");
  }
}

void PnPsolver::ensure_solver() {
  if (mpGpu) return;
  const int n = (int)mvSigma2.size();
  const orbx_pnp_problem prob{n, n ? mvP3Dw.data() : nullptr, n ? mvP2D.data() : nullptr,
                              n ? mvSigma2.data() : nullptr, fu, fv, uc, vc};
  check(orbx_pnp_create(&prob, &mParams, gOrbxDevice, &mpGpu), "orbx_pnp_create");
  int mi = 0;
  float eps = 0;
  check(orbx_pnp_get_params(mpGpu, &mi, &mRansacMaxIts, &eps), "orbx_pnp_get_params");
}

cv::Mat PnPsolver::find(std::vector<bool>& vbInliers, int& nInliers) {
  ensure_solver();
  bool bFlag;
  return iterate(mRansacMaxIts, bFlag, vbInliers, nInliers);  // src/PnPsolver.cc:181-185
}

cv::Mat PnPsolver::iterate(int nIterations, bool& bNoMore, std::vector<bool>& vbInliers, int& nInliers) {
  ensure_solver();
  bNoMore = false;
  vbInliers.clear();
  nInliers = 0;
  const int n = (int)mvSigma2.size();
  std::vector<uint8_t> inl(n > 0 ? n : 1, 0);
  float T[16];
  int no_more = 0, ni = 0, found = 0;
  {
    std::lock_guard<std::mutex> lock(g_rand_mu);
    check(orbx_pnp_iterate_stream(mpGpu, nIterations, &g_rand, &no_more, T, inl.data(), &ni, &found),
          "orbx_pnp_iterate_stream");
  }
  bNoMore = no_more != 0;
  if (!found) return cv::Mat();
  nInliers = ni;
  vbInliers.assign(mvpMapPointMatches.size(), false);  // :261-266 / :283-288
  for (int i = 0; i < n; i++)
    if (inl[i]) vbInliers[mvKeyPointIndices[i]] = true;
  cv::Mat Tcw(4, 4, CV_32F);
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++) Tcw.at<float>(r, c) = T[4 * r + c];
  return Tcw;
}

// ------------------------------------------------------------------ Optimizer
void (*Optimizer::mpfnGatheredHook)(const LocalBAProblem&, const std::vector<KeyFrame*>&) = nullptr;

int Optimizer::PoseOptimization(Frame* pFrame) {
  // src/Optimizer.cc:287-528: one edge per feature with a MapPoint, in feature order (:318-410);
  // mvbOutlier of those features reset to false; below 3 correspondences the pose is left as is
  const int N = pFrame->N;
  std::vector<float> obs, Xw, isig;
  std::vector<int> idx;
  for (int i = 0; i < N; i++) {
    MapPoint* pMP = pFrame->mvpMapPoints[i];
    if (!pMP) continue;
    pFrame->mvbOutlier[i] = false;
    const cv::KeyPoint& kpUn = pFrame->mvKeysUn[i];
    obs.push_back(kpUn.pt.x);
    obs.push_back(kpUn.pt.y);
    obs.push_back(pFrame->mvuRight[i]);  // < 0: EdgeSE3ProjectXYZOnlyPose, else the stereo edge
    const cv::Mat X = pMP->GetWorldPos();
    for (int k = 0; k < 3; k++) Xw.push_back(X.at<float>(k, 0));
    isig.push_back(pFrame->mvInvLevelSigma2[kpUn.octave]);
    idx.push_back(i);
  }
  const int n = (int)idx.size();
  if (n < 3) return 0;  // :424-425
  orbx_pose_problem p;
  std::memset(&p, 0, sizeof(p));
  p.n = n;
  p.obs = obs.data();
  p.Xw = Xw.data();
  p.inv_sigma2 = isig.data();
  p.fx = Frame::fx;
  p.fy = Frame::fy;
  p.cx = Frame::cx;
  p.cy = Frame::cy;
  p.bf = pFrame->mbf;
  copy_mat44(pFrame->mTcw, p.Tcw);
  float T[16];
  std::vector<uint8_t> outlier(n);
  int32_t ngood = 0;
  p.Tcw_out = T;
  p.outlier = outlier.data();
  p.ngood = &ngood;
  check(orbx_pose_optimization(&p, gOrbxDevice), "orbx_pose_optimization");
  for (int k = 0; k < n; k++) pFrame->mvbOutlier[idx[k]] = outlier[k] != 0;
  cv::Mat pose(4, 4, CV_32F);
  for (int i = 0; i < 16; i++) pose.at<float>(i / 4, i % 4) = T[i];
  pFrame->SetPose(pose);
  return ngood;
}

void Optimizer::LocalBundleAdjustment(KeyFrame* pKF, bool* pbStopFlag, Map* pMap) {
  // src/Optimizer.cc:532-551: the local KeyFrames (pKF and its non-bad covisibles)
  std::list<KeyFrame*> lLocalKeyFrames;
  lLocalKeyFrames.push_back(pKF);
  pKF->mnBALocalForKF = pKF->mnId;
  const std::vector<KeyFrame*> vNeighKFs = pKF->GetVectorCovisibleKeyFrames();
  for (KeyFrame* pKFi : vNeighKFs) {
    pKFi->mnBALocalForKF = pKF->mnId;
    if (!pKFi->isBad()) lLocalKeyFrames.push_back(pKFi);
  }
  // :553-572: the local MapPoints, first seen first
  std::list<MapPoint*> lLocalMapPoints;
  for (KeyFrame* pKFl : lLocalKeyFrames) {
    const std::vector<MapPoint*> vpMPs = pKFl->GetMapPointMatches();
    for (MapPoint* pMP : vpMPs)
      if (pMP && !pMP->isBad() && pMP->mnBALocalForKF != pKF->mnId) {
        lLocalMapPoints.push_back(pMP);
        pMP->mnBALocalForKF = pKF->mnId;
      }
  }
  // :574-592: KeyFrames that observe local MapPoints but are not local -> fixed
  std::list<KeyFrame*> lFixedCameras;
  for (MapPoint* pMP : lLocalMapPoints) {
    const std::map<KeyFrame*, size_t> observations = pMP->GetObservations();
    for (const auto& ob : observations) {
      KeyFrame* pKFi = ob.first;
      if (pKFi->mnBALocalForKF != pKF->mnId && pKFi->mnBAFixedForKF != pKF->mnId) {
        pKFi->mnBAFixedForKF = pKF->mnId;
        if (!pKFi->isBad()) lFixedCameras.push_back(pKFi);
      }
    }
  }
  // :608-640: vertices -- local poses (fixed iff mnId == 0), then the fixed cameras
  LocalBAProblem P;
  std::vector<KeyFrame*> cams;
  std::map<KeyFrame*, int> cam_index;
  auto add_cam = [&](KeyFrame* pKFi, bool fixed) {
    cam_index[pKFi] = (int)cams.size();
    cams.push_back(pKFi);
    LocalBAProblem::Camera C;
    C.Tcw = pKFi->GetPose();
    C.fixed = fixed;
    C.fx = pKFi->fx;
    C.fy = pKFi->fy;
    C.cx = pKFi->cx;
    C.cy = pKFi->cy;
    C.bf = pKFi->mbf;
    P.cameras.push_back(C);
  };
  for (KeyFrame* pKFi : lLocalKeyFrames) add_cam(pKFi, pKFi->mnId == 0);
  for (KeyFrame* pKFi : lFixedCameras) add_cam(pKFi, true);
  // :656-745: one point vertex per local MapPoint, one edge per observation by a non-bad KeyFrame
  // (GetObservations() order), monocular when mvuRight < 0
  std::vector<MapPoint*> points(lLocalMapPoints.begin(), lLocalMapPoints.end());
  std::vector<std::pair<KeyFrame*, MapPoint*>> edge_obj;
  for (size_t p = 0; p < points.size(); p++) {
    MapPoint* pMP = points[p];
    P.points.push_back(pMP->GetWorldPos());
    const std::map<KeyFrame*, size_t> observations = pMP->GetObservations();
    for (const auto& ob : observations) {
      KeyFrame* pKFi = ob.first;
      if (pKFi->isBad()) continue;
      const cv::KeyPoint& kpUn = pKFi->mvKeysUn[ob.second];
      LocalBAProblem::Observation o;
      o.point = (int)p;
      o.camera = cam_index.at(pKFi);
      o.u = kpUn.pt.x;
      o.v = kpUn.pt.y;
      o.ur = pKFi->mvuRight[ob.second];
      o.invSigma2 = pKFi->mvInvLevelSigma2[kpUn.octave];
      P.observations.push_back(o);
      edge_obj.emplace_back(pKFi, pMP);
    }
  }
  if (mpfnGatheredHook) mpfnGatheredHook(P, cams);
  // :747-751: a stop requested before the optimisation leaves the map untouched
  if (pbStopFlag && *pbStopFlag) return;
  LocalBAResult R;
  LocalBundleAdjustment(P, pbStopFlag, R, gOrbxDevice);
  // the flag may have gone up between the check above and the library's own poll: the library then
  // skipped optimize(5), and the reference would have returned here with the map untouched (:749-751)
  if (!R.ran) return;
  // :803-847 vToErase (the library's per-edge verdict after the last phase), then :849-884
  std::unique_lock<std::mutex> lock(pMap->mMutexMapUpdate);
  for (size_t e = 0; e < edge_obj.size(); e++) {
    if (!R.erase[e]) continue;
    KeyFrame* pKFi = edge_obj[e].first;
    MapPoint* pMPi = edge_obj[e].second;
    pKFi->EraseMapPointMatch(pMPi);
    pMPi->EraseObservation(pKFi);
  }
  for (KeyFrame* pKFl : lLocalKeyFrames) pKFl->SetPose(R.Tcw[cam_index.at(pKFl)]);
  for (size_t p = 0; p < points.size(); p++) {
    points[p]->SetWorldPos(R.points[p]);
    points[p]->UpdateNormalAndDepth();
  }
}

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
  // the LocalMapping thread keeps one solver (device buffers and stream reused across calls),
  // released when that thread exits
  struct BaDeleter {
    void operator()(orbx_ba* h) const { orbx_ba_destroy(h); }
  };
  static thread_local std::unique_ptr<orbx_ba, BaDeleter> ba;
  static thread_local int ba_device = -1;
  if (ba && ba_device != device) ba.reset();
  if (!ba) {
    orbx_ba* h = nullptr;
    check(orbx_ba_create(device, &h), "orbx_ba_create");
    ba.reset(h);
    ba_device = device;
  }
  check(orbx_ba_run_bool(ba.get(), &prob, &res, pbStopFlag), "orbx_ba_run");
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
  R.ran = res.ran != 0;
}

}  // namespace ORB_SLAM2
