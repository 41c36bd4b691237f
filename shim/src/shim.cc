// shim.cc -- the reference's hot-path classes (ORBextractor, Frame's ORB/stereo part, ORBmatcher's
// SearchByBoW / DescriptorDistance, PnPsolver, Optimizer::LocalBundleAdjustment) as thin C++ over
// the C ABI of liborbx.so (include/orbx.h).  Argument meaning and error behaviour follow the
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

#include "ORBextractor.h"
#include "ORBmatcher.h"
#include "Objects.h"
#include "Optimizer.h"
#include "PnPsolver.h"
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
float Frame::fx = 0.f, Frame::fy = 0.f, Frame::cx = 0.f, Frame::cy = 0.f, Frame::invfx = 0.f, Frame::invfy = 0.f;

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
  // scale tables (src/Frame.cc:66-73) and the static intrinsics (:111-126)
  mnScaleLevels = mpORBextractorLeft->GetLevels();
  mfScaleFactor = mpORBextractorLeft->GetScaleFactor();
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

// ------------------------------------------------------------------ PnPsolver
int PnPsolver::mnDevice = 0;

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
  check(orbx_pnp_create(&prob, &mParams, mnDevice, &mpGpu), "orbx_pnp_create");
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
int Optimizer::mnDevice = 0;
void (*Optimizer::mpfnGatheredHook)(const LocalBAProblem&, const std::vector<KeyFrame*>&) = nullptr;

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
  LocalBundleAdjustment(P, pbStopFlag, R, mnDevice);
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
