/*
 * orbx.h -- C ABI of the MI355X-native ORB-SLAM2 hot path (liborbx.so).
 *
 * Plain C, plain pointers and sizes; never throws; every call returns an
 * orbx_status (0 = ok, <0 = error).  Each handle owns one HIP stream, so two
 * handles may be driven from two host threads concurrently (the reference
 * runs the left and right extractors on two std::threads,
 * src/Frame.cc:80-84).  A single handle is not thread-safe, exactly like the
 * reference's ORBextractor (shared mvImagePyramid).
 *
 * Entry point -> reference interface it replaces:
 *   orbx_extractor_create       ORBextractor::ORBextractor      src/ORBextractor.cc:416-490, include/ORBextractor.h:61
 *   orbx_extractor_scale_tables GetScaleFactors/GetInverseScaleFactors/GetScaleSigmaSquares/
 *                               GetInverseScaleSigmaSquares     include/ORBextractor.h:85-103
 *   orbx_extractor_get_levels   GetLevels                       include/ORBextractor.h:81
 *   orbx_extractor_tables       protected mnFeaturesPerLevel/umax/pattern
 *                                                               src/ORBextractor.cc:416-490, include/ORBextractor.h:118,132,135
 *   orbx_extractor_set_pyramid_readback
 *                               mvImagePyramid refreshed by every operator()  src/ORBextractor.cc:1215-1250
 *   orbx_extract                ORBextractor::operator()        src/ORBextractor.cc:1138-1211, include/ORBextractor.h:77-78
 *   orbx_pyramid_level          public mvImagePyramid[level]    include/ORBextractor.h:104 (read at src/Frame.cc:556,681,694,700)
 *   orbx_extract_batch_device   frame-batch form of operator() (one launch per stage for n images)
 *   orbx_stereo_match           Frame::ComputeStereoMatches     src/Frame.cc:547-788, include/Frame.h:111
 *   orbx_stereo_frames_device   extract(L)+extract(R)+ComputeStereoMatches for n stereo frames
 *   orbx_frame_stereo           the ORB part of Frame's stereo constructor: ExtractORB(0/1) on two
 *                               threads + ComputeStereoMatches  src/Frame.cc:62-123 (:80-84, :121)
 *   orbx_descriptor_distance_device
 *                               ORBmatcher::DescriptorDistance  src/ORBmatcher.cc:1844-1860, include/ORBmatcher.h:50
 *   orbx_search_by_bow_kf_f     ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&)
 *                                                               src/ORBmatcher.cc:175-325, include/ORBmatcher.h:114
 *   orbx_search_by_bow_kf_kf    ORBmatcher::SearchByBoW(KeyFrame*, KeyFrame*, vector<MapPoint*>&)
 *                                                               src/ORBmatcher.cc:589-736, include/ORBmatcher.h:116
 *   orbx_search_by_bow_device   batch of the two above (one block per problem); ComputeThreeMaxima
 *                               (src/ORBmatcher.cc:1797-1839) runs inside
 *   orbx_pnp_create             PnPsolver::PnPsolver + SetRansacParameters
 *                                                               src/PnPsolver.cc:67-179, include/PnPsolver.h:66,71
 *   orbx_pnp_iterate            PnPsolver::iterate              src/PnPsolver.cc:182-384, include/PnPsolver.h:77
 *   orbx_voc_load_text          TemplatedVocabulary::loadFromTextFile (ORBVocabulary)
 *                                                               Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1338-1420
 *   orbx_voc_transform          TemplatedVocabulary::transform(features, BowVector, FeatureVector, levelsup)
 *                                                               :1125-1196, 1218-1259 (Frame::ComputeBoW src/Frame.cc:462-469)
 *   orbx_search_by_projection   ORBmatcher::SearchByProjection x3 (+ Frame::isInFrustum, GetFeaturesInArea)
 *                                                               src/ORBmatcher.cc:46-142, 1489-1795, include/ORBmatcher.h:64-95
 *   orbx_search_by_projection_device   batch of the above (one block per problem)
 *   orbx_search_for_triangulation  ORBmatcher::SearchForTriangulation src/ORBmatcher.cc:738-925, include/ORBmatcher.h:134
 *   orbx_search_by_sim3            ORBmatcher::SearchBySim3 src/ORBmatcher.cc:1238-1487, include/ORBmatcher.h:139
 *   orbx_search_for_initialization ORBmatcher::SearchForInitialization src/ORBmatcher.cc:442-587, include/ORBmatcher.h:130
 *   orbx_pose_optimization     Optimizer::PoseOptimization     src/Optimizer.cc:287-528, include/Optimizer.h:71
 *   orbx_pose_optimization_device      batch of the above (one block per frame)
 *   orbx_distinctive_descriptors[_device]  MapPoint::ComputeDistinctiveDescriptors src/MapPoint.cc:249-320
 *   orbx_undistort_keypoints[_device]      Frame::UndistortKeyPoints src/Frame.cc:471-506 (cv::undistortPoints)
 *   orbx_local_ba / orbx_ba_*   Optimizer::LocalBundleAdjustment src/Optimizer.cc:530-885, include/Optimizer.h:61
 *                               (g2o graph build, optimize(5), outlier levels, optimize(10), vToErase;
 *                               the Map mutex/recovery part stays on the caller's side)
 */
#ifndef ORBX_H
#define ORBX_H
#include <stddef.h>
#include <stdint.h>
#ifndef __cplusplus
#include <stdbool.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

typedef int orbx_status;
#define ORBX_OK 0
#define ORBX_ERR_ARG (-1)        /* bad argument / null pointer               */
#define ORBX_ERR_CAPACITY (-2)   /* caller buffer too small                   */
#define ORBX_ERR_HIP (-3)        /* HIP runtime error (launch, alloc, copy)   */
#define ORBX_ERR_NODEV (-4)      /* no usable gfx950 device                   */
#define ORBX_ERR_SIZE (-5)       /* image geometry outside supported range    */
#define ORBX_ERR_STATE (-6)      /* call requires a previous extraction       */

/* stream argument of the handle-owning device entry points (extractor, vocabulary): NULL picks the
 * handle's own (non-blocking) stream, this value the device's legacy null stream, which is what a
 * caller on PyTorch's default stream must pass so its own work stays ordered with the library's. */
#define ORBX_STREAM_NULL ((void*)1)

/* Layout-identical to cv::KeyPoint (28 bytes). class_id is always -1. */
typedef struct {
  float x, y, size, angle, response;
  int32_t octave, class_id;
} orbx_keypoint;

/* ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST) */
typedef struct {
  int nfeatures;
  float scale_factor;
  int nlevels;     /* 1..16 */
  int ini_th_fast;
  int min_th_fast;
} orbx_extractor_params;

typedef struct orbx_extractor orbx_extractor;

orbx_status orbx_extractor_create(const orbx_extractor_params* params, int device, orbx_extractor** out);
void orbx_extractor_destroy(orbx_extractor* h);
int orbx_extractor_get_levels(const orbx_extractor* h);
/* Any output pointer may be NULL; arrays hold nlevels floats. */
orbx_status orbx_extractor_scale_tables(const orbx_extractor* h, float* scale, float* inv_scale,
                                        float* sigma2, float* inv_sigma2);
/* The constructor's remaining tables (src/ORBextractor.cc:416-490; the protected members
 * mnFeaturesPerLevel, umax and pattern of include/ORBextractor.h:118,132,135): features_per_level
 * holds nlevels ints, umax 16 (HALF_PATCH_SIZE + 1), pattern 1024 (the 512 (x, y) sample points of the
 * 256 rBRIEF pairs, bit_pattern_31_).  Any pointer may be NULL. */
orbx_status orbx_extractor_tables(const orbx_extractor* h, int* features_per_level, int* umax, int* pattern);
/* mvImagePyramid readback (include/ORBextractor.h:104; the reference rebuilds it on every operator()
 * call, src/ORBextractor.cc:1215-1250).  With on != 0 every orbx_extract also copies the pyramid it
 * built into pinned host memory in the same stream, before its single synchronisation, and
 * orbx_pyramid_level(h, 0, l, ...) then reads that copy with no device call.  Off by default (a
 * caller that never reads the levels on the host does not pay the copy). */
orbx_status orbx_extractor_set_pyramid_readback(orbx_extractor* h, int on);
/* Upper bound on keypoints per image for this geometry (size kps/desc buffers with it). */
int orbx_extractor_max_keypoints(orbx_extractor* h, int width, int height);

/* Drop-in ORBextractor::operator(): host image in, host keypoints/descriptors out.
 * An empty image (w or h == 0, or img == NULL) returns ORBX_OK with *n = 0,
 * mirroring the reference's silent return. desc receives n*32 bytes, row i <-> kps[i].
 * Output order is level-major, exactly the reference's. */
orbx_status orbx_extract(orbx_extractor* h, const uint8_t* img, int width, int height, size_t stride,
                         orbx_keypoint* kps, int cap, uint8_t* desc, int* n);

/* Copy level `level` of image `image` of the last extraction to host memory
 * (dst may be NULL to query the size). */
orbx_status orbx_pyramid_level(orbx_extractor* h, int image, int level, uint8_t* dst, size_t dst_stride,
                               int* width, int* height);

/* Device-resident batch: n_images u8 images of width x height, image i at
 * d_images + i*image_pitch (row stride = width).  Outputs on device: image i
 * writes d_counts[i] keypoints to d_kps + i*kp_capacity and descriptors to
 * d_desc + i*kp_capacity*32.  stream: hipStream_t (NULL = the handle's own; ORBX_STREAM_NULL = the
 * device's legacy null stream, e.g. PyTorch's default stream).
 * Asynchronous; the input buffer must stay alive until the stream completes
 * and, for orbx_stereo_* on the same batch, until those complete too
 * (level 0 of the pyramid is the input itself). */
orbx_status orbx_extract_batch_device(orbx_extractor* h, int n_images, const uint8_t* d_images, int width,
                                      int height, size_t image_pitch, orbx_keypoint* d_kps, uint8_t* d_desc,
                                      int32_t* d_counts, int kp_capacity, void* stream);

/* Drop-in Frame::ComputeStereoMatches: host keypoints/descriptors, pyramids
 * from the last extraction of `left` and `right`.  bf = baseline*fx (mbf),
 * baseline = mb.  Writes uRight[nL], depth[nL] (-1 = no match).
 * The last call on each handle must be orbx_extract and kpsL/kpsR must be the
 * keypoints it returned (checked by count and fingerprint): otherwise the
 * pyramid no longer belongs to them and ORBX_ERR_STATE is returned. */
orbx_status orbx_stereo_match(orbx_extractor* left, orbx_extractor* right, const orbx_keypoint* kpsL,
                              const uint8_t* descL, int nL, const orbx_keypoint* kpsR, const uint8_t* descR,
                              int nR, float bf, float baseline, float* uRight, float* depth);

/* The ORB part of the stereo Frame constructor in one call (src/Frame.cc:62-123: ExtractORB(0, imLeft)
 * and ExtractORB(1, imRight) on two threads, then ComputeStereoMatches), host images in and host
 * results out: both images go through `h` as one batch of two (the reference builds its left and
 * right extractors with the same parameters, src/Tracking.cc:113-126; results are those of two
 * orbx_extract calls + orbx_stereo_match), the matcher runs on the device right behind them and
 * everything returns in one copy with one synchronisation.  nL / nR keypoints and descriptors into
 * kpsL / descL (capacity capL) and kpsR / descR (capR); uRight[nL], depth[nL] (-1 = no match).
 * Afterwards orbx_pyramid_level(h, 0 / 1, ...) reads the left / right pyramid, and h's last
 * extraction is no longer an orbx_extract result (orbx_stereo_match on it returns ORBX_ERR_STATE). */
orbx_status orbx_frame_stereo(orbx_extractor* h, const uint8_t* imL, size_t strideL, const uint8_t* imR,
                              size_t strideR, int width, int height, float bf, float baseline, orbx_keypoint* kpsL,
                              uint8_t* descL, int capL, int* nL, orbx_keypoint* kpsR, uint8_t* descR, int capR,
                              int* nR, float* uRight, float* depth);

/* Device-resident stereo frames: d_images holds 2*n_frames images ordered
 * L0,R0,L1,R1,... (pitch image_pitch).  Runs extraction of all 2n images and
 * the stereo matcher of every frame.  Per image i: d_counts[i], d_kps/d_desc as
 * in orbx_extract_batch_device.  Per frame f: d_uright/d_depth + f*kp_capacity
 * hold the left keypoints' results; d_nmatches[f] = surviving matches. */
orbx_status orbx_stereo_frames_device(orbx_extractor* h, int n_frames, const uint8_t* d_images, int width,
                                      int height, size_t image_pitch, orbx_keypoint* d_kps, uint8_t* d_desc,
                                      int32_t* d_counts, int kp_capacity, float bf, float baseline,
                                      float* d_uright, float* d_depth, int32_t* d_nmatches, void* stream);

/* Batched ORBmatcher::DescriptorDistance on device: d_out[i] = popcount(a_i ^ b_i). */
orbx_status orbx_descriptor_distance_device(const uint8_t* d_a, const uint8_t* d_b, int n, int32_t* d_out,
                                            void* stream);

/* One side of SearchByBoW: n features (descriptors n x 32, keypoint angles),
 * MapPoint validity valid[i] = (mvpMapPoints[i] && !isBad()) (NULL = all valid;
 * ignored for the Frame side), and the DBoW2::FeatureVector as CSR: n_nodes
 * ascending node ids, node_off[n_nodes+1], feat[] = feature indices of each
 * node in vector order. */
typedef struct {
  int n;
  const uint8_t* desc;
  const float* angle;
  const uint8_t* valid;
  int n_nodes;
  const uint32_t* node_id;
  const int32_t* node_off;
  const int32_t* feat;
} orbx_bow_side;

/* Host pointers in and out.  KF-F: match_f[f->n] = KF feature index matched to
 * each frame feature (the reference stores KF MapPoint*), -1 otherwise.
 * KF-KF: match12[kf1->n] = KF2 feature index or -1.  *nmatches = the return
 * value of the reference.  nnratio/check_ori = ORBmatcher(nnratio, checkOri). */
orbx_status orbx_search_by_bow_kf_f(const orbx_bow_side* kf, const orbx_bow_side* f, float nnratio, int check_ori,
                                    int32_t* match_f, int* nmatches, int device);
orbx_status orbx_search_by_bow_kf_kf(const orbx_bow_side* kf1, const orbx_bow_side* kf2, float nnratio,
                                     int check_ori, int32_t* match12, int* nmatches, int device);

/* Batched, device-resident: problems[] is a HOST array whose pointers are device
 * pointers; mode 0 = KF-F, 1 = KF-KF.  Each problem writes match[] and *nmatches. */
typedef struct {
  orbx_bow_side a, b;
  float nnratio;
  int check_ori;
  int mode;
  int32_t* match;
  int32_t* nmatches;
  /* optional (NULL: use the side's fields): feature and FeatureVector node counts as an earlier
   * kernel of the stream left them (e.g. orbx_voc_transform_device's n_fv and the extraction's
   * counts); the side's n / n_nodes are then the capacities and the counts are min'd with them */
  const int32_t* a_n_dev;
  const int32_t* a_nodes_dev;
  const int32_t* b_n_dev;
  const int32_t* b_nodes_dev;
} orbx_bow_problem;
orbx_status orbx_search_by_bow_device(const orbx_bow_problem* problems, int n, void* stream);

/* DBoW2 vocabulary (ORBVocabulary = TemplatedVocabulary<FORB::TDescriptor, FORB>)
 * from the text format of loadFromTextFile: header "k L scoring weighting",
 * then one line per node "parent isLeaf d0..d31 weight" in node-id order.  A
 * blank line ends the node list.  The tree lives on `device`. */
typedef struct orbx_voc orbx_voc;
orbx_status orbx_voc_load_text(const char* text, size_t len, int device, orbx_voc** out);
orbx_status orbx_voc_destroy(orbx_voc* v);
/* info = {k, L, scoring, weighting, n_nodes (incl. root), n_words} */
orbx_status orbx_voc_info(const orbx_voc* v, int32_t info[6]);
/* transform(features, BowVector, FeatureVector, levelsup) for n_sets descriptor
 * sets in one call: set s = rows set_off[s] .. set_off[s+1]-1 of desc (32 B
 * each, set_off[0] = 0, at most 8192 rows per set).  Host pointers.  Per set s:
 *   BowVector     n_bow[s] entries at bow_words/bow_values + set_off[s], word ids
 *                 ascending (std::map order), values after the vocabulary's
 *                 weighting/normalisation;
 *   FeatureVector n_fv[s] nodes at fv_nodes + set_off[s] (ascending), the
 *                 features of node j at fv_feat[set_off[s] + fv_off[set_off[s] + s + j]
 *                 .. + fv_off[set_off[s] + s + j + 1]) as indices within the set,
 *                 ascending -- the CSR that orbx_bow_side takes. */
orbx_status orbx_voc_transform(orbx_voc* v, const uint8_t* desc, const int32_t* set_off, int n_sets, int levelsup,
                               uint32_t* bow_words, double* bow_values, int32_t* n_bow, uint32_t* fv_nodes,
                               int32_t* fv_off, int32_t* fv_feat, int32_t* n_fv);
/* The same on a device batch, e.g. the left images of orbx_stereo_frames_device (Frame::ComputeBoW
 * for every frame of the batch at once): set s is rows s*stride .. s*stride + count[s*count_step]-1
 * of d_desc (at most cap <= 8192 rows; the stereo batch's left images: stride = 2*cap,
 * count_step = 2).  Outputs as above with set_off[s] = s*cap (fv_off of set s starts at
 * s*(cap+1)).  All pointers device pointers, queued on `stream` (NULL: the vocabulary's own;
 * ORBX_STREAM_NULL: the device's legacy null stream),
 * no host synchronisation. */
orbx_status orbx_voc_transform_device(orbx_voc* v, const uint8_t* d_desc, int cap, long long stride,
                                      const int32_t* d_count, int count_step, int n_sets, int levelsup,
                                      uint32_t* d_bow_words, double* d_bow_values, int32_t* d_n_bow,
                                      uint32_t* d_fv_nodes, int32_t* d_fv_off, int32_t* d_fv_feat, int32_t* d_n_fv,
                                      void* stream);

/* Optimizer::LocalBundleAdjustment on g2o semantics (BlockSolver_6_3 +
 * LinearSolverEigen + Levenberg, Huber kernels, two phases), FP64 on the GPU.
 * The caller gathers lLocalKeyFrames (not fixed unless mnId==0),
 * lFixedCameras (fixed) and lLocalMapPoints with their observations exactly
 * as src/Optimizer.cc:530-650 does, and writes back poses, points and erases
 * the flagged observations under the map mutex (:817-885).
 *   cameras: Tcw row-major 3x4 float, fixed flag, intrinsics fx,fy,cx,cy,bf
 *   edges:   point, camera, obs (u, v, ur; ur < 0 -> monocular
 *            EdgeSE3ProjectXYZ, else EdgeStereoSE3ProjectXYZ), invSigma2 */
typedef struct {
  int n_cams;
  const float* Tcw;
  const uint8_t* fixed;
  const float* intr;
  int n_points;
  const float* Xw;
  int n_edges;
  const int32_t* edge_point;
  const int32_t* edge_cam;
  const float* obs;
  const float* inv_sigma2;
} orbx_ba_problem;

typedef struct {
  float* Tcw;             /* n_cams x 12 (Converter::toCvMat of the optimised SE3Quat) */
  float* Xw;              /* n_points x 3 */
  uint8_t* edge_outlier;  /* n_edges: observation to erase (vToErase, :817-847) */
  double* Tcw_d;          /* optional FP64 copies (NULL to skip) */
  double* Xw_d;
  int iterations[2];      /* LM iterations run by optimize(5) and optimize(10) */
  int trials;             /* LM inner trials in total */
  double chi2[2];         /* active robust chi2 at the end of each phase */
  int ran;                /* 1: the optimisation ran and the outputs are the optimised state; 0: the stop
                           * flag was up before optimize(5) (src/Optimizer.cc:749-751) -- the reference
                           * then returns with the map untouched, so a caller must skip its write-back */
} orbx_ba_result;

typedef struct orbx_ba orbx_ba;
/* A solver handle keeps its device buffers and HIP stream across calls. */
orbx_status orbx_ba_create(int device, orbx_ba** out);
/* The same with the handle's stream at a HIP stream priority: 0 the default, < 0 higher (clamped to
 * the device's greatest priority).  LocalMapping's LocalBA (src/LocalMapping.cc:99-101) runs beside
 * Tracking's extraction on the same GPU: a high-priority stream lets its short, latency-bound trial
 * kernels take the compute units the extraction launches free up before further extraction blocks. */
orbx_status orbx_ba_create_priority(int device, int priority, orbx_ba** out);
/* The same with the handle's stream restricted to a set of compute units (cu_mask: cu_mask_words
 * 32-bit words, bit i = CU i as the HIP runtime numbers them; NULL or 0 words = all CUs): a
 * LocalMapping handle and the Tracking extraction streams (orbx_stream_create below) can take
 * disjoint CU sets, so neither waits for units the other holds. */
orbx_status orbx_ba_create_masked(int device, const uint32_t* cu_mask, int cu_mask_words, orbx_ba** out);
/* A HIP stream of `device` restricted to a CU set (as above), for the *_device entry points' stream
 * arguments; orbx_stream_destroy synchronises and releases it. */
orbx_status orbx_stream_create(int device, const uint32_t* cu_mask, int cu_mask_words, void** stream);
void orbx_stream_destroy(void* stream);
orbx_status orbx_ba_destroy(orbx_ba* h);
/* *stop_flag != 0 (the reference's pbStopFlag / setForceStopFlag) is polled
 * before the run and between LM trials -- by the device itself while the LM
 * loop runs there: the flag's page is mapped into the GPU's address space
 * (pinned memory as is, any other page registered once per handle). */
orbx_status orbx_ba_run(orbx_ba* h, const orbx_ba_problem* problem, orbx_ba_result* result,
                        const volatile int* stop_flag);
/* The same with the reference's own flag type: LocalBundleAdjustment(KeyFrame*, bool* pbStopFlag, Map*)
 * (include/Optimizer.h:61), set from LocalMapping::InterruptBA on another thread. */
orbx_status orbx_ba_run_bool(orbx_ba* h, const orbx_ba_problem* problem, orbx_ba_result* result,
                             const volatile bool* stop_flag);
/* K independent LocalBundleAdjustment problems in one call (e.g. one local map
 * per sequence): every LM trial kernel runs once for all of them, each on its
 * own arrays and LM state, so K problems cost about one problem's launches.
 * Results are bit-identical to K orbx_ba_run calls.  problems/results are
 * arrays of n; one stop flag for all. */
orbx_status orbx_ba_run_many(orbx_ba* h, int n, const orbx_ba_problem* problems, orbx_ba_result* results,
                             const volatile int* stop_flag);
/* A stop flag owned by the handle, in pinned host memory the device reads
 * directly (no page registration): set it from another thread to interrupt
 * orbx_ba_run(h, ..., flag) like LocalMapping::InterruptBA sets mbAbortBA. */
orbx_status orbx_ba_stop_flag(orbx_ba* h, volatile int** flag);
/* One-shot form: create, run, destroy. */
orbx_status orbx_local_ba(const orbx_ba_problem* problem, orbx_ba_result* result, const volatile int* stop_flag,
                          int device);

/* PnPsolver (src/PnPsolver.cc).  The caller gathers the correspondences
 * exactly like the constructor (:67-125): for each frame keypoint i with a
 * valid, non-bad MapPoint, p2d = mvKeysUn[i].pt, sigma2 = mvLevelSigma2[octave],
 * p3d = MapPoint world position, and keeps i (mvKeyPointIndices) to map the
 * returned inlier bytes back to frame indices. */
typedef struct {
  int n;
  const float* p3d;    /* n x 3 */
  const float* p2d;    /* n x 2 */
  const float* sigma2; /* n */
  float fx, fy, cx, cy;
} orbx_pnp_problem;

typedef struct { /* SetRansacParameters arguments (Tracking: 0.99, 10, 300, 4, 0.5, 5.991) */
  double probability;
  int min_inliers;
  int max_iterations;
  int min_set; /* 1..16 */
  float epsilon;
  float th2;
} orbx_pnp_params;

typedef struct orbx_pnp orbx_pnp;
orbx_status orbx_pnp_create(const orbx_pnp_problem* problem, const orbx_pnp_params* params, int device,
                            orbx_pnp** out);
/* n solvers at once (one per relocalisation candidate, or one per frame of a batch): the same as n
 * orbx_pnp_create calls with one parameter set, the correspondences in one upload.  out[n]; each
 * solver is released with orbx_pnp_destroy. */
orbx_status orbx_pnp_create_many(const orbx_pnp_problem* problems, int n, const orbx_pnp_params* params, int device,
                                 orbx_pnp** out);
/* The same from device-resident correspondences (e.g. the matches a device SearchByBoW produced):
 * problem i is rows offsets[i] .. offsets[i+1]-1 of d_p3d (x3), d_p2d (x2), d_sigma2 (device
 * pointers); offsets[n+1] and intr[4n] (fx, fy, cx, cy per problem) are host arrays. */
orbx_status orbx_pnp_create_many_device(const float* d_p3d, const float* d_p2d, const float* d_sigma2,
                                        const int32_t* offsets, const float* intr, int n,
                                        const orbx_pnp_params* params, int device, orbx_pnp** out);
orbx_status orbx_pnp_destroy(orbx_pnp* h);
/* PnPsolver::SetRansacParameters (src/PnPsolver.cc:136-179, include/PnPsolver.h:71) on an existing
 * solver, at any time: the derived parameters and maxError = sigma2 * th2 (sigma2: the n values given
 * at creation, host) are recomputed in place; mnIterations, the best inlier set and pose are kept. */
orbx_status orbx_pnp_set_ransac_parameters(orbx_pnp* h, const float* sigma2, const orbx_pnp_params* params);
/* Derived RANSAC parameters (mRansacMinInliers, mRansacMaxIts, mRansacEpsilon). */
orbx_status orbx_pnp_get_params(const orbx_pnp* h, int* min_inliers, int* max_iterations, float* epsilon);
/* iterate(nIterations, bNoMore, vbInliers, nInliers).  rand_vals: the next
 * rand() outputs of the caller's stream (the reference draws
 * DUtils::Random::RandomInt from the process rand()); supply at least
 * min_set * max(maxIts - done, nIterations) values; *used = values consumed,
 * so the caller advances its stream by exactly that.  *found = 1 when a pose
 * (Tcw, row-major 4x4) is returned; inliers[n] = 1 per inlier correspondence. */
orbx_status orbx_pnp_iterate(orbx_pnp* h, int n_iterations, const int32_t* rand_vals, int n_rand, int* used,
                             int* no_more, float Tcw[16], uint8_t* inliers, int* n_inliers, int* found);

/* glibc rand() (random_r TYPE_3) as a copyable stream: the reference's
 * RandomInt draws from the unseeded process rand() (seed 1).  POD state, so
 * a caller can snapshot it. */
typedef struct {
  uint32_t r[34];
  int32_t i;
} orbx_rand_state;
void orbx_rand_seed(orbx_rand_state* s, uint32_t seed);
int32_t orbx_rand_next(orbx_rand_state* s);
/* iterate() drawing from *rng and advancing it by exactly the values the
 * reference would consume. */
orbx_status orbx_pnp_iterate_stream(orbx_pnp* h, int n_iterations, orbx_rand_state* rng, int* no_more,
                                    float Tcw[16], uint8_t* inliers, int* n_inliers, int* found);

/* Several solvers per call.  Per solver: */
typedef struct {
  int no_more;    /* bNoMore */
  int found;      /* a pose was returned */
  int n_inliers;  /* nInliers */
  int used;       /* rand() values this call drew for the solver */
  float Tcw[16];  /* row-major 4x4 when found */
} orbx_pnp_result;
/* Tracking::Relocalization's candidate loop (src/Tracking.cc:1738-1757): iterate(n_iterations)
 * on solvers[0], solvers[1], ... in order, all drawing from the one stream *rng, stopping after
 * the first solver that returns a pose (*stopped = its index, n when none did).  Exactly the
 * calls the reference makes, so the solvers' state and *rng advance as they would; solvers
 * after *stopped are untouched (their results zeroed).  One hypothesis launch and one check
 * launch span all solvers (a solver that returns no pose consumes all of its iterations, so
 * where each one starts in the stream is known up front).  inliers[s] (may be NULL, or any
 * entry NULL): solvers[s]->n bytes, written when results[s].found.  Same device for all. */
orbx_status orbx_pnp_iterate_candidates(orbx_pnp* const* solvers, int n, int n_iterations, orbx_rand_state* rng,
                                        orbx_pnp_result* results, uint8_t* const* inliers, int* stopped);
/* Independent solvers, each with its own rand() stream rngs[s] (distinct pointers), e.g. one
 * relocalising frame per sequence of a multi-sequence batch: iterate(n_iterations) on every
 * solver, results as above; hypotheses, inlier checks and Refine() calls of all solvers are
 * batched into shared launches. */
orbx_status orbx_pnp_iterate_many(orbx_pnp* const* solvers, int n, int n_iterations, orbx_rand_state* const* rngs,
                                  orbx_pnp_result* results, uint8_t* const* inliers);

/* ORBmatcher::SearchByProjection -- the three overloads run on every tracked
 * frame -- with Frame::AssignFeaturesToGrid / GetFeaturesInArea
 * (src/Frame.cc:254-271, 388-453) and, for the local map, Frame::isInFrustum
 * (src/Frame.cc:315-375) fused in front:
 *   ORBX_PROJ_LOCAL      SearchByProjection(Frame&, const vector<MapPoint*>&, th)
 *                                                   src/ORBmatcher.cc:46-142, include/ORBmatcher.h:64
 *                        (frustum = 1: Tracking::SearchLocalPoints' isInFrustum(pMP, 0.5)
 *                        loop first, src/Tracking.cc:1427-1443)
 *   ORBX_PROJ_LAST_FRAME SearchByProjection(Frame&, const Frame&, th, bMono)
 *                                                   src/ORBmatcher.cc:1489-1646, include/ORBmatcher.h:76
 *   ORBX_PROJ_KEYFRAME   SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>&, th, ORBdist)
 *                                                   src/ORBmatcher.cc:1648-1795, include/ORBmatcher.h:95
 *   ORBX_PROJ_FUSE       the matching half of Fuse(KeyFrame*, const vector<MapPoint*>&, th)
 *                                                   src/ORBmatcher.cc:944-1054, include/ORBmatcher.h:148
 *                        (f = the KeyFrame, bounds = its int mnMinX.. as float; point_match[k] =
 *                        bestIdx when bestDist <= TH_LOW, *nmatches = nFused.  The caller then
 *                        applies Replace/AddObservation in point order, :1057-1086, re-querying
 *                        any later point whose descriptor a Replace recomputed)
 *   ORBX_PROJ_SIM3       SearchByProjection(KeyFrame*, cv::Mat Scw, const vector<MapPoint*>&,
 *                        vector<MapPoint*>& vpMatched, th)   src/ORBmatcher.cc:327-440
 *                        (LoopClosing::ComputeSim3, src/LoopClosing.cc:504; f = the KeyFrame with
 *                        f.Tcw = the 4x4 Sim3 Scw, bounds = its int mnMinX.. as float; occ[i] != 0 =
 *                        vpMatched[i] on entry; flags bit0 = !isBad() && not in vpMatched;
 *                        frame_out[i] = k: vpMatched[i] = point k; *nmatches = nmatches)
 *   ORBX_PROJ_FUSE_SIM3  the matching half of Fuse(KeyFrame*, cv::Mat Scw, const vector<MapPoint*>&,
 *                        th, vector<MapPoint*>& vpReplacePoint)   src/ORBmatcher.cc:1094-1236
 *                        (LoopClosing::SearchAndFuse, src/LoopClosing.cc:837; f as for SIM3, occ
 *                        unused; flags bit0 = !isBad() && !spAlreadyFound.count(pMP) with
 *                        spAlreadyFound = pKF->GetMapPoints() at entry; point_match[k] = bestIdx
 *                        when bestDist <= TH_LOW, *nmatches = nFused; the caller applies the
 *                        replace / AddMapPoint block, :1210-1229, in point order)
 *   ORBX_PROJ_BY_SIM3    one direction of SearchBySim3 (src/ORBmatcher.cc:1283-1340; orbx_search_by_sim3
 *                        below runs both): f = the other KeyFrame (its own Tcw unused), f.Tcw = the
 *                        points' KeyFrame pose [Riw | tiw], last_Tcw = [sRji | tji]; flags bit0 =
 *                        pMP && !vbAlreadyMatched && !isBad(); point_match[k] = bestIdx (<= TH_HIGH)
 * The current Frame (orbx_proj_frame) and the projected MapPoints are SoA
 * arrays the caller gathers from its object graph; the Frame's mvpMapPoints
 * on entry is summarised per feature as occ[i]: 0 NULL, 1 a MapPoint with
 * Observations() == 0, 2 a MapPoint with Observations() > 0. */
#define ORBX_GRID_COLS 64 /* FRAME_GRID_COLS, include/Frame.h:39 */
#define ORBX_GRID_ROWS 48 /* FRAME_GRID_ROWS, include/Frame.h:38 */
#define ORBX_PROJ_LOCAL 0
#define ORBX_PROJ_LAST_FRAME 1
#define ORBX_PROJ_KEYFRAME 2
#define ORBX_PROJ_FUSE 3
#define ORBX_PROJ_SIM3 4
#define ORBX_PROJ_FUSE_SIM3 5
#define ORBX_PROJ_BY_SIM3 6
#define ORBX_PROJ_MAX_FEATURES 8192 /* Frame::N per problem */

typedef struct {
  int n;                           /* N */
  const orbx_keypoint* keys_un;    /* mvKeysUn (pt, octave, angle) */
  const uint8_t* desc;             /* mDescriptors, n x 32 */
  const float* u_right;            /* mvuRight, NULL = monocular (all -1) */
  const int8_t* occ;               /* mvpMapPoints on entry (see above), NULL = all NULL */
  float min_x, max_x, min_y, max_y;/* mnMinX, mnMaxX, mnMinY, mnMaxY */
  float grid_inv_w, grid_inv_h;    /* mfGridElementWidthInv, mfGridElementHeightInv */
  int nlevels;                     /* mnScaleLevels (<= 16) */
  float scale_factors[16];         /* mvScaleFactors */
  float inv_level_sigma2[16];      /* mvInvLevelSigma2 (FUSE) */
  float log_scale_factor;          /* mfLogScaleFactor */
  float fx, fy, cx, cy, bf, b;     /* fx, fy, cx, cy, mbf, mb */
  float Tcw[16];                   /* mTcw, row-major 4x4 */
  /* the bounds the feature grid was built with, when they differ from min_x / min_y: a KeyFrame keeps
   * integer mnMinX / mnMinY (include/KeyFrame.h, GetFeaturesInArea's cell range, IsInImage) while its
   * mGrid is the Frame's, built from the float Frame::mnMinX / mnMinY (src/Frame.cc:388-395 PosInGrid);
   * grid_min_set = 0: the grid uses min_x / min_y */
  float grid_min_x, grid_min_y;
  int grid_min_set;
} orbx_proj_frame;

typedef struct {
  int kind;                 /* ORBX_PROJ_* */
  int frustum;              /* LOCAL: 1 = compute track[]/track_level[] by isInFrustum first */
  orbx_proj_frame f;
  int n_points;
  const uint8_t* desc;      /* MapPoint::GetDescriptor(), n_points x 32 */
  const uint8_t* flags;     /* bit0 = the point takes part (LOCAL: mbTrackInView && !isBad(), or with
                               frustum: mnLastFrameSeen != mnId && !isBad(); LAST_FRAME: pMP &&
                               !mvbOutlier[i]; KEYFRAME: pMP && !isBad() && !sAlreadyFound.count(pMP);
                               FUSE: pMP && !isBad() && !IsInKeyFrame(pKF); SIM3: !isBad() &&
                               !spAlreadyFound.count(pMP));
                               bit1 = Observations() > 0 */
  const float* pos;         /* GetWorldPos(), n_points x 3 (frustum, LAST_FRAME, KEYFRAME, FUSE*, SIM3) */
  const float* normal;      /* GetNormal(), n_points x 3 (frustum, FUSE*, SIM3) */
  const float* dist_minmax; /* mfMinDistance, mfMaxDistance, n_points x 2 (frustum, KEYFRAME, FUSE*, SIM3) */
  const float* angle;       /* LastFrame.mvKeysUn[i].angle / pKF->mvKeysUn[i].angle (LAST_FRAME, KEYFRAME) */
  const int32_t* octave;    /* LastFrame.mvKeys[i].octave (LAST_FRAME) */
  float* track;             /* LOCAL, n_points x 4: mTrackProjX, mTrackProjY, mTrackProjXR, mTrackViewCos
                               (input, or output when frustum) */
  int32_t* track_level;     /* LOCAL: mnTrackScaleLevel (input; with frustum output, -1 = not in view) */
  float th;                 /* th */
  float nnratio;            /* ORBmatcher mfNNratio (LOCAL) */
  float view_cos_limit;     /* isInFrustum viewingCosLimit (0.5 in SearchLocalPoints) */
  int check_ori;            /* ORBmatcher mbCheckOrientation (LAST_FRAME, KEYFRAME) */
  int mono;                 /* bMono (LAST_FRAME) */
  int orb_dist;             /* ORBdist (KEYFRAME) */
  float last_Tcw[16];       /* LastFrame.mTcw (LAST_FRAME) */
  int32_t* frame_out;       /* f.n: the Frame's mvpMapPoints on return: -1 unchanged by this call,
                               -2 set to NULL by the rotation check, k >= 0 = point k */
  int32_t* point_match;     /* n_points: feature index point k was assigned to (before the
                               rotation check), -1 none */
  int32_t* nmatches;        /* the reference's return value */
  /* Device batches only (orbx_search_by_projection_device; NULL/0 otherwise): sizes and pose that
   * an earlier kernel of the same stream produced, so no host round trip sizes the problem. */
  const int32_t* f_n_dev;   /* N = min(*f_n_dev, f.n): f.n is then the capacity */
  const int32_t* n_points_dev; /* n_points = min(*n_points_dev, n_points) */
  const float* Tcw_dev;     /* 16 floats replacing f.Tcw */
  const int32_t* gate;      /* run only if *gate < gate_below (else every output is left as is): */
  int gate_below;           /* Tracking's "if(nmatches<20) search again with 2*th" (src/Tracking.cc:1071-1076) */
} orbx_proj_problem;

/* One problem; every pointer in *p is a HOST pointer (outputs are written back). */
orbx_status orbx_search_by_projection(const orbx_proj_problem* p, int device);
/* Batched, device-resident: problems[] is a HOST array whose pointers are
 * device pointers; one launch for the whole batch, stream-ordered. */
orbx_status orbx_search_by_projection_device(const orbx_proj_problem* problems, int n, void* stream);

/* ORBmatcher::SearchBySim3(KeyFrame* pKF1, KeyFrame* pKF2, vector<MapPoint*>& vpMatches12, s12, R12,
 * t12, th) -- src/ORBmatcher.cc:1238-1487, include/ORBmatcher.h:139 (caller LoopClosing::ComputeSim3,
 * src/LoopClosing.cc:422).  kf1 / kf2: the KeyFrames (keys_un, desc, bounds = int mnMinX.. as float,
 * grid, levels, fx.., Tcw = GetPose()); per feature i of KF j the MapPoint GetMapPointMatches()[i]:
 * descj/posj/dist_minmaxj (MapPoint descriptor, world position, mfMinDistance/mfMaxDistance) and flagsj
 * bit0 = pMP && !vbAlreadyMatchedj[i] && !pMP->isBad() (vbAlreadyMatched from vpMatches12 on entry,
 * :1262-1273).  match12[i1] = idx2 where the two directions agree (vpMatches12[i1] =
 * vpMapPoints2[idx2]), -1 elsewhere; *nfound = nFound. */
typedef struct {
  orbx_proj_frame kf1, kf2;
  const uint8_t* desc1;
  const float* pos1;
  const float* dist_minmax1;
  const uint8_t* flags1;
  const uint8_t* desc2;
  const float* pos2;
  const float* dist_minmax2;
  const uint8_t* flags2;
  float s12;
  float R12[9];   /* row-major */
  float t12[3];
  float th;
  int32_t* match12; /* kf1.n */
  int32_t* nfound;
} orbx_sim3_problem;
orbx_status orbx_search_by_sim3(const orbx_sim3_problem* p, int device); /* host pointers */

/* ORBmatcher::SearchForInitialization(Frame& F1, Frame& F2, vector<cv::Point2f>& vbPrevMatched,
 * vector<int>& vnMatches12, int windowSize) -- src/ORBmatcher.cc:442-587, include/ORBmatcher.h:130
 * (caller Tracking::MonocularInitialization, src/Tracking.cc:711).  f1: keys_un (octave >= 0, angle), desc; f2: keys_un,
 * desc and the grid fields (min_x, min_y, grid_inv_w/h); the other frame fields are unused.
 * prev_matched: f1.n (x, y) pairs, updated in place as vbPrevMatched; match12[i1] = vnMatches12[i1];
 * nnratio = the ORBmatcher's mfNNratio (0.9 in the reference's initializer), check_ori =
 * mbCheckOrientation.  n1, n2 <= ORBX_PROJ_MAX_FEATURES. */
typedef struct {
  orbx_proj_frame f1, f2;
  float* prev_matched;
  int window;
  float nnratio;
  int check_ori;
  int32_t* match12;
  int32_t* nmatches;
} orbx_init_problem;
orbx_status orbx_search_for_initialization(const orbx_init_problem* p, int device); /* host pointers */

/* ORBmatcher::SearchForTriangulation(KeyFrame*, KeyFrame*, cv::Mat F12,
 * vector<pair<size_t,size_t>>&, bOnlyStereo) -- src/ORBmatcher.cc:738-925,
 * include/ORBmatcher.h:134 (caller LocalMapping::CreateNewMapPoints,
 * src/LocalMapping.cc:363).  Each KeyFrame: mvKeysUn, descriptors, mvuRight
 * (NULL = monocular), has_mp[i] = (GetMapPoint(i) != NULL) and its
 * FeatureVector as CSR (as orbx_bow_side).  match12[i] = KF2 index matched to
 * KF1 feature i after the rotation check (-1 none): vMatchedPairs is
 * {(i, match12[i]) : match12[i] >= 0} in ascending i. */
typedef struct {
  int n;
  const orbx_keypoint* keys_un;
  const uint8_t* desc;
  const float* u_right;
  const uint8_t* has_mp;
  int n_nodes;
  const uint32_t* node_id;
  const int32_t* node_off;
  const int32_t* feat;
} orbx_tri_kf;

typedef struct {
  orbx_tri_kf kf1, kf2;
  float F12[9];             /* row-major 3x3 (LocalMapping::ComputeF12) */
  float C1w[3];             /* pKF1->GetCameraCenter() */
  float T2w[16];            /* pKF2 Tcw, row-major */
  float fx, fy, cx, cy;     /* pKF2 intrinsics */
  float scale_factors2[16]; /* pKF2->mvScaleFactors */
  float level_sigma2_2[16]; /* pKF2->mvLevelSigma2 */
  int only_stereo;          /* bOnlyStereo */
  int check_ori;            /* ORBmatcher mbCheckOrientation */
  int32_t* match12;         /* kf1.n */
  int32_t* nmatches;        /* return value */
} orbx_tri_problem;

orbx_status orbx_search_for_triangulation(const orbx_tri_problem* p, int device); /* host pointers */
orbx_status orbx_search_for_triangulation_device(const orbx_tri_problem* problems, int n, void* stream);

/* Optimizer::PoseOptimization(Frame*) -- src/Optimizer.cc:287-528, include/Optimizer.h:71:
 * one SE3 vertex, EdgeSE3ProjectXYZOnlyPose (monocular) / EdgeStereoSE3ProjectXYZOnlyPose
 * (mvuRight >= 0) edges with Huber kernels, four rounds of optimize(10) restarting from
 * mTcw, outlier levels between rounds, kernels dropped after round 2.  The caller gathers
 * one edge per feature with a MapPoint, in feature order (the reference's edge insertion
 * order), exactly as src/Optimizer.cc:318-410 does, and writes back pFrame->SetPose(Tcw_out)
 * and mvbOutlier[feature of edge k] = outlier[k]. */
typedef struct {
  int n;                    /* edges = nInitialCorrespondences */
  const float* obs;         /* n x 3: mvKeysUn[i].pt.x, .y, mvuRight[i] (< 0: monocular edge) */
  const float* Xw;          /* n x 3: MapPoint::GetWorldPos() */
  const float* inv_sigma2;  /* n: mvInvLevelSigma2[mvKeysUn[i].octave] */
  float fx, fy, cx, cy, bf; /* Frame fx, fy, cx, cy, mbf */
  float Tcw[16];            /* pFrame->mTcw on entry, row-major */
  float* Tcw_out;           /* 16: the optimised pose (Converter::toCvMat) */
  uint8_t* outlier;         /* n: mvbOutlier of each edge's feature on return */
  int32_t* ngood;           /* the return value nInitialCorrespondences - nBad */
  int32_t* iterations;      /* optional [4]: LM iterations run by each round's optimize(10) */
  /* Device batches only (NULL otherwise): the edge count and the starting pose as an earlier kernel
   * of the stream left them -- n is then the capacity and n = min(*n_dev, n) */
  const int32_t* n_dev;
  const float* Tcw_dev;     /* 16 floats replacing Tcw */
} orbx_pose_problem;

/* One problem, HOST pointers. */
orbx_status orbx_pose_optimization(const orbx_pose_problem* p, int device);
/* Batched, device-resident: problems[] is a HOST array whose pointers are device
 * pointers; one block per problem runs all four rounds on the GPU (no host round trips). */
orbx_status orbx_pose_optimization_device(const orbx_pose_problem* problems, int n, void* stream);

/* Tracking::TrackReferenceKeyFrame's gather (src/Tracking.cc:910-969) between SearchByBoW(KF, F)
 * and PoseOptimization(&F), on a device batch: PoseOptimization's edge per current-frame feature
 * with a MapPoint, in feature order (src/Optimizer.cc:318-410).  The reference KeyFrame's MapPoints
 * are its stereo points as StereoInitialization creates them (src/Tracking.cc:590-668): feature k has
 * one iff kf_depth[k] > 0, at
 * Frame::UnprojectStereo(k) (src/Frame.cc:823-839: mvKeysUn[k], mRwc*x3Dc+mOw -- cv::gemm with the
 * addend on OpenCV 3.2's small-matrix path: the dot product in float, then a float add) with pose Twc.
 * (KeyFrame::UnprojectStereo, src/KeyFrame.cc:758-780, reads mvKeys instead; the two agree whenever
 * mvKeysUn == mvKeys, i.e. for rectified input without distortion -- KITTI, rectified EuRoC.)  Writes obs / Xw / inv_sigma2 (and the feature of each edge) compacted, and
 * *n_edges -- the inputs of an orbx_pose_problem.  Device pointers; problems[] is a HOST array. */
typedef struct {
  const orbx_keypoint* f_kps;      /* current frame mvKeysUn */
  const float* f_uright;           /* current frame mvuRight (NULL: monocular) */
  const int32_t* f_count;          /* current frame N (device) */
  const int32_t* match;            /* SearchByBoW KF-F output: KF feature per frame feature, or -1 */
  const orbx_keypoint* kf_kps;     /* reference KeyFrame mvKeysUn */
  const float* kf_depth;           /* reference KeyFrame mvDepth */
  float Twc[12];                   /* reference KeyFrame pose, camera to world, row-major 3x4 */
  float fx, fy, cx, cy;            /* KeyFrame intrinsics */
  const float* inv_level_sigma2;   /* current frame mvInvLevelSigma2 (device, per octave) */
  float* obs;                      /* out: capacity N x 3 */
  float* Xw;                       /* out: capacity N x 3 */
  float* inv_sigma2;               /* out: capacity N */
  int32_t* edge_feature;           /* out (optional): capacity N */
  int32_t* n_edges;                /* out: 1 */
} orbx_track_gather;
orbx_status orbx_track_gather_device(const orbx_track_gather* problems, int n, void* stream);

/* The MapPoints StereoInitialization creates (src/Tracking.cc:590-668: one per feature with mvDepth > 0;
 * CreateNewKeyFrame, :1311-1401, and UpdateLastFrame, :971-1040, instead stop at the first point past
 * mThDepth once more than 100 exist, so this models an initial keyframe as the last frame) as the SoA
 * a SearchByProjection problem takes, for the
 * frame's features 0..N-1 (point i = feature i, the frame's descriptors are the points' descriptors):
 *   pos      Frame::UnprojectStereo(i) (src/Frame.cc:823-839) with pose Twc
 *   normal, dist_minmax  MapPoint::UpdateNormalAndDepth with the one observation (src/MapPoint.cc
 *            UpdateNormalAndDepth): PC = pos - Ow, normal = PC / cv::norm(PC), mfMaxDistance =
 *            |PC| * mvScaleFactors[octave], mfMinDistance = mfMaxDistance / mvScaleFactors[nlevels-1]
 *   angle, octave  mvKeysUn[i].angle / .octave (LastFrame.mvKeysUn / mvKeys in SearchByProjection)
 *   flags    bit0 = mvDepth[i] > 0 (a MapPoint, not an outlier), bit1 = 1 (observed by its KeyFrame)
 * Device pointers, capacity cap per frame; problems[] is a HOST array. */
typedef struct {
  const orbx_keypoint* kps;   /* mvKeysUn */
  const float* depth;         /* mvDepth */
  const int32_t* count;       /* N (device) */
  int cap;
  float Twc[12];              /* row-major 3x4: Rwc | Ow */
  float fx, fy, cx, cy;
  int nlevels;
  float scale_factors[16];
  float* pos;                 /* cap x 3 */
  float* normal;              /* cap x 3 */
  float* dist_minmax;         /* cap x 2 */
  float* angle;               /* cap */
  int32_t* octave;            /* cap */
  uint8_t* flags;             /* cap */
} orbx_frame_points;
orbx_status orbx_frame_points_device(const orbx_frame_points* problems, int n, void* stream);

/* Tracking::TrackWithMotionModel + TrackLocalMap bookkeeping between the device launches
 * (src/Tracking.cc:1049-1170, 1403-1468), one block per tracked frame, on the frame's MapPoint
 * table fmap[i] (point index held by feature i, -1 = NULL):
 *   ORBX_TRACK_AFTER_MOTION  fmap = SearchByProjection(F, LastFrame)'s frame_out; lost = nmatches <
 *                            min_matches (:1078-1079); every point now held is marked seen
 *                            (mnLastFrameSeen = current); PoseOptimization edges from fmap
 *   ORBX_TRACK_AFTER_POSE    the edges PoseOptimization flagged outliers leave fmap (:1093-1107);
 *                            lost |= ngood < min_good (nmatchesMap >= 10, :1135); then the inputs of
 *                            SearchLocalPoints: occ (mvpMapPoints, Observations() > 0) and the local
 *                            points' flags (bit0 = a MapPoint not seen in this frame, :1408-1430)
 *   ORBX_TRACK_AFTER_LOCAL   fmap += SearchByProjection(F, local points)'s frame_out; edges again
 * Edges (obs / Xw / inv_sigma2 / edge_feature / n_edges: orbx_pose_problem inputs) are in feature
 * order; a lost frame gets n_edges = 0.  Device pointers; problems[] is a HOST array. */
#define ORBX_TRACK_AFTER_MOTION 0
#define ORBX_TRACK_AFTER_POSE 1
#define ORBX_TRACK_AFTER_LOCAL 2
typedef struct {
  int op;
  int cap;                        /* feature capacity of the frame and of the point table */
  const int32_t* count;           /* current frame N */
  const orbx_keypoint* kps;       /* current frame mvKeysUn */
  const float* u_right;           /* current frame mvuRight (NULL: monocular) */
  const float* inv_level_sigma2;  /* mvInvLevelSigma2 (device, per octave) */
  const int32_t* n_points;        /* points in the table (device) */
  const float* pos;               /* the points' world positions (cap x 3) */
  const uint8_t* flags;           /* the points' flags as orbx_frame_points wrote them */
  const int32_t* frame_out;       /* AFTER_MOTION / AFTER_LOCAL: the search's frame_out */
  const int32_t* nmatches;        /* AFTER_MOTION: the search's return value */
  int min_matches;                /* AFTER_MOTION: 20 */
  const uint8_t* outlier;         /* AFTER_POSE: PoseOptimization's per-edge outlier flags */
  const int32_t* ngood;           /* AFTER_POSE: PoseOptimization's return value */
  int min_good;                   /* AFTER_POSE: 10 */
  int32_t* fmap;                  /* cap */
  uint8_t* seen;                  /* cap (points) */
  uint8_t* local_flags;           /* cap (points): AFTER_POSE output */
  int8_t* occ;                    /* cap (features): AFTER_POSE output */
  int32_t* lost;                  /* 1 */
  float* obs;                     /* cap x 3 */
  float* Xw;                      /* cap x 3 */
  float* inv_sigma2;              /* cap */
  int32_t* edge_feature;          /* cap */
  int32_t* n_edges;               /* 1 */
} orbx_track_step;
orbx_status orbx_track_step_device(const orbx_track_step* problems, int n, void* stream);

/* MapPoint::ComputeDistinctiveDescriptors() -- src/MapPoint.cc:249-320, include/MapPoint.h:83,
 * for a batch of MapPoints.  Point p's observed descriptors (pKF->mDescriptors.row(idx) for
 * each (pKF, idx) of mObservations in map order, bad KeyFrames skipped, :270-276) are rows
 * obs_off[p] .. obs_off[p+1]-1 of desc (32 B each; at most 65535 per point).  best[p] =
 * BestIdx within that list (-1: no observation, mDescriptor unchanged); out_desc (optional,
 * n_points x 32) = the new mDescriptor. */
orbx_status orbx_distinctive_descriptors(const uint8_t* desc, const int32_t* obs_off, int n_points, int32_t* best,
                                         uint8_t* out_desc, int device); /* host pointers */
orbx_status orbx_distinctive_descriptors_device(const uint8_t* desc, const int32_t* obs_off, int n_points,
                                                int32_t* best, uint8_t* out_desc, void* stream);

/* Frame::UndistortKeyPoints() -- src/Frame.cc:471-506, include/Frame.h:242 (cv::undistortPoints
 * with P = K) and the corner pass of Frame::ComputeImageBounds (:508-537, four keypoints at the
 * image corners).  K = mK row-major (float), dist = mDistCoef (k1, k2, p1, p2[, k3]). */
typedef struct {
  float K[9];
  float dist[5];
  int n_dist; /* 4 or 5 */
} orbx_camera;

orbx_status orbx_undistort_keypoints(const orbx_keypoint* keys, int n, const orbx_camera* cam,
                                     orbx_keypoint* keys_un, int device); /* host pointers */
/* Frame batch, device pointers: frame f's keypoints are keys[frame_off[f] .. frame_off[f+1]),
 * at most max_keys each; cams[n_frames] is device-resident. */
orbx_status orbx_undistort_keypoints_device(const orbx_keypoint* keys, const int32_t* frame_off, int n_frames,
                                            int max_keys, const orbx_camera* cams, orbx_keypoint* keys_un,
                                            void* stream);

/* Per-stage HIP-event timers (the g2o G2OBatchStatistics analogue,
 * Thirdparty/g2o/g2o/core/batch_stats.h:38-79).  When enabled, every kernel
 * launch of the handle is bracketed by events on its stream.
 * orbx_profile_read(h, -1, ...) returns the number of stages; for stage >= 0 it
 * fills the accumulated milliseconds, launch count and kernel name. */
orbx_status orbx_profile_enable(orbx_extractor* h, int enable);
orbx_status orbx_profile_reset(orbx_extractor* h);
int orbx_profile_read(orbx_extractor* h, int stage, double* total_ms, long long* launches, const char** name);

/* Library/device info: returns the number of visible HIP devices (<=0: none). */
int orbx_device_count(void);
const char* orbx_version(void);
/* sizeof of a struct of this header by name ("orbx_proj_problem", ...), -1 if unknown: bindings
 * (ctypes, cgo, JNA) check their layouts against it. */
long long orbx_sizeof(const char* type);

#ifdef __cplusplus
}
#endif
#endif /* ORBX_H */
