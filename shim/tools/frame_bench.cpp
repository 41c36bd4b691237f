// frame_bench.cpp -- per-frame latency of the drop-in path as ORB-SLAM2 drives it: one stereo
// Frame per TrackStereo call (Examples/Stereo/stereo_kitti.cc:82-99 times exactly that call on the
// Tracking thread), i.e. the shim's Frame stereo constructor -- two extraction threads on two
// ORBextractor handles (src/Frame.cc:80-84), UndistortKeyPoints, ComputeStereoMatches -- on
// host images, with results returned to host vectors.  Extractors are built once, as Tracking does.
//
// usage: frame_bench FILE W H N_UNIQUE N_FRAMES WARMUP NFEATURES BF FX [mono]
//   FILE holds N_UNIQUE stereo pairs (L then R, W*H bytes each); frame f uses pair f % N_UNIQUE.
//   mono (BASELINE config 1, TUM): FILE holds N_UNIQUE images and each call is one
//   ORBextractor::operator()(image, cv::Mat(), keypoints, descriptors) -- the extraction Frame's
//   monocular constructor makes (src/Frame.cc:186-205 -> ExtractORB, :273-279); BF/FX unused.
// Prints one JSON line: per-frame milliseconds (after WARMUP) and the keypoint / match counts.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ORBextractor.h"
#include "orbx_shim.h"
#include "Objects.h"

using namespace ORB_SLAM2;

int main(int argc, char** argv) {
  if (argc < 10) {
    std::fprintf(stderr, "usage: frame_bench FILE W H N_UNIQUE N_FRAMES WARMUP NFEATURES BF FX\n");
    return 2;
  }
  const int W = std::atoi(argv[2]), H = std::atoi(argv[3]), U = std::atoi(argv[4]);
  const int NF = std::atoi(argv[5]), WU = std::atoi(argv[6]), nfeat = std::atoi(argv[7]);
  const float bf = (float)std::atof(argv[8]), fx = (float)std::atof(argv[9]);
  const bool mono = argc > 10 && std::strcmp(argv[10], "mono") == 0;
  std::vector<uint8_t> data((size_t)U * (mono ? 1 : 2) * W * H);
  FILE* f = std::fopen(argv[1], "rb");
  if (!f || std::fread(data.data(), 1, data.size(), f) != data.size()) {
    std::fprintf(stderr, "cannot read %s\n", argv[1]);
    return 2;
  }
  std::fclose(f);
  try {
    if (mono) {
      ORBextractor ex(nfeat, 1.2f, 8, 20, 7);  // Tracking's mono extractor (src/Tracking.cc:120,125)
      std::vector<double> ms;
      long long kp = 0;
      std::vector<cv::KeyPoint> keys;
      cv::Mat desc;
      for (int i = 0; i < WU + NF; i++) {
        cv::Mat im(H, W, CV_8U, data.data() + (size_t)(i % U) * W * H);
        const auto t0 = std::chrono::steady_clock::now();
        ex(im, cv::Mat(), keys, desc);
        const auto t1 = std::chrono::steady_clock::now();
        if (i >= WU) {
          ms.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
          kp += (long long)keys.size();
        }
      }
      std::vector<double> s = ms;
      std::sort(s.begin(), s.end());
      double mean = 0;
      for (double v : ms) mean += v;
      mean /= ms.size();
      std::printf("{\"frames\": %d, \"median_ms\": %.4f, \"p90_ms\": %.4f, \"mean_ms\": %.4f, \"min_ms\": %.4f, "
                  "\"keypoints_per_frame\": %.1f}\n",
                  NF, s[s.size() / 2], s[std::min(s.size() - 1, (size_t)(0.9 * s.size()))], mean, s.front(),
                  (double)kp / NF);
      return 0;
    }
    // "threads": the reference's two extraction threads + the matcher instead of one orbx_frame_stereo
    gOrbxFrameStereoFused = !(argc > 10 && std::strcmp(argv[10], "threads") == 0);
    ORBextractor exL(nfeat, 1.2f, 8, 20, 7), exR(nfeat, 1.2f, 8, 20, 7);  // Tracking's (src/Tracking.cc:120-126)
    cv::Mat K(3, 3, CV_32F), dist(4, 1, CV_32F);
    std::memset(K.data, 0, 36);
    std::memset(dist.data, 0, 16);
    K.at<float>(0, 0) = fx;
    K.at<float>(1, 1) = fx;
    K.at<float>(0, 2) = W / 2.f;
    K.at<float>(1, 2) = H / 2.f;
    K.at<float>(2, 2) = 1.f;
    std::vector<double> ms;
    long long kp = 0, matched = 0;
    for (int i = 0; i < WU + NF; i++) {
      const int u = i % U;
      cv::Mat imL(H, W, CV_8U, data.data() + (size_t)(2 * u) * W * H);
      cv::Mat imR(H, W, CV_8U, data.data() + (size_t)(2 * u + 1) * W * H);
      const auto t0 = std::chrono::steady_clock::now();
      Frame F(imL, imR, &exL, &exR, K, dist, bf, 35.f * bf / fx);
      const auto t1 = std::chrono::steady_clock::now();
      if (i >= WU) {
        ms.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
        kp += F.N;
        for (float v : F.mvuRight) matched += v >= 0;
      }
    }
    std::vector<double> s = ms;
    std::sort(s.begin(), s.end());
    const double med = s[s.size() / 2], p90 = s[std::min(s.size() - 1, (size_t)(0.9 * s.size()))];
    double mean = 0;
    for (double v : ms) mean += v;
    mean /= ms.size();
    std::printf("{\"frames\": %d, \"median_ms\": %.4f, \"p90_ms\": %.4f, \"mean_ms\": %.4f, \"min_ms\": %.4f, "
                "\"keypoints_per_frame\": %.1f, \"matches_per_frame\": %.1f}\n",
                NF, med, p90, mean, s.front(), (double)kp / NF, (double)matched / NF);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "exception: %s\n", e.what());
    return 3;
  }
  return 0;
}
