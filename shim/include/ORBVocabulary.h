// ORBVocabulary.h -- drop-in ORB_SLAM2::ORBVocabulary (include/ORBVocabulary.h:
// DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB>) for the members the hot path uses:
//   loadFromTextFile(filename)                  TemplatedVocabulary.h:1338-1420 (the ORBvoc.txt format)
//   transform(features, BowVector, FeatureVector, levelsup)   TemplatedVocabulary.h:1125-1196
// The tree lives on the MI355X (orbx_voc_*); transform descends every descriptor there.
#pragma once
#include <string>
#include <vector>

#include "Objects.h"
#include "opencv_min.hpp"
#include "orbx.h"
#include "orbx_shim.h"

namespace ORB_SLAM2 {

class ORBVocabulary {
 public:
  // the reference's `new ORBVocabulary()` (System.cc); the tree goes to device gOrbxDevice when loaded
  ORBVocabulary() = default;
  ~ORBVocabulary();
  ORBVocabulary(const ORBVocabulary&) = delete;
  ORBVocabulary& operator=(const ORBVocabulary&) = delete;

  // false when the file cannot be read; a malformed file throws std::runtime_error
  bool loadFromTextFile(const std::string& filename);
  bool loadFromText(const std::string& text);
  // features: one 1x32 CV_8U row per feature (Converter::toDescriptorVector of mDescriptors)
  void transform(const std::vector<cv::Mat>& features, DBoW2::BowVector& v, DBoW2::FeatureVector& fv,
                 int levelsup) const;
  // the same for the rows of an N x 32 descriptor matrix (no per-row Mats)
  void transform(const cv::Mat& descriptors, DBoW2::BowVector& v, DBoW2::FeatureVector& fv, int levelsup) const;

  unsigned int size() const { return (unsigned)mInfo[5]; }  // number of words
  int getBranchingFactor() const { return mInfo[0]; }
  int getDepthLevels() const { return mInfo[1]; }
  bool empty() const { return mpGpu == nullptr || mInfo[5] == 0; }
  orbx_voc* gpu() const { return mpGpu; }

 private:
  orbx_voc* mpGpu = nullptr;
  int32_t mInfo[6] = {0, 0, 0, 0, 0, 0};
};

}  // namespace ORB_SLAM2
