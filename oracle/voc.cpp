// oracle/voc.cpp -- TEST INFRASTRUCTURE ONLY (CPU checker; never linked into
// the product).  Restatement of DBoW2's vocabulary text loader and
// transform() as ORB-SLAM2 uses them (Frame::ComputeBoW src/Frame.cc:462-469,
// KeyFrame::ComputeBoW src/KeyFrame.cc:65-78: transform(desc, BowVec,
// FeatVec, 4)).
//
//   loadFromTextFile   Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1338-1420
//   transform (batch)  :1125-1196;  transform (one feature) :1218-1259
//   BowVector::addWeight / addIfNotExist / normalize, FeatureVector::addFeature
//       (BowVector.cpp / FeatureVector.cpp are absent from the reference:
//       upstream DBoW2's published bodies, restated -- std::map order,
//       first insert stores the value, later ones add; L1 norm = sum |v| in
//       word-id order, L2 = sqrt(sum v^2); divide only when norm > 0)
//   FORB::distance     FORB.h:47 (FORB.cpp absent: the bit-count Hamming of
//       ORBmatcher::DescriptorDistance, src/ORBmatcher.cc:1844-1860)
//   FORB::fromString   FORB.h:61 (32 whitespace-separated byte values)
//
// Parity is unpinned against the genuine DBoW2 build (no vocabulary file or
// fixture ships with the reference); tests pin this restatement with a
// literal pure-Python transform on small synthetic vocabularies.
//
// Defined behaviour where the reference has none: the loader stops at the
// first blank line (the reference's `while(!f.eof())` would parse a trailing
// empty line into a node with an uninitialised parent); a descent that ends
// in a leaf above the FeatureVector level files the feature under that leaf
// (the reference leaves the NodeId uninitialised).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <sstream>
#include <string>
#include <vector>

namespace {

struct VNode {
  int parent = -1;
  std::vector<int> children;
  uint8_t desc[32] = {};
  double weight = 0;
  int word_id = -1;
};

struct Voc {
  int k = 0, L = 0, scoring = 0, weighting = 0;
  std::vector<VNode> nodes;
  int n_words = 0;
};

int hamming(const uint8_t* a, const uint8_t* b) {
  int d = 0;
  for (int i = 0; i < 32; i++) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
  return d;
}

// TemplatedVocabulary::transform(feature, word_id, weight, nid, levelsup)
void transform_one(const Voc& v, const uint8_t* f, int levelsup, int* word, double* weight, int* nid) {
  const int nid_level = v.L - levelsup;
  if (nid_level <= 0) *nid = 0;
  int final_id = 0, level = 0;
  do {
    ++level;
    const std::vector<int>& ch = v.nodes[final_id].children;
    final_id = ch[0];
    double best_d = hamming(f, v.nodes[final_id].desc);
    for (size_t i = 1; i < ch.size(); i++) {
      const double d = hamming(f, v.nodes[ch[i]].desc);
      if (d < best_d) {
        best_d = d;
        final_id = ch[i];
      }
    }
    if (level == nid_level) *nid = final_id;
  } while (!v.nodes[final_id].children.empty());
  if (nid_level > level) *nid = final_id;  // leaf above nid_level: the reference leaves nid unset
  *word = v.nodes[final_id].word_id;
  *weight = v.nodes[final_id].weight;
}

}  // namespace

extern "C" {

void* oracle_voc_load(const char* text, long len) {
  Voc* v = new Voc();
  std::string all(text, (size_t)len);
  std::istringstream f(all);
  std::string s;
  std::getline(f, s);
  std::stringstream ss(s);
  int n1 = -1, n2 = -1;
  ss >> v->k >> v->L >> n1 >> n2;
  if (v->k < 0 || v->k > 20 || v->L < 1 || v->L > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3) {
    delete v;
    return nullptr;
  }
  v->scoring = n1;
  v->weighting = n2;
  v->nodes.resize(1);
  while (std::getline(f, s)) {
    if (s.find_first_not_of(" \t\r") == std::string::npos) break;
    std::stringstream sn(s);
    const int nid = (int)v->nodes.size();
    v->nodes.resize(nid + 1);
    int pid = 0, leaf = 0;
    sn >> pid >> leaf;
    if (pid < 0 || pid >= nid) {
      delete v;
      return nullptr;
    }
    v->nodes[nid].parent = pid;
    v->nodes[pid].children.push_back(nid);
    for (int i = 0; i < 32; i++) {
      int b = 0;
      sn >> b;
      v->nodes[nid].desc[i] = (uint8_t)b;
    }
    sn >> v->nodes[nid].weight;
    if (leaf > 0) v->nodes[nid].word_id = v->n_words++;
  }
  return v;
}

void oracle_voc_free(void* h) { delete (Voc*)h; }

void oracle_voc_info(void* h, int* out /* k, L, scoring, weighting, n_nodes, n_words */) {
  const Voc* v = (const Voc*)h;
  out[0] = v->k;
  out[1] = v->L;
  out[2] = v->scoring;
  out[3] = v->weighting;
  out[4] = (int)v->nodes.size();
  out[5] = v->n_words;
}

// TemplatedVocabulary::transform(features, BowVector, FeatureVector, levelsup).
// Outputs in map order: bow (word ascending, value), fv CSR (node ascending,
// features ascending).  Returns 0, or -1 when the vocabulary is empty.
int oracle_voc_transform(void* h, const uint8_t* desc, int n, int levelsup, int* bow_words, double* bow_values,
                         int* n_bow, int* fv_nodes, int* fv_off, int* fv_feat, int* n_fv) {
  const Voc* v = (const Voc*)h;
  *n_bow = *n_fv = 0;
  if (v->nodes.empty() || v->nodes[0].children.empty()) return -1;
  // scoring object: mustNormalize (ScoringObject.h:69-89): DOT_PRODUCT does not
  const bool must = v->scoring != 5;
  const bool l2 = v->scoring == 1;
  std::map<int, double> bow;
  std::map<int, std::vector<int>> fv;
  for (int i = 0; i < n; i++) {
    int word = 0, nid = 0;
    double w = 0;
    transform_one(*v, desc + 32 * (size_t)i, levelsup, &word, &w, &nid);
    if (w > 0) {
      if (v->weighting == 0 || v->weighting == 1) {  // TF_IDF, TF: addWeight
        auto it = bow.find(word);
        if (it != bow.end())
          it->second += w;
        else
          bow.emplace(word, w);
      } else {  // IDF, BINARY: addIfNotExist
        bow.emplace(word, w);
      }
      fv[nid].push_back(i);
    }
  }
  if ((v->weighting == 0 || v->weighting == 1) && !bow.empty() && !must) {
    const double nd = (double)bow.size();
    for (auto& kv : bow) kv.second /= nd;
  }
  if (must) {
    double norm = 0.0;
    if (!l2) {
      for (auto& kv : bow) norm += std::fabs(kv.second);
    } else {
      for (auto& kv : bow) norm += kv.second * kv.second;
      norm = std::sqrt(norm);
    }
    if (norm > 0.0)
      for (auto& kv : bow) kv.second /= norm;
  }
  int b = 0;
  for (auto& kv : bow) {
    bow_words[b] = kv.first;
    bow_values[b] = kv.second;
    b++;
  }
  *n_bow = b;
  int q = 0, o = 0;
  for (auto& kv : fv) {
    fv_nodes[q] = kv.first;
    fv_off[q] = o;
    for (int f : kv.second) fv_feat[o++] = f;
    q++;
  }
  fv_off[q] = o;
  *n_fv = q;
  return 0;
}

}  // extern "C"
