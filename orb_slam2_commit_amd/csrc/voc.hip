// voc.hip -- DBoW2 TemplatedVocabulary<FORB> (ORBVocabulary) on the GPU:
// the text-format loader and transform(features, BowVector, FeatureVector,
// levelsup) that Frame::ComputeBoW / KeyFrame::ComputeBoW call with
// levelsup = 4 (src/Frame.cc:462-469, src/KeyFrame.cc:65-78).
//
//   loadFromTextFile  Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1338-1420
//                     (host parse; nodes as SoA in HBM, children as CSR)
//   k_voc_descend     one thread per descriptor: transform(feature, word,
//                     weight, nid, levelsup) :1218-1259 -- at each level the
//                     Hamming distance (FORB::distance) to every child, first
//                     strict minimum wins, the node at level L - levelsup is
//                     the FeatureVector key
//   k_voc_build       one block per descriptor set: BowVector (std::map by
//                     word: addWeight / addIfNotExist in feature order, then
//                     L1/L2 normalize or the TF mean) and FeatureVector
//                     (std::map by node: features in order) :1125-1196, as
//                     ascending-key sorts in LDS; the norm is summed by one
//                     thread in word order, so values are bit-identical to
//                     the std::map restatement (oracle/voc.cpp).
// BowVector.cpp / FeatureVector.cpp / FORB.cpp are absent from the reference;
// their upstream DBoW2 bodies are restated (oracle/voc.cpp header).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/orbx.h"
#include "orbx_scratch.h"

namespace orbx {

constexpr int kVocBuildThreads = 512;
constexpr int kVocMaxSet = 8192;  // descriptors per set (LDS sort); ORB-SLAM2 frames carry <= nfeatures

struct VocDev {
  const uint64_t* desc;     // n_nodes x 4
  const double* weight;     // n_nodes
  const int* word_id;       // n_nodes (-1: not a word)
  const int* child_off;     // n_nodes + 1
  const int* child;         // children in file order
  int L, scoring, weighting;
};

__device__ __forceinline__ int hamming4(const uint64_t f[4], const uint64_t* d) {
  return __popcll(f[0] ^ d[0]) + __popcll(f[1] ^ d[1]) + __popcll(f[2] ^ d[2]) + __popcll(f[3] ^ d[3]);
}

// set_cnt != nullptr: strided sets -- output row i is row r = i % cap of set s = i / cap, read
// from input row s * stride + r, live while r < set_cnt[s * cnt_step] (the device batch layout:
// each image's descriptors at a fixed capacity stride with its count on the device)
__global__ __launch_bounds__(256) void k_voc_descend(VocDev V, const uint64_t* __restrict__ feats, int total,
                                                     int levelsup, int* __restrict__ word, double* __restrict__ weight,
                                                     int* __restrict__ nid, const int32_t* __restrict__ set_cnt,
                                                     int cap, long long stride, int cnt_step) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  size_t row = (size_t)i;
  if (set_cnt) {
    const int s = i / cap, r = i - s * cap;
    if (r >= set_cnt[(size_t)s * cnt_step]) return;
    row = (size_t)s * stride + r;
  }
  const uint64_t f[4] = {feats[4 * row], feats[4 * row + 1], feats[4 * row + 2], feats[4 * row + 3]};
  const int nid_level = V.L - levelsup;
  int nv = 0, node = 0, level = 0;
  for (;;) {
    ++level;
    const int c0 = V.child_off[node], c1 = V.child_off[node + 1];
    int best = V.child[c0];
    int best_d = hamming4(f, V.desc + 4 * (size_t)best);
    for (int c = c0 + 1; c < c1; c++) {
      const int id = V.child[c];
      const int d = hamming4(f, V.desc + 4 * (size_t)id);
      if (d < best_d) {  // the reference compares doubles of these ints: same order
        best_d = d;
        best = id;
      }
    }
    if (level == nid_level) nv = best;
    node = best;
    if (V.child_off[node + 1] == V.child_off[node]) break;  // leaf
  }
  if (nid_level > level) nv = node;  // leaf above the FeatureVector level (reference: unset)
  word[i] = V.word_id[node];
  weight[i] = V.weight[node];
  nid[i] = nv;
}

// ascending bitonic sort of P (power of two) keys in LDS
__device__ void bitonic_asc(uint64_t* k, int P) {
  for (int size = 2; size <= P; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < P / 2; t += kVocBuildThreads) {
        const int lo = 2 * t - (t & (stride - 1)), hi = lo + stride;
        const bool up = (lo & size) == 0;
        const uint64_t a = k[lo], b = k[hi];
        if (up ? a > b : a < b) {
          k[lo] = b;
          k[hi] = a;
        }
      }
      __syncthreads();
    }
}

// Exclusive block scan of one int per thread (kVocBuildThreads); returns the
// thread's offset and *total.
__device__ int block_scan_excl(int v, int* sh, int* total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[wv] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0;
    for (int w = 0; w < kVocBuildThreads / 64; w++) {
      const int t = sh[w];
      sh[w] = s;
      s += t;
    }
    sh[kVocBuildThreads / 64] = s;
  }
  __syncthreads();
  const int r = sh[wv] + x - v;
  *total = sh[kVocBuildThreads / 64];
  __syncthreads();
  return r;
}

// Sorts (key_hi << 32 | feature) of the features with weight > 0 and marks
// the first entry of every key run; returns the number of valid entries and
// the run starts in rs[0..n_runs).
__device__ void sort_runs(uint64_t* keys, int* rs, int* sh, const int* key_hi, const double* w, int n, int P,
                          int* n_valid, int* n_runs) {
  for (int i = threadIdx.x; i < P; i += kVocBuildThreads)
    keys[i] = (i < n && w[i] > 0) ? ((uint64_t)(uint32_t)key_hi[i] << 32 | (uint32_t)i) : ~0ull;
  __syncthreads();
  bitonic_asc(keys, P);
  // per thread a contiguous chunk of P / threads entries
  const int per = (P + kVocBuildThreads - 1) / kVocBuildThreads;
  const int a = threadIdx.x * per, b = min(a + per, P);
  int cnt_valid = 0, cnt_runs = 0;
  for (int i = a; i < b; i++) {
    if (keys[i] == ~0ull) continue;
    cnt_valid++;
    cnt_runs += i == 0 || (keys[i] >> 32) != (keys[i - 1] >> 32);
  }
  int tv = 0, tr = 0;
  (void)block_scan_excl(cnt_valid, sh, &tv);
  int off = block_scan_excl(cnt_runs, sh, &tr);
  for (int i = a; i < b; i++)
    if (keys[i] != ~0ull && (i == 0 || (keys[i] >> 32) != (keys[i - 1] >> 32))) rs[off++] = i;
  __syncthreads();
  *n_valid = tv;
  *n_runs = tr;
}

struct VocSetOut {
  uint32_t* bow_words;
  double* bow_values;
  int32_t* n_bow;
  uint32_t* fv_nodes;
  int32_t* fv_off;
  int32_t* fv_feat;
  int32_t* n_fv;
};

__global__ __launch_bounds__(kVocBuildThreads) void k_voc_build(VocDev V, const int32_t* __restrict__ set_off,
                                                                const int* __restrict__ word,
                                                                const double* __restrict__ weight,
                                                                const int* __restrict__ nid, VocSetOut O,
                                                                const int32_t* __restrict__ set_cnt, int cap,
                                                                int cnt_step) {
  extern __shared__ __attribute__((aligned(16))) uint64_t keys[];  // P keys, then P run starts (int)
  __shared__ int sh[kVocBuildThreads / 64 + 1];
  const int s = blockIdx.x;
  const int o = set_cnt ? s * cap : set_off[s];
  const int n = set_cnt ? min(set_cnt[(size_t)s * cnt_step], cap) : set_off[s + 1] - o;
  int P = 1;
  while (P < n) P <<= 1;
  int* rs = reinterpret_cast<int*>(keys + P);
  const double* w = weight + o;
  // ---- BowVector
  int m = 0, nr = 0;
  sort_runs(keys, rs, sh, word + o, w, n, P, &m, &nr);
  const bool tf = V.weighting == 0 || V.weighting == 1;  // TF_IDF / TF: addWeight; IDF / BINARY: addIfNotExist
  // run values in registers (runs r = tid + q * threads), then staged in LDS
  // over the consumed keys for the sequential norm
  constexpr int kRuns = kVocMaxSet / kVocBuildThreads;
  double vr[kRuns];
  uint32_t wr[kRuns];
#pragma unroll
  for (int q = 0; q < kRuns; q++) {
    const int r = threadIdx.x + q * kVocBuildThreads;
    vr[q] = 0.0;
    wr[q] = 0;
    if (r < nr) {
      const int a = rs[r], b = r + 1 < nr ? rs[r + 1] : m;
      double v = w[(uint32_t)keys[a]];
      if (tf)
        for (int j = a + 1; j < b; j++) v += w[(uint32_t)keys[j]];
      vr[q] = v;
      wr[q] = (uint32_t)(keys[a] >> 32);
    }
  }
  __syncthreads();
  double* vals = reinterpret_cast<double*>(keys);  // nr <= P
#pragma unroll
  for (int q = 0; q < kRuns; q++) {
    const int r = threadIdx.x + q * kVocBuildThreads;
    if (r < nr) vals[r] = vr[q];
  }
  __syncthreads();
  const bool must = V.scoring != 5, l2 = V.scoring == 1;  // ScoringObject.h:69-89
  __shared__ double scale;
  if (threadIdx.x == 0) {
    double norm = 0.0;
    if (must) {  // BowVector::normalize: the map order is word order; 8 LDS loads in flight
      int r = 0;
      for (; r + 8 <= nr; r += 8) {
        double t[8];
#pragma unroll
        for (int u = 0; u < 8; u++) t[u] = l2 ? vals[r + u] * vals[r + u] : fabs(vals[r + u]);
#pragma unroll
        for (int u = 0; u < 8; u++) norm += t[u];
      }
      for (; r < nr; r++) norm += l2 ? vals[r] * vals[r] : fabs(vals[r]);
      if (l2) norm = sqrt(norm);
    } else if (tf && nr > 0) {
      norm = (double)nr;  // the TF mean when no normalisation follows
    }
    scale = norm;
    O.n_bow[s] = nr;
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kRuns; q++) {
    const int r = threadIdx.x + q * kVocBuildThreads;
    if (r < nr) {
      O.bow_words[o + r] = wr[q];
      O.bow_values[o + r] = scale > 0.0 ? vr[q] / scale : vr[q];
    }
  }
  __syncthreads();
  // ---- FeatureVector
  sort_runs(keys, rs, sh, nid + o, w, n, P, &m, &nr);
  int32_t* foff = O.fv_off + o + s;
  for (int r = threadIdx.x; r < nr; r += kVocBuildThreads) {
    O.fv_nodes[o + r] = (uint32_t)(keys[rs[r]] >> 32);
    foff[r] = rs[r];
  }
  for (int j = threadIdx.x; j < m; j += kVocBuildThreads) O.fv_feat[o + j] = (int32_t)(uint32_t)keys[j];
  if (threadIdx.x == 0) {
    foff[nr] = m;
    O.n_fv[s] = nr;
  }
}

}  // namespace orbx

// ------------------------------------------------------------------ host / C ABI
struct orbx_voc {
  int device = 0;
  hipStream_t st = nullptr;
  int k = 0, L = 0, scoring = 0, weighting = 0, n_nodes = 0, n_words = 0;
  bool empty = true;
  void* d_mem = nullptr;
  orbx::VocDev dev{};
  // No per-handle scratch: ORB-SLAM2 shares one vocabulary between the Tracking and LocalMapping
  // threads (Frame::ComputeBoW / KeyFrame::ComputeBoW), so every call brings its own -- a scratch
  // lease (host API) or stream-ordered allocations on the caller's stream (device API).
};

namespace {

inline size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

// one integer token; false at end of line
bool next_int(const char*& p, const char* e, long* out) {
  while (p < e && (*p == ' ' || *p == '\t' || *p == '\r')) p++;
  if (p >= e || *p == '\n') return false;
  char* q = nullptr;
  const long v = std::strtol(p, &q, 10);
  if (q == p) return false;
  p = q;
  *out = v;
  return true;
}
bool next_double(const char*& p, const char* e, double* out) {
  while (p < e && (*p == ' ' || *p == '\t' || *p == '\r')) p++;
  if (p >= e || *p == '\n') return false;
  std::string tok;
  while (p < e && *p != ' ' && *p != '\t' && *p != '\r' && *p != '\n') tok.push_back(*p++);
  char* q = nullptr;
  *out = std::strtod(tok.c_str(), &q);  // correctly rounded, as istream >> double
  return q != tok.c_str();
}

#define VOC_CHECK(x)                            \
  do {                                          \
    if ((x) != hipSuccess) return ORBX_ERR_HIP; \
  } while (0)

}  // namespace

extern "C" {

orbx_status orbx_voc_load_text(const char* text, size_t len, int device, orbx_voc** out) {
  if (!text || !out) return ORBX_ERR_ARG;
  *out = nullptr;
  const char* p = text;
  const char* e = text + len;
  long hdr[4];
  for (int i = 0; i < 4; i++)
    if (!next_int(p, e, &hdr[i])) return ORBX_ERR_ARG;
  if (hdr[0] < 0 || hdr[0] > 20 || hdr[1] < 1 || hdr[1] > 10 || hdr[2] < 0 || hdr[2] > 5 || hdr[3] < 0 || hdr[3] > 3)
    return ORBX_ERR_ARG;  // "Vocabulary loading failure: This is not a correct text file!"
  while (p < e && *p != '\n') p++;
  if (p < e) p++;
  std::vector<int> parent(1, -1), word(1, -1);
  std::vector<uint64_t> desc(4, 0);
  std::vector<double> weight(1, 0.0);
  int n_words = 0;
  while (p < e) {
    const char* line = p;
    while (p < e && *p != '\n') p++;
    const char* le = p;
    if (p < e) p++;
    const char* q = line;
    long pid = 0, leaf = 0;
    if (!next_int(q, le, &pid)) break;  // blank line ends the node list (defined; see oracle/voc.cpp)
    const int nid = (int)parent.size();
    if (!next_int(q, le, &leaf) || pid < 0 || pid >= nid) return ORBX_ERR_ARG;
    uint8_t d[32];
    for (int i = 0; i < 32; i++) {
      long b = 0;
      if (!next_int(q, le, &b)) return ORBX_ERR_ARG;
      d[i] = (uint8_t)b;
    }
    double wv = 0;
    if (!next_double(q, le, &wv)) return ORBX_ERR_ARG;
    parent.push_back((int)pid);
    uint64_t d64[4];
    std::memcpy(d64, d, 32);
    desc.insert(desc.end(), d64, d64 + 4);
    weight.push_back(wv);
    word.push_back(leaf > 0 ? n_words++ : -1);
  }
  const int n = (int)parent.size();
  // children CSR in file order (m_nodes[pid].children.push_back(nid))
  std::vector<int> child_off(n + 1, 0), child(std::max(n - 1, 1), 0);
  for (int i = 1; i < n; i++) child_off[parent[i] + 1]++;
  for (int i = 0; i < n; i++) child_off[i + 1] += child_off[i];
  {
    std::vector<int> fill(child_off.begin(), child_off.end() - 1);
    for (int i = 1; i < n; i++) child[fill[parent[i]]++] = i;
  }
  int nd = 0;
  if (hipGetDeviceCount(&nd) != hipSuccess || nd <= 0) return ORBX_ERR_NODEV;
  if (device < 0 || device >= nd) return ORBX_ERR_ARG;
  if (hipSetDevice(device) != hipSuccess) return ORBX_ERR_HIP;
  orbx_voc* v = new (std::nothrow) orbx_voc();
  if (!v) return ORBX_ERR_HIP;
  v->device = device;
  v->k = (int)hdr[0];
  v->L = (int)hdr[1];
  v->scoring = (int)hdr[2];
  v->weighting = (int)hdr[3];
  v->n_nodes = n;
  v->n_words = n_words;
  v->empty = child_off[1] == 0;
  const size_t b_desc = a256(32 * (size_t)n), b_w = a256(8 * (size_t)n), b_word = a256(4 * (size_t)n),
               b_off = a256(4 * (size_t)(n + 1)), b_child = a256(4 * child.size());
  std::vector<uint8_t> stage(b_desc + b_w + b_word + b_off + b_child);
  std::memcpy(stage.data(), desc.data(), 32 * (size_t)n);
  std::memcpy(stage.data() + b_desc, weight.data(), 8 * (size_t)n);
  std::memcpy(stage.data() + b_desc + b_w, word.data(), 4 * (size_t)n);
  std::memcpy(stage.data() + b_desc + b_w + b_word, child_off.data(), 4 * (size_t)(n + 1));
  std::memcpy(stage.data() + b_desc + b_w + b_word + b_off, child.data(), 4 * child.size());
  hipError_t he = hipStreamCreateWithFlags(&v->st, hipStreamNonBlocking);
  if (he == hipSuccess) he = hipMalloc(&v->d_mem, stage.size());
  if (he == hipSuccess) he = hipMemcpy(v->d_mem, stage.data(), stage.size(), hipMemcpyHostToDevice);
  if (he != hipSuccess) {
    if (v->d_mem) (void)hipFree(v->d_mem);
    if (v->st) (void)hipStreamDestroy(v->st);
    delete v;
    return ORBX_ERR_HIP;
  }
  uint8_t* base = (uint8_t*)v->d_mem;
  v->dev.desc = (const uint64_t*)base;
  v->dev.weight = (const double*)(base + b_desc);
  v->dev.word_id = (const int*)(base + b_desc + b_w);
  v->dev.child_off = (const int*)(base + b_desc + b_w + b_word);
  v->dev.child = (const int*)(base + b_desc + b_w + b_word + b_off);
  v->dev.L = v->L;
  v->dev.scoring = v->scoring;
  v->dev.weighting = v->weighting;
  *out = v;
  return ORBX_OK;
}

orbx_status orbx_voc_destroy(orbx_voc* v) {
  if (!v) return ORBX_ERR_ARG;
  (void)hipSetDevice(v->device);
  if (v->d_mem) (void)hipFree(v->d_mem);
  if (v->st) (void)hipStreamDestroy(v->st);
  delete v;
  return ORBX_OK;
}

orbx_status orbx_voc_info(const orbx_voc* v, int32_t info[6]) {
  if (!v || !info) return ORBX_ERR_ARG;
  info[0] = v->k;
  info[1] = v->L;
  info[2] = v->scoring;
  info[3] = v->weighting;
  info[4] = v->n_nodes;
  info[5] = v->n_words;
  return ORBX_OK;
}

orbx_status orbx_voc_transform(orbx_voc* v, const uint8_t* desc, const int32_t* set_off, int n_sets, int levelsup,
                               uint32_t* bow_words, double* bow_values, int32_t* n_bow, uint32_t* fv_nodes,
                               int32_t* fv_off, int32_t* fv_feat, int32_t* n_fv) {
  if (!v || !set_off || n_sets < 0 || !n_bow || !n_fv) return ORBX_ERR_ARG;
  if (n_sets == 0) return ORBX_OK;
  const int total = set_off[n_sets];
  if (set_off[0] != 0 || total < 0) return ORBX_ERR_ARG;
  int maxn = 0;
  for (int s = 0; s < n_sets; s++) {
    const int n = set_off[s + 1] - set_off[s];
    if (n < 0) return ORBX_ERR_ARG;
    maxn = std::max(maxn, n);
  }
  if (maxn > orbx::kVocMaxSet) return ORBX_ERR_SIZE;
  if (total > 0 && (!desc || !bow_words || !bow_values || !fv_nodes || !fv_feat)) return ORBX_ERR_ARG;
  if (!fv_off) return ORBX_ERR_ARG;
  if (v->empty || total == 0) {  // transform() returns empty vectors
    for (int s = 0; s < n_sets; s++) {
      n_bow[s] = n_fv[s] = 0;
      fv_off[set_off[s] + s] = 0;
    }
    return ORBX_OK;
  }
  if (hipSetDevice(v->device) != hipSuccess) return ORBX_ERR_HIP;
  // device scratch: desc | set_off | word | weight | nid | outputs
  const size_t nt = (size_t)total, ns = (size_t)n_sets;
  const size_t b_desc = a256(32 * nt), b_soff = a256(4 * (ns + 1)), b_word = a256(4 * nt), b_w = a256(8 * nt),
               b_nid = a256(4 * nt), b_bw = a256(4 * nt), b_bv = a256(8 * nt), b_nb = a256(4 * ns),
               b_fn = a256(4 * nt), b_fo = a256(4 * (nt + ns)), b_ff = a256(4 * nt), b_nf = a256(4 * ns);
  const size_t need = b_desc + b_soff + b_word + b_w + b_nid + b_bw + b_bv + b_nb + b_fn + b_fo + b_ff + b_nf;
  // a per-call lease (own stream + arena): concurrent callers never share scratch
  orbx::ScratchGuard g(v->device);
  if (!g.l) return ORBX_ERR_HIP;
  VOC_CHECK(g.l->reserve(need, 0));
  uint8_t* w = g.l->d;
  uint64_t* d_desc = (uint64_t*)w;
  w += b_desc;
  int32_t* d_soff = (int32_t*)w;
  w += b_soff;
  int* d_word = (int*)w;
  w += b_word;
  double* d_wt = (double*)w;
  w += b_w;
  int* d_nid = (int*)w;
  w += b_nid;
  orbx::VocSetOut O;
  O.bow_words = (uint32_t*)w;
  w += b_bw;
  O.bow_values = (double*)w;
  w += b_bv;
  O.n_bow = (int32_t*)w;
  w += b_nb;
  O.fv_nodes = (uint32_t*)w;
  w += b_fn;
  O.fv_off = (int32_t*)w;
  w += b_fo;
  O.fv_feat = (int32_t*)w;
  w += b_ff;
  O.n_fv = (int32_t*)w;
  hipStream_t st = g.l->st;
  VOC_CHECK(hipMemcpyAsync(d_desc, desc, 32 * nt, hipMemcpyHostToDevice, st));
  VOC_CHECK(hipMemcpyAsync(d_soff, set_off, 4 * (ns + 1), hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(orbx::k_voc_descend, dim3((total + 255) / 256), dim3(256), 0, st, v->dev, d_desc, total,
                     levelsup, d_word, d_wt, d_nid, nullptr, 1, 1LL, 1);
  int P = 1;
  while (P < maxn) P <<= 1;
  const size_t smem = (size_t)P * 8 + (size_t)P * 4;
  if (smem > 64 * 1024)
    VOC_CHECK(hipFuncSetAttribute((const void*)orbx::k_voc_build, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)smem));
  hipLaunchKernelGGL(orbx::k_voc_build, dim3(n_sets), dim3(orbx::kVocBuildThreads), smem, st, v->dev, d_soff,
                     d_word, d_wt, d_nid, O, nullptr, 0, 1);
  VOC_CHECK(hipGetLastError());
  VOC_CHECK(hipMemcpyAsync(bow_words, O.bow_words, 4 * nt, hipMemcpyDeviceToHost, st));
  VOC_CHECK(hipMemcpyAsync(bow_values, O.bow_values, 8 * nt, hipMemcpyDeviceToHost, st));
  VOC_CHECK(hipMemcpyAsync(n_bow, O.n_bow, 4 * ns, hipMemcpyDeviceToHost, st));
  VOC_CHECK(hipMemcpyAsync(fv_nodes, O.fv_nodes, 4 * nt, hipMemcpyDeviceToHost, st));
  VOC_CHECK(hipMemcpyAsync(fv_off, O.fv_off, 4 * (nt + ns), hipMemcpyDeviceToHost, st));
  VOC_CHECK(hipMemcpyAsync(fv_feat, O.fv_feat, 4 * nt, hipMemcpyDeviceToHost, st));
  VOC_CHECK(hipMemcpyAsync(n_fv, O.n_fv, 4 * ns, hipMemcpyDeviceToHost, st));
  VOC_CHECK(hipStreamSynchronize(st));
  return ORBX_OK;
}

orbx_status orbx_voc_transform_device(orbx_voc* v, const uint8_t* d_desc, int cap, long long stride,
                                      const int32_t* d_count, int count_step, int n_sets, int levelsup,
                                      uint32_t* d_bow_words, double* d_bow_values, int32_t* d_n_bow,
                                      uint32_t* d_fv_nodes, int32_t* d_fv_off, int32_t* d_fv_feat, int32_t* d_n_fv,
                                      void* stream) {
  if (!v || n_sets < 0 || cap <= 0 || stride < cap || count_step < 1 || (n_sets > 0 && (!d_desc || !d_count)))
    return ORBX_ERR_ARG;
  if (n_sets == 0) return ORBX_OK;
  if (!d_bow_words || !d_bow_values || !d_n_bow || !d_fv_nodes || !d_fv_off || !d_fv_feat || !d_n_fv)
    return ORBX_ERR_ARG;
  if (cap > orbx::kVocMaxSet) return ORBX_ERR_SIZE;
  if (v->empty) return ORBX_ERR_STATE;
  if (hipSetDevice(v->device) != hipSuccess) return ORBX_ERR_HIP;
  hipStream_t st = stream == ORBX_STREAM_NULL ? (hipStream_t)0 : stream ? (hipStream_t)stream : v->st;
  const size_t nt = (size_t)n_sets * cap;
  if (nt > (size_t)0x7FFFFFFF) return ORBX_ERR_SIZE;
  const size_t need = a256(4 * nt) + a256(8 * nt) + a256(4 * nt);  // word | weight | nid
  // stream-ordered scratch on the caller's stream: freed after k_voc_build in stream order, so a
  // later call (any thread, any stream) can never overwrite what a queued build still reads
  int P = 1;
  while (P < cap) P <<= 1;
  const size_t smem = (size_t)P * 8 + (size_t)P * 4;
  if (smem > 64 * 1024)
    VOC_CHECK(hipFuncSetAttribute((const void*)orbx::k_voc_build, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)smem));
  uint8_t* w = nullptr;
  VOC_CHECK(hipMallocAsync((void**)&w, need, st));
  int* d_word = (int*)w;
  double* d_wt = (double*)(w + a256(4 * nt));
  int* d_nid = (int*)(w + a256(4 * nt) + a256(8 * nt));
  orbx::VocSetOut O{d_bow_words, d_bow_values, d_n_bow, d_fv_nodes, d_fv_off, d_fv_feat, d_n_fv};
  hipLaunchKernelGGL(orbx::k_voc_descend, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, st, v->dev,
                     (const uint64_t*)d_desc, (int)nt, levelsup, d_word, d_wt, d_nid, d_count, cap, stride,
                     count_step);
  hipLaunchKernelGGL(orbx::k_voc_build, dim3(n_sets), dim3(orbx::kVocBuildThreads), smem, st, v->dev, nullptr,
                     d_word, d_wt, d_nid, O, d_count, cap, count_step);
  const hipError_t e1 = hipGetLastError();
  const hipError_t e2 = hipFreeAsync(w, st);
  return (e1 == hipSuccess && e2 == hipSuccess) ? ORBX_OK : ORBX_ERR_HIP;
}

}  // extern "C"
