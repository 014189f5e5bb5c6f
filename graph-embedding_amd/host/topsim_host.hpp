// C++ host mirror of the reference's TopSim Java API
// (DeepSim/TopSimAll/src/{conf,structures,simrank,utils}), over the
// libgraphwalk C ABI (include/graphwalk.h).  Same class names, argument
// meaning and error behaviour, so a Java driver such as
// benchmark/Test_u_u_TopSim_singleSample.java:25-71 translates line by line
// (see test_u_u_topsim_singlesample.cpp).  All compute runs on the GPU.
#pragma once
#include <stdint.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/graphwalk.h"

namespace conf {
// MyConfiguration.java:16-22
struct MyConfiguration {
  static inline std::string SEPARATOR = ",";
  static inline const std::string SEPARATOR_KV = ":";
  static inline int TOPK = 20;
  static inline double MIN = 0.000000001;
  static inline double C = 0.6;
  static inline std::vector<int> testTopK = {20};
};
}  // namespace conf

namespace gw {
// Java exceptions on this path, as C++ types carrying the GW_* code.
struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};
struct IOException : Error { using Error::Error; };
struct NumberFormatException : Error { using Error::Error; };
struct ArrayIndexOutOfBoundsException : Error { using Error::Error; };
struct DeviceException : Error { using Error::Error; };
void check(int rc, const gw_graph* g = nullptr);
}  // namespace gw

namespace structures {
// structures.Graph (Graph.java:16-93): undirected multigraph, insertion order.
class Graph {
 public:
  Graph(const std::string& graphPath, int V, const std::string& separator = conf::MyConfiguration::SEPARATOR,
        int device = 0);
  ~Graph();
  Graph(const Graph&) = delete;
  Graph& operator=(const Graph&) = delete;
  int degree(int v) const { return (int)(offsets_[v + 1] - offsets_[v]); }
  std::vector<int> neighbors(int v) const;
  int getVCount() const { return vCount; }
  long getECount() const { return eCount; }
  gw_graph* handle() const { return g_; }
  int device() const { return device_; }

 private:
  gw_graph* g_ = nullptr;
  int vCount = 0;
  long eCount = 0;
  int device_ = 0;
  std::vector<int64_t> offsets_;
  std::vector<int32_t> nbrs_;
};
}  // namespace structures

namespace simrank {
// Shared by TopSim_singleSample / TopSim_Enumerate / SingleRandomWalk.
class TopSimBase {
 public:
  TopSimBase(structures::Graph& g, int sample, int step, int variant, uint64_t seed);
  virtual ~TopSimBase() = default;
  // compute(): every source (TopSim_singleSample.java:47-54).  Keeps dense
  // rows when V*V doubles fit `dense_limit_bytes`, else top-TOPK rows.
  virtual void compute();
  void compute(const std::vector<int32_t>& sources);
  // double[][] getResult() (:235-237); throws when only top-k rows exist.
  const std::vector<double>& getResult() const;
  // sparse top-k rows: ids[src*k + j] (-1 padded), scores likewise
  void topK(int k, std::vector<int32_t>& ids, std::vector<double>& scores,
            const std::vector<int32_t>* sources = nullptr) const;
  // compute() + Print.printByOrder(sim, outPath, topk) for rows too large to
  // keep dense: the same Philox walks as sparse rows, FixedMaxPQ replayed
  // exactly (gw_topsim_write_text)
  void writeText(const std::string& outPath, int topk, const std::string& sep, int decimals) const;
  gw_topsim_stats_t stats() const { return stats_; }
  const std::vector<int32_t>& sources() const { return sources_; }
  bool dense() const { return dense_; }
  int topk_rows_k() const { return topk_k_; }
  const std::vector<int32_t>& topk_ids() const { return ids_; }
  const std::vector<double>& topk_scores() const { return scores_; }
  int getVCount() const { return g_.getVCount(); }
  static inline int64_t dense_limit_bytes = int64_t(1) << 30;

 protected:
  structures::Graph& g_;
  int SAMPLE, STEP, variant_;
  uint64_t seed_;
  std::vector<int32_t> sources_;
  std::vector<double> sim_;
  std::vector<int32_t> ids_;
  std::vector<double> scores_;
  int topk_k_ = 0;
  bool dense_ = false;
  gw_topsim_stats_t stats_{};
};

class TopSim_singleSample : public TopSimBase {
 public:
  TopSim_singleSample(structures::Graph& g, int sample, int step, uint64_t seed = 0)
      : TopSimBase(g, sample, step, GW_TOPSIM_SINGLE_SAMPLE, seed) {}
};
using TopSim_Basic = TopSim_singleSample;  // TopSim_Basic.java: same algorithm

class TopSim_Enumerate : public TopSimBase {
 public:
  TopSim_Enumerate(structures::Graph& g, int sample, int step, uint64_t seed = 0)
      : TopSimBase(g, sample, step, GW_TOPSIM_ENUMERATE, seed) {}
  void compute() override { TopSimBase::compute(std::vector<int32_t>{0}); }  // :46-53 walks node 0
};

class SingleRandomWalk : public TopSimBase {
 public:
  SingleRandomWalk(structures::Graph& g, int sample, int step, uint64_t seed = 0)
      : TopSimBase(g, sample, step, GW_TOPSIM_SINGLE_RW, seed) {}
};

// simrank.TopSim_singleSample_M / SingleRandomWalk_M: FixedCacheMap rows
// (capacity = TOPK * M), iteration order (ascending), STEP = 5 as the reference.
class TopSimM {
 public:
  TopSimM(structures::Graph& g, int M, int sample, int variant, uint64_t seed, int step)
      : g_(g), capacity(conf::MyConfiguration::TOPK * M), SAMPLE(sample), STEP(step), variant_(variant), seed_(seed) {}
  void compute();  // every vertex
  int getCapacity() const { return capacity; }
  int getVCount() const { return g_.getVCount(); }
  // row v: size(v) entries keys()[v*capacity + i], values()[...] ascending
  int size(int v) const { return sizes_[v]; }
  const std::vector<int32_t>& keys() const { return keys_; }
  const std::vector<float>& values() const { return vals_; }
  gw_topsim_stats_t stats() const { return stats_; }

 private:
  structures::Graph& g_;
  int capacity, SAMPLE, STEP, variant_;
  uint64_t seed_;
  std::vector<int32_t> keys_, sizes_;
  std::vector<float> vals_;
  gw_topsim_stats_t stats_{};
};
struct TopSim_singleSample_M : TopSimM {  // TopSim_singleSample_M.java:33-54
  TopSim_singleSample_M(structures::Graph& g, int M, int sample, uint64_t seed = 0, int step = 5)
      : TopSimM(g, M, sample, GW_TOPSIM_SINGLE_SAMPLE, seed, step) {}
};
struct SingleRandomWalk_M : TopSimM {  // SingleRandomWalk_M.java:24-42
  SingleRandomWalk_M(structures::Graph& g, int M, int sample, uint64_t seed = 0, int step = 5)
      : TopSimM(g, M, sample, GW_TOPSIM_SINGLE_RW, seed, step) {}
};

// Double-walk variants (§8f-4): dense V*V results, row-major.
class DoubleWalkBase {
 public:
  const std::vector<double>& getResult() const { return sim_; }
  int getVCount() const { return g_.getVCount(); }

 protected:
  DoubleWalkBase(structures::Graph& g, uint64_t seed) : g_(g), seed_(seed) {}
  void run(int kind, int sample, int step, int topK, int singleStep, const int32_t* cand);
  structures::Graph& g_;
  uint64_t seed_;
  std::vector<double> sim_;
};
// simrank.TopSim_doubleSample (TopSim_doubleSample.java:30-197)
class TopSim_doubleSample : public DoubleWalkBase {
 public:
  TopSim_doubleSample(structures::Graph& g, int sample, int step, uint64_t seed = 0)
      : DoubleWalkBase(g, seed), SAMPLE(sample), STEP(step) {}
  void compute() { run(GW_DOUBLE_SAMPLE, SAMPLE, STEP, 0, 0, nullptr); }

 private:
  int SAMPLE, STEP;
};
// simrank.DoubleRandomWalk (DoubleRandomWalk.java:25-95)
class DoubleRandomWalk : public DoubleWalkBase {
 public:
  DoubleRandomWalk(structures::Graph& g, int sample, int step, uint64_t seed = 0)
      : DoubleWalkBase(g, seed), SAMPLE(sample), STEP(step) {}
  void compute() { run(GW_DOUBLE_RANDOM_WALK, SAMPLE, STEP, 0, 0, nullptr); }

 private:
  int SAMPLE, STEP;
};
// simrank.TopSim_Dev (TopSim_Dev.java:31-95): compute(candidate V*V)
class TopSim_Dev : public DoubleWalkBase {
 public:
  TopSim_Dev(structures::Graph& g, int sample, int step, int topK, int singleStep, uint64_t seed = 0)
      : DoubleWalkBase(g, seed), sample_(sample), STEP(step), singleK(topK), singleStep_(singleStep) {}
  void compute(const std::vector<double>& candidate);

 private:
  int sample_, STEP, singleK, singleStep_;
};

// simrank.SimRank (SimRank.java:15-82): naive all-pairs SimRank on the GPU.
class SimRank {
 public:
  explicit SimRank(structures::Graph& g, int step = 3) : g_(g), STEP(step) {}  // STEP = 3 (:16)
  void compute();                                                            // :36-57 + postProcess
  double sim(int v, int w) const;                                            // :67-77, one round
  const std::vector<double>& getResult() const { return sim_; }              // :79-81, V*V row-major
  int getVCount() const { return g_.getVCount(); }

 private:
  structures::Graph& g_;
  int STEP;
  std::vector<double> sim_;
};
}  // namespace simrank

namespace utils {
struct Print {
  // Print.printByOrder(double[][] sim, outPath, topk, testTopK) (Print.java:25-53)
  static void printByOrder(const simrank::TopSimBase& sim, const std::string& outPath, int topk, int testTopK);
  static void printByOrder(const std::vector<double>& sim, int64_t V, const std::string& outPath, int topk,
                           int testTopK);
  // Print.printByOrder(FixedCacheMap[] sim, outPath, topk) (Print.java:94-124)
  static void printByOrder(const simrank::TopSimM& sim, const std::string& outPath, int topk);
  // Print.printByOrderAll (Print.java:55-84): same with "%.7f"
  static void printByOrderAll(const std::vector<double>& sim, int64_t V, const std::string& outPath, int topk,
                              int testTopK);
};
struct Eval {
  // Eval.precision(path1, path2, prePath, K) (Eval.java:81-131)
  static std::string precision(const std::string& path1, const std::string& path2, const std::string& prePath,
                               int K);
};
}  // namespace utils
