// C++ host mirror of the TopSim Java API over the libgraphwalk C ABI.
#include "topsim_host.hpp"

#include <stdio.h>

#include <algorithm>
#include <fstream>
#include <iostream>
#include <limits>
#include <set>
#include <sstream>

namespace gw {
void check(int rc, const gw_graph* g) {
  if (rc == GW_OK) return;
  std::string msg = gw_last_error(g);
  switch (rc) {
    case GW_ERR_IO: throw IOException(rc, msg);
    case GW_ERR_PARSE: throw NumberFormatException(rc, msg);
    case GW_ERR_RANGE: throw ArrayIndexOutOfBoundsException(rc, msg);
    case GW_ERR_DEVICE: throw DeviceException(rc, msg);
    default: throw Error(rc, std::string(gw_strerror(rc)) + ": " + msg);
  }
}
}  // namespace gw

namespace structures {
Graph::Graph(const std::string& graphPath, int V, const std::string& separator, int device)
    : vCount(V), device_(device) {
  gw::check(gw_graph_load_edgelist(graphPath.c_str(), separator.c_str(), GW_SEM_JAVA_MULTI, 0, 0, V, &g_));
  gw_graph_info_t inf;
  gw::check(gw_graph_info(g_, &inf), g_);
  offsets_.resize(inf.n + 1);
  nbrs_.resize(inf.nnz);
  gw::check(gw_graph_export_csr(g_, offsets_.data(), nbrs_.data(), nullptr, nullptr, nullptr), g_);
  eCount = (long)(inf.nnz / 2);  // addEdge increments once per line (Graph.java:56)
  gw::check(gw_graph_to_device(g_, device_), g_);
}

Graph::~Graph() {
  if (g_) gw_graph_free(g_);
}

std::vector<int> Graph::neighbors(int v) const {
  return std::vector<int>(nbrs_.begin() + offsets_[v], nbrs_.begin() + offsets_[v + 1]);
}
}  // namespace structures

namespace simrank {
TopSimBase::TopSimBase(structures::Graph& g, int sample, int step, int variant, uint64_t seed)
    : g_(g), SAMPLE(sample), STEP(step), variant_(variant), seed_(seed) {}

void TopSimBase::compute() {
  std::vector<int32_t> all(g_.getVCount());
  for (int i = 0; i < g_.getVCount(); ++i) all[i] = i;
  compute(all);
}

void TopSimBase::compute(const std::vector<int32_t>& sources) {
  sources_ = sources;
  const int64_t V = g_.getVCount();
  const int64_t ns = (int64_t)sources.size();
  int64_t st[4] = {0, 0, 0, 0};
  dense_ = ns * V * 8 <= dense_limit_bytes;
  if (dense_) {
    sim_.assign(ns * V, 0.0);
    ids_.clear();
    scores_.clear();
    gw::check(gw_topsim_host(g_.handle(), variant_, SAMPLE, STEP, conf::MyConfiguration::C, seed_, sources.data(),
                             ns, 0, nullptr, nullptr, sim_.data(), st),
              g_.handle());
  } else {
    sim_.clear();
    topk_k_ = conf::MyConfiguration::TOPK;
    ids_.assign(ns * topk_k_, -1);
    scores_.assign(ns * topk_k_, 0.0);
    gw::check(gw_topsim_host(g_.handle(), variant_, SAMPLE, STEP, conf::MyConfiguration::C, seed_, sources.data(),
                             ns, topk_k_, ids_.data(), scores_.data(), nullptr, st),
              g_.handle());
  }
  stats_.extensions = st[0];
  stats_.pair_updates = st[1];
  stats_.max_frontier = st[2];
  stats_.walkers = st[3];
}

void TopSimBase::writeText(const std::string& outPath, int topk, const std::string& sep, int decimals) const {
  gw::check(gw_topsim_write_text(g_.handle(), variant_, SAMPLE, STEP, conf::MyConfiguration::C, seed_, sources_.data(),
                                 (int64_t)sources_.size(), topk, outPath.c_str(), sep.c_str(), decimals, nullptr),
            g_.handle());
}

const std::vector<double>& TopSimBase::getResult() const {
  if (!dense_) throw gw::Error(GW_ERR_STATE, "dense result not kept (V too large); use topK()");
  return sim_;
}

void TopSimBase::topK(int k, std::vector<int32_t>& ids, std::vector<double>& scores,
                      const std::vector<int32_t>* sources) const {
  const std::vector<int32_t>& src = sources ? *sources : sources_;
  ids.assign(src.size() * (size_t)k, -1);
  scores.assign(src.size() * (size_t)k, 0.0);
  int64_t st[4];
  gw::check(gw_topsim_host(g_.handle(), variant_, SAMPLE, STEP, conf::MyConfiguration::C, seed_, src.data(),
                           (int64_t)src.size(), k, ids.data(), scores.data(), nullptr, st),
            g_.handle());
}

void TopSimM::compute() {
  const int64_t V = g_.getVCount();
  std::vector<int32_t> src((size_t)V);
  for (int64_t i = 0; i < V; ++i) src[(size_t)i] = (int32_t)i;
  keys_.assign((size_t)(V * capacity), -1);
  vals_.assign((size_t)(V * capacity), 0.f);
  sizes_.assign((size_t)V, 0);
  int64_t st[4] = {0, 0, 0, 0};
  gw::check(gw_topsim_m_host(g_.handle(), variant_, capacity, SAMPLE, STEP, conf::MyConfiguration::C, seed_,
                             src.data(), V, keys_.data(), vals_.data(), sizes_.data(), st),
            g_.handle());
  stats_.extensions = st[0];
  stats_.pair_updates = st[1];
  stats_.max_frontier = st[2];
  stats_.walkers = st[3];
}

void DoubleWalkBase::run(int kind, int sample, int step, int topK, int singleStep, const int32_t* cand) {
  const int64_t V = g_.getVCount();
  sim_.assign((size_t)(V * V), 0.0);
  gw::check(gw_double_sim_host(g_.handle(), kind, sample, step, topK, singleStep, conf::MyConfiguration::C, seed_,
                               cand, sim_.data()),
            g_.handle());
}

void TopSim_Dev::compute(const std::vector<double>& candidate) {
  const int64_t V = g_.getVCount();
  std::vector<int32_t> cand((size_t)(V * singleK), -1);
  gw::check(gw_select_fixed_max_pq(candidate.data(), V, V, singleK, conf::MyConfiguration::MIN, cand.data()));
  run(GW_DOUBLE_DEV, sample_, STEP, singleK, singleStep_, cand.data());
}

void SimRank::compute() {
  const int64_t V = g_.getVCount();
  sim_.assign((size_t)(V * V), 0.0);
  gw::check(gw_simrank_naive_host(g_.handle(), conf::MyConfiguration::C, STEP, sim_.data()), g_.handle());
}

double SimRank::sim(int v, int w) const {
  if (v == w) return 1;
  const int dv = g_.degree(v), dw = g_.degree(w);
  if (dv == 0 || dw == 0) return 0;
  const int64_t V = g_.getVCount();
  double result = 0;
  for (int vn : g_.neighbors(v))
    for (int wn : g_.neighbors(w))
      result += sim_.empty() ? (vn == wn ? 1.0 : 0.0) : sim_[(size_t)vn * V + wn];
  return conf::MyConfiguration::C * result / (dv * dw);
}
}  // namespace simrank

namespace utils {
void Print::printByOrder(const simrank::TopSimBase& sim, const std::string& outPath, int topk, int) {
  const std::string& sep = conf::MyConfiguration::SEPARATOR;
  if (sim.dense()) {
    const auto& rows = sim.getResult();
    gw::check(gw_write_sim_text_dense(outPath.c_str(), rows.data(), sim.sources().data(),
                                      (int64_t)sim.sources().size(), sim.getVCount(), topk, sep.c_str(), 6));
  } else {
    sim.writeText(outPath, topk, sep, 6);  // Java-exact from sparse rows
  }
}

void Print::printByOrder(const std::vector<double>& sim, int64_t V, const std::string& outPath, int topk, int) {
  gw::check(gw_write_sim_text_dense(outPath.c_str(), sim.data(), nullptr, (int64_t)(sim.size() / V), V, topk,
                                    conf::MyConfiguration::SEPARATOR.c_str(), 6));
}

void Print::printByOrder(const simrank::TopSimM& sim, const std::string& outPath, int topk) {
  std::vector<int32_t> sizes((size_t)sim.getVCount());
  for (int v = 0; v < sim.getVCount(); ++v) sizes[(size_t)v] = sim.size(v);
  gw::check(gw_write_sim_text_cachemap(outPath.c_str(), sim.keys().data(), sim.values().data(), sizes.data(),
                                       nullptr, sim.getVCount(), sim.getCapacity(), topk,
                                       conf::MyConfiguration::SEPARATOR.c_str()));
}

void Print::printByOrderAll(const std::vector<double>& sim, int64_t V, const std::string& outPath, int topk, int) {
  gw::check(gw_write_sim_text_dense(outPath.c_str(), sim.data(), nullptr, (int64_t)(sim.size() / V), V, topk,
                                    conf::MyConfiguration::SEPARATOR.c_str(), 7));
}

static std::vector<std::string> split(const std::string& s, const std::string& sep) {
  std::vector<std::string> out;
  size_t b = 0;
  for (;;) {
    size_t p = s.find(sep, b);
    if (p == std::string::npos) {
      out.push_back(s.substr(b));
      break;
    }
    out.push_back(s.substr(b, p - b));
    b = p + sep.size();
  }
  while (!out.empty() && out.back().empty()) out.pop_back();  // Java split drops trailing empties
  return out;
}

// Java's Double.toString (libgraphwalk gw_format_java_double)
static std::string java_double(double v) {
  char buf[64];
  if (gw_format_java_double(v, buf, sizeof buf) != GW_OK) return "NaN";
  return buf;
}

std::string Eval::precision(const std::string& path1, const std::string& path2, const std::string& prePath, int K) {
  (void)K;  // the reference uses MyConfiguration.TOPK (Eval.java:112)
  std::ifstream in1(path1), in2(path2);
  if (!in1 || !in2) throw gw::IOException(GW_ERR_IO, "cannot open " + path1 + " or " + path2);
  std::ofstream out(prePath, std::ios::binary);
  const std::string& sep = conf::MyConfiguration::SEPARATOR;
  const std::string& kv = conf::MyConfiguration::SEPARATOR_KV;
  double sum = 0, mn = std::numeric_limits<double>::max();  // Double.MAX_VALUE (Eval.java:89)
  long total = 0;
  std::string l1, l2;
  while (std::getline(in1, l1)) {
    if (!std::getline(in2, l2)) l2.clear();
    if (!l1.empty() && l1.back() == '\r') l1.pop_back();
    if (!l2.empty() && l2.back() == '\r') l2.pop_back();
    auto t1 = split(l1, sep), t2 = split(l2, sep);
    if (t1.empty() || t2.empty() || t1[0] != t2[0]) {
      std::cout << "error !" << (t1.empty() ? "" : t1[0]) << "\t" << (t2.empty() ? "" : t2[0]) << std::endl;
      continue;
    }
    std::set<std::string> s1, s2;
    for (size_t i = 1; i < t1.size(); ++i) {
      auto p = split(t1[i], kv);
      if (p.size() >= 2 && std::stod(p[1]) >= conf::MyConfiguration::MIN) s1.insert(p[0]);
    }
    for (size_t i = 1; i < t2.size(); ++i) {
      auto p = split(t2[i], kv);
      if (p.size() >= 2 && std::stod(p[1]) >= conf::MyConfiguration::MIN) s2.insert(p[0]);
    }
    const int realK = std::min<int>(conf::MyConfiguration::TOPK, (int)s1.size());
    double pre;
    if (realK == 0) {
      pre = 1.0;
    } else {
      int inter = 0;
      for (auto& x : s1) inter += s2.count(x) ? 1 : 0;
      pre = 1.0 * inter / realK;
    }
    sum += pre;
    out << t1[0] << sep << java_double(pre) << "\r\n";  // Java "" + double (Eval.java:118)
    ++total;
    mn = std::min(mn, pre);
  }
  const double avg = sum / (double)total;  // NaN for an empty gold file, as in Java (0.0 / 0)
  std::cout << "total nodes:" << total << "\tavg precision: " << java_double(avg)
            << "\tmin pre: " << java_double(mn) << std::endl;  // min stays Double.MAX_VALUE when empty
  return java_double(avg);
}
}  // namespace utils
