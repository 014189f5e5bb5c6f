// Port of the reference benchmark driver
// DeepSim/TopSimAll/src/benchmark/Test_u_u_TopSim_singleSample.java:25-71 to
// the C++ host mirror (GPU TopSim).  The Java driver hard-codes its inputs in
// MyConfiguration; here they are flags with the same defaults:
//
//   test_u_u_topsim_singlesample --graph blog.txt --V 10313 [--sep ,]
//       [--gold gold_prefix] [--out out_prefix] [--steps 5]
//       [--samples 1000,2500,5000,10000,20000,40000] [--topk 20] [--seed 0]
//       [--sources first:last]
//
// Per (step, sample): new TopSim_singleSample(g, sample, step); compute();
// Print.printByOrder(result, out_..._top{k}_step{s}_sample{n}.txt, TOPK, k);
// and, when --gold is given, Eval.precision(gold.sim.txt, out.sim.txt, ...).
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "topsim_host.hpp"

static std::vector<int> parse_list(const std::string& s) {
  std::vector<int> v;
  std::stringstream ss(s);
  std::string t;
  while (std::getline(ss, t, ',')) v.push_back(atoi(t.c_str()));
  return v;
}

int main(int argc, char** argv) {
  std::string graph, gold, out = "topSimSingle", sep = conf::MyConfiguration::SEPARATOR, srcrange;
  int V = -1, device = 0;
  uint64_t seed = 0;
  std::vector<int> steps = {5};
  std::vector<int> samples = {1000, 2500, 5000, 10000, 20000, 40000};  // :38
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&]() -> std::string {
      if (i + 1 >= argc) {
        std::cerr << "missing value for " << a << std::endl;
        exit(2);
      }
      return argv[++i];
    };
    if (a == "--graph") graph = val();
    else if (a == "--V") V = atoi(val().c_str());
    else if (a == "--sep") { sep = val(); if (sep == "\\t" || sep == "tab") sep = "\t"; }
    else if (a == "--gold") gold = val();
    else if (a == "--out") out = val();
    else if (a == "--steps") steps = parse_list(val());
    else if (a == "--samples") samples = parse_list(val());
    else if (a == "--topk") conf::MyConfiguration::TOPK = atoi(val().c_str());
    else if (a == "--seed") seed = strtoull(val().c_str(), nullptr, 10);
    else if (a == "--device") device = atoi(val().c_str());
    else if (a == "--sources") srcrange = val();
    else if (a == "--C") conf::MyConfiguration::C = atof(val().c_str());
    else {
      std::cerr << "unknown flag " << a << std::endl;
      return 2;
    }
  }
  if (graph.empty() || V < 0) {
    std::cerr << "usage: " << argv[0] << " --graph PATH --V COUNT [--sep ,] [--gold PREFIX] [--out PREFIX]\n";
    return 2;
  }
  conf::MyConfiguration::SEPARATOR = sep;
  conf::MyConfiguration::testTopK = {conf::MyConfiguration::TOPK};
  try {
    structures::Graph g(graph, V, sep, device);  // :46
    std::vector<int32_t> sources;
    if (!srcrange.empty()) {
      int a = atoi(srcrange.c_str()), b = atoi(strchr(srcrange.c_str(), ':') + 1);
      for (int s = a; s < b && s < V; ++s) sources.push_back(s);
    }
    for (int step : steps) {
      for (int sample : samples) {  // :48-52
        simrank::TopSim_singleSample srw(g, sample, step, seed);
        auto t0 = std::chrono::steady_clock::now();
        if (sources.empty()) srw.compute();
        else srw.compute(sources);
        double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        auto st = srw.stats();
        for (int k : conf::MyConfiguration::testTopK) {
          std::cout << "Step:" << step << " Sample:" << sample << " TopK:" << k << " computation done! "
                    << sec << " s, extensions " << st.extensions << ", pair-updates " << st.pair_updates
                    << std::endl;
          std::string outPath = out + "_topSimSingle_top" + std::to_string(k) + "_step" + std::to_string(step) +
                                "_sample" + std::to_string(sample) + ".txt";
          utils::Print::printByOrder(srw, outPath, conf::MyConfiguration::TOPK, k);  // :61
          if (!gold.empty()) {
            std::string prePath = out + "_topSimSingle_top" + std::to_string(k) + "_step" + std::to_string(step) +
                                  "_sample" + std::to_string(sample) + "precision.txt";
            std::cout << "precision: " << utils::Eval::precision(gold + ".sim.txt", outPath + ".sim.txt", prePath, k)
                      << std::endl;  // :64
          }
        }
      }
    }
  } catch (const gw::Error& e) {
    std::cerr << "error " << e.code << ": " << e.what() << std::endl;
    return 1;
  }
  return 0;
}
