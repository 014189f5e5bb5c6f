// C++ driver for the SimRank variants beyond TopSim_singleSample, over the
// host mirror (topsim_host.hpp) — the shapes of the reference mains:
//   SimRank.main               (SimRank.java:85-105)    --algo simrank
//   TopSim_singleSample_M      (TopSim_singleSample_M.java:33-54) --algo topsim_m
//   SingleRandomWalk_M         (SingleRandomWalk_M.java:24-42)    --algo srw_m
//   TopSim_doubleSample        (TopSim_doubleSample.java:30-56)   --algo double
//   TopSim_Dev                 (TopSim_Dev.java:31-95)            --algo dev
//   DoubleRandomWalk           (DoubleRandomWalk.java:25-48)      --algo drw
//
//   simrank_variants --graph PATH --V N [--sep ,] --algo A --out PREFIX
//       [--sample N] [--step N] [--M N] [--topk K] [--single S] [--seed S]
//
// simrank writes Print.printByOrderAll(sim, out, 1000, 10); topsim_m / srw_m
// write Print.printByOrder(FixedCacheMap[], out, TOPK); the dense variants
// write the V*V doubles to out.bin (dev: candidates from a naive SimRank).
#include <stdio.h>
#include <stdlib.h>

#include <iostream>
#include <string>
#include <vector>

#include "topsim_host.hpp"

static void dump(const std::string& path, const std::vector<double>& v) {
  FILE* f = fopen(path.c_str(), "wb");
  if (!f || fwrite(v.data(), sizeof(double), v.size(), f) != v.size()) {
    std::cerr << "cannot write " << path << std::endl;
    exit(1);
  }
  fclose(f);
}

int main(int argc, char** argv) {
  std::string graph, algo, out = "out", sep = conf::MyConfiguration::SEPARATOR;
  int V = -1, sample = 1000, step = 3, M = 5, single = 1, device = 0;
  uint64_t seed = 0;
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
    else if (a == "--algo") algo = val();
    else if (a == "--out") out = val();
    else if (a == "--sample") sample = atoi(val().c_str());
    else if (a == "--step") step = atoi(val().c_str());
    else if (a == "--M") M = atoi(val().c_str());
    else if (a == "--topk") conf::MyConfiguration::TOPK = atoi(val().c_str());
    else if (a == "--single") single = atoi(val().c_str());
    else if (a == "--seed") seed = strtoull(val().c_str(), nullptr, 10);
    else if (a == "--device") device = atoi(val().c_str());
    else if (a == "--C") conf::MyConfiguration::C = atof(val().c_str());
    else {
      std::cerr << "unknown flag " << a << std::endl;
      return 2;
    }
  }
  if (graph.empty() || V < 0 || algo.empty()) {
    std::cerr << "usage: " << argv[0] << " --graph PATH --V N --algo simrank|topsim_m|srw_m|double|dev|drw\n";
    return 2;
  }
  conf::MyConfiguration::SEPARATOR = sep;
  try {
    structures::Graph g(graph, V, sep, device);
    if (algo == "simrank") {
      simrank::SimRank sr(g, step);
      sr.compute();
      utils::Print::printByOrderAll(sr.getResult(), V, out, 1000, 10);
    } else if (algo == "topsim_m" || algo == "srw_m") {
      if (algo == "topsim_m") {
        simrank::TopSim_singleSample_M ts(g, M, sample, seed, step);
        ts.compute();
        utils::Print::printByOrder(ts, out, conf::MyConfiguration::TOPK);
      } else {
        simrank::SingleRandomWalk_M ts(g, M, sample, seed, step);
        ts.compute();
        utils::Print::printByOrder(ts, out, conf::MyConfiguration::TOPK);
      }
    } else if (algo == "double") {
      simrank::TopSim_doubleSample ds(g, sample, step, seed);
      ds.compute();
      dump(out + ".bin", ds.getResult());
    } else if (algo == "drw") {
      simrank::DoubleRandomWalk dw(g, sample, step, seed);
      dw.compute();
      dump(out + ".bin", dw.getResult());
    } else if (algo == "dev") {
      simrank::SimRank sr(g);  // candidate matrix
      sr.compute();
      simrank::TopSim_Dev dev(g, sample, step, conf::MyConfiguration::TOPK, single, seed);
      dev.compute(sr.getResult());
      dump(out + ".bin", dev.getResult());
    } else {
      std::cerr << "unknown --algo " << algo << std::endl;
      return 2;
    }
  } catch (const gw::Error& e) {
    std::cerr << "error " << e.code << ": " << e.what() << std::endl;
    return 1;
  }
  return 0;
}
