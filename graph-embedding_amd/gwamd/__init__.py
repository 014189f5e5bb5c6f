"""gwamd — MI355X-native node2vec walk generation and TopSim SimRank.

Host-side mirror of the reference interfaces over the libgraphwalk C ABI
(include/graphwalk.h):

* `gwamd.node2vec`  — node2vec/src/node2vec.py (Graph, alias_setup, alias_draw)
* `gwamd.topsim`    — DeepSim/TopSimAll structures.Graph, TopSim_singleSample,
                      TopSim_Enumerate, SingleRandomWalk, SimRank (naive),
                      Print.printByOrder/printByOrderAll,
                      Eval.precision
* `gwamd.graph`     — owning handle over a gw_graph (edgelist / networkx /
                      R-MAT constructors)
* `gwamd.io`        — save_list / read_list / read_simrank formats
"""
from . import _lib
from ._lib import device_count, lib
from .graph import GWGraph

__all__ = ["GWGraph", "device_count", "lib", "_lib"]
__version__ = "0.1.0"
