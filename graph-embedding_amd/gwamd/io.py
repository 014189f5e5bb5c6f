"""Reference file formats on the walk / SimRank boundary.

* walks out:  DeepSim/src/main.py:237-243 `save_list` — every id followed by
  '\\t' (trailing tab included), one walk per line.
* walks in:   DeepSim/src/main.py:245-254 `read_list` — strip, split on '\\t',
  ids stay strings.
* sims in:    DeepSim/src/main.py:83-107 `read_simrank` — the consumer of the
  TopSim `.sim.txt` file: per line, `v,id:val,...`; pairs with val <= 1e-8
  are dropped; (id, val) kept as strings.
"""
import ctypes

import numpy as np

from . import _lib as C


def save_walks(graph, path, walks, lens=None):
    """Write dense-id walks (numpy [W, L] int32, -1 padded) of a GWGraph in
    the save_list format (labels)."""
    walks = np.ascontiguousarray(walks, np.int32)
    ln = None if lens is None else np.ascontiguousarray(lens, np.int32)
    C.check(C.lib().gw_write_walks_text(graph.handle, str(path).encode(), C.ptr(walks), C.ptr(ln),
                                        walks.shape[0], walks.shape[1]))


def save_list(walks, file_path):
    """save_list for python lists of labels (DeepSim/src/main.py:237-243)."""
    with open(file_path, "w") as f:
        for walk in walks:
            for t in walk:
                f.write(str(t))
                f.write("\t")
            f.write("\n")


def read_list(file_path):
    """DeepSim/src/main.py:245-254."""
    walks = []
    with open(file_path, "r") as f:
        for line in f.readlines():
            line = line.strip()
            walks.append([w for w in line.split("\t")])
    return walks


def read_simrank(path):
    """DeepSim/src/main.py:83-107 (the `.sim.txt` consumer)."""
    simrank = []
    with open(path) as f:
        for line in f.readlines():
            words = line.split(",")
            sim = []
            for i in range(1, len(words)):
                if i == len(words) - 1:
                    words[i] = words[i][:-1]
                ts = words[i].split(":")
                if float(ts[1]) <= 0.00000001:
                    continue
                sim.append((ts[0], ts[1]))
            simrank.append(sim)
    return simrank


__all__ = ["save_walks", "save_list", "read_list", "read_simrank", "ctypes"]
