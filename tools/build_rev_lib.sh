#!/bin/bash
# Build libgraphwalk from the sources of a git revision into
# graph-embedding_amd/gwamd/ab/libgraphwalk_<rev>.so (for in-process A/B with
# tools/ab_inproc.py; the .so travels to the GPU box, git ignores it).
#   tools/build_rev_lib.sh <rev>
set -e
rev=$1
root=$(cd "$(dirname "$0")/.." && pwd)
work=/tmp/gw_rev_$rev
rm -rf "$work" && mkdir -p "$work"
git -C "$root" archive "$rev" graph-embedding_amd/csrc include | tar -x -C "$work"
out="$root/graph-embedding_amd/gwamd/ab"
mkdir -p "$out"
flags="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -munsafe-fp-atomics -Wno-unused-result -I$work/include"
objs=""
for s in gw_n2v gw_n2v_bitset gw_topsim gw_simrank gw_topsim_m gw_topsim_d; do
  /opt/rocm/bin/hipcc $flags -c "$work/graph-embedding_amd/csrc/$s.hip" -o "$work/$s.o" &
  objs="$objs $work/$s.o"
done
for s in gw_graph_host gw_capi gw_comm; do
  g++ -O3 -std=c++17 -fPIC -fopenmp -ffp-contract=off -I$work/include -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ \
      -c "$work/graph-embedding_amd/csrc/$s.cpp" -o "$work/$s.o" &
  objs="$objs $work/$s.o"
done
wait
g++ -shared -o "$out/libgraphwalk_$rev.so" $objs -L/opt/rocm/lib -lamdhip64 -fopenmp -ldl -Wl,-rpath,/opt/rocm/lib -Wl,--no-undefined
echo "$out/libgraphwalk_$rev.so"
