#!/bin/bash
# Build an A/B variant of libgraphwalk.so: one replaced HIP translation unit
# (+ optional extra hipcc flags) linked with the in-tree objects of the rest.
#   tools/build_variant.sh <name> <replaced unit, e.g. gw_n2v_bitset> <variant.hip> [extra hipcc flags...]
# Output: abv/<name>.so (git-ignored, travels to the GPU box; select with GW_LIB=abv/<name>.so)
set -e
cd "$(dirname "$0")/.."
name=$1; base=$2; src=$3; shift 3
mkdir -p abv
ROCM=${ROCM_PATH:-/opt/rocm}
# the variant source may live anywhere: compile it with csrc on the include path
$ROCM/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -munsafe-fp-atomics -Wno-unused-result \
  -Iinclude -Igraph-embedding_amd/csrc "$@" -c "$src" -o abv/$name.o
objs=$(ls graph-embedding_amd/build/*.o | grep -v "/${base}.hip.o")
g++ -shared -o abv/$name.so abv/$name.o $objs -L$ROCM/lib -lamdhip64 -fopenmp -Wl,-rpath,$ROCM/lib -Wl,--no-undefined
echo abv/$name.so
