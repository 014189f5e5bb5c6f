#!/bin/bash
# ASan + UBSan run of the host code: the edge-list parsers, graph
# builders, writers and C-ABI argument checks (gw_graph_host.cpp, gw_capi.cpp,
# gw_comm.cpp) and the oracle (oracle.c) compiled with
# -fsanitize=address,undefined, linked with the unchanged HIP objects (device
# code is not sanitized: GPU ASan is not available on this pool), then the CPU
# test suite (pytest -m "not gpu") under the sanitizer runtimes.
#   bash tools/sanitize.sh [pytest args...]     (log: profiles/r02/sanitize_cpu.log)
set -e
cd "$(dirname "$0")/.."
python graph-embedding_amd/build.py > /dev/null
B=graph-embedding_amd/build_san
mkdir -p $B
SAN="-O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined"
for f in gw_graph_host gw_capi gw_comm; do
  g++ $SAN -std=c++17 -fPIC -fopenmp -ffp-contract=off -Wall -Wno-unused-function -Iinclude -I/opt/rocm/include \
      -D__HIP_PLATFORM_AMD__ -c graph-embedding_amd/csrc/$f.cpp -o $B/$f.o &
done
gcc $SAN -fPIC -fopenmp -ffp-contract=off -std=gnu11 -shared -o $B/liboracle_san.so oracle/oracle.c -lm &
wait
g++ -shared -fsanitize=address,undefined -o $B/libgraphwalk_san.so $B/gw_graph_host.o $B/gw_capi.o $B/gw_comm.o \
    graph-embedding_amd/build/*.hip.o -L/opt/rocm/lib -lamdhip64 -fopenmp -ldl -Wl,-rpath,/opt/rocm/lib
ASAN_RT=$(gcc -print-file-name=libasan.so)
UBSAN_RT=$(gcc -print-file-name=libubsan.so)
mkdir -p profiles/r02
{
  echo "# tools/sanitize.sh $(date -u +%FT%TZ): $(g++ --version | head -1)"
  echo "# libs: $B/libgraphwalk_san.so (host objects: $SAN), $B/liboracle_san.so"
  LD_PRELOAD=$ASAN_RT:$UBSAN_RT ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 \
    UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 GW_SANITIZED=1 \
    GW_LIB=$PWD/$B/libgraphwalk_san.so GW_ORACLE_LIB=$PWD/$B/liboracle_san.so \
    python -m pytest tests -q -m "not gpu" -p no:cacheprovider "$@" 2>&1
} | tee profiles/r02/sanitize_cpu.log | tail -5
rm -rf $B  # (16 MB of instrumented objects: not shipped with the tree)
grep -q " passed" profiles/r02/sanitize_cpu.log && ! grep -q "ERROR: AddressSanitizer\|runtime error:" profiles/r02/sanitize_cpu.log
