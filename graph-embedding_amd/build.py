"""Build libgraphwalk.so in-tree (hipcc for gfx950 + g++ for host code).

    python graph-embedding_amd/build.py [--force] [--verbose]

Output: graph-embedding_amd/gwamd/libgraphwalk.so (git-ignored, travels to
the GPU box with the repo snapshot).  No CMake: the product is a handful of
translation units.
"""
import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "build")
OUT = os.path.join(HERE, "gwamd", "libgraphwalk.so")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("GW_OFFLOAD_ARCH", "gfx950")

HIP_SRCS = ["gw_n2v.hip", "gw_n2v_bitset.hip", "gw_topsim.hip", "gw_simrank.hip", "gw_topsim_m.hip", "gw_topsim_d.hip"]
CXX_SRCS = ["gw_graph_host.cpp", "gw_capi.cpp", "gw_comm.cpp"]
HEADERS = ["gw_internal.h", "gw_philox.h", "gw_device_common.h"]

HIPCC_FLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
    "-ffp-contract=off",        # bitwise parity with the host restatement
    "-munsafe-fp-atomics",      # native global/LDS f64 atomic add
    "-Wno-unused-result",
    f"-I{os.path.join(ROOT, 'include')}",
]
CXX_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-fopenmp", "-ffp-contract=off",
             "-Wall", "-Wno-unused-function", f"-I{os.path.join(ROOT, 'include')}",
             f"-I{ROCM}/include", "-D__HIP_PLATFORM_AMD__"]


def _newer(obj, deps):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"build step failed: {' '.join(cmd[:3])} ...")
    return r


def build(force=False, verbose=False, diag=False):
    """diag=True: the timing-experiment build (-DGW_DIAG: GW_DIAG_* knobs, some of
    which return wrong walks on purpose) into gwamd/libgraphwalk_diag.so; the
    release library never carries those paths."""
    BUILD = os.path.join(HERE, "build_diag" if diag else "build")
    OUT = os.path.join(HERE, "gwamd", "libgraphwalk_diag.so" if diag else "libgraphwalk.so")
    hip_flags = HIPCC_FLAGS + (["-DGW_DIAG"] if diag else [])
    cxx_flags = CXX_FLAGS + (["-DGW_DIAG"] if diag else [])
    os.makedirs(BUILD, exist_ok=True)
    hdrs = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(ROOT, "include", "graphwalk.h")]
    jobs = []
    objs = []
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    for s in HIP_SRCS:
        src = os.path.join(CSRC, s)
        obj = os.path.join(BUILD, s + ".o")
        objs.append(obj)
        if force or _newer(obj, [src] + hdrs + [__file__]):
            jobs.append([hipcc] + hip_flags + ["-c", src, "-o", obj])
    cxx = shutil.which("g++") or "g++"
    for s in CXX_SRCS:
        src = os.path.join(CSRC, s)
        obj = os.path.join(BUILD, s + ".o")
        objs.append(obj)
        if force or _newer(obj, [src] + hdrs + [__file__]):
            jobs.append([cxx] + cxx_flags + ["-c", src, "-o", obj])
    with cf.ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        list(ex.map(lambda c: _run(c, verbose), jobs))
    if force or jobs or _newer(OUT, objs):
        _run([cxx, "-shared", "-o", OUT] + objs +
             [f"-L{ROCM}/lib", "-lamdhip64", "-fopenmp", "-ldl", f"-Wl,-rpath,{ROCM}/lib",
              "-Wl,--no-undefined"], verbose)
    if diag:
        return OUT
    # JNI shim for a Java host (north_star): only where a JDK provides jni.h
    jh = os.environ.get("JAVA_HOME")
    if jh and os.path.exists(os.path.join(jh, "include", "jni.h")):
        jni_src = os.path.join(HERE, "jni", "graphwalk_jni.c")
        jni_out = os.path.join(HERE, "gwamd", "libgraphwalk_jni.so")
        if force or _newer(jni_out, [jni_src, OUT, os.path.join(ROOT, "include", "graphwalk.h")]):
            _run(["gcc", "-O2", "-shared", "-fPIC", "-Wall", f"-I{jh}/include", f"-I{jh}/include/linux",
                  f"-I{os.path.join(ROOT, 'include')}", jni_src, f"-L{os.path.dirname(OUT)}", "-lgraphwalk",
                  "-Wl,-rpath,$ORIGIN", "-o", jni_out], verbose)
    # C++ host mirror of the Java TopSim API + the benchmark driver binary
    host = os.path.join(HERE, "host")
    bindir = os.path.join(HERE, "bin")
    os.makedirs(bindir, exist_ok=True)
    hsrc = [os.path.join(host, "topsim_host.cpp")]
    hhdr = [os.path.join(host, "topsim_host.hpp"), os.path.join(ROOT, "include", "graphwalk.h")]
    for drv in ["test_u_u_topsim_singlesample", "simrank_variants"]:
        exe = os.path.join(bindir, drv)
        dsrc = os.path.join(host, drv + ".cpp")
        if force or _newer(exe, hsrc + hhdr + [dsrc, OUT, __file__]):
            _run([cxx, "-O2", "-std=c++17", "-Wall", f"-I{os.path.join(ROOT, 'include')}", "-o", exe, dsrc] + hsrc +
                 [f"-L{os.path.dirname(OUT)}", "-lgraphwalk", "-Wl,-rpath,$ORIGIN/../gwamd",
                  f"-L{ROCM}/lib", "-lamdhip64", f"-Wl,-rpath,{ROCM}/lib"], verbose)
    return OUT


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--diag", action="store_true", help="timing-experiment library (-DGW_DIAG)")
    a = ap.parse_args()
    print(build(force=a.force, verbose=a.verbose, diag=a.diag))
