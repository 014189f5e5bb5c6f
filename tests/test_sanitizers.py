"""CPU: the host code under AddressSanitizer + UndefinedBehaviorSanitizer.

tools/sanitize.sh rebuilds gw_graph_host.cpp / gw_capi.cpp / gw_comm.cpp and
oracle.c with -fsanitize=address,undefined and runs the host-side tests (the
edge-list loaders incl. malformed / truncated / oversized inputs, writers,
C-ABI argument checks, oracle vs golden vectors) with the sanitizer runtimes
preloaded; any report aborts the run.  (The full `-m "not gpu"` suite under
the same build: `bash tools/sanitize.sh`, log in profiles/r02/sanitize_cpu.log.)
"""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


@pytest.mark.skipif(os.environ.get("GW_SANITIZED") == "1", reason="already inside the sanitized run")
@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_host_code_is_clean_under_asan_ubsan(tmp_path):
    env = dict(os.environ)
    log = os.path.join(ROOT, "profiles", "r02", "sanitize_cpu.log")
    keep = open(log).read() if os.path.exists(log) else None
    try:
        p = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize.sh"), "-k", "capi or oracle_golden"],
                           capture_output=True, text=True, timeout=900, env=env, cwd=ROOT)
        out = open(log).read()
    finally:
        if keep is not None:  # the committed log is the full-suite run
            open(log, "w").write(keep)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
    assert " passed" in out and "runtime error:" not in out and "AddressSanitizer" not in out
