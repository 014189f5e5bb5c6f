"""Kernel-trace duration of the exact dispatch each bench line timed.

    python tools/kt_lines.py KERNEL_TRACE_CSV BENCH_JSON OUT_JSON

Lines whose `roofline.pmc_match` carries `nth` (bench.py ts_dispatch: the
ordinal of the timed dispatch among the process's dispatches of that kernel,
e.g. the 18 config-3 sweep points, several of which share one kernel) get the
rocprofv3 duration, scratch and VGPRs of that dispatch, next to the bench's
own HIP-event kernel_ms.  The trace must come from the same bench command
(tools/gpu_run.sh kt).
"""
import csv
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import lines, norm  # noqa: E402


def main():
    path, bjson, out = sys.argv[1:4]
    trace = list(csv.DictReader(open(path)))
    bench = [json.loads(ln) for ln in open(bjson) if ln.startswith("{")][-1]
    res = {}
    for roof in lines(bench):
        m = roof.get("pmc_match") or {}
        if m.get("nth") is None:
            continue
        rx = re.compile(m["kernel"])
        disp = sorted((int(r["Dispatch_Id"]), r) for r in trace if rx.match(norm(r["Kernel_Name"])))
        got = []
        for k in m["nth"]:
            if k < len(disp):
                r = disp[k][1]
                got.append({"ms": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6,
                            "scratch_bytes": int(r["Scratch_Size"]), "vgprs": int(r["VGPR_Count"]),
                            "grid": int(r["Grid_Size_X"]), "dispatch_id": int(r["Dispatch_Id"])})
        key = f"{roof.get('pmc_tag')}#{m['nth']}"
        res[key] = {"kernel": roof.get("kernel"), "bench_kernel_ms": roof.get("kernel_ms"), "dispatches": got}
        if got:
            print(f"{key:48s} rocprof {got[0]['ms']:9.3f} ms  bench {roof.get('kernel_ms') or 0:9.3f} ms  "
                  f"scratch {got[0]['scratch_bytes']} B  vgprs {got[0]['vgprs']}  {roof.get('kernel')}")
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
