"""Per-(kernel, grid) dispatch statistics from a rocprofv3 kernel trace.

    python tools/kt_summary.py KERNEL_TRACE_CSV OUT_JSON [NAME_REGEX]

rocprofv3 --stats averages every dispatch of a kernel; bench.py launches the
same walk kernel on two graphs (the headline R-MAT-20 and the north_star
10M-vertex graph), so this splits the trace by grid size: each workload's
average duration can be set beside bench.py's HIP-event kernel_ms.
"""
import csv
import json
import re
import sys


def main():
    path, out = sys.argv[1:3]
    rx = re.compile(sys.argv[3] if len(sys.argv) > 3 else r"k_walk|k_topsim|k_sr_|k_bs_")
    acc = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        if not rx.search(name):
            continue
        key = f"{name} grid={r['Grid_Size_X']}x{r['Grid_Size_Y']} wg={r['Workgroup_Size_X']}"
        ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        e = acc.setdefault(key, {"calls": 0, "total_ns": 0, "min_ns": ns, "max_ns": ns,
                                 "lds_bytes": int(r["LDS_Block_Size"]), "vgprs": int(r["VGPR_Count"]),
                                 "scratch_bytes": int(r["Scratch_Size"])})
        e["calls"] += 1
        e["total_ns"] += ns
        e["min_ns"] = min(e["min_ns"], ns)
        e["max_ns"] = max(e["max_ns"], ns)
    for e in acc.values():
        e["avg_ms"] = e["total_ns"] / e["calls"] / 1e6
    json.dump(dict(sorted(acc.items())), open(out, "w"), indent=1)
    for k, e in sorted(acc.items(), key=lambda x: -x[1]["total_ns"]):
        print(f"{e['avg_ms']:10.3f} ms x{e['calls']:3d}  {k}")


if __name__ == "__main__":
    main()
