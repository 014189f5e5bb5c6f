"""Per-kernel PMC means from a rocprofv3 --pmc directory, per walk-step of the
headline launch: python tools/pmc_lines.py PMC_DIR BENCH_JSON"""
import csv
import glob
import json
import sys


def main():
    d, bj = sys.argv[1], sys.argv[2]
    b = json.load(open(bj))
    units = b["roofline"]["units_per_launch"]
    acc = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "")
            acc.setdefault((k, r.get("Grid_Size", "")), {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for (k, grid), cs in sorted(acc.items()):
        means = {c: sum(v) / len(v) for c, v in cs.items()}
        out = {c: round(v) for c, v in means.items()}
        if "TCC_EA0_RDREQ_sum" in means:
            out["rdreq_per_step"] = round(means["TCC_EA0_RDREQ_sum"] / units, 4)
        print(k, grid, json.dumps(out))


if __name__ == "__main__":
    main()
