#!/usr/bin/env python3
"""Summarise a `tools/gpu_run.sh calib` run (rounds 1-4: tools/gpu_calib.sh) into profiles/calib_<tag>.json.

The PMC runs launch, per (table size, read size), one warm-up and one timed
dispatch of k_coop<RB,1> in the order the sweep prints its lines; rocprofv3's
counter CSV lists dispatches in order, so dispatch pairs map to those lines.
"""
import csv
import glob
import json
import os
import re
import sys


def load_jsonl(p):
    with open(p) as f:
        return [json.loads(x) for x in f if x.startswith("{")]


def pmc(dirp):
    fs = glob.glob(os.path.join(dirp, "**", "*counter_collection.csv"), recursive=True)
    rows = {}
    for f in fs:
        for r in csv.DictReader(open(f)):
            if "k_coop" not in r["Kernel_Name"]:
                continue
            d = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)
            rows.setdefault(d, {"kernel": r["Kernel_Name"]})
            rows[d][r["Counter_Name"]] = rows[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [rows[k] for k in sorted(rows)]


def main():
    src, tag = sys.argv[1], sys.argv[2]
    sweep = load_jsonl(os.path.join(src, "sweep.jsonl"))
    out = {"tool": "tools/calib/calib_sweep.hip via tools/gpu_run.sh calib", "tag": tag,
           "definition": "random RB-byte blocks (RB-aligned), read cooperatively (RB/16 lanes per block), "
                         "DEP=1: next address depends on the data read; W waves per SIMD forced by LDS",
           "sweep": sweep, "pmc": []}
    for name in ("pmc_rdreq", "pmc_hit", "pmc_fetch"):
        lines = load_jsonl(os.path.join(src, name + ".jsonl"))
        disp = pmc(os.path.join(src, name))
        # two dispatches (warm + timed) per printed line
        for i, ln in enumerate(lines):
            if 2 * i + 1 >= len(disp):
                break
            c = disp[2 * i + 1]
            rec = next((p for p in out["pmc"] if p["rb"] == ln["rb"] and p["table_mb"] == ln["table_mb"]), None)
            if rec is None:
                rec = {"rb": ln["rb"], "table_mb": ln["table_mb"], "waves": ln["waves"], "dep": ln["dep"],
                       "reads": ln["reads"]}
                out["pmc"].append(rec)
            for k, v in c.items():
                if k != "kernel":
                    rec[k] = v
                    rec[k + "_per_read"] = v / ln["reads"]
    # the walk kernels' denominator: dependent 64 B blocks at 5 waves/SIMD per table size
    peak = {}
    for r in sweep:
        if r["dep"] == 1 and r["waves"] == 5:
            peak.setdefault(str(r["rb"]), {})[str(r["table_mb"])] = r["blocks_per_s"]
    out["dep_w5_blocks_per_s"] = peak
    best = {}
    for r in sweep:
        k = f'{r["rb"]}/{r["table_mb"]}'
        if r["dep"] == 1 and (k not in best or r["blocks_per_s"] > best[k]["blocks_per_s"]):
            best[k] = r
    out["dep_best_over_waves"] = {k: {"blocks_per_s": v["blocks_per_s"], "waves": v["waves"]} for k, v in best.items()}
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "profiles", f"calib_{tag}.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(os.path.abspath(dst))
    for k, v in sorted(best.items(), key=lambda kv: (int(kv[0].split("/")[0]), int(kv[0].split("/")[1]))):
        print(f"rb {k:12s} best {v['blocks_per_s']:.3g} blocks/s at {v['waves']} waves  ({v['bytes_per_s']/1e12:.2f} TB/s)")
    for p in out["pmc"]:
        print({k: (round(v, 3) if isinstance(v, float) else v) for k, v in p.items() if "per_read" in k or k in ("rb", "table_mb")})


if __name__ == "__main__":
    main()
