"""Summarise rocprofv3 PMC passes of the bench into profiles/pmc_summary.json.

    python tools/pmc_summary.py FETCH_DIR WRITE_DIR RDREQ_DIR BENCH_JSON

Each *_DIR holds one `rocprofv3 --pmc ... --output-format csv -d DIR -o pmc`
run of the same bench command (separate passes: FETCH_SIZE; WRITE_SIZE;
TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum).  Every measurement line of the
bench JSON (headline and secondaries) that carries `roofline.pmc_tag` and
`roofline.pmc_match` {kernel regex, grid threads or null} gets an entry keyed
by the tag, with the library sha the bench reports, so bench.py quotes it only
for that exact build and workload size:

  fetch/write_bytes_per_launch   FETCH_SIZE / WRITE_SIZE (KiB) x 1024, mean over
                                 the matching dispatches
  fabric_read_requests_per_launch  TCC_EA0_RDREQ_sum
  hbm_bytes_per_launch           2 x FETCH_SIZE + WRITE_SIZE: FETCH_SIZE tallies
                                 64 B per read request (FETCH_SIZE ==
                                 TCC_EA0_RDREQ x 64 B), while a request moves a
                                 128 B line (MI355X_MICROARCH.md §HBM gfx950
                                 correction; profiles/calib_r02.json: a random
                                 128 B block costs one request, 256 B two).
                                 Infinity-Cache hits are counted (same guide).
"""
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def norm(name):
    return name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0].strip()


def rows(d):
    out = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def matching(rs, kre, grid, nth=None):
    """Rows of the dispatches a line measured: kernel regex and grid, and with
    `nth` only those dispatches' ordinals among the regex's matches in
    dispatch order (bench.py ts_dispatch: lines sharing one kernel)."""
    m = [r for r in rs if re.match(kre, norm(r["Kernel_Name"]))
         and (grid is None or int(r.get("Grid_Size", -1)) == grid)]
    if nth is not None:
        ids = sorted({int(r["Dispatch_Id"]) for r in m})
        keep = {ids[k] for k in nth if k < len(ids)}
        m = [r for r in m if int(r["Dispatch_Id"]) in keep]
    return m


def mean_counter(rs, counter, kre, grid, nth=None):
    v = [float(r["Counter_Value"]) for r in matching(rs, kre, grid, nth) if r["Counter_Name"] == counter]
    return (sum(v) / len(v), len(v)) if v else (None, 0)


def lines(bench):
    """Every roofline dict of a bench line: the headline, each secondary (and
    its `more` entries) and the one-shot rejection-sampler legs
    (`end_to_end_rejection.roofline`)."""
    def of(d):
        d = d or {}
        yield d.get("roofline") or {}
        yield (d.get("end_to_end_rejection") or {}).get("roofline") or {}
    yield from of(bench)
    for v in (bench.get("secondary") or {}).values():
        yield from of(v)
        for m in ((v or {}).get("more", []) or []) + ((v or {}).get("points", []) or []):
            yield from of(m)


def main():
    fdir, wdir, rdir, bjson = sys.argv[1:5]
    bench = [json.loads(ln) for ln in open(bjson) if ln.startswith("{")][-1]
    sha = (bench.get("roofline") or {}).get("lib_sha256")
    F, W, R = rows(fdir), rows(wdir), rows(rdir)
    out_path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        summ = json.load(open(out_path))
    except Exception:
        summ = {}
    for roof in lines(bench):
        tag, m = roof.get("pmc_tag"), roof.get("pmc_match")
        if not tag or not m:
            continue
        kre, grid, nth = m["kernel"], m.get("grid"), m.get("nth")
        fb, nf = mean_counter(F, "FETCH_SIZE", kre, grid, nth)
        wb, nw = mean_counter(W, "WRITE_SIZE", kre, grid, nth)
        rq, nr = mean_counter(R, "TCC_EA0_RDREQ_sum", kre, grid, nth)
        hit, _ = mean_counter(R, "TCC_HIT_sum", kre, grid, nth)
        miss, _ = mean_counter(R, "TCC_MISS_sum", kre, grid, nth)
        sel = matching(F, kre, grid, nth)
        if fb is None or wb is None:
            print(f"{tag}: no matching dispatches for {kre} grid {grid}", file=sys.stderr)
            continue
        units = roof.get("units_per_launch")
        e = {
            "kernel": kre, "grid": grid, "nth": nth, "dispatches": [nf, nw, nr], "lib_sha256": sha,
            "scratch_bytes": max(int(r.get("Scratch_Size") or 0) for r in sel) if sel else None,
            "vgprs": max(int(r.get("VGPR_Count") or 0) for r in sel) if sel else None,
            "units_per_launch": units,
            "fetch_bytes_per_launch": fb * 1024, "write_bytes_per_launch": wb * 1024,
            "hbm_bytes_per_launch": 2 * fb * 1024 + wb * 1024,
            "fabric_read_requests_per_launch": rq,
            "l2_hit_rate": hit / (hit + miss) if hit is not None and miss and hit + miss > 0 else None,
            "algorithmic_bytes_per_launch": roof.get("algorithmic_bytes") or (
                roof.get("bytes_per_unit", 0) * (units or 0)),
            "note": "2 x FETCH_SIZE + WRITE_SIZE (KiB x 1024), mean over matching dispatches of separate --pmc "
                    "passes; FETCH_SIZE counts 64 B per 128 B read request (tools/pmc_summary.py)",
        }
        if units:
            e["fabric_read_requests_per_unit"] = rq / units if rq else None
            e["hbm_bytes_per_unit"] = e["hbm_bytes_per_launch"] / units
        summ[tag] = e
        print(tag, json.dumps({k: e[k] for k in ("units_per_launch", "hbm_bytes_per_launch",
                                                 "fabric_read_requests_per_launch", "l2_hit_rate")}))
    json.dump(summ, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
