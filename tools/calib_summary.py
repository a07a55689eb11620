"""Summarise tools/fetch_calib.sh output into profiles/<tag>_fetch_calibration.json: per calibration
case, the known bytes, the mean FETCH_SIZE bytes per dispatch, their ratio (the correction factor
for that access pattern) and the L2 hit rate; plus the gather-rate sweep by table size.
Usage: python tools/calib_summary.py r02"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def dispatch_values(src, counter):
    """Counter values of the calib_* dispatches in dispatch order."""
    recs = []
    for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            recs += [r for r in csv.DictReader(fh) if r.get("Counter_Name") == counter and "calib_" in r["Kernel_Name"]]
    recs.sort(key=lambda r: int(r["Dispatch_Id"]))
    return [float(r["Counter_Value"]) for r in recs]


def main():
    tag = sys.argv[1]
    src = os.path.join(ROOT, "gpurun_out", f"calib_{tag}")
    cases, order = {}, []
    for line in open(os.path.join(src, "timing.txt")):
        p = line.split()
        if len(p) < 3 or "ms" not in p:
            continue
        ms = float(p[p.index("ms") - 1])
        if p[0].startswith("sweep_"):
            name = f"{p[0]}_{p[2]}MiB"
            nbytes = None
        else:
            name = p[0]
            nbytes = int(p[2])
        t = {"ms": ms, "rate_TBs": float(p[p.index("ms") + 1])}
        if nbytes is not None:
            t["bytes"] = nbytes
        if p[1] == "gathered_bytes":
            t["unique_bytes"] = int(p[4])
        cases[name] = t
        order.append(name)
    per = 2  # the PMC passes run the binary with reps=1: a warm-up and one timed dispatch per case
    for counter, sub in (("FETCH_SIZE", "fetch"), ("TCC_HIT_sum", "hitmiss"), ("TCC_MISS_sum", "hitmiss")):
        vals = dispatch_values(os.path.join(src, sub), counter)
        if len(vals) != per * len(order):
            print(f"warning: {len(vals)} {counter} dispatches for {len(order)} cases", file=sys.stderr)
            continue
        for j, name in enumerate(order):
            cases[name][counter] = vals[per * j + 1]
    for name, c in cases.items():
        if "FETCH_SIZE" in c and "bytes" in c:
            c["known_over_fetch_size"] = c["bytes"] / (c["FETCH_SIZE"] * 1024) if c["FETCH_SIZE"] else None
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            h, m = c["TCC_HIT_sum"], c["TCC_MISS_sum"]
            c["l2_hit_rate"] = h / (h + m) if h + m else None
    sweep = {n.split("_", 2)[2]: c["rate_TBs"] for n, c in cases.items() if n.startswith("sweep_256")}
    doc = {"method": "tools/fetch_calib.hip: known-byte reads in the SpMM's access pattern (16 lanes x 16 B per "
                     "256-B row, 32 x 16 B per 512-B row); rocprofv3 --pmc FETCH_SIZE and --pmc TCC_HIT_sum "
                     "TCC_MISS_sum in separate passes (tools/fetch_calib.sh); known_over_fetch_size = the factor "
                     "that turns FETCH_SIZE (KB * 1024) into bytes read for that pattern; sweep = gather rate of "
                     "uniformly random 256-B rows by table size (timing only)",
           "cases": cases, "sweep_256": sweep}
    dst = os.path.join(ROOT, "profiles", f"{tag}_fetch_calibration.json")
    with open(dst, "w") as fh:
        json.dump(doc, fh, indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
