"""Summarise tools/fetch_calib.sh output into profiles/<tag>_fetch_calibration.json: per calibration
kernel, the known bytes, the mean FETCH_SIZE bytes per dispatch, their ratio (the correction factor
for that access pattern) and the L2 hit rate.  Usage: python tools/calib_summary.py r02"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {"calib_stream": "stream", "calib_gather_once<256": "once_256", "calib_gather_once<512": "once_512"}


def case_of(name, occurrence):
    if "calib_stream" in name:
        return "stream"
    m = re.search(r"calib_gather_once<(\d+)", name)
    if m:
        return f"once_{m.group(1)}"
    if "calib_gather_hot" in name:
        return ("hot_mall", "hot_l2")[occurrence]
    return None


def rows(src, counter):
    out = defaultdict(list)
    for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
        seen_hot = []
        with open(f) as fh:
            recs = [r for r in csv.DictReader(fh) if r.get("Counter_Name") == counter]
        # the hot kernel runs twice per pass (mall then l2), each 1 + reps dispatches in order
        hot = [r for r in recs if "calib_gather_hot" in r["Kernel_Name"]]
        hot.sort(key=lambda r: int(r.get("Dispatch_Id", r.get("Correlation_Id", 0)) or 0))
        half = len(hot) // 2
        for j, r in enumerate(hot):
            out["hot_mall" if j < half else "hot_l2"].append(float(r["Counter_Value"]))
        for r in recs:
            c = case_of(r["Kernel_Name"], 0)
            if c and not c.startswith("hot"):
                out[c].append(float(r["Counter_Value"]))
    return out


def main():
    tag = sys.argv[1]
    src = os.path.join(ROOT, "gpurun_out", f"calib_{tag}")
    timing = {}
    for line in open(os.path.join(src, "timing.txt")):
        p = line.split()
        if len(p) > 2 and p[1] in ("known_read_bytes", "gathered_bytes"):
            t = {"bytes": int(p[2])}
            if p[1] == "gathered_bytes":
                t["unique_bytes"] = int(p[4])
            ms = float(p[p.index("ms") - 1])
            t["ms"] = ms
            t["rate_TBs"] = t["bytes"] / ms / 1e9
            timing[p[0]] = t
    fetch = rows(os.path.join(src, "fetch"), "FETCH_SIZE")
    hit = rows(os.path.join(src, "hitmiss"), "TCC_HIT_sum")
    miss = rows(os.path.join(src, "hitmiss"), "TCC_MISS_sum")
    cases = {}
    for c, t in timing.items():
        d = dict(t)
        if fetch.get(c):
            fb = sum(fetch[c]) / len(fetch[c]) * 1024
            d["fetch_size_bytes"] = fb
            d["known_over_fetch_size"] = t["bytes"] / fb if fb else None
        if hit.get(c) and miss.get(c):
            h, m = sum(hit[c]) / len(hit[c]), sum(miss[c]) / len(miss[c])
            d["l2_hit_rate"] = h / (h + m) if h + m else None
        cases[c] = d
    doc = {"method": "tools/fetch_calib.hip: known-byte reads in the SpMM's access pattern; rocprofv3 --pmc "
                     "FETCH_SIZE and --pmc TCC_HIT_sum TCC_MISS_sum in separate passes; known_over_fetch_size = "
                     "the factor that turns FETCH_SIZE (KB * 1024) into bytes read for that pattern",
           "cases": cases}
    dst = os.path.join(ROOT, "profiles", f"{tag}_fetch_calibration.json")
    with open(dst, "w") as fh:
        json.dump(doc, fh, indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
