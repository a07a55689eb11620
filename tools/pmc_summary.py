"""Summarise tools/profile_round.sh output (gpurun_out/prof_<tag>/) into profiles/<tag>_<config>_*:
kernel stats, the raw PMC rows of our kernels, and per-launch HBM traffic
(2 * FETCH_SIZE + WRITE_SIZE, KB -> bytes; the x2 is the gfx950 correction for 16-B/lane reads in
MI355X_MICROARCH.md).  Usage: python tools/pmc_summary.py r01 [--config synth10m] [--src DIR] [--dst DIR]"""
import csv
import glob
import json
import os
import re
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name: str) -> str:
    m = re.search(r"::(\w+)<", name) or re.search(r"(\w+)\(", name)
    return m.group(1) if m else name


def pmc_rows(path_glob, counter):
    rows = []
    for f in glob.glob(path_glob, recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r.get("Counter_Name") == counter and "lgx::" in r.get("Kernel_Name", ""):
                    rows.append(r)
    return rows


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--config", default="synth10m")
    ap.add_argument("--src", default=None, help="default gpurun_out/prof_<tag>")
    ap.add_argument("--dst", default=os.path.join(ROOT, "profiles"))
    args = ap.parse_args()
    tag, config = args.tag, args.config
    src = args.src or os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = args.dst
    os.makedirs(dst, exist_ok=True)
    pre = os.path.join(dst, f"{tag}_{config}_")
    stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], pre + "kernel_stats.csv")
    for name in ("bench.json", "bench_under_rocprof.json"):
        if os.path.exists(os.path.join(src, name)):
            shutil.copy(os.path.join(src, name), pre + name.replace("bench.json", "bench_line.json")
                        if name == "bench.json" else pre + name)
    # kernels keyed by workload leg: the bf16 / f32 SpMM instantiations and the scoring kernels
    per = defaultdict(lambda: {"FETCH_SIZE": [], "WRITE_SIZE": []})
    for counter, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        rows = pmc_rows(os.path.join(src, sub, "**", "*counter_collection.csv"), counter)
        with open(pre + f"pmc_{counter.lower()}.csv", "w", newline="") as fh:
            if rows:
                w = csv.DictWriter(fh, fieldnames=list(rows[0].keys()))
                w.writeheader()
                w.writerows(rows)
        # legs: the propagation kernels by storage type; the scoring sweeps by kernel (f32 leg:
        # score_topk_f32_lds, bf16 leg: score_topk_bf16_lds); a finalize belongs to the leg of the
        # sweep dispatched before it
        last_scoring = "scoring"
        for r in sorted(rows, key=lambda r: int(r.get("Dispatch_Id", 0) or 0)):
            name = r["Kernel_Name"]
            k = short(name)
            if k == "score_topk_f32_lds":
                leg = last_scoring = "scoring_f32"
            elif k == "score_topk_bf16_lds":
                leg = last_scoring = "scoring"
            elif "score" in k:
                leg = last_scoring
            else:
                leg = "bf16" if "unsigned short" in name else "f32"
            per[(leg, k)][counter].append(float(r["Counter_Value"]))
    kernels = defaultdict(dict)
    for (leg, k), v in per.items():
        if not v["FETCH_SIZE"] or not v["WRITE_SIZE"]:
            continue
        f = sum(v["FETCH_SIZE"]) / len(v["FETCH_SIZE"])
        w = sum(v["WRITE_SIZE"]) / len(v["WRITE_SIZE"])
        kernels[leg][k] = {"FETCH_SIZE_KB_mean": f, "WRITE_SIZE_KB_mean": w, "dispatches": len(v["FETCH_SIZE"]),
                           "hbm_bytes_per_launch": (2 * f + w) * 1024}
    import hashlib
    h = hashlib.sha256(open(os.path.join(ROOT, "factors_of_serendipity_recommendation_amd", "liblgx.so"), "rb").read())
    # the scoring legs' sizes as the profiled bench line reports them (not a hard-coded string)
    legs = "scoring legs: see the bench line"
    try:
        line = json.load(open(os.path.join(src, "bench_under_rocprof.json")))
        legs = "; ".join(f"scoring {x['dtype']} d={x['d']}: {x['users_per_step']} users x {x['n_items']} items"
                         for x in (line.get("scoring"), line.get("scoring_bf16")) if x)
    except (OSError, ValueError, KeyError, TypeError):
        pass
    doc = {"workload": f"{config} (bench.py: propagation K=3 d=128 f32 and bf16; {legs}), n_gpus=1",
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (tools/profile_round.sh); "
                     "bytes = (2*FETCH_SIZE + WRITE_SIZE) KB * 1024, the x2 measured for streaming reads and for "
                     "random 256-B / 512-B row gathers (profiles/r02_fetch_calibration.json). FETCH_SIZE counts "
                     "L2 misses served by the Infinity Cache as well as HBM reads (same calibration), so this is "
                     "L2-miss traffic, an upper bound on HBM traffic",
           "lib_sha256_16": h.hexdigest()[:16],
           "kernels": kernels}
    with open(pre + "pmc_traffic.json", "w") as fh:
        json.dump(doc, fh, indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
