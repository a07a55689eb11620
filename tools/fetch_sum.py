"""Development: sum one rocprofv3 --pmc counter over the dispatches of each kernel in a
counter_collection.csv tree, per library call (FETCH_SIZE / WRITE_SIZE are in KB).

  python tools/fetch_sum.py <rocprof output dir> <calls> [--counter FETCH_SIZE]
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def main():
    src, calls = sys.argv[1], int(sys.argv[2])
    counter = sys.argv[sys.argv.index("--counter") + 1] if "--counter" in sys.argv else "FETCH_SIZE"
    tot, n = defaultdict(float), defaultdict(int)
    for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r.get("Counter_Name") != counter:
                    continue
                m = re.search(r"::(\w+)<", r["Kernel_Name"]) or re.search(r"(\w+)\(", r["Kernel_Name"])
                name = m.group(1) if m else r["Kernel_Name"]
                tot[name] += float(r["Counter_Value"])
                n[name] += 1
    out = {k: {"dispatches": n[k], "kb_per_call": tot[k] / calls, "gb_per_call_x2": 2 * tot[k] * 1024 / calls / 1e9}
           for k in tot}
    print(json.dumps({"src": src, "counter": counter, "calls": calls, "kernels": out}))


if __name__ == "__main__":
    main()
