"""MFMA busy fraction of the bf16 scoring walk from one rocprofv3 --pmc pass (tools/gpu_evidence.sh).

    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
        --kernel-include-regex score_topk_bf16_lds -d <dir> -o run -- python3 bench.py --no-propagation ...
    python3 tools/mfma_busy.py <dir> > profiles/<tag>_scoring_pmc_mfma.txt

SQ_VALU_MFMA_BUSY_CYCLES is summed over the SIMDs (1024 on MI355X), SQ_BUSY_CYCLES over the shader
engines (32): busy = (MFMA busy cycles per SIMD) / (busy cycles per SE); the shader clock follows from
SQ_BUSY_CYCLES per SE over the kernels' wall time.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    src = sys.argv[1]
    per = defaultdict(lambda: defaultdict(float))
    spans = {}
    for path in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as fh:
            for r in csv.DictReader(fh):
                if "score_topk_bf16_lds" not in r.get("Kernel_Name", ""):
                    continue
                key = (path, r["Dispatch_Id"])
                per[key][r["Counter_Name"]] += float(r["Counter_Value"])
                spans[key] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    if not per:
        sys.exit("no score_topk_bf16_lds dispatches found")
    tot = defaultdict(float)
    for c in per.values():
        for k, v in c.items():
            tot[k] += v
    ns = sum(e - s for s, e in spans.values())
    mfma, busy = tot["SQ_VALU_MFMA_BUSY_CYCLES"], tot["SQ_BUSY_CYCLES"]
    print(f"dispatches {len(per)}, kernel time {ns / 1e6:.1f} ms")
    for k in sorted(tot):
        print(f"{k:26s} {tot[k]:.4e}")
    frac = (mfma / 1024) / (busy / 32)
    clock = busy / 32 / (ns * 1e-9) / 1e9
    print(f"MFMA busy per SIMD / busy cycles per SE = ({mfma:.3e} / 1024) / ({busy:.3e} / 32) = {frac:.3f}")
    print(f"shader clock over the kernel time: {clock:.2f} GHz")


if __name__ == "__main__":
    main()
