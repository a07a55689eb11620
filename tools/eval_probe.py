"""Development: the fused score + mask + top-k launch at the evaluation shapes of Procedure.Test
(Gowalla: 27 522 test users x 40 981 items, d=64; Amazon-book: 52 643 x 91 599, d=128; fp32)
beside the same walk with no top-k (lgx_score_minmax) and the top-k without the mask, to split the
launch into the walk and its events.  HIP events, median of 5.

  python tools/eval_probe.py [--lib other/liblgx.so] [--only gowalla|amazon] [--f32]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import factors_of_serendipity_recommendation_amd as lgx  # noqa: E402
from factors_of_serendipity_recommendation_amd import _lib, ops  # noqa: E402

if "--lib" in sys.argv:
    _lib.LIB_PATH = os.path.abspath(sys.argv[sys.argv.index("--lib") + 1])
    _lib._lib = None
    _lib.ALLOW_MISSING = True
ONLY = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None
DTYPES = (torch.float32,) if "--f32" in sys.argv else (torch.float32, torch.bfloat16)


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


for name, B, I, d, npos in (("gowalla", 27522, 40981, 64, 27), ("amazon", 52643, 91599, 128, 46)):
    if ONLY and name != ONLY:
        continue
    for dt in DTYPES:
        Q = lgx.fill_normal((B, d), 0.1, 7, dtype=dt)
        items = lgx.fill_normal((I, d), 0.1, 8, dtype=dt)
        g = torch.Generator(device="cuda")
        g.manual_seed(3)
        pos = torch.randint(0, I, (B, npos), device="cuda", generator=g).sort(dim=1).values
        mask = (torch.arange(0, B + 1, device="cuda", dtype=torch.int64) * npos, pos.reshape(-1).to(torch.int32))
        flops = 2.0 * B * I * d
        peak = 157.3e12 if dt == torch.float32 else 2.5e15
        row = {}
        row["topk+mask"] = timed(lambda: ops.score_topk(Q, items, 20, mask=mask, mask_value=-1024.0, apply_sigmoid=True))
        row["topk"] = timed(lambda: ops.score_topk(Q, items, 20))
        row["top1"] = timed(lambda: ops.score_topk(Q, items, 1))
        row["minmax walk"] = timed(lambda: ops.score_minmax(Q, items))
        print(f"{name} {str(dt)[6:]} B={B} I={I} d={d}: {ops.score_topk_plan(B, I, d, dt, 20)}", flush=True)
        print("   " + "  ".join(f"{k} {v:.2f} ms ({flops / v * 1e3 / peak:.2f})" for k, v in row.items()), flush=True)
