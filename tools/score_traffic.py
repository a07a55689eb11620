"""Development: the bench's bf16 scoring call (bench.py bench_scoring: d=256, 1M items, top-20, 50
masked items per user, the same seeds) on B users, for counter collection and A/B timing of
liblgx.so builds.  One warm-up call, then --calls timed calls (HIP events); prints one JSON line.

  python tools/score_traffic.py [--lib other/liblgx.so] [--users 262144] [--calls 1] [--dtype bf16]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from factors_of_serendipity_recommendation_amd import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
ap.add_argument("--users", type=int, default=262_144)
ap.add_argument("--calls", type=int, default=1)
ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
args = ap.parse_args()
if args.lib:
    _lib.LIB_PATH = os.path.abspath(args.lib)
    _lib._lib = None
    _lib.ALLOW_MISSING = True
import factors_of_serendipity_recommendation_amd as lgx  # noqa: E402
from factors_of_serendipity_recommendation_amd import ops  # noqa: E402

dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
d, n_items, k, B, per = 256, 1_000_000, 20, args.users, 50
items = lgx.fill_normal((n_items, d), 1.0 / 16, 4242, dtype=dt)
Q = lgx.fill_normal((B, d), 1.0 / 16, 777, dtype=dt)
g = torch.Generator(device="cuda")
g.manual_seed(99)
pos = torch.randint(0, n_items, (B, per), device="cuda", generator=g).sort(dim=1).values
mask = (torch.arange(0, B + 1, device="cuda", dtype=torch.int64) * per, pos.reshape(-1).to(torch.int32))
ops.score_topk(Q, items, k, mask=mask)
torch.cuda.synchronize()
ts = []
for _ in range(args.calls):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    ops.score_topk(Q, items, k, mask=mask)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
ms = float(np.median(ts))
peak = 2.5e15 if dt == torch.bfloat16 else 157.3e12
print(json.dumps({"lib": args.lib or _lib.LIB_PATH, "users": B, "dtype": args.dtype, "ms": ms,
                  "frac": 2.0 * B * n_items * d / (ms / 1e3) / peak, "calls_incl_warmup": args.calls + 1,
                  "plan": ops.score_topk_plan(B, n_items, d, dt, k)}), flush=True)
