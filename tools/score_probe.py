"""Development: the bench's bf16 scoring leg shape (B users x 1M items, d=256, top-20, 50 masked
items per user) timed with HIP events; run under rocprofv3 --kernel-trace --stats for the per-kernel
split (floor pass, the seeded stages, the split tail, the finalize).

  python tools/score_probe.py [B] [dtype] [--lib other/liblgx.so]   (--lib: time another build)
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import factors_of_serendipity_recommendation_amd as lgx  # noqa: E402
from factors_of_serendipity_recommendation_amd import _lib, ops  # noqa: E402

if "--lib" in sys.argv:
    j = sys.argv.index("--lib")
    _lib.LIB_PATH = os.path.abspath(sys.argv[j + 1])
    _lib._lib = None
    _lib.ALLOW_MISSING = True
    del sys.argv[j:j + 2]

B = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
dt = torch.float32 if len(sys.argv) > 2 and sys.argv[2] == "f32" else torch.bfloat16
I, d, k = 1_000_000, 256, 20
items = lgx.fill_normal((I, d), 1 / 16, 4242, dtype=dt)
Q = lgx.fill_normal((B, d), 1 / 16, 777, dtype=dt)
g = torch.Generator(device="cuda")
g.manual_seed(99)
pos = torch.randint(0, I, (B, 50), device="cuda", generator=g).sort(dim=1).values
mask = (torch.arange(0, B + 1, device="cuda", dtype=torch.int64) * 50, pos.reshape(-1).to(torch.int32))
print(ops.score_topk_plan(B, I, d, dt, k), flush=True)
ops.score_topk(Q, items, k, mask=mask)
torch.cuda.synchronize()
ts = []
for _ in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    ops.score_topk(Q, items, k, mask=mask)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
ms = float(np.median(ts))
peak = 157.3e12 if dt == torch.float32 else 2.5e15
print(f"B={B} {dt}: {ms:.2f} ms  {2.0 * B * I * d / ms / 1e9:.1f} TF/s  frac {2.0 * B * I * d / ms * 1e3 / peak:.3f}",
      flush=True)
