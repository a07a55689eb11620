"""Development: one scoring launch on the C5 shape for counter collection (B users, 1M items)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import factors_of_serendipity_recommendation_amd as lgx  # noqa: E402
from factors_of_serendipity_recommendation_amd import ops  # noqa: E402

B = int(os.environ.get("ABL_B", "131072"))
items = lgx.fill_normal((1_000_000, 256), 1 / 16, 1, dtype=torch.bfloat16)
Q = lgx.fill_normal((B, 256), 1 / 16, 2, dtype=torch.bfloat16)
for _ in range(2):
    ops.score_topk(Q, items, 20)
torch.cuda.synchronize()
print("done", flush=True)
