"""Development: time lgx_score_topk variants on the C5 shape (bf16, d=256, 1M items, top-20)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from factors_of_serendipity_recommendation_amd import _lib  # noqa: E402

if os.environ.get("LGX_LIB"):  # A/B against another build of the library on the same box
    _lib.LIB_PATH = os.path.abspath(os.environ["LGX_LIB"])
import factors_of_serendipity_recommendation_amd as lgx  # noqa: E402
from factors_of_serendipity_recommendation_amd import ops  # noqa: E402


def run(B, n_items=int(os.environ.get("ABL_ITEMS", "1000000")), d=256, k=20, masked=True, reps=3):
    items = lgx.fill_normal((n_items, d), 1 / 16, 1, dtype=torch.bfloat16)
    Q = lgx.fill_normal((B, d), 1 / 16, 2, dtype=torch.bfloat16)
    mask = None
    if masked:
        pos = torch.randint(0, n_items, (B, 50), device="cuda").sort(dim=1).values
        mask = (torch.arange(B + 1, device="cuda", dtype=torch.int64) * 50, pos.reshape(-1).to(torch.int32))
    ops.score_topk(Q, items, k, mask=mask)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        ops.score_topk(Q, items, k, mask=mask)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / reps
    tf = 2 * B * n_items * d / t / 1e12
    tag = os.path.basename(os.environ.get("LGX_LIB", "liblgx.so"))
    print(f"{tag} I={n_items} B={B} masked={masked} ablate={os.environ.get('LGX_SCORE_ABLATE', '0')}: {t * 1e3:.1f} ms  {tf:.0f} TF/s",
          flush=True)


if __name__ == "__main__":
    for B in [int(x) for x in os.environ.get("ABL_B", "131072,32768").split(",")]:
        run(B, masked=True)
        run(B, masked=False)
