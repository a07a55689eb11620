"""Development: where the fused top-k's time goes at the evaluation shapes on propagated LightGCN
tables (tools/bench_rows.py's synthetic Gowalla / Amazon-book datasets, the test users, their train
positives as the mask, top-20, fp32): masked vs unmasked, top-1, the bare walk, and the masked call
restricted to users whose mask holds at most 32 / 64 / 128 items -- power-law users with hundreds
of masked items saturate the 256-bit Bloom filter, so every candidate of theirs needs an exact test.
HIP events, median of 5.

  python tools/mask_probe.py [--lib other/liblgx.so]
"""
import os
import sys
import tempfile

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import bench_rows as br  # noqa: E402
from factors_of_serendipity_recommendation_amd import _lib, evaluator, ops  # noqa: E402

if "--lib" in sys.argv:
    _lib.LIB_PATH = os.path.abspath(sys.argv[sys.argv.index("--lib") + 1])
    _lib._lib = None
    _lib.ALLOW_MISSING = True
from factors_of_serendipity_recommendation_amd.model import LightGCN  # noqa: E402


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


def sub_mask(mask, sel):
    ip, ix = mask
    lens = (ip[1:] - ip[:-1])[sel]
    nip = torch.zeros(sel.numel() + 1, dtype=torch.int64, device=ip.device)
    nip[1:] = torch.cumsum(lens, 0)
    rid = torch.repeat_interleave(torch.arange(sel.numel(), device=ip.device), lens)
    pos = ip[sel][rid] + torch.arange(rid.numel(), device=ip.device) - nip[rid]
    return nip, ix[pos].contiguous()


with tempfile.TemporaryDirectory() as tmp:
    for name in ("gowalla", "amazon"):
        cfg = br.CONFIGS[name]
        ds = br._eval_dataset(cfg, tmp)
        conf = {"latent_dim_rec": cfg.d, "lightGCN_n_layers": cfg.K, "keep_prob": 0.6, "A_split": False,
                "pretrain": 0, "dropout": 0}
        torch.manual_seed(0)
        model = LightGCN(conf, ds).to("cuda").eval()
        with torch.no_grad():
            U, I = model.computer()
        tl = evaluator._TestLists.get(ds, I.shape[0], U.device)
        rows, mask = tl.rows, tl.mask
        lens = (mask[0][1:] - mask[0][:-1])
        q = torch.quantile(lens.double(), torch.tensor([0.5, 0.9, 0.99, 1.0], dtype=torch.float64, device=lens.device))
        res = {"masked": timed(lambda: ops.score_topk(U, I, 20, user_rows=rows, mask=mask, mask_value=-1024.0,
                                                      apply_sigmoid=True)),
               "unmasked": timed(lambda: ops.score_topk(U, I, 20, user_rows=rows)),
               "top1": timed(lambda: ops.score_topk(U, I, 1, user_rows=rows)),
               "walk": timed(lambda: ops.score_minmax(U[rows], I))}
        for lim in (32, 64, 128):
            sel = torch.nonzero(lens <= lim).flatten()
            m2 = sub_mask(mask, sel)
            r2 = rows[sel].contiguous()
            t = timed(lambda: ops.score_topk(U, I, 20, user_rows=r2, mask=m2, mask_value=-1024.0, apply_sigmoid=True))
            tu = timed(lambda: ops.score_topk(U, I, 20, user_rows=r2))
            res[f"mask<={lim} ({sel.numel()} users)"] = f"{t:.2f} / unmasked {tu:.2f}"
        print(f"{name}: {rows.numel()} test users, mask length p50/p90/p99/max "
              f"{'/'.join(str(int(x)) for x in q.tolist())}; plan {ops.score_topk_plan(rows.numel(), I.shape[0], cfg.d, torch.float32, 20)}",
              flush=True)
        print("   " + " | ".join(f"{k} {v:.2f} ms" if isinstance(v, float) else f"{k} {v} ms" for k, v in res.items()),
              flush=True)
        del model, ds
        torch.cuda.empty_cache()
