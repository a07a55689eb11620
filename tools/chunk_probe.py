"""Development: the evaluator's route at the evaluation shapes (propagated tables) with the dense
route's chunk at 256 MiB (the default) and larger, at the default threshold and a few others.
HIP events, median of 5.

  python tools/chunk_probe.py
"""
import os
import sys
import tempfile

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import bench_rows as br  # noqa: E402
from factors_of_serendipity_recommendation_amd import evaluator, ops  # noqa: E402
from factors_of_serendipity_recommendation_amd.model import LightGCN  # noqa: E402

_orig = ops.dense_chunk_users


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
        for mb in (256, 1024, 4096):
            ops.dense_chunk_users = lambda n, chunk_bytes=0, _mb=mb: _orig(n, _mb << 20)
            line = []
            for thr in (None, 128, 256, 1024):
                r = evaluator._Route(tl.rows, tl.mask, I.shape[0], 20, cfg.d, thr)
                t = timed(lambda: r.topk(U, I, 20, -1024.0, True))
                td = timed(lambda: ops.score_topk_dense_masked(U, I, 20, r.heavy_rows, r.heavy_mask,
                                                               offsets=r.heavy_offsets)) if r.n_heavy else 0.0
                line.append(f"thr {r.thr}{'*' if thr is None else ''} ({r.n_heavy} dense): {t:.2f} (dense {td:.2f})")
            print(f"{name}, chunk {mb} MiB: " + " | ".join(line), flush=True)
        ops.dense_chunk_users = _orig
        del model, ds
        torch.cuda.empty_cache()
