"""Development: the evaluator's score + mask + top-20 step at the evaluation shapes on propagated
LightGCN tables (tools/bench_rows.py's synthetic Gowalla / Amazon-book datasets): every test user
through the fused launch, against the evaluator's route (the fused launch for users with at most
DENSE_MASK_MIN masked items, dense rows for the rest) at several thresholds, with the two parts
timed apart.  HIP events, median of 5.

  python tools/route_probe.py [--lib other/liblgx.so]
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
        n = tl.rows.numel()
        fused = timed(lambda: ops.score_topk(U, I, 20, user_rows=tl.rows, mask=tl.mask, mask_value=-1024.0,
                                             apply_sigmoid=True))
        print(f"{name}: {n} test users, all fused: {fused:.2f} ms  [{ops.score_topk_plan(n, I.shape[0], cfg.d, torch.float32, 20)}]",
              flush=True)
        for thr in (32, 64, 128, 256, 1024, None):
            r = evaluator._Route(tl.rows, tl.mask, I.shape[0], 20, cfg.d, thr)
            tot = timed(lambda: r.topk(U, I, 20, -1024.0, True))
            if r.n_heavy:
                tf = timed(lambda: ops.score_topk(U, I, 20, user_rows=r.light_rows, mask=r.light_mask,
                                                  mask_value=-1024.0, apply_sigmoid=True))
                td = timed(lambda: ops.score_topk_dense_masked(U, I, 20, r.heavy_rows, r.heavy_mask,
                                                               offsets=r.heavy_offsets))
                plan = ops.score_topk_plan(n - r.n_heavy, I.shape[0], cfg.d, torch.float32, 20)
            else:
                tf, td, plan = tot, 0.0, "-"
            print(f"   threshold {r.thr}{' (the rule)' if thr is None else ''}: {r.n_heavy} dense users, route {tot:.2f} ms = fused {tf:.2f} + dense {td:.2f}  [{plan}]",
                  flush=True)
        del model, ds
        torch.cuda.empty_cache()
