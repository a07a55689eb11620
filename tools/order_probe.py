"""Development: does sweeping the catalog in descending item-norm order cut the fused top-k's event
cost at the evaluation shapes?  Builds tools/bench_rows.py's synthetic Gowalla / Amazon-book datasets,
propagates them with the LightGCN module, and times lgx_score_topk (masked top-20, the test users)
on the item table as is and with its rows permuted by descending norm (timing only: the permuted
call's ids are in the permuted space).  HIP events, median of 5.

  python tools/order_probe.py [--lib other/liblgx.so]
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
        norm = I.norm(dim=1)
        perm = torch.argsort(norm, descending=True)
        Ip = I[perm].contiguous()
        rperm = torch.randperm(I.shape[0], device=I.device)
        Ir = I[rperm].contiguous()
        run = lambda T: ops.score_topk(U, T, 20, user_rows=tl.rows, mask=tl.mask, mask_value=-1024.0,  # noqa: E731
                                       apply_sigmoid=True)
        t0, t1, t2 = timed(lambda: run(I)), timed(lambda: run(Ip)), timed(lambda: run(Ir))
        tw = timed(lambda: ops.score_minmax(U[tl.rows], I))
        cv = float(norm.std() / norm.mean())
        print(f"{name}: as is {t0:.2f} ms | norm-descending {t1:.2f} ms | random order {t2:.2f} ms | "
              f"bare walk (min/max) {tw:.2f} ms | item-norm cv {cv:.3f}; corr(norm, id) "
              f"{float(np.corrcoef(norm.cpu().numpy(), np.arange(I.shape[0]))[0, 1]):.3f}", flush=True)
