"""Development: every test user of the evaluation shapes through the dense route (score_dense +
-inf scatter + topk_rows, ops.score_topk_dense_masked) at several chunk sizes, against the
evaluator's route (fused walk + dense rows for long masks), on propagated LightGCN tables
(tools/bench_rows.py's synthetic Gowalla / Amazon-book datasets).  HIP events, median of 5.

  python tools/dense_probe.py [--lib other/liblgx.so]
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
        n, ni = tl.rows.numel(), I.shape[0]
        r = evaluator._Route(tl.rows, tl.mask, ni, 20, cfg.d)
        route = timed(lambda: r.topk(U, I, 20, -1024.0, True))
        ref = r.topk(U, I, 20, -1024.0, True)
        print(f"{name}: {n} test users x {ni} items, d={cfg.d}: evaluator route {route:.2f} ms", flush=True)
        for cb in (256 << 20, 1 << 30, 4 << 30):
            step = ops.dense_chunk_users(ni, cb)
            offs = [ops.dense_mask_offsets(tl.mask, ni, c0, min(n, c0 + step)) for c0 in range(0, n, step)]
            t = timed(lambda: ops.score_topk_dense_masked(U, I, 20, tl.rows, tl.mask, chunk_bytes=cb, offsets=offs))
            got = ops.score_topk_dense_masked(U, I, 20, tl.rows, tl.mask, chunk_bytes=cb, offsets=offs)
            same = torch.equal(got.sort(dim=1).values, ref.sort(dim=1).values)
            if not same:
                # users whose sets differ: the float64 scores of the swapped items against each set's
                # float64 k-th score (an f32 near-tie flips with the summation order of the kernel)
                bad = torch.nonzero((got.sort(dim=1).values != ref.sort(dim=1).values).any(dim=1)).flatten()
                gap = 0.0
                for u in bad.tolist():
                    q = U[tl.rows[u]].double()
                    a64 = (I[got[u].long()].double() @ q)
                    b64 = (I[ref[u].long()].double() @ q)
                    gap = max(gap, abs(float(a64.min() - b64.min())) / max(1e-30, abs(float(b64.min()))))
                print(f"   {bad.numel()} users differ; largest relative gap between the two sets' float64 k-th scores {gap:.2e}",
                      flush=True)
            rows = tl.rows[:step]
            ts = timed(lambda: ops.score_dense(U, I, user_rows=rows))
            S = ops.score_dense(U, I, user_rows=rows)
            tk = timed(lambda: ops.topk_rows(S, 20))
            del S
            torch.cuda.empty_cache()
            fl = 2.0 * step * ni * cfg.d / (ts * 1e-3) / 1e12
            print(f"   all dense, chunks of {step} users ({cb >> 20} MiB): {t:.2f} ms; one chunk: score_dense {ts:.3f} ms "
                  f"({fl:.1f} TF/s), topk_rows {tk:.3f} ms; same top-20 sets as the route: {same}", flush=True)
        del model, ds
        torch.cuda.empty_cache()
