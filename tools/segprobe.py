"""SpMM layer time vs seg_len on the small BASELINE shapes (configs[0..2]) -- tuning probe for
graph.choose_seg_len.  Run on the GPU box: python tools/segprobe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import factors_of_serendipity_recommendation_amd as lgx  # noqa: E402
from factors_of_serendipity_recommendation_amd import ops  # noqa: E402
from factors_of_serendipity_recommendation_amd.graph import choose_seg_len  # noqa: E402
from factors_of_serendipity_recommendation_amd.synth import CONFIGS, synth_edges  # noqa: E402

DEV = "cuda:0"
for name in ("gowalla", "ml1m", "amazon"):
    cfg = CONFIGS[name]
    u, i = synth_edges(cfg, 2020, DEV)
    dt = torch.bfloat16 if cfg.dtype == "bf16" else torch.float32
    X = (torch.randn(cfg.n_users + cfg.n_items, cfg.d, device=DEV) * 0.1).to(dt)
    res = []
    for sl in (16, 32, 64, 128, 256, 512, 1024):
        A = lgx.build_norm_adj(u, i, cfg.n_users, cfg.n_items, dedup=True, device=DEV, seg_len=sl)
        for _ in range(3):
            ops.spmm(A, X)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            ops.spmm(A, X)
        e1.record()
        torch.cuda.synchronize()
        res.append(f"{sl}:{e0.elapsed_time(e1) / 50 * 1000:.1f}us")
    print(name, "nnz", A.nnz, "default seg_len", choose_seg_len(A.nnz), " ".join(res), flush=True)
