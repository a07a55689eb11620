"""Development: propagation latency on the small configs -- GPU-event time per call in a back-to-back
loop (throughput), host wall per synchronised call (latency), and the kernels alone.
  python tools/small_latency.py"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import factors_of_serendipity_recommendation_amd as lgx  # noqa: E402
from factors_of_serendipity_recommendation_amd import ops  # noqa: E402
from factors_of_serendipity_recommendation_amd.synth import CONFIGS, synth_graph  # noqa: E402


def main():
    for name in ("ml1m", "gowalla", "amazon"):
        cfg = CONFIGS[name]
        A = synth_graph(cfg, seed=2020, device="cuda")
        dt = torch.bfloat16 if cfg.dtype == "bf16" else torch.float32
        E0 = lgx.fill_normal((cfg.n_users + cfg.n_items, cfg.d), 0.1, 7, dtype=dt)
        out = torch.empty((E0.shape[0], cfg.d), dtype=torch.float32, device="cuda")
        for _ in range(20):
            ops.propagate(A, E0, cfg.K, out=out)
        torch.cuda.synchronize()
        n = 200
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            ops.propagate(A, E0, cfg.K, out=out)
        e1.record()
        torch.cuda.synchronize()
        thr = e0.elapsed_time(e1) / n * 1e3
        lat = []
        for _ in range(100):
            t0 = time.perf_counter()
            ops.propagate(A, E0, cfg.K, out=out)
            torch.cuda.synchronize()
            lat.append(time.perf_counter() - t0)
        host = []
        for _ in range(100):
            t0 = time.perf_counter()
            ops.propagate(A, E0, cfg.K, out=out)
            host.append(time.perf_counter() - t0)
            torch.cuda.synchronize()
        print(f"{name:8s} nnz={A.nnz:9d} seg_len={A.plan.seg_len:5d} splits={len(A.plan.split_row):6d} "
              f"throughput {thr:8.1f} us/call  latency {np.median(lat) * 1e6:8.1f} us  host issue "
              f"{np.median(host) * 1e6:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
