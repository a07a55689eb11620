"""Development: lgx_foldout_metrics and the users' mean (lgx_column_mean_f32) at batch_test's
evaluation shapes (27 522 / 52 643 users, top-20, ~6 / ~10 truth items each), HIP events, median of 5,
with the op wrappers' host work (ops.foldout_metrics builds the 1/log2 table per call) timed apart.

  python tools/foldout_probe.py [--lib other/liblgx.so]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from factors_of_serendipity_recommendation_amd import _lib  # noqa: E402

if "--lib" in sys.argv:
    _lib.LIB_PATH = os.path.abspath(sys.argv[sys.argv.index("--lib") + 1])
    _lib._lib = None
    _lib.ALLOW_MISSING = True
from factors_of_serendipity_recommendation_amd import ops  # noqa: E402


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


for name, B, I, nt in (("gowalla", 27522, 40981, 6), ("amazon", 52643, 91599, 11)):
    rng = np.random.default_rng(1)
    lists = [sorted(rng.choice(I, rng.integers(1, 2 * nt), replace=False).tolist()) for _ in range(B)]
    truth = ops.lists_to_device_csr(lists, "cuda", sort=False)
    idx = torch.randint(0, I, (B, 20), device="cuda", dtype=torch.int32)
    tl = ops.inv_log2_table(20, "cuda")
    out = torch.empty((B, 100), dtype=torch.float32, device="cuda")
    L = _lib.lib()
    st = torch.cuda.current_stream().cuda_stream
    k_only = timed(lambda: L.lgx_foldout_metrics(idx.data_ptr(), B, 20, truth[0].data_ptr(), truth[1].data_ptr(),
                                                 tl.data_ptr(), out.data_ptr(), st))
    op = timed(lambda: ops.foldout_metrics(idx, truth))
    mean = timed(lambda: ops.column_mean(out)) if hasattr(L, "lgx_column_mean_f32") else float("nan")
    print(f"{name}: {B} users: foldout kernel {k_only:.3f} ms, ops.foldout_metrics {op:.3f} ms, column mean "
          f"{mean:.3f} ms", flush=True)
