"""Development: lgx_column_mean_f32 (batch_test's np.mean over users) alone at the evaluation shapes'
curve widths, HIP events, median of 7.

  python tools/cm_probe.py [--lib other/liblgx.so]
"""
import sys, torch, numpy as np
import os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from factors_of_serendipity_recommendation_amd import _lib
if "--lib" in sys.argv:
    _lib.LIB_PATH = os.path.abspath(sys.argv[sys.argv.index("--lib") + 1])
    _lib._lib = None
    _lib.ALLOW_MISSING = True
from factors_of_serendipity_recommendation_amd import ops  # noqa: E402
def t(fn, reps=7):
    fn(); torch.cuda.synchronize(); ts=[]
    for _ in range(reps):
        a=torch.cuda.Event(enable_timing=True); b=torch.cuda.Event(enable_timing=True)
        a.record(); fn(); b.record(); torch.cuda.synchronize(); ts.append(a.elapsed_time(b))
    return float(np.median(ts))
for rows, cols in ((52643, 100), (52643, 64), (210572, 64), (27522, 100), (1000, 100)):
    x = torch.rand((rows, cols), device="cuda")
    k = t(lambda: ops.column_mean(x))
    c = t(lambda: ops.column_mean(x).cpu())
    print(f"[{rows}, {cols}]: kernel {k:.3f} ms, with .cpu() {c:.3f} ms, {k / rows * 1e6:.2f} ns/row", flush=True)
