"""Development: the C4 bf16 SpMM layer (PLAIN and STACK) with the default library and the
LGX_SPMM_NT build (CSR streamed with non-temporal loads), HIP events, best of reps.
  python tools/nt_probe.py [--lib tools/liblgx_nt.so]"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
args = ap.parse_args()
import factors_of_serendipity_recommendation_amd as lgx  # noqa: E402
from factors_of_serendipity_recommendation_amd import _lib, ops  # noqa: E402
if args.lib:
    _lib.LIB_PATH = os.path.abspath(args.lib)
from factors_of_serendipity_recommendation_amd.synth import CONFIGS, synth_graph  # noqa: E402

print("lib:", _lib.LIB_PATH, flush=True)
cfg = CONFIGS["synth10m"]
A = synth_graph(cfg, seed=2020, device="cuda")
N, d = cfg.n_users + cfg.n_items, cfg.d
E0 = lgx.fill_normal((N, d), 0.1, 2020, dtype=torch.bfloat16)
Y1 = torch.empty((N, d), dtype=torch.bfloat16, device="cuda")
Y2 = torch.empty((N, d), dtype=torch.bfloat16, device="cuda")
out = torch.empty((N, d), dtype=torch.float32, device="cuda")


def timed(fn, reps=4):
    fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best


print(f"PLAIN {timed(lambda: ops.propagate_layer(A, E0, _lib.LGX_LAYER_PLAIN, Y=Y1)):.3f} ms", flush=True)
print(f"STACK {timed(lambda: ops.propagate_layer_stack(A, Y2, E0, [Y1, Y2], out, 4.0)):.3f} ms", flush=True)
