"""Development probe: does a degree-ordered numbering of the C4 graph (users and items each sorted by
descending degree) change the SpMM layer time, alone and with non-temporal cold gathers?

  python tools/renum_probe.py

Times the fused MID layer (bf16 d=128) on the original and the renumbered graph; with the ntcold
library, also with gathers of users ranked >= Hu and items ranked >= Hi non-temporal (H pairs
from --cuts).  The renumbered CSR is rebuilt canonically (rows in the new order, columns sorted).
"""
import argparse
import ctypes
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--dtype", default="bf16")
args = ap.parse_args()
from factors_of_serendipity_recommendation_amd import _lib  # noqa: E402
if args.lib:
    _lib.LIB_PATH = os.path.abspath(args.lib)
import factors_of_serendipity_recommendation_amd as lgx  # noqa: E402
from factors_of_serendipity_recommendation_amd import ops  # noqa: E402
from factors_of_serendipity_recommendation_amd.synth import CONFIGS, synth_graph  # noqa: E402


def timed(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return min(ts)


cfg = CONFIGS["synth10m"]
U, I, d = cfg.n_users, cfg.n_items, cfg.d
N = U + I
dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
print("lib:", _lib.LIB_PATH, flush=True)
t0 = time.time()
A = synth_graph(cfg, seed=2020, device="cuda")
print(f"graph nnz={A.nnz} in {time.time() - t0:.1f}s", flush=True)
E0 = lgx.fill_normal((N, d), 0.1, 2020, dtype=dt)
Y = torch.empty((N, d), dtype=dt, device="cuda")
acc = torch.zeros((N, d), dtype=torch.float32, device="cuda")
out = torch.empty((N, d), dtype=torch.float32, device="cuda")


def layer(G):
    return timed(lambda: ops.propagate_layer(G, E0, _lib.LGX_LAYER_MID, Y=Y, E0=E0, acc=acc, out=out, n_mean=4.0),
                 args.reps)


print(f"original numbering    MID {layer(A):8.3f} ms", flush=True)
t0 = time.time()
deg = torch.diff(A.indptr)
order = torch.cat([torch.argsort(-deg[:U], stable=True), U + torch.argsort(-deg[U:], stable=True)])
inv = torch.empty_like(order)
inv[order] = torch.arange(N, device="cuda")
rows = torch.repeat_interleave(torch.arange(N, device="cuda"), deg)
key = inv[rows] * N + inv[A.indices.long()]
del rows
key, perm = torch.sort(key)
vals = A.vals[perm]
del perm
ncol = (key % N).to(torch.int32)
nrow = key // N
del key
indptr = torch.zeros(N + 1, dtype=torch.int64, device="cuda")
indptr[1:] = torch.cumsum(torch.bincount(nrow, minlength=N), 0)
del nrow, A
torch.cuda.empty_cache()
B = lgx.from_csr_arrays(indptr, ncol, vals, device="cuda", n_users=U, n_items=I)
print(f"renumbered in {time.time() - t0:.1f}s", flush=True)
print(f"degree-ordered        MID {layer(B):8.3f} ms", flush=True)
print("probe done", flush=True)
