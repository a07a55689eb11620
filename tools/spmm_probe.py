"""Development probe: where the C4 SpMM layer spends its time (not part of the library).

  python tools/spmm_probe.py [--blocks 8,16]

Builds the synth10m graph (10M users x 1M items, 1e9 nnz, d=128 bf16) and times, with HIP events:
  * the full fused layer (MID mode), as the bench runs it;
  * its two halves: user rows gathering the 256 MB item table (A_pull) and item rows gathering the
    2.56 GB user table (A_push), each as one PLAIN launch;
  * A_push cut into column blocks of the user table (one PARTIAL launch per block), to price a
    cache-blocked schedule before building it.
Each line: ms per launch (min of reps) and the algorithmic rate (layer_bytes / t).
"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
ap.add_argument("--blocks", default="8,20")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--phase", action="store_true", help="time phase-ordered plans (items then users)")
ap.add_argument("--hot", default="", help="hot-column set sizes to split off, e.g. 4096,16384")
ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
args = ap.parse_args()

from factors_of_serendipity_recommendation_amd import _lib  # noqa: E402

if args.lib:
    _lib.LIB_PATH = os.path.abspath(args.lib)
import factors_of_serendipity_recommendation_amd as lgx  # noqa: E402
from factors_of_serendipity_recommendation_amd import ops  # noqa: E402
from factors_of_serendipity_recommendation_amd.distributed import _planned, make_shard  # noqa: E402
from factors_of_serendipity_recommendation_amd.synth import CONFIGS, synth_graph  # noqa: E402


def layer_bytes(nnz, rows, d, s, out_s=None):
    return nnz * (4 + 4 + d * s) + rows * d * (out_s or s) + 8 * (rows + 1)


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


def report(name, ms, nbytes):
    print(f"{name:<40s} {ms:9.3f} ms  {nbytes / ms / 1e9:7.3f} TB/s algorithmic", flush=True)


cfg = CONFIGS["synth10m"]
U, I, d = cfg.n_users, cfg.n_items, cfg.d
print("lib:", _lib.LIB_PATH, flush=True)
t0 = time.time()
A = synth_graph(cfg, seed=2020, device="cuda")
print(f"graph nnz={A.nnz} in {time.time() - t0:.1f}s seg_len={A.plan.seg_len}", flush=True)
N = U + I
DT = torch.bfloat16 if args.dtype == "bf16" else torch.float32
ES = 2 if args.dtype == "bf16" else 4
E0 = lgx.fill_normal((N, d), 0.1, 2020, dtype=DT)
Y = torch.empty((N, d), dtype=DT, device="cuda")
acc = torch.zeros((N, d), dtype=torch.float32, device="cuda")
out = torch.empty((N, d), dtype=torch.float32, device="cuda")
ms = timed(lambda: ops.propagate_layer(A, E0, _lib.LGX_LAYER_MID, Y=Y, E0=E0, acc=acc, out=out, n_mean=4.0), args.reps)
report("full layer (MID)", ms, layer_bytes(A.nnz, N, d, ES))
if args.phase:
    from factors_of_serendipity_recommendation_amd.graph import make_plan  # noqa: E402
    ms = timed(lambda: ops.propagate_layer(A, E0, _lib.LGX_LAYER_PLAIN, Y=Y), args.reps)
    report("full layer (PLAIN)", ms, layer_bytes(A.nnz, N, d, ES))
    ip_host = A.indptr.cpu().numpy()
    for tag, ph in (("items then users", [(U, N), (0, U)]), ("users then items", [(0, U), (U, N)])):
        A.plan = make_plan(ip_host, A.plan.seg_len, phases=ph)
        A._dev_plan.clear()
        A.ensure_plan()
        for mname, mode in (("PLAIN", _lib.LGX_LAYER_PLAIN), ("MID", _lib.LGX_LAYER_MID)):
            ms = timed(lambda: ops.propagate_layer(A, E0, mode, Y=Y, E0=E0, acc=acc, out=out, n_mean=4.0), args.reps)
            report(f"phased {tag} ({mname})", ms, layer_bytes(A.nnz, N, d, ES))
    for sl in (8192, 16384, 32768):
        A.plan = make_plan(ip_host, sl, phases=[(0, U), (U, N)])
        A._dev_plan.clear()
        A.ensure_plan()
        ms = timed(lambda: ops.propagate_layer(A, E0, _lib.LGX_LAYER_MID, Y=Y, E0=E0, acc=acc, out=out, n_mean=4.0), args.reps)
        report(f"phased users/items seg_len {sl} (MID)", ms, layer_bytes(A.nnz, N, d, ES))

sh = make_shard(A, U, I, 0, 1)
del A, acc, out
torch.cuda.empty_cache()
Xi, Xu = E0[U:].contiguous(), E0[:U].contiguous()
Yu = torch.empty((U, d), dtype=DT, device="cuda")
Yi = torch.empty((I, d), dtype=DT, device="cuda")
ms = timed(lambda: ops.propagate_layer(sh.A_pull, Xi, _lib.LGX_LAYER_PLAIN, Y=Yu), args.reps)
report("user rows <- item table (A_pull)", ms, layer_bytes(sh.A_pull.nnz, U, d, ES))
ms = timed(lambda: ops.propagate_layer(sh.A_push, Xu, _lib.LGX_LAYER_PLAIN, Y=Yi), args.reps)
report("item rows <- user table (A_push)", ms, layer_bytes(sh.A_push.nnz, I, d, ES))



def split_csr(G, keep_col):
    """(hot, cold) CSRs of G: edges whose column is / is not in keep_col (bool [n_cols])."""
    r = torch.repeat_interleave(torch.arange(G.n_rows, device="cuda", dtype=torch.int64), torch.diff(G.indptr))
    hot = keep_col[G.indices.to(torch.int64)]
    outs = []
    for sel in (hot, ~hot):
        ip = torch.zeros(G.n_rows + 1, dtype=torch.int64, device="cuda")
        ip[1:] = torch.cumsum(torch.bincount(r[sel], minlength=G.n_rows), 0)
        outs.append(_planned(ip, G.indices[sel], G.vals[sel], G.n_rows, G.n_cols, None))
    return outs


for name, G, X, n_out in (("A_pull", sh.A_pull, Xi, U), ("A_push", sh.A_push, Xu, I)):
    if not args.hot:
        break
    deg = torch.bincount(G.indices.to(torch.int64), minlength=G.n_cols)
    order = torch.argsort(deg, descending=True)
    outb = torch.empty((n_out, d), dtype=torch.float32, device="cuda")
    for H in [int(x) for x in args.hot.split(",")]:
        keep = torch.zeros(G.n_cols, dtype=torch.bool, device="cuda")
        keep[order[:H]] = True
        hot, cold = split_csr(G, keep)
        torch.cuda.synchronize()
        ms_h = timed(lambda: ops.propagate_layer(hot, X, _lib.LGX_LAYER_PARTIAL, out=outb), args.reps)
        ms_c = timed(lambda: ops.propagate_layer(cold, X, _lib.LGX_LAYER_PARTIAL, out=outb), args.reps)
        report(f"{name} hot {H} cols ({hot.nnz / G.nnz:.2f} of nnz)", ms_h, layer_bytes(hot.nnz, n_out, d, ES, 4))
        report(f"{name} cold rest", ms_c, layer_bytes(cold.nnz, n_out, d, ES, 4))
        del hot, cold
        torch.cuda.empty_cache()
    del outb

P = sh.A_push
rows = torch.repeat_interleave(torch.arange(P.n_rows, device="cuda", dtype=torch.int64), torch.diff(P.indptr))
Pout = torch.empty((I, d), dtype=torch.float32, device="cuda")
for nb in [int(x) for x in args.blocks.split(",") if x]:
    edges = torch.linspace(0, U, nb + 1, device="cuda").round().to(torch.int64)
    blk = torch.bucketize(P.indices.to(torch.int64), edges[1:], right=True)
    subs = []
    for c in range(nb):
        sel = blk == c
        r = rows[sel]
        ip = torch.zeros(P.n_rows + 1, dtype=torch.int64, device="cuda")
        ip[1:] = torch.cumsum(torch.bincount(r, minlength=P.n_rows), 0)
        subs.append(_planned(ip, P.indices[sel], P.vals[sel], P.n_rows, U, None))
        del sel, r
    torch.cuda.synchronize()

    def run():
        for g in subs:
            ops.propagate_layer(g, Xu, _lib.LGX_LAYER_PARTIAL, out=Pout)

    ms = timed(run, args.reps)
    report(f"A_push in {nb} user-column blocks", ms, layer_bytes(P.nnz, I, d, ES))
    del subs
    torch.cuda.empty_cache()
print("probe done", flush=True)
