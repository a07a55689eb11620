"""Multi-GPU readiness on ONE GPU: the per-rank work of the C4 propagation at world = 8 (or --world),
timed rank by rank with the real kernels, plus the per-layer collective volumes of
distributed.ShardedPropagation.  Prints one JSON document with a predicted per-layer and per-step
time at two assumed RCCL rates (one xGMI link, and the sum of the 7 links at an assumed efficiency).

  python tools/shard_probe.py [--world 8] [--ranks 0,7] [--dtype bf16] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import factors_of_serendipity_recommendation_amd as lgx  # noqa: E402
from factors_of_serendipity_recommendation_amd import _lib, ops  # noqa: E402
from factors_of_serendipity_recommendation_amd.distributed import make_shard  # noqa: E402
from factors_of_serendipity_recommendation_amd.synth import CONFIGS, synth_graph  # noqa: E402

LINK_GBS = 153.0       # one xGMI link per direction (task brief: 7 links x ~153 GB/s per GPU)
LINKS = 7


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--ranks", default="0,7")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--link-efficiency", type=float, default=0.6)
    args = ap.parse_args()
    cfg = CONFIGS["synth10m"]
    U, I, d, K, w = cfg.n_users, cfg.n_items, cfg.d, cfg.K, args.world
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    s = 2 if dt == torch.bfloat16 else 4
    t0 = time.time()
    A = synth_graph(cfg, seed=2020, device="cuda")
    print(f"graph nnz={A.nnz} in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    # the single-GPU layer for reference (same graph, same kernels)
    E0 = lgx.fill_normal((U + I, d), 0.1, 2020, dtype=dt)
    Y = torch.empty_like(E0)
    acc = torch.zeros((U + I, d), dtype=torch.float32, device="cuda")
    out = torch.empty((U + I, d), dtype=torch.float32, device="cuda")
    one_gpu = timed(lambda: ops.propagate_layer(A, E0, _lib.LGX_LAYER_MID, Y=Y, E0=E0, acc=acc, out=out,
                                                n_mean=float(K + 1)), args.reps)
    del Y, acc, out
    torch.cuda.empty_cache()
    ranks = []
    for r in (int(x) for x in args.ranks.split(",")):
        t0 = time.time()
        sh = make_shard(A, U, I, r, w)
        build = time.time() - t0
        nu, mi = sh.n_u_local, sh.mi
        Xu = lgx.fill_normal((nu, d), 0.1, 7 + r, dtype=dt)
        Xi = lgx.fill_normal((w * mi, d), 0.1, 11, dtype=dt)
        P = torch.empty((w * mi, d), dtype=torch.float32, device="cuda")
        Yu = torch.empty((nu, d), dtype=dt, device="cuda")
        acc_u = torch.zeros((nu, d), dtype=torch.float32, device="cuda")
        out_u = torch.empty((nu, d), dtype=torch.float32, device="cuda")
        yi = torch.randn((mi, d), dtype=torch.float32, device="cuda")
        Yi = torch.empty((mi, d), dtype=dt, device="cuda")
        acc_i = torch.zeros((mi, d), dtype=torch.float32, device="cuda")
        out_i = torch.empty((mi, d), dtype=torch.float32, device="cuda")
        E0i = Xi[:mi]
        push = timed(lambda: ops.propagate_layer(sh.A_push, Xu, _lib.LGX_LAYER_PARTIAL, out=P), args.reps)
        pull = timed(lambda: ops.propagate_layer(sh.A_pull, Xi, _lib.LGX_LAYER_MID, Y=Yu, E0=Xu, acc=acc_u,
                                                 out=out_u, n_mean=float(K + 1)), args.reps)
        epi = timed(lambda: ops.layer_epilogue(yi, _lib.LGX_LAYER_MID, Y=Yi, E0=E0i, acc=acc_i, out=out_i,
                                               n_mean=float(K + 1)), args.reps)
        rs_bytes = (w - 1) / w * (w * mi) * d * 4      # reduce-scatter of the fp32 push partials
        ag_bytes = (w - 1) / w * (w * mi) * d * s      # all-gather of the item block of the layer
        ranks.append({"rank": r, "users": nu, "pull_nnz": sh.A_pull.nnz, "push_nnz": sh.A_push.nnz,
                      "shard_build_s": round(build, 2), "push_ms": push, "pull_ms": pull, "item_epilogue_ms": epi,
                      "reduce_scatter_bytes": int(rs_bytes), "all_gather_bytes": int(ag_bytes)})
        print(json.dumps(ranks[-1]), file=sys.stderr, flush=True)
        del sh, Xu, Xi, P, Yu, acc_u, out_u, yi, Yi, acc_i, out_i
        torch.cuda.empty_cache()
    worst = max(ranks, key=lambda x: x["push_ms"] + x["pull_ms"] + x["item_epilogue_ms"])
    compute = worst["push_ms"] + worst["pull_ms"] + worst["item_epilogue_ms"]
    pred = {}
    for name, gbs in (("one_link", LINK_GBS), (f"{LINKS}_links_x{args.link_efficiency}", LINKS * LINK_GBS * args.link_efficiency)):
        rs = worst["reduce_scatter_bytes"] / gbs / 1e6
        ag = worst["all_gather_bytes"] / gbs / 1e6
        # schedule (distributed.py): RS(k) hides under pull(k), AG(k) under push(k+1); exposed = the excess
        exposed = max(0.0, rs - worst["pull_ms"]) + max(0.0, ag - worst["push_ms"])
        layer = compute + exposed
        step = K * compute + max(0.0, rs - worst["pull_ms"]) * K + max(0.0, ag - worst["push_ms"]) * (K - 1)
        pred[name] = {"rccl_GBs_assumed": gbs, "reduce_scatter_ms": rs, "all_gather_ms": ag,
                      "exposed_comm_ms_per_layer": exposed, "layer_ms": layer, "step_ms": step,
                      "speedup_vs_1gpu": (K * one_gpu) / step}
    print(json.dumps({"workload": f"synth10m {args.dtype} K={K} d={d}, world={w}", "one_gpu_layer_ms": one_gpu,
                      "ranks": ranks, "critical_rank": worst["rank"], "compute_ms_per_layer": compute,
                      "prediction": pred,
                      "note": "per-rank kernels timed on one MI355X (HIP events, best of reps); collective "
                              "times are volumes / assumed RCCL rates, not measurements"}, indent=1), flush=True)


if __name__ == "__main__":
    main()
