"""Benchmark of the LightGCN hot path on MI355X (contract: one JSON line from rank 0).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config synth10m] [--score-users 65536]
  N>1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Workload (BASELINE.json): the propagation metric is quoted at 1/2/4/8 GPUs on configs[3]
("Synthetic 10M users x 1M items, 500M edges, K=3, d=128, row-sharded with RCCL all-gather"),
which fits one MI355X (CSR 8 GB + tables < 30 GB of 288 GB), so it is the N=1 workload too and the
total graph is fixed as N grows (strong scaling).  One step = one full K-layer propagation
(LightGCN.computer(), model.py:145-177) with bf16 embedding storage and fp32 accumulation.
The scoring metric (configs[4]: user x item MFMA scoring + train mask + top-20, d=256 bf16, 1M
items) is reported in the same line under "scoring": one step scores a fixed batch of query users
against the full catalog, the batch split across ranks.

value = K * nnz(A^) * steps / t  (edges/s), t = max over ranks of the barrier-bracketed loop.
roofline.achieved = algorithmic bytes per SpMM launch / mean launch time (HIP events on the
compute stream), bytes per layer = nnz*(4 + 4 + d*s) + rows*d*s + 8*(rows+1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import factors_of_serendipity_recommendation_amd as lgx  # noqa: E402
from factors_of_serendipity_recommendation_amd import _lib, ops  # noqa: E402
from factors_of_serendipity_recommendation_amd.distributed import ShardedPropagation, make_shard  # noqa: E402
from factors_of_serendipity_recommendation_amd.synth import CONFIGS, synth_graph  # noqa: E402

HBM_PEAK = 8.0e12        # MI355X HBM3E spec (MI355X_MICROARCH.md)
BF16_MFMA_PEAK = 2.5e15  # dense bf16 MFMA spec
METRIC = "LightGCN prop edges/s + full-catalog score items/s at 1/2/4/8 MI355X"


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def barrier_sync(world):
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def measured_traffic(config: str, world: int, kernels) -> tuple:
    """HBM bytes per launch from the newest committed rocprofv3 PMC summary for this workload
    (profiles/rNN_<config>_pmc_traffic.json; (2*FETCH_SIZE + WRITE_SIZE) per MI355X_MICROARCH.md).
    Returns (GB per launch or None, source file)."""
    import glob
    if world != 1:
        return None, None
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{config}_pmc_traffic.json")))
    if not files:
        return None, None
    doc = json.load(open(files[-1]))
    try:
        b = sum(doc["kernels"][k]["hbm_bytes_per_launch"] for k in kernels)
    except KeyError:
        return None, None
    return b / 1e9, os.path.relpath(files[-1], ROOT)


def layer_bytes(nnz: int, rows: int, d: int, s: int, out_s: int = 0) -> int:
    """col id + value + one gathered row per nonzero, one output row per row, indptr."""
    return nnz * (4 + 4 + d * s) + rows * d * (out_s or s) + 8 * (rows + 1)


def bench_propagation(args, rank, world):
    cfg = CONFIGS[args.config]
    dtype = torch.bfloat16 if (args.dtype or cfg.dtype) == "bf16" else torch.float32
    es = 2 if dtype == torch.bfloat16 else 4
    t0 = time.time()
    A = synth_graph(cfg, seed=2020, device="cuda")
    N = cfg.n_users + cfg.n_items
    log(f"[bench] graph {cfg.name}: N={N} nnz={A.nnz} built in {time.time() - t0:.1f}s")
    E0 = lgx.fill_normal((N, cfg.d), 0.1, 2020, dtype=dtype)
    K, d = cfg.K, cfg.d
    timings = []  # (start, end) events around every SpMM layer launch on the compute stream

    if world == 1:
        out = torch.empty((N, d), dtype=torch.float32, device="cuda")
        bufs = [torch.empty((N, d), dtype=dtype, device="cuda") for _ in range(2)]
        acc = torch.empty((N, d), dtype=torch.float32, device="cuda")
        local_nnz, local_rows = A.nnz, N

        def step(record):
            X = E0
            for k in range(1, K + 1):
                mode = (_lib.LGX_LAYER_ONLY if K == 1 else _lib.LGX_LAYER_FIRST if k == 1
                        else _lib.LGX_LAYER_LAST if k == K else _lib.LGX_LAYER_MID)
                Y = bufs[k & 1] if k < K else None
                if record:
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                ops.propagate_layer(A, X, mode, Y=Y, E0=E0, acc=acc, out=out, n_mean=float(K + 1))
                if record:
                    e1.record()
                    timings.append((e0, e1, layer_bytes(A.nnz, A.n_rows, d, es)))
                X = Y
    else:
        shard = make_shard(A, cfg.n_users, cfg.n_items, rank, world)
        del A
        torch.cuda.empty_cache()
        prop = ShardedPropagation(shard, E0[:cfg.n_users], E0[cfg.n_users:], K)
        del E0
        local_nnz = shard.A_pull.nnz + shard.A_push.nnz  # every edge of the rank's users, both directions
        local_rows = shard.n_u_local + shard.n_i_local

        def layer_fn(Aop, X, mode, **kw):
            if step.record:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
            ops.propagate_layer(Aop, X, mode, **kw)
            if step.record:
                e1.record()
                # the push launch writes fp32 partial sums
                out_s = 4 if mode == _lib.LGX_LAYER_PARTIAL else es
                timings.append((e0, e1, layer_bytes(Aop.nnz, Aop.n_rows, d, es, out_s)))

        prop.layer_fn = layer_fn

        def step(record):
            step.record = record
            prop.step()
        step.record = False

    nnz_all = local_nnz
    if world > 1:
        t = torch.tensor([local_nnz], dtype=torch.int64, device="cuda")
        dist.all_reduce(t)
        nnz_all = int(t.item())

    for _ in range(args.warmup):
        step(False)
    barrier_sync(world)
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    barrier_sync(world)
    elapsed = max_over_ranks(time.perf_counter() - t_start, world)
    # per-launch time of the dominant kernel family (spmm_segments + its fix-up pass)
    launch_ms = [e0.elapsed_time(e1) for e0, e1, _ in timings]
    mean_launch_s = float(np.mean(launch_ms)) / 1e3
    bytes_per_launch = float(np.mean([b for _, _, b in timings]))
    achieved = bytes_per_launch / mean_launch_s
    edges = K * nnz_all * args.steps
    traffic, traffic_src = measured_traffic(cfg.name, world, ["spmm_segments", "spmm_fixup"])
    res = {
        "cfg": cfg, "dtype": "bf16" if es == 2 else "f32", "value": edges / elapsed,
        "ms_per_step": elapsed / args.steps * 1e3, "nnz": nnz_all,
        "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK, "traffic": traffic, "traffic_unit": "GB/launch",
                     "traffic_source": traffic_src,
                     "kernel": "spmm_segments (+spmm_fixup)", "bytes_per_launch": int(bytes_per_launch),
                     "mean_launch_ms": mean_launch_s * 1e3,
                     # achieved counts every gathered row as an HBM read, so the caches that serve part
                     # of them can lift frac above 1; the PMC bytes over the same launch time are the
                     # HBM rate the kernel really pulls
                     "traffic_rate_gbs": traffic / mean_launch_s if traffic else None,
                     "traffic_frac": traffic * 1e9 / mean_launch_s / HBM_PEAK if traffic else None},
        "graph": A if world == 1 else None, "E0": E0 if world == 1 else None,
    }
    return res


def cpu_baseline(res, args):
    """oracle/torch_ref.py (torch.sparse.mm on the host, model.py:163-175) on a bounded row block
    of the same graph against the full fp32 table."""
    from oracle import torch_ref
    A, E0 = res["graph"], res["E0"]
    cfg = res["cfg"]
    threads = min(os.cpu_count() or 1, 16)
    ip = A.indptr.cpu().numpy()
    target = args.cpu_nnz
    r1 = int(np.searchsorted(ip, target))
    r1 = max(1, min(r1, A.n_rows))
    nnz = int(ip[r1])
    G = torch_ref.coo_from_csr(ip[:r1 + 1], A.indices[:nnz].cpu().numpy(), A.vals[:nnz].cpu().numpy(), A.n_cols)
    X = E0.float().cpu()
    r = torch_ref.time_spmm_rows(G, X, cfg.K, threads)
    return {"value": r["edges_per_s"], "unit": "edges/s", "cores": threads, "kind": "port",
            "sample": f"rows [0,{r1}) of the same graph ({nnz} nnz, {cfg.K} x torch.sparse.mm against the full "
                      f"fp32 [{A.n_cols},{cfg.d}] table, {r['seconds']:.1f}s)"}


def bench_scoring(args, rank, world):
    """configs[4]: d=256 bf16, 1M items, top-20 with a train mask; users split over ranks."""
    d, n_items, k = 256, args.score_items, 20
    B_total = args.score_users
    B = B_total // world
    items = lgx.fill_normal((n_items, d), 1.0 / 16, 4242, dtype=torch.bfloat16)
    Q = lgx.fill_normal((B, d), 1.0 / 16, 777 + rank, dtype=torch.bfloat16)
    g = torch.Generator(device="cuda")
    g.manual_seed(99 + rank)
    per = 50
    pos = torch.randint(0, n_items, (B, per), device="cuda", generator=g).sort(dim=1).values
    mask = (torch.arange(0, B + 1, device="cuda", dtype=torch.int64) * per, pos.reshape(-1).to(torch.int32))
    for _ in range(max(1, args.warmup // 2)):
        ops.score_topk(Q, items, k, mask=mask)
    barrier_sync(world)
    ev = []
    t_start = time.perf_counter()
    steps = max(1, args.score_steps)
    for _ in range(steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.score_topk(Q, items, k, mask=mask)
        e1.record()
        ev.append((e0, e1))
    barrier_sync(world)
    elapsed = max_over_ranks(time.perf_counter() - t_start, world)
    mean_launch = float(np.mean([a.elapsed_time(b) for a, b in ev])) / 1e3
    flops = 2.0 * B * n_items * d
    traffic, traffic_src = measured_traffic(args.config, world, ["score_topk_bf16_lds"])
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = scoring_cpu_baseline(Q, items, pos, k, args.cpu_score_users)
    return {"value": B_total * n_items * steps / elapsed, "unit": "items/s", "users_per_step": B_total,
            "n_items": n_items, "d": d, "k": k, "dtype": "bf16", "ms_per_step": elapsed / steps * 1e3,
            "roofline": {"bound": "mfma", "achieved": flops / mean_launch / 1e12, "peak": BF16_MFMA_PEAK / 1e12,
                         "unit": "TFLOP/s", "frac": flops / mean_launch / BF16_MFMA_PEAK, "traffic": traffic,
                         "traffic_unit": "GB/launch", "traffic_source": traffic_src,
                         "kernel": "score_topk_bf16_lds (+ score_topk_finalize, both inside the timed launch)"},
            "cpu_baseline": cpu}


def scoring_cpu_baseline(Q, items, pos, k, n_users):
    """The reference's CPU scoring procedure (Procedure.py:121-135 per 100-user batch: fp32 matmul,
    sigmoid, train mask, torch.topk) on the first n_users query users of the same batch."""
    from oracle import torch_ref
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    Qc = Q[:n_users].float().cpu()
    Ic = items.float().cpu()
    masks = [row for row in pos[:n_users].cpu().numpy()]
    torch_ref.score_topk_cpu(Qc[:100], Ic, k, masks[:100])  # warm-up
    _, t = torch_ref.score_topk_cpu(Qc, Ic, k, masks)
    return {"value": n_users * items.shape[0] / t, "unit": "items/s", "cores": threads, "kind": "port",
            "sample": f"{n_users} of the query users x {items.shape[0]} items, d={items.shape[1]} fp32, "
                      f"top-{k} with the same train masks ({t:.1f}s)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="synth10m", choices=sorted(CONFIGS))
    ap.add_argument("--dtype", default=None, choices=[None, "bf16", "f32"])
    ap.add_argument("--score-users", type=int, default=1_000_000)
    ap.add_argument("--score-items", type=int, default=1_000_000)
    ap.add_argument("--score-steps", type=int, default=2)
    ap.add_argument("--cpu-nnz", type=int, default=40_000_000)
    ap.add_argument("--cpu-score-users", type=int, default=4000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-scoring", action="store_true")
    ap.add_argument("--no-propagation", action="store_true", help="development: scoring leg only")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    local_rank %= max(1, torch.cuda.device_count())  # identity on a real node; rehearsal ranks share a GPU
    torch.cuda.set_device(local_rank)
    if world > 1:
        # LGX_BENCH_BACKEND=gloo: rehearsal of the N>1 path with ranks sharing one GPU (RCCL refuses
        # that); measurements are always taken over RCCL ("nccl")
        backend = os.environ.get("LGX_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)
    if world != args.gpus:
        log(f"[bench] warning: --gpus {args.gpus} but WORLD_SIZE={world}")

    if args.no_propagation:
        sc = bench_scoring(args, rank, world)
        if rank == 0:
            print(json.dumps({"metric": METRIC, "scoring": sc}), flush=True)
        return
    res = bench_propagation(args, rank, world)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(res, args)
    res.pop("graph", None)
    res.pop("E0", None)
    torch.cuda.empty_cache()
    scoring = None if args.no_scoring else bench_scoring(args, rank, world)
    cfg = res["cfg"]
    line = {
        "metric": METRIC, "value": res["value"], "unit": "edges/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": res["ms_per_step"], "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": res["dtype"], "data": "synthetic (seeded power-law bipartite graph)",
        "config": {"workload": f"{cfg.name}: {cfg.n_users} users x {cfg.n_items} items, {cfg.n_edges} edges "
                               f"(nnz {res['nnz']}), K={cfg.K}, d={cfg.d}, {res['dtype']} storage / fp32 accumulate",
                   "parallelism": f"row-shard{world}" if world > 1 else "single"},
        "roofline": res["roofline"], "cpu_baseline": cpu, "scoring": scoring,
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
