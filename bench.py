"""Benchmark of the LightGCN hot path on MI355X (contract: one JSON line from rank 0).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config synth10m] [--score-users 1000000]
  N>1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N
       or just `python bench.py --gpus N`: without WORLD_SIZE in the environment it starts the N
       ranks itself (torch.distributed.run as a child process) and forwards rank 0's line; a
       WORLD_SIZE that differs from --gpus is an error (exit 2), never a silent one-rank run.

Workload (BASELINE.json): the propagation metric is quoted at 1/2/4/8 GPUs on configs[3]
("Synthetic 10M users x 1M items, 500M edges, K=3, d=128, row-sharded with RCCL all-gather"),
which fits one MI355X (CSR 8 GB + tables < 30 GB of 288 GB), so it is the N=1 workload too and the
total graph is fixed as N grows (strong scaling).  One step = one full K-layer propagation
(LightGCN.computer(), model.py:145-177).  `value` / `dtype` are the fp32-storage run, the
reference's precision (model.py:163-176); the same line carries the bf16-storage / fp32-accumulate
run ("fp32 parity; bf16 perf") under "bf16".  The scoring metric (configs[4]: user x
item MFMA scoring + train mask + top-20, d=256, 1M items) is reported under "scoring" in fp32 (the
reference's precision, model.py:183) and under "scoring_bf16" (SURVEY C5's bf16 inputs), both on
SURVEY C5's 1M query users: one step scores a fixed batch of query
users against the full catalog, the batch split across ranks.

value = K * nnz(A^) * steps / t  (edges/s), t = max over ranks of the barrier-bracketed loop.

SpMM roofline (per launch of spmm_segments + spmm_fixup, HIP events on the compute stream):
  * achieved = model bytes / mean launch time, where the model is cache-aware: the CSR stream
    (8 B/nnz + indptr), the layer's epilogue I/O (mode-dependent), and every gathered table row
    EXCEPT those of the hottest rows that fit one XCD's 4 MiB L2 (by column degree, per table).
    Those rows are served from L2 at 19.4 TB/s (profiles/r02_fetch_calibration.json sweep), so a
    schedule cannot be made to pull them from HBM; every other gather is counted as one HBM row
    read.  This stays below the kernel's measured L2-miss traffic, so frac <= 1.
  * floor_bytes = nnz*8 + 2*N*d*s (SURVEY 8(d) compulsory floor); gathered_bytes = every gathered
    row counted (the SURVEY 8(d) figure, which can exceed the HBM peak on cached rows).
  * traffic = calibrated rocprofv3 counter bytes per launch (2 x FETCH_SIZE + WRITE_SIZE; the x2
    measured for this access pattern in profiles/r02_fetch_calibration.json) from this round's PMC
    profile, used only when that profile was taken from the same liblgx.so build (sha256).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import math
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
from factors_of_serendipity_recommendation_amd.distributed import ShardedPropagation, make_shard_from_edges  # noqa: E402
from factors_of_serendipity_recommendation_amd.synth import CONFIGS, synth_edges, synth_graph  # noqa: E402

HBM_PEAK = 8.0e12        # MI355X HBM3E spec (MI355X_MICROARCH.md)
BF16_MFMA_PEAK = 2.5e15  # dense bf16 MFMA spec
F32_MFMA_PEAK = 157.3e12  # f32-input MFMA (v_mfma_f32_32x32x2_f32), MI355X_MICROARCH.md:42
L2_BYTES = 4 << 20       # per XCD
METRIC = "LightGCN prop edges/s + full-catalog score items/s at 1/2/4/8 MI355X"
CALIB = "profiles/r02_fetch_calibration.json"


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


def lib_sha() -> str:
    h = hashlib.sha256()
    with open(_lib.LIB_PATH, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()[:16]


def measured_traffic(config: str, dtype: str, world: int, kernels, calls_from=None) -> tuple:
    """Calibrated counter bytes per launch from the newest committed PMC summary of this workload
    (profiles/rNN_<config>_pmc_traffic.json), if it was collected from the library build that is
    running now.  Returns (GB per launch or None, source or reason).  calls_from = (kernel, its
    dispatches per call): the bytes of every dispatch of `kernels` per library call instead (a call
    that launches a kernel several times, as lgx_score_topk's seeded stages do)."""
    import glob
    if world != 1:
        return None, "PMC profiles are single-GPU"
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{config}_pmc_traffic.json")))
    if not files:
        return None, "no PMC profile"
    doc = json.load(open(files[-1]))
    src = os.path.relpath(files[-1], ROOT)
    if doc.get("lib_sha256_16") != lib_sha():
        return None, f"{src} was taken from another liblgx.so build"
    try:
        ks = doc["kernels"][dtype]
        if calls_from:
            calls = ks[calls_from[0]]["dispatches"] / calls_from[1]
            b = sum(ks[k]["hbm_bytes_per_launch"] * ks[k]["dispatches"] for k in kernels) / calls
        else:
            b = sum(ks[k]["hbm_bytes_per_launch"] for k in kernels)
    except KeyError:
        return None, f"{src} has no {dtype} entry"
    return b / 1e9, src


def epilogue_bytes(mode: int, rows: int, d: int, s: int, n_prev: int = 0) -> int:
    """Bytes the layer epilogue moves per mode (ops.propagate_layer modes, spmm.hip finish_chunk)."""
    t, f = rows * d * s, rows * d * 4
    return {_lib.LGX_LAYER_PLAIN: t, _lib.LGX_LAYER_FIRST: t + t + f, _lib.LGX_LAYER_MID: t + 2 * f,
            _lib.LGX_LAYER_LAST: 2 * f, _lib.LGX_LAYER_ONLY: t + f, _lib.LGX_LAYER_PARTIAL: f,
            _lib.LGX_LAYER_STACK: t * (1 + n_prev) + f}[mode]


def cold_gather_rows(A, d: int, s: int) -> tuple:
    """Gathers per layer of rows outside each table's L2-resident hot set: (cold nnz, hot rows,
    hot fraction).  Column degree == row degree (A^ symmetric); the user rows gather the item table
    and the item rows the user table, each its own hot set."""
    deg = torch.diff(A.indptr)
    R = max(1, L2_BYTES // (d * s))
    U, I = A.n_users, A.n_items
    tables = [deg[:U], deg[U:]] if U > 0 and I > 0 else [deg]
    total = int(deg.sum())
    hot = sum(int(torch.topk(t, min(R, t.numel())).values.sum()) for t in tables if t.numel())
    return total - hot, R, hot / max(1, total)


def cold_gather_cols(Aop, d: int, s: int) -> tuple:
    """cold_gather_rows for a rectangular shard operator (N>1): it gathers ONE table (its columns),
    whose L2 hot set is the top-R columns by in-operator count (bincount of the column ids)."""
    cnt = torch.bincount(Aop.indices.to(torch.int64), minlength=Aop.n_cols)
    R = max(1, L2_BYTES // (d * s))
    total = int(cnt.sum())
    hot = int(torch.topk(cnt, min(R, cnt.numel())).values.sum()) if cnt.numel() else 0
    return total - hot, R, hot / max(1, total)


def layer_models(A, d: int, s: int, mode: int, n_prev: int = 0, shard_op: bool = False) -> dict:
    """Byte models of one layer launch of operator A (the same conventions at N=1 and N>1): CSR
    stream + epilogue + gathers of rows outside the per-XCD L2 hot set of each gathered table."""
    nnz, rows, N = A.nnz, A.n_rows, A.n_cols
    csr = nnz * 8 + 8 * (rows + 1)
    epi = epilogue_bytes(mode, rows, d, s, n_prev)
    cold, R, hot_frac = cold_gather_cols(A, d, s) if shard_op else cold_gather_rows(A, d, s)
    floor = nnz * 8 + (rows + N) * d * s if shard_op else nnz * 8 + 2 * N * d * s
    # column-blocked item rows: the f32 row sums carried between the nb block launches (written by
    # blocks 0..nb-2, read by blocks 1..nb-1) plus the nb-1 extra block pointers per item row
    nb = A.col_block_count(d, s)
    carry = (2 * (nb - 1) * A.n_items * d * 4 + 8 * (nb - 1) * A.n_items) if nb > 1 else 0
    return {"model": csr + epi + carry + cold * d * s, "gathered": csr + epi + carry + nnz * d * s,
            "floor": floor, "hot_rows": R, "hot_frac": hot_frac, "col_blocks": nb,
            "kernel": ops.spmm_kernel_name(d, torch.bfloat16 if s == 2 else torch.float32, A.plan.seg_len)}


def calibration() -> dict:
    path = os.path.join(ROOT, CALIB)
    if not os.path.exists(path):
        return {}
    doc = json.load(open(path))
    c = doc["cases"]
    return {"source": CALIB, "fetch_size_factor_random_256B_rows": round(c["once_256"]["known_over_fetch_size"], 3),
            "fetch_size_counts_mall_hits": c["hot_mall"]["known_over_fetch_size"] < 3.0,
            "gather_rate_by_table_size_tbs": doc.get("sweep_256", {})}


def make_step(A, E0, K, d, dtype, world, cfg, rank, timings):
    es = 2 if dtype == torch.bfloat16 else 4
    N = A.n_rows if world == 1 else None
    if world == 1:
        # lgx_propagate's schedule: layers 1..K-1 keep their tables (PLAIN), the last layer forms the
        # mean from E0 and them (STACK) -- no f32 running sum moved by every layer
        out = torch.empty((N, d), dtype=torch.float32, device="cuda")
        bufs = [torch.empty((N, d), dtype=dtype, device="cuda") for _ in range(max(1, K - 1))]
        models = {}

        def step(record):
            X = E0
            for k in range(1, K + 1):
                mode = (_lib.LGX_LAYER_ONLY if K == 1 else _lib.LGX_LAYER_STACK if k == K else _lib.LGX_LAYER_PLAIN)
                if record:
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                if mode == _lib.LGX_LAYER_STACK:
                    ops.propagate_layer_stack(A, X, E0, bufs[:K - 1], out, float(K + 1))
                else:
                    ops.propagate_layer(A, X, mode, Y=bufs[k - 1] if k < K else None, E0=E0, out=out,
                                        n_mean=float(K + 1))
                if record:
                    e1.record()
                    if mode not in models:
                        models[mode] = layer_models(A, d, es, mode, K - 1)
                    timings.append((e0, e1, models[mode]))
                if k < K:
                    X = bufs[k - 1]
        return step, A.nnz, A.n_rows
    # N > 1: A is this rank's shard (built from the edge list, never the full operator)
    shard = A
    E0u, E0i = E0  # this rank's user rows, the full item table
    prop = ShardedPropagation(shard, E0u, E0i, K, local_user_rows=True)
    models = {}

    # the N=1 conventions per shard operator: cache-aware model (hot set of the table it gathers),
    # kernel named from the operator's own launch plan
    def layer_fn(Aop, X, mode, **kw):
        if step.record:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        ops.propagate_layer(Aop, X, mode, **kw)
        if step.record:
            e1.record()
            key = (id(Aop), mode)
            if key not in models:
                models[key] = layer_models(Aop, d, es, mode, shard_op=True)
            timings.append((e0, e1, models[key]))

    def stack_fn(Aop, X, E0r, prev, out, n_mean):
        if step.record:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        ops.propagate_layer_stack(Aop, X, E0r, prev, out, n_mean)
        if step.record:
            e1.record()
            key = (id(Aop), _lib.LGX_LAYER_STACK)
            if key not in models:
                models[key] = layer_models(Aop, d, es, _lib.LGX_LAYER_STACK, len(prev), shard_op=True)
            timings.append((e0, e1, models[key]))

    prop.layer_fn = layer_fn
    prop.stack_fn = stack_fn

    def step(record):
        step.record = record
        prop.record_phases = record  # per-phase stamps on the compute stream (distributed.PhaseRecorder)
        prop.step()
    step.record = False
    step.prop = prop
    return step, shard.A_pull.nnz + shard.A_push.nnz, shard.n_u_local + shard.n_i_local


def bench_propagation(args, rank, world, A, cfg, dtype, steps, warmup):
    es = 2 if dtype == torch.bfloat16 else 4
    dname = "bf16" if es == 2 else "f32"
    K, d = cfg.K, cfg.d
    N = cfg.n_users + cfg.n_items
    if world == 1:
        E0 = lgx.fill_normal((N, d), 0.1, 2020, dtype=dtype)
    else:
        # the rows of the N=1 table this rank reads: its own users (no replicated 10 M-row table)
        # and the whole item table (the padded layer-0 item table every rank pulls from)
        u0, u1 = int(A.user_bounds[rank]), int(A.user_bounds[rank + 1])
        E0 = (lgx.fill_normal((u1 - u0, d), 0.1, 2020, dtype=dtype, first=u0 * d),
              lgx.fill_normal((cfg.n_items, d), 0.1, 2020, dtype=dtype, first=cfg.n_users * d))
    timings = []
    step, local_nnz, _ = make_step(A, E0, K, d, dtype, world, cfg, rank, timings)
    nnz_all = local_nnz
    if world > 1:
        t = torch.tensor([local_nnz], dtype=torch.int64, device="cuda")
        dist.all_reduce(t)
        nnz_all = int(t.item())
    for _ in range(warmup):
        step(False)
    barrier_sync(world)
    t_start = time.perf_counter()
    for _ in range(steps):
        step(True)
    barrier_sync(world)
    elapsed = max_over_ranks(time.perf_counter() - t_start, world)
    launch_s = np.array([e0.elapsed_time(e1) for e0, e1, _ in timings]) / 1e3
    mean_launch_s = float(launch_s.mean())
    mean = {key: float(np.mean([m[key] for _, _, m in timings])) for key in ("model", "gathered", "floor")}
    hot_rows = timings[0][2]["hot_rows"]
    hot_frac = float(np.mean([m["hot_frac"] for _, _, m in timings]))
    kernels = sorted({m["kernel"] for _, _, m in timings})
    col_blocks = max(m.get("col_blocks", 0) for _, _, m in timings)
    # per layer call: with column blocks one call is 1 + nb dispatches of spmm_segments
    traffic, tsrc = measured_traffic(cfg.name, dname, world, ["spmm_segments", "spmm_fixup"],
                                     calls_from=("spmm_segments", 1 + col_blocks) if col_blocks > 1 else None)
    achieved = mean["model"] / mean_launch_s
    roof = {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
            "frac": achieved / HBM_PEAK, "traffic": traffic,
            "kernel": "spmm_segments (+spmm_fixup): " + ", ".join(kernels)
                      + (f"; item rows in {col_blocks} column blocks (1 + {col_blocks} launches per layer)"
                         if col_blocks > 1 else ""),
            "mean_launch_ms": mean_launch_s * 1e3,
            "bytes_model": "cache-aware: CSR + epilogue + gathers of rows outside the per-XCD L2 hot set "
                           f"(top {hot_rows} rows per gathered table = {hot_frac:.3f} of gathers)"
                           + ("" if world == 1 else "; per-rank pull / push operators, each its own hot set"),
            "bytes_per_launch": int(mean["model"]),
            "floor_bytes_per_launch": int(mean["floor"]), "floor_rate_gbs": mean["floor"] / mean_launch_s / 1e9,
            "floor_frac": mean["floor"] / mean_launch_s / HBM_PEAK,
            "gathered_bytes_per_launch": int(mean["gathered"]),
            "gathered_rate_gbs": mean["gathered"] / mean_launch_s / 1e9,
            "traffic_unit": "GB/launch", "traffic_source": tsrc,
            "traffic_rate_gbs": traffic / mean_launch_s if traffic else None,
            "traffic_frac": traffic * 1e9 / mean_launch_s / HBM_PEAK if traffic else None}
    out = {"dtype": dname, "value": K * nnz_all * steps / elapsed, "unit": "edges/s",
           "ms_per_step": elapsed / steps * 1e3, "steps": steps, "warmup": warmup, "nnz": nnz_all,
           "roofline": roof, "E0": E0 if world == 1 else None}
    if world == 1:
        roof["calibration"] = calibration()
    else:
        # where a step's time goes on each rank's compute stream, max over ranks per phase: push /
        # pull / reduce / epilogue are kernels, allgather_wait / exchange_wait the time the stream
        # sat behind a collective (the communication the schedule left exposed)
        ph = step.prop.phase_summary()
        names = ["push", "allgather_wait", "pull", "exchange_wait", "exchange_sync", "reduce", "epilogue",
                 "comm_exposed_ms"]
        mx = {n: max_over_ranks(float(ph.get(n, 0.0)), world) for n in names}
        out["comm_exposed_ms"] = mx.pop("comm_exposed_ms")
        out["phases_ms"] = mx
        sync = ("; gloo has no device all-to-all: each exchange is a host-staged, host-synchronous "
                "all-to-all (exchange_sync), so this line is a rehearsal of the schedule, not of RCCL's overlap"
                if not step.prop._a2a_native else "")
        out["phases_note"] = (f"ms per step on the compute stream, max over {world} ranks; push in "
                              f"{len(step.prop.push_chunks)} chunks, each exchanged by its own all-to-all{sync}")
        out["per_rank"] = gather_rank_stats(world, {
            "rank": rank, "users": A.n_u_local, "pull_nnz": A.A_pull.nnz, "push_nnz": step.prop.push_nnz,
            "peak_mem_gb": torch.cuda.max_memory_allocated() / 1e9,
            "build_peak_mem_gb": getattr(A, "build_peak_gb", None), "build_s": getattr(A, "build_s", None),
            "layer_launch_ms_mean": mean_launch_s * 1e3,
            "kernel_ms_per_step": sum(v for kk, v in ph.items() if kk in ("push", "pull", "reduce", "epilogue"))})
    return out


def gather_rank_stats(world: int, mine: dict) -> list:
    """Every rank's dict on rank 0 (all_gather_object over the bench's group), in rank order."""
    got = [None] * world
    dist.all_gather_object(got, mine)
    return got


# ------------------------------------------------------------------------------------ CPU baseline
def host_cpus() -> tuple:
    """CPUs this process may run on: the affinity set, capped by a cgroup-v2 CPU quota if any."""
    n = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(p)
    except (OSError, ValueError):
        pass
    if quota is not None:
        n = max(1, min(n, int(math.ceil(quota))))
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return n, model, quota


def cpu_baseline(A, E0, cfg, target_nnz):
    """oracle/torch_ref.py (torch.sparse.mm on the host, model.py:163-175) on a bounded sample of
    BOTH row kinds of the same graph -- the first user rows (gathering the item table) and the first
    item rows (gathering the user table) -- against the full fp32 table; rate extrapolated per edge."""
    from oracle import torch_ref
    threads, model, quota = host_cpus()
    ip = A.indptr.cpu().numpy()
    X = E0.float().cpu()
    U = cfg.n_users
    secs, edges, parts = 0.0, 0, []
    for name, r0 in (("user", 0), ("item", U)):
        base = int(ip[r0])
        r1 = int(np.searchsorted(ip, base + target_nnz // 2))
        r1 = max(r0 + 1, min(r1, A.n_rows))
        s, e = int(ip[r0]), int(ip[r1])
        G = torch_ref.coo_from_csr(ip[r0:r1 + 1] - s, A.indices[s:e].cpu().numpy(), A.vals[s:e].cpu().numpy(),
                                   A.n_cols)
        r = torch_ref.time_spmm_rows(G, X, cfg.K, threads)
        secs += r["seconds"]
        edges += r["edges"]
        parts.append(f"{name} rows [{r0},{r1}) ({e - s} nnz)")
        del G
    return {"value": edges / secs, "unit": "edges/s", "cores": threads, "kind": "port", "extrapolated": True,
            "cpu_model": model, "os_cpu_count": os.cpu_count(), "cgroup_cpu_quota": quota,
            "sample": f"{cfg.K} x torch.sparse.mm of " + " + ".join(parts) + f" against the full fp32 "
                      f"[{A.n_cols},{cfg.d}] table, {secs:.1f}s; per-edge rate extrapolated to the whole graph"}


def bench_scoring(args, rank, world, dtype, B_total, steps, with_cpu):
    """configs[4]: d=256, 1M items, top-20 with a 50-item train mask; users split over ranks.
    dtype float32 = the reference's precision (model.py:183 fp32 matmul; score_topk_f32_lds,
    v_mfma_f32_16x16x4_f32, against the 157.3 TF f32 MFMA peak); bfloat16 = SURVEY C5's inputs
    (score_topk_bf16_lds, against 2.5 PF)."""
    d, n_items, k = 256, args.score_items, 20
    B = B_total // world
    f32 = dtype == torch.float32
    items = lgx.fill_normal((n_items, d), 1.0 / 16, 4242, dtype=dtype)
    Q = lgx.fill_normal((B, d), 1.0 / 16, 777 + rank, dtype=dtype)
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
    steps = max(1, steps)
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
    plan = ops.score_topk_plan(B, n_items, d, dtype, k)
    peak = F32_MFMA_PEAK if f32 else BF16_MFMA_PEAK
    sweep = plan.split("<", 1)[0]  # the sweep kernel the plan launches (score_topk_f32_lds / _bf16_lds)
    # per lgx_score_topk call: every stage of every user range (finalize runs once per range)
    traffic, tsrc = measured_traffic(args.config, "scoring_f32" if f32 else "scoring", world,
                                     [sweep, "score_topk_finalize"],
                                     calls_from=("score_topk_finalize", plan.count("; ") + 1))
    cpu = None
    if with_cpu and rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = scoring_cpu_baseline(Q, items, pos, k, args.cpu_score_users)
    return {"value": B * world * n_items * steps / elapsed, "unit": "items/s", "users_per_step": B * world,
            "n_items": n_items, "d": d, "k": k, "dtype": "f32" if f32 else "bf16",
            "ms_per_step": elapsed / steps * 1e3, "steps": steps, "plan": plan,
            "roofline": {"bound": "mfma", "achieved": flops / mean_launch / 1e12, "peak": peak / 1e12,
                         "unit": "TFLOP/s", "frac": flops / mean_launch / peak, "traffic": traffic,
                         "traffic_unit": "GB/call", "traffic_source": tsrc,
                         "kernel": f"{sweep} (+ score_topk_finalize, both inside the timed launch)",
                         "launch": "one lgx_score_topk call: every launch of its plan (seeded stages, split tail)"},
            "cpu_baseline": cpu}


def scoring_cpu_baseline(Q, items, pos, k, n_users):
    """The reference's CPU scoring procedure (Procedure.py:121-135 per 100-user batch: fp32 matmul,
    sigmoid, train mask, torch.topk) on the first n_users query users of the same batch."""
    from oracle import torch_ref
    threads, model, _ = host_cpus()
    torch.set_num_threads(threads)
    Qc = Q[:n_users].float().cpu()
    Ic = items.float().cpu()
    masks = [row for row in pos[:n_users].cpu().numpy()]
    torch_ref.score_topk_cpu(Qc[:100], Ic, k, masks[:100])  # warm-up
    _, t = torch_ref.score_topk_cpu(Qc, Ic, k, masks)
    return {"value": n_users * items.shape[0] / t, "unit": "items/s", "cores": threads, "kind": "port",
            "extrapolated": True, "cpu_model": model,
            "sample": f"{n_users} of the query users x {items.shape[0]} items, d={items.shape[1]} fp32, "
                      f"top-{k} with the same train masks ({t:.1f}s); per-item rate extrapolated"}


def launch_ranks(n: int, argv) -> int:
    """`bench.py --gpus N` (N > 1) started without a launcher: run N ranks under
    torch.distributed.run as CHILD processes (this process never touches the GPU: it is called
    before any torch.cuda use, and it does not exec), forward rank 0's JSON line to stdout and
    return non-zero if any rank failed or no line came back."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]
    print(f"[bench] launching {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, bufsize=1)
    line = None
    for raw in p.stdout:
        s = raw.strip()
        if s.startswith("{") and '"metric"' in s:
            try:
                json.loads(s)
                line = s
                continue
            except ValueError:
                pass
        sys.stderr.write(raw)
        sys.stderr.flush()
    rc = p.wait()
    if rc != 0 or line is None:
        print(f"[bench] rank launch failed (exit {rc}, result line {'present' if line else 'missing'})",
              file=sys.stderr, flush=True)
        return rc if rc != 0 else 1
    print(line, flush=True)
    return 0


def launch_check(args, world: int, rank: int) -> None:
    """--launch-check: the rank-launch path without a GPU (CPU tests): join a gloo group, report it."""
    if world > 1:
        dist.init_process_group("gloo")
    if os.environ.get("LGX_LAUNCH_CHECK_FAIL_RANK") == str(rank):  # tests: one rank dies
        sys.exit(3)
    pg = {"world_size": dist.get_world_size(), "backend": dist.get_backend()} if world > 1 else None
    if rank == 0:
        print(json.dumps({"metric": METRIC, "n_gpus": world, "process_group": pg}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="synth10m", choices=sorted(CONFIGS))
    ap.add_argument("--dtype", default="f32", choices=["bf16", "f32"],
                    help="storage dtype of the headline propagation run (f32 = the reference's, model.py:163-176)")
    ap.add_argument("--score-users", type=int, default=1_000_000, help="bf16 scoring leg users (configs[4])")
    ap.add_argument("--score-f32-users", type=int, default=1_000_000, help="fp32 scoring leg users (configs[4])")
    ap.add_argument("--score-items", type=int, default=1_000_000)
    ap.add_argument("--score-steps", type=int, default=2)
    ap.add_argument("--cpu-nnz", type=int, default=40_000_000)
    ap.add_argument("--cpu-score-users", type=int, default=4000)
    ap.add_argument("--extra-steps", type=int, default=10, help="timed steps of the other-dtype propagation run")
    ap.add_argument("--no-extra-dtype", action="store_true", help="skip the other-dtype propagation run")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-scoring", action="store_true")
    ap.add_argument("--no-propagation", action="store_true", help="development: scoring legs only")
    ap.add_argument("--launch-check", action="store_true", help="tests: rank launch only, no GPU work")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no external launcher: start the N ranks here, before anything initialises the GPU
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        log(f"[bench] error: --gpus {args.gpus} but WORLD_SIZE={world}; the line would not be the "
            f"{args.gpus}-GPU measurement")
        sys.exit(2)
    if args.launch_check:
        launch_check(args, world, rank)
        return
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
        log(f"[bench] world {dist.get_world_size()} over {dist.get_backend()}")

    def scoring_legs():
        if args.no_scoring:
            return None, None
        f32 = bench_scoring(args, rank, world, torch.float32, args.score_f32_users, args.score_steps, True)
        torch.cuda.empty_cache()
        bf16 = bench_scoring(args, rank, world, torch.bfloat16, args.score_users, args.score_steps, False)
        bf16["cpu_baseline"] = "see scoring.cpu_baseline (the reference's fp32 procedure)"
        torch.cuda.empty_cache()
        return f32, bf16

    if args.no_propagation:
        sc, sc16 = scoring_legs()
        if rank == 0:
            print(json.dumps({"metric": METRIC, "scoring": sc, "scoring_bf16": sc16}), flush=True)
        return
    cfg = CONFIGS[args.config]
    main_dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    t0 = time.time()
    if world == 1:
        A = synth_graph(cfg, seed=2020, device="cuda")
        log(f"[bench] graph {cfg.name}: N={cfg.n_users + cfg.n_items} nnz={A.nnz} built in {time.time() - t0:.1f}s")
    else:
        # every rank draws the same seeded edge list and builds only its own rows.  Ranks that share
        # a GPU (one-GPU rehearsals) build one after another behind barriers, so that the edge
        # draws' transient peaks (~30 GB at C4) do not coincide; on a node every rank has its own.
        shared = world > max(1, torch.cuda.device_count())
        A = None
        for turn in range(world if shared else 1):
            if not shared or turn == rank:
                u, i = synth_edges(cfg, seed=2020, device="cuda")
                A = make_shard_from_edges(u, i, cfg.n_users, cfg.n_items, rank, world)
                del u, i
                torch.cuda.synchronize()
                torch.cuda.empty_cache()
                print(f"[bench] rank {rank}: shard built ({time.time() - t0:.1f}s since start)",
                      file=sys.stderr, flush=True)
            if shared:
                dist.barrier()
        build_peak = torch.cuda.max_memory_allocated() / 1e9
        A.build_peak_gb = build_peak
        A.build_s = time.time() - t0
        torch.cuda.reset_peak_memory_stats()
        log(f"[bench] shard {rank}/{world} of {cfg.name}: {A.n_u_local} users, pull nnz {A.A_pull.nnz} "
            f"built in {time.time() - t0:.1f}s ({'rank-serialised' if shared else 'in parallel'}, "
            f"build peak {build_peak:.1f} GB)")
    res = bench_propagation(args, rank, world, A, cfg, main_dtype, args.steps, args.warmup)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(A, res["E0"], cfg, args.cpu_nnz)
    res.pop("E0", None)
    torch.cuda.empty_cache()
    extra = None
    if not args.no_extra_dtype:
        other = torch.float32 if main_dtype == torch.bfloat16 else torch.bfloat16
        extra = bench_propagation(args, rank, world, A, cfg, other, max(1, args.extra_steps),
                                  max(1, min(2, args.warmup)))
        extra.pop("E0", None)
        extra["note"] = ("bf16 embedding storage / fp32 accumulation (SURVEY C4's perf mode), same graph and "
                         "kernel family" if other == torch.bfloat16 else
                         "fp32 embedding storage (the reference's precision), same graph and kernel family")
    del A
    torch.cuda.empty_cache()
    scoring, scoring16 = scoring_legs()
    line = {
        "metric": METRIC, "value": res["value"], "unit": "edges/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": res["ms_per_step"], "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": res["dtype"], "data": "synthetic (seeded power-law bipartite graph)",
        "config": {"workload": f"{cfg.name}: {cfg.n_users} users x {cfg.n_items} items, {cfg.n_edges} edges "
                               f"(nnz {res['nnz']}), K={cfg.K}, d={cfg.d}, {res['dtype']} storage / fp32 accumulate",
                   "parallelism": f"row-shard{world}" if world > 1 else "single"},
        "process_group": ({"world_size": dist.get_world_size(), "backend": dist.get_backend()} if world > 1
                          else None),
        "roofline": res["roofline"], "cpu_baseline": cpu,
        **({"phases_ms": res["phases_ms"], "comm_exposed_ms": res["comm_exposed_ms"],
            "phases_note": res["phases_note"], "per_rank": res["per_rank"],
            "per_rank_note": "peak_mem_gb = torch.cuda.max_memory_allocated over the timed propagation (shard, "
                             "tables, push chunks, exchange buffers; the shard build's transient peak is reset "
                             "before it); kernel_ms_per_step = push + pull + reduce + epilogue on that rank"}
           if world > 1 else {}),
        ("bf16" if extra and extra["dtype"] == "bf16" else "fp32"): extra,
        "scoring": scoring, "scoring_bf16": scoring16,
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
