"""Multi-GPU readiness on ONE GPU: the per-rank work of the C4 propagation at world = 8 (or --world),
timed rank by rank with the real kernels and the real schedule of distributed.ShardedPropagation
(push in n_chunks launches, pull, the rank-order slab sums, the item epilogue, K layers with the
STACK mean in the last pull), with the collectives stubbed out.  Prints one JSON document: the
per-rank phase times, the single-GPU step on the same graph, the collective volumes per layer, and
a predicted step time and speedup at two assumed RCCL rates.

  python tools/shard_probe.py [--world 8] [--ranks all] [--dtype f32] [--reps 3] [--chunks 4] [--contend]

--contend also times every rank with the collectives replaced by device copies of their bytes on a
side stream (_CopyComm): the SpMM under the HBM traffic and CU use of the exchanges.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import factors_of_serendipity_recommendation_amd as lgx  # noqa: E402
from factors_of_serendipity_recommendation_amd import ops  # noqa: E402
from factors_of_serendipity_recommendation_amd.distributed import (ShardedPropagation,  # noqa: E402
                                                                    make_shard_from_edges)
from factors_of_serendipity_recommendation_amd.synth import CONFIGS, synth_edges, synth_graph  # noqa: E402

LINK_GBS = 153.0       # one xGMI link per direction (task brief: 7 links x ~153 GB/s per GPU)
LINKS = 7


class _NoComm(ShardedPropagation):
    """The product schedule with the exchanges and all-gathers left out (kernels only)."""

    def _exchange(self, c0, m):
        return None

    def _all_gather(self, table):
        return None


class _Done:
    """A collective handle whose wait() makes the compute stream wait for a side-stream event."""

    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)


class _CopyComm(ShardedPropagation):
    """The product schedule with every collective replaced by device copies of the bytes it moves
    through this GPU's HBM, issued on a side stream at the collective's place in the schedule and
    waited for where the collective is waited for: chunk c's all-to-all reads its [world, mc, d]
    send slabs and writes the received ones (R <- P), the all-gather writes the world-1 peer blocks
    of the padded item table.  The link time is not in it (no peer); the interference of that
    traffic and of the copy kernels' CUs with the overlapped SpMM is."""

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.side = torch.cuda.Stream()
        self._a2a_native = True  # async handles, as RCCL's: no host-synchronous exchange stamps

    def _side(self, fn):
        ev = torch.cuda.Event()
        ev.record()
        self.side.wait_event(ev)
        with torch.cuda.stream(self.side):
            fn()
            done = torch.cuda.Event()
            done.record()
        return _Done(done)

    def _exchange(self, c0, m):
        P, R = self._chunk_views(c0, m)
        return self._side(lambda: R.copy_(P))

    def _all_gather(self, table):
        s = self.s
        blocks = table.view(s.world, s.mi, self.d)

        def fn():
            for q in range(s.world):
                if q != s.rank:
                    blocks[q].copy_(self.send_i)
        return self._side(fn)


def timed_steps(fn, reps):
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
    ap.add_argument("--ranks", default="all")
    ap.add_argument("--contend", action="store_true")
    ap.add_argument("--dtype", default="f32", choices=["bf16", "f32"])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--chunks", type=int, default=4)
    ap.add_argument("--link-efficiency", type=float, default=0.6)
    ap.add_argument("--no-one-gpu", action="store_true")
    args = ap.parse_args()
    cfg = CONFIGS["synth10m"]
    U, I, d, K, w = cfg.n_users, cfg.n_items, cfg.d, cfg.K, args.world
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    s = 2 if dt == torch.bfloat16 else 4
    # a one-process gloo group: ShardedPropagation asks the backend; no collective is issued
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29611")
    dist.init_process_group("gloo", rank=0, world_size=1)
    E0 = lgx.fill_normal((U + I, d), 0.1, 2020, dtype=dt)
    one_gpu = None
    if not args.no_one_gpu:
        t0 = time.time()
        A = synth_graph(cfg, seed=2020, device="cuda")
        print(f"graph nnz={A.nnz} in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
        out = torch.empty((U + I, d), dtype=torch.float32, device="cuda")
        one_gpu = timed_steps(lambda: ops.propagate(A, E0, K, out=out), args.reps)
        print(f"one GPU step {one_gpu:.2f} ms", file=sys.stderr, flush=True)
        del A, out
        torch.cuda.empty_cache()
    u, i = synth_edges(cfg, seed=2020, device="cuda")
    ranks = []
    rank_ids = range(w) if args.ranks == "all" else [int(x) for x in args.ranks.split(",")]
    for r in rank_ids:
        t0 = time.time()
        sh = make_shard_from_edges(u, i, U, I, r, w)
        build = time.time() - t0
        contended = None
        if args.contend:
            cp = _CopyComm(sh, E0[:U], E0[U:], K, force_collectives=True, n_chunks=args.chunks)
            contended = timed_steps(cp.step, args.reps)
            cp.record_phases = True
            for _ in range(args.reps):
                cp.step()
            cph = cp.phase_summary()
            del cp
        torch.cuda.reset_peak_memory_stats()
        prop = _NoComm(sh, E0[:U], E0[U:], K, force_collectives=True, n_chunks=args.chunks)
        step_ms = timed_steps(prop.step, args.reps)
        prop.record_phases = True
        for _ in range(args.reps):
            prop.step()
        ph = prop.phase_summary()
        mi = sh.mi
        a2a_bytes = (w - 1) / w * (w * mi) * d * 4       # fp32 push partials out (and in) per layer
        ag_bytes = (w - 1) * mi * d * s                  # item blocks received per layer
        rec = {"rank": r, "users": sh.n_u_local, "pull_nnz": sh.A_pull.nnz, "push_nnz": sh.A_push.nnz,
               "push_chunks": len(prop.push_chunks), "shard_build_s": round(build, 2), "step_ms": step_ms,
               "phases_ms_per_step": {k: v for k, v in ph.items() if k in ("push", "pull", "reduce", "epilogue")},
               "all_to_all_bytes_per_layer": int(a2a_bytes), "all_gather_bytes_per_layer": int(ag_bytes),
               "peak_mem_gb_schedule": torch.cuda.max_memory_allocated() / 1e9}
        if contended is not None:
            rec["step_ms_with_copy_collectives"] = contended
            rec["phases_ms_with_copy_collectives"] = {k: v for k, v in cph.items() if k != "begin"}
        ranks.append(rec)
        print(json.dumps(rec), file=sys.stderr, flush=True)
        del sh, prop
        torch.cuda.empty_cache()
    worst = max(ranks, key=lambda x: x["step_ms"])
    worst_c = max(ranks, key=lambda x: x.get("step_ms_with_copy_collectives", 0.0))
    ph = worst["phases_ms_per_step"]
    push_l, pull_l = ph["push"] / K, ph["pull"] / K
    nch = worst["push_chunks"]
    pred = {}
    for name, per_peer_gbs in (("one_link_total", LINK_GBS / (w - 1)),
                               (f"{LINKS}_links_x{args.link_efficiency}", LINK_GBS * args.link_efficiency)):
        # all-to-all: each peer pair has its own link, carrying 1/(w-1) of the out bytes; all-gather:
        # one block from each peer.  "one_link_total" = the whole volume through one link's rate.
        a2a = worst["all_to_all_bytes_per_layer"] / (w - 1) / per_peer_gbs / 1e6
        ag = worst["all_gather_bytes_per_layer"] / (w - 1) / per_peer_gbs / 1e6
        # schedule: chunk c's exchange starts after its push launch and must end before the
        # reduce; it runs under the later chunks' pushes and the pull.  The all-gather of layer k
        # runs under the push of layer k+1 (K-1 of them per step).
        window_a2a = push_l * (nch - 1) / nch + pull_l
        exposed = K * max(0.0, a2a - window_a2a) + (K - 1) * max(0.0, ag - push_l)
        step = worst["step_ms"] + exposed
        pred[name] = {"per_peer_GBs_assumed": per_peer_gbs, "all_to_all_ms_per_layer": a2a,
                      "all_gather_ms_per_layer": ag, "exposed_comm_ms_per_step": exposed, "step_ms": step,
                      "speedup_vs_1gpu": (one_gpu / step) if one_gpu else None}
        if "step_ms_with_copy_collectives" in worst_c:
            # the slowest rank with the exchanges' HBM traffic and copy kernels running beside it
            # (measured) plus the link time the windows do not cover (modelled as above)
            step_c = worst_c["step_ms_with_copy_collectives"] + exposed
            pred[name]["step_ms_with_copy_contention"] = step_c
            pred[name]["speedup_vs_1gpu_with_copy_contention"] = (one_gpu / step_c) if one_gpu else None
    print(json.dumps({"workload": f"synth10m {args.dtype} K={K} d={d}, world={w}", "one_gpu_step_ms": one_gpu,
                      "ranks_timed": [x["rank"] for x in ranks],
                      "ranks": ranks, "critical_rank": worst["rank"], "kernel_ms_per_step": worst["step_ms"],
                      "kernel_ms_per_step_by_rank": [round(x["step_ms"], 3) for x in ranks],
                      "critical_rank_with_copy_collectives": worst_c["rank"] if args.contend else None,
                      "prediction": pred,
                      "note": "per-rank kernels of ShardedPropagation.step (collectives stubbed out) timed on one "
                              "MI355X with HIP events, best of reps; collective times are volumes / assumed "
                              "RCCL rates, not measurements"}, indent=1), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
