"""Row-sharded multi-GPU propagation: one process per GPU, RCCL collectives over xGMI.

The reference's only scale-out device is row-folding A^ into 100 blocks on one device
(dataloader.py:319-329, model.py:164-168; LightGCN-tf/LightGCN.py:201-213, 243-247).  Here the
layer is split across GPUs, and the bipartite structure decides which side moves.

Partition.  Users are sharded into contiguous nnz-balanced blocks (rank r owns users [u_r, u_{r+1})
and ALL of their edges); items into equal row blocks of mi = ceil(I / world) rows (rank r owns
items [r*mi, (r+1)*mi), so an item's padded coordinate is its own id).  A rank holds its users'
edges twice:
    A_pull : local users x items        (rows of A^; columns are item ids)
    A_push : items x local users        (the transpose; A^ is symmetric, so same values)

Layer k.  With U (10M) >> I (1M) the user table is the big one, so it never moves:
  * users pull:  U^k[own] = A_pull . I^{k-1}  -- needs the full item table (all-gathered, I*d*s bytes)
  * items push:  P = A_push . U^{k-1}[own]    -- fp32 partial sums for EVERY item from this rank's
                 users only; an all-to-all hands rank q the partials of its own item block, which it
                 adds in rank order (lgx_sum_slabs: a reduce-scatter whose sum does not depend on
                 the collective's ring / channel order, nor on the chunking below); the layer
                 epilogue (bf16 store, layer sum, mean) runs on that block, which is then
                 all-gathered for the next pull.
Per rank and layer the wire carries ~(world-1)/world * I*d*(4 + s) bytes, against
(world-1)/world * (U + I)*d*s for all-gathering both tables: 3.7x less at C4 (10M x 1M, d=128 bf16).

Overlap.  The push runs in n_chunks launches, chunk c covering rows [c*mc, (c+1)*mc) of EVERY
rank's item block (its rows re-ordered chunk-major, so a chunk's partials are one contiguous
[world, mc, d] slab set); chunk c's exchange starts while chunks c+1.. compute, and the exchanges
finish under the pull of layer k; the all-gather of item layer k runs under the push of layer k+1.
A chunk's rows keep the unchunked operator's segment length, so every row is summed exactly as in
one launch: chunked and unchunked layers are equal bit for bit.  The last layer is never gathered:
each rank keeps the fp32 layer means of its own users and items (gather_outputs() assembles the
full tables).

Diagnostics.  With record_phases set, every step stamps the compute stream after each phase
(push, allgather_wait, pull, exchange_wait, reduce, epilogue); the waits are the time the stream
sat behind a collective, i.e. the communication the schedule left exposed (phase_summary()).  Under
gloo with device tensors (one-GPU rehearsals) the exchange is a host-staged, host-synchronous
all-to-all: its time is stamped as exchange_sync, and counts as exposed.

The SpMM and epilogue callables are injectable so that the CPU tests drive the same schedule over
gloo with an oracle SpMM.
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from .graph import CSRGraph, make_plan


def balanced_bounds(indptr: np.ndarray, lo: int, hi: int, world: int) -> np.ndarray:
    """Contiguous row blocks of rows [lo, hi) with ~equal nonzeros (prefix-sum split)."""
    cum = indptr[lo:hi + 1].astype(np.int64) - int(indptr[lo])
    total = int(cum[-1])
    targets = (np.arange(1, world, dtype=np.float64) * total / world)
    cuts = np.searchsorted(cum, targets, side="left")
    b = np.concatenate([[0], cuts, [hi - lo]]).astype(np.int64)
    b = np.maximum.accumulate(b)
    return b + lo


def equal_bounds(n: int, world: int) -> Tuple[np.ndarray, int]:
    """Equal row blocks of mi = ceil(n / world) rows (the last may be short or empty)."""
    mi = max(1, -(-n // world))
    return np.minimum(np.arange(world + 1, dtype=np.int64) * mi, n), mi


@dataclass
class Shard:
    rank: int
    world: int
    n_users: int
    n_items: int
    user_bounds: np.ndarray  # [world+1] global user ids, nnz-balanced
    item_bounds: np.ndarray  # [world+1] global item ids, equal blocks of mi rows
    mi: int                  # item block rows
    A_pull: CSRGraph         # local users -> item ids (world*mi columns)
    A_push: CSRGraph         # item ids (world*mi rows) -> local users

    @property
    def n_u_local(self) -> int:
        return int(self.user_bounds[self.rank + 1] - self.user_bounds[self.rank])

    @property
    def n_i_local(self) -> int:
        return int(self.item_bounds[self.rank + 1] - self.item_bounds[self.rank])


def _planned(indptr, indices, vals, n_rows, n_cols, seg_len) -> CSRGraph:
    g = CSRGraph(indptr.contiguous(), indices.contiguous(), vals.contiguous(), n_rows, n_cols)
    g.plan = make_plan(indptr.cpu().numpy(), seg_len)
    g.ensure_plan()
    return g


def _transpose(G: CSRGraph, n_rows_out: int, seg_len: Optional[int]) -> CSRGraph:
    """CSR transpose (rows sorted, columns ascending within a row) -- sort by (col, row)."""
    dev = G.indptr.device
    counts = torch.diff(G.indptr)
    rows = torch.repeat_interleave(torch.arange(G.n_rows, device=dev, dtype=torch.int64), counts)
    cols = G.indices.to(torch.int64)
    perm = torch.argsort(cols * max(1, G.n_rows) + rows)
    indptr = torch.zeros(n_rows_out + 1, dtype=torch.int64, device=dev)
    indptr[1:] = torch.cumsum(torch.bincount(cols, minlength=n_rows_out), 0)
    return _planned(indptr, rows[perm].to(torch.int32), G.vals[perm], n_rows_out, G.n_rows, seg_len)


def make_shard(A: CSRGraph, n_users: int, n_items: int, rank: int, world: int,
               seg_len: Optional[int] = None) -> Shard:
    """Cut the square operator (users first, then items) into this rank's pull / push operators."""
    ip = A.indptr.cpu().numpy()
    ub = balanced_bounds(ip, 0, n_users, world)
    ib, mi = equal_bounds(n_items, world)
    r0, r1 = int(ub[rank]), int(ub[rank + 1])
    s, e = int(ip[r0]), int(ip[r1])
    indptr = (A.indptr[r0:r1 + 1] - s).contiguous()
    items = (A.indices[s:e].to(torch.int64) - n_users).to(torch.int32)  # item id == padded coordinate
    A_pull = _planned(indptr, items, A.vals[s:e], r1 - r0, world * mi, seg_len)
    A_push = _transpose(A_pull, world * mi, seg_len)
    return Shard(rank, world, n_users, n_items, ub, ib, mi, A_pull, A_push)


def make_shard_from_edges(users: torch.Tensor, items: torch.Tensor, n_users: int, n_items: int, rank: int,
                          world: int, seg_len: Optional[int] = None) -> Shard:
    """make_shard() without materialising the full operator: from the unique edge list sorted by
    (user, item) (what synth_edges returns), build only this rank's rows.  The degrees are global
    (bincounts of the edge list), the values those of lgx_build_norm_adj with dedup
    (d = (float)(1/sqrt((double)deg)), val = (d_u * 1) * d_i in f32), so the shard is bit for bit
    the one make_shard cuts from the full operator.  Saves every rank the 1e9-nnz CSR build at C4."""
    dev = users.device
    u64 = users.to(torch.int64)
    if u64.numel() > 1:
        # sorted by (user, item) AND unique: a repeated edge would double-count both degrees and
        # keep both entries, unsorted items would break the CSR order -- either way not make_shard's
        # operator.  One vectorised comparison of the packed keys.
        key = u64 * n_items + items.to(torch.int64)
        if bool((key[1:] <= key[:-1]).any()):
            raise ValueError("make_shard_from_edges: edges must be unique and sorted by (user, item)")
    deg_u = torch.bincount(u64, minlength=n_users).cpu().numpy()
    deg_i = torch.bincount(items.to(torch.int64), minlength=n_items).cpu().numpy()
    ip = np.zeros(n_users + 1, dtype=np.int64)
    np.cumsum(deg_u, out=ip[1:])
    ub = balanced_bounds(ip, 0, n_users, world)
    ib, mi = equal_bounds(n_items, world)
    r0, r1 = int(ub[rank]), int(ub[rank + 1])
    s, e = int(ip[r0]), int(ip[r1])

    def dinv(deg):  # IEEE double sqrt and division, rounded once: the builder's d_r
        d = deg.astype(np.float64)
        with np.errstate(divide="ignore"):
            v = np.where(d > 0, 1.0 / np.sqrt(d), 0.0)
        return torch.from_numpy(v.astype(np.float32)).to(dev)

    du, di = dinv(deg_u), dinv(deg_i)
    cols = items[s:e].contiguous()
    vals = (du[u64[s:e]] * 1.0) * di[cols.to(torch.int64)]
    indptr = torch.from_numpy(ip[r0:r1 + 1] - s).to(dev)
    A_pull = _planned(indptr, cols.to(torch.int32), vals, r1 - r0, world * mi, seg_len)
    A_push = _transpose(A_pull, world * mi, seg_len)
    return Shard(rank, world, n_users, n_items, ub, ib, mi, A_pull, A_push)


def pad_table(full: torch.Tensor, bounds: np.ndarray, pad: int) -> torch.Tensor:
    """[n, d] table in global row order -> [world*pad, d] padded layout (zeros in the gaps)."""
    world = len(bounds) - 1
    out = torch.zeros((world * pad, full.shape[1]), dtype=full.dtype, device=full.device)
    for q in range(world):
        a, b = int(bounds[q]), int(bounds[q + 1])
        out[q * pad:q * pad + (b - a)] = full[a:b]
    return out


def _row_gather(G: CSRGraph, rows: torch.Tensor) -> CSRGraph:
    """The rows `rows` of G, in that order, as a CSR (columns keep their order within each row)."""
    dev = G.indptr.device
    rows = rows.to(device=dev, dtype=torch.int64)
    lens = torch.diff(G.indptr)[rows]
    indptr = torch.zeros(rows.numel() + 1, dtype=torch.int64, device=dev)
    torch.cumsum(lens, 0, out=indptr[1:])
    rid = torch.repeat_interleave(torch.arange(rows.numel(), device=dev, dtype=torch.int64), lens)
    pos = G.indptr[rows][rid] + torch.arange(rid.numel(), device=dev, dtype=torch.int64) - indptr[rid]
    return CSRGraph(indptr, G.indices[pos].contiguous(), G.vals[pos].contiguous(), rows.numel(), G.n_cols)


def chunk_push_operator(A_push: CSRGraph, world: int, mi: int, n_chunks: int) -> List[Tuple[CSRGraph, int, int]]:
    """Cut the push operator (world * mi item rows) into chunks: chunk c = rows q*mi + c*mc + j of
    every rank block q (j < its mc_c rows), in (q, j) order, so that its output is the [world, mc_c,
    d] slab set one all-to-all exchanges.  Returns [(operator, first row of the chunk in a block,
    mc_c)].  Every chunk keeps A_push's segment length, so each row is summed as in one launch."""
    mc = max(1, -(-mi // max(1, n_chunks)))
    seg_len = A_push.plan.seg_len if A_push.plan is not None else None
    out = []
    dev = A_push.indptr.device
    for c0 in range(0, mi, mc):
        m = min(mc, mi - c0)
        rows = (torch.arange(world, dtype=torch.int64)[:, None] * mi + c0 + torch.arange(m)[None, :]).reshape(-1)
        G = _row_gather(A_push, rows.to(dev))
        G.plan = make_plan(G.indptr.cpu().numpy(), seg_len)
        G.ensure_plan()
        out.append((G, c0, m))
    return out


class PhaseRecorder:
    """Per-step stamps on the compute stream (HIP events; host clock for CPU tensors): the time
    between two stamps is charged to the label of the later one.  At most `keep` steps hold their
    events; older ones are folded into running totals (waiting for their last event, which is long
    done by then), so a recorder left on through a training run stays bounded."""

    def __init__(self, cuda: bool, keep: int = 32):
        self.cuda = cuda
        self.keep = keep
        self.steps: List[List[Tuple[str, object]]] = []
        self._cur: Optional[List[Tuple[str, object]]] = None
        self._tot: Dict[str, float] = {}
        self._n = 0

    def _stamp(self):
        if self.cuda:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            return ev
        return time.perf_counter()

    def begin(self) -> None:
        self._cur = [("begin", self._stamp())]

    def mark(self, label: str) -> None:
        if self._cur is not None:
            self._cur.append((label, self._stamp()))

    def end(self) -> None:
        if self._cur is not None:
            self.steps.append(self._cur)
            self._cur = None
            while len(self.steps) > self.keep:
                self._fold(self.steps.pop(0))

    def _fold(self, st) -> None:
        if self.cuda:
            st[-1][1].synchronize()
        for (_, a), (label, b) in zip(st[:-1], st[1:]):
            dt = a.elapsed_time(b) if self.cuda else (b - a) * 1e3
            self._tot[label] = self._tot.get(label, 0.0) + dt
        self._n += 1

    def summary(self) -> Dict[str, float]:
        """Mean milliseconds per step by label (call after the stream has drained)."""
        for st in self.steps:
            self._fold(st)
        self.steps = []
        n = max(1, self._n)
        return {k: v / n for k, v in self._tot.items()}


LayerFn = Callable[..., None]


def _default_layer_fn(A, X, mode, Y=None, E0=None, acc=None, out=None, n_mean=1.0):
    from .ops import propagate_layer
    propagate_layer(A, X, mode, Y=Y, E0=E0, acc=acc, out=out, n_mean=n_mean)


def _default_epilogue_fn(y, mode, Y=None, E0=None, acc=None, out=None, n_mean=1.0):
    from .ops import layer_epilogue
    layer_epilogue(y, mode, Y=Y, E0=E0, acc=acc, out=out, n_mean=n_mean)


def _default_stack_fn(A, X, E0, prev, out, n_mean):
    from .ops import propagate_layer_stack
    propagate_layer_stack(A, X, E0, prev, out, n_mean)


def _default_sum_fn(src, out):
    from .ops import sum_slabs
    sum_slabs(src, out)


def _host_sum(src, out):
    """lgx_sum_slabs' order on the host (CPU tests): src[0] + src[1] + ... left to right."""
    acc = src[0].clone()
    for j in range(1, src.shape[0]):
        acc += src[j]
    out.copy_(acc)


class ShardedPropagation:
    """K-layer LightGCN propagation of a row-sharded graph (see module docstring)."""

    def __init__(self, shard: Shard, E0_user: torch.Tensor, E0_item: torch.Tensor, K: int,
                 group=None, layer_fn: Optional[LayerFn] = None, epilogue_fn: Optional[LayerFn] = None,
                 stack_fn: Optional[LayerFn] = None, force_collectives: bool = False,
                 n_chunks: Optional[int] = None, sum_fn: Optional[Callable] = None,
                 local_user_rows: bool = False):
        """E0_user / E0_item: the FULL layer-0 tables in global row order (replicated input, as every
        rank holds the embedding parameters); dtype f32 or bf16.  local_user_rows: E0_user holds only
        this rank's users [user_bounds[rank], user_bounds[rank+1]) -- the propagation never reads
        another rank's user rows, so a caller need not hold the full [U, d] table (C4 fp32: 5.1 GB).  The user side keeps its K-1 layer
        tables and forms the mean in the last pull (stack_fn = lgx_propagate_layer_stack), as the
        single-GPU lgx_propagate does; the item side keeps the f32 running sum of its own block.

        force_collectives: issue the exchange / all-gather even at world 1 (where they are copies),
        so that a one-GPU RCCL group runs the async collective stream ordering the overlap depends on.

        n_chunks: push launches per layer (default 4 with collectives, else 1), each followed by its
        own all-to-all.  The chunk operators hold copies of the push rows (C4 / 8: ~1 GB per rank
        beside shard.A_push); a caller that keeps no other use for shard.A_push may drop it after
        construction (self.push_nnz keeps its count).  sum_fn(src [n, rows, d], out [rows, d]): the ordered slab sum (default
        lgx_sum_slabs on the GPU, the same left-to-right adds on the host)."""
        self.s = shard
        self.K = K
        self.group = group
        self.layer_fn = layer_fn or _default_layer_fn
        self.epilogue_fn = epilogue_fn or _default_epilogue_fn
        self.stack_fn = stack_fn or _default_stack_fn
        s = shard
        d = E0_user.shape[1]
        self.d = d
        dev, dt = E0_user.device, E0_user.dtype
        u0, u1 = int(s.user_bounds[s.rank]), int(s.user_bounds[s.rank + 1])
        i0, i1 = int(s.item_bounds[s.rank]), int(s.item_bounds[s.rank + 1])
        if local_user_rows:
            if E0_user.shape[0] != u1 - u0:
                raise ValueError(f"ShardedPropagation: local_user_rows expects {u1 - u0} rows, got {E0_user.shape[0]}")
            self.E0u = E0_user.contiguous()
        else:
            self.E0u = E0_user[u0:u1].contiguous()
        self.E0i = E0_item[i0:i1].contiguous()
        # users: local rows only, layers 0..K-1 kept; items: full padded tables, layer ping-pong
        self.Xu = [self.E0u] + [torch.zeros((s.n_u_local, d), dtype=dt, device=dev) for _ in range(max(1, K - 1))]
        self.Xi = [pad_table(E0_item, s.item_bounds, s.mi)] + \
                  [torch.zeros((s.world * s.mi, d), dtype=dt, device=dev) for _ in range(2)]
        self.P = torch.zeros((s.world * s.mi, d), dtype=torch.float32, device=dev)  # push partials
        self.yi = torch.zeros((s.mi, d), dtype=torch.float32, device=dev)           # own item block sums
        self.send_i = torch.zeros((s.mi, d), dtype=dt, device=dev)
        self.acc_i = torch.zeros((s.n_i_local, d), dtype=torch.float32, device=dev)
        self.out_u = torch.zeros((s.n_u_local, d), dtype=torch.float32, device=dev)
        self.out_i = torch.zeros((s.n_i_local, d), dtype=torch.float32, device=dev)
        self._collective = s.world > 1 or force_collectives
        # gloo has no all-to-all of device tensors: staged through host tensors there (tests and
        # rehearsals only), the same slabs in the same order, hence the same sums
        self._a2a_native = self._collective and not (dev.type == "cuda" and dist.get_backend(group) == "gloo")
        if n_chunks is None:
            n_chunks = 4 if self._collective else 1
        self.push_chunks = chunk_push_operator(s.A_push, s.world, s.mi, n_chunks) if n_chunks > 1 else \
            [(s.A_push, 0, s.mi)]
        self.push_nnz = sum(c[0].nnz for c in self.push_chunks)
        self.R = torch.zeros_like(self.P)  # received partials: chunk c = [world, mc_c, d] slabs
        self.sum_fn = sum_fn or (_default_sum_fn if dev.type == "cuda" else _host_sum)
        self.record_phases = False
        self.phases = PhaseRecorder(dev.type == "cuda")

    @staticmethod
    def _buf(k: int) -> int:
        return 0 if k == 0 else 1 + (k + 1) % 2

    def _mode(self, k: int) -> int:
        if self.K == 1:
            return _lib.LGX_LAYER_ONLY
        if k == 1:
            return _lib.LGX_LAYER_FIRST
        if k == self.K:
            return _lib.LGX_LAYER_LAST
        return _lib.LGX_LAYER_MID

    def _chunk_views(self, c0: int, m: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """P / R storage of the chunk starting at block row c0: [world, m, d] each, contiguous."""
        w, d = self.s.world, self.d
        off = w * c0 * d
        n = w * m * d
        return self.P.view(-1)[off:off + n].view(w, m, d), self.R.view(-1)[off:off + n].view(w, m, d)

    def _exchange(self, c0: int, m: int):
        """Rank q receives slab r of every rank r's chunk (the partials of q's own item rows)."""
        P, R = self._chunk_views(c0, m)
        if not self._collective:
            R.copy_(P)
            return None
        if self._a2a_native:
            return dist.all_to_all_single(R, P, group=self.group, async_op=True)
        # gloo with device tensors (rehearsals): the same all-to-all through host buffers, blocking;
        # each rank moves the bytes RCCL would move, not the world-fold of an all-gather
        Rh = torch.empty(R.shape, dtype=R.dtype)
        dist.all_to_all_single(Rh, P.cpu(), group=self.group)
        R.copy_(Rh)
        return None

    def _reduce(self, c0: int, m: int) -> None:
        """yi[c0:c0+m] = sum over ranks of the received slabs, in rank order."""
        _, R = self._chunk_views(c0, m)
        self.sum_fn(R, self.yi[c0:c0 + m])

    def _all_gather(self, table: torch.Tensor):
        if not self._collective:
            table.copy_(self.send_i)
            return None
        return dist.all_gather_into_tensor(table, self.send_i, group=self.group, async_op=True)

    def schedule(self) -> List[Tuple[str, int]]:
        """Per layer: push (items, chunked, each chunk exchanged), pull (users), item sums + epilogue +
        all-gather."""
        order = []
        for k in range(1, self.K + 1):
            order.extend([("push", k), ("pull", k), ("items", k)])
        return order

    def step(self) -> Tuple[torch.Tensor, torch.Tensor]:
        """One full propagation; returns this rank's (out_user, out_item) fp32 layer means."""
        s = self.s
        n_mean = float(self.K + 1)
        rec = self.phases if self.record_phases else None
        if rec:
            rec.begin()
        ag = None  # all-gather publishing the item table of the previous layer
        for k in range(1, self.K + 1):
            mode = self._mode(k)
            # push: item partial sums from this rank's users at layer k-1, chunk by chunk, each
            # chunk's exchange issued as soon as its launch is queued
            ex = []
            blocking = rec is not None and self._collective and not self._a2a_native
            for Ac, c0, m in self.push_chunks:
                self.layer_fn(Ac, self.Xu[k - 1], _lib.LGX_LAYER_PARTIAL,
                              out=self._chunk_views(c0, m)[0].view(s.world * m, self.d))
                if blocking:
                    rec.mark("push")
                ex.append(self._exchange(c0, m))
                if blocking:  # gloo: the exchange returned on the host only once done
                    rec.mark("exchange_sync")
            if rec:
                rec.mark("push")
            # pull: this rank's user rows from the full item table of layer k-1
            if ag is not None:
                ag.wait()
                if rec:
                    rec.mark("allgather_wait")
            Xi = self.Xi[self._buf(k - 1)]
            if self.K == 1:
                self.layer_fn(s.A_pull, Xi, _lib.LGX_LAYER_ONLY, E0=self.E0u, out=self.out_u, n_mean=n_mean)
            elif k < self.K:
                self.layer_fn(s.A_pull, Xi, _lib.LGX_LAYER_PLAIN, Y=self.Xu[k])
            else:
                self.stack_fn(s.A_pull, Xi, self.E0u, self.Xu[1:self.K], self.out_u, n_mean)
            if rec:
                rec.mark("pull")
            # items: the ordered cross-rank sums of the own block, its epilogue, then publish it
            for (_, c0, m), h in zip(self.push_chunks, ex):
                if h is not None:
                    h.wait()
                    if rec:
                        rec.mark("exchange_wait")
                self._reduce(c0, m)
                if rec:
                    rec.mark("reduce")
            n_i = s.n_i_local
            Yi = self.send_i[:n_i] if k < self.K else None
            self.epilogue_fn(self.yi[:n_i], mode, Y=Yi, E0=self.E0i, acc=self.acc_i, out=self.out_i,
                             n_mean=n_mean)
            if rec:
                rec.mark("epilogue")
            ag = self._all_gather(self.Xi[self._buf(k)]) if k < self.K else None
        if rec:
            rec.end()
        return self.out_u, self.out_i

    def phase_summary(self) -> Dict[str, float]:
        """Mean ms per recorded step by phase, plus comm_exposed_ms = allgather_wait +
        exchange_wait + exchange_sync (the stream's time behind collectives).  Synchronises the
        device."""
        if self.phases.cuda:
            torch.cuda.synchronize()
        ph = self.phases.summary()
        ph.pop("begin", None)
        ph["comm_exposed_ms"] = ph.get("allgather_wait", 0.0) + ph.get("exchange_wait", 0.0) + \
            ph.get("exchange_sync", 0.0)
        return ph

    def gather_outputs(self) -> Tuple[torch.Tensor, torch.Tensor]:
        """All-gather the sharded layer means into full [U, d] / [I, d] fp32 tables."""
        s = self.s
        mu = max(1, int(np.diff(s.user_bounds).max()))
        outs = []
        for loc, bounds, pad in ((self.out_u, s.user_bounds, mu), (self.out_i, s.item_bounds, s.mi)):
            slab = torch.zeros((pad, self.d), dtype=torch.float32, device=loc.device)
            slab[:loc.shape[0]] = loc
            full = torch.empty((s.world * pad, self.d), dtype=torch.float32, device=loc.device)
            if self._collective:
                dist.all_gather_into_tensor(full, slab, group=self.group)
            else:
                full.copy_(slab)
            parts = [full[q * pad:q * pad + int(bounds[q + 1] - bounds[q])] for q in range(s.world)]
            outs.append(torch.cat(parts))
        return outs[0], outs[1]
