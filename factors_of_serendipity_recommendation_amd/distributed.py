"""Row-sharded multi-GPU propagation: one process per GPU, RCCL all-gather of each layer's table
over xGMI.

The reference's only scale-out device is row-folding A^ into 100 blocks on one device
(dataloader.py:319-329, model.py:164-168; LightGCN-tf/LightGCN.py:201-213, 243-247).  Here the
folds become per-GPU row shards and the exchange step is a per-layer all-gather.

Partition.  User rows and item rows are sharded SEPARATELY into contiguous, nnz-balanced blocks
(rank r owns users [u_r, u_{r+1}) and items [i_r, i_{r+1})).  Because the graph is bipartite a
user row only references item columns and vice versa, so each rank holds two local operators:
    A_ui : local user rows -> item columns,  A_iu : local item rows -> user columns
with their column ids rewritten once into PADDED coordinates: rank q's item block lives at rows
[q*mi, q*mi + n_q) of an item table of world*mi rows (mi = max block size), likewise for users.
A layer's local output is written to a [mi, d] send buffer which is exactly this rank's
all_gather_into_tensor input, and the gathered table needs no reshuffle.  Send buffers ping-pong
by layer parity (the gather of layer k may still be reading one while layer k+1 of the same side
is computed into the other).

Overlap.  Layer k+1 of the users needs layer k of the items and vice versa, so the K layers form
two independent chains (I0 -> U1 -> I2 -> U3 ... and U0 -> I1 -> U2 -> I3 ...).  Steps are issued
alternating between the chains (U1, I1, I2, U2, U3, I3, ...): every step consumes the table
gathered two steps earlier, so each all-gather runs under the next step's SpMM.  The last layer
writes the layer mean of the rank's own rows (fp32) and is never gathered.

Buffers (per rank): layer-0 tables (the replicated E0), two ping-pong padded tables per side for
layers >= 1, fp32 layer sums for the local rows.  No data-path collective other than the
all-gathers.  The compute callable is injectable so that the CPU tests drive the same schedule
over gloo with an oracle SpMM.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Optional, Tuple

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


@dataclass
class Shard:
    rank: int
    world: int
    n_users: int
    n_items: int
    user_bounds: np.ndarray  # [world+1] global user ids
    item_bounds: np.ndarray  # [world+1] global item ids
    mu: int  # padded user block rows
    mi: int  # padded item block rows
    A_ui: CSRGraph  # local users -> padded item columns
    A_iu: CSRGraph  # local items -> padded user columns

    @property
    def n_u_local(self) -> int:
        return int(self.user_bounds[self.rank + 1] - self.user_bounds[self.rank])

    @property
    def n_i_local(self) -> int:
        return int(self.item_bounds[self.rank + 1] - self.item_bounds[self.rank])


def _remap_cols(cols: torch.Tensor, col_base: int, bounds: np.ndarray, pad: int) -> torch.Tensor:
    """Global column ids (in [col_base, col_base + n)) -> padded coordinates owner*pad + offset."""
    c = cols.to(torch.int64) - col_base
    b = torch.as_tensor(bounds, dtype=torch.int64, device=cols.device)
    owner = torch.searchsorted(b, c, right=True) - 1
    return (owner * pad + (c - b[owner])).to(torch.int32)


def _slice_rows(A: CSRGraph, r0: int, r1: int, col_base: int, bounds: np.ndarray, pad: int,
                n_cols_padded: int, seg_len: Optional[int]) -> CSRGraph:
    ip = A.indptr[r0:r1 + 1]
    s, e = int(ip[0]), int(ip[-1])
    indptr = (ip - s).contiguous()
    indices = _remap_cols(A.indices[s:e], col_base, bounds, pad).contiguous()
    vals = A.vals[s:e].contiguous()
    g = CSRGraph(indptr, indices, vals, r1 - r0, n_cols_padded)
    g.plan = make_plan(indptr.cpu().numpy(), seg_len)
    g.ensure_plan()
    return g


def make_shard(A: CSRGraph, n_users: int, n_items: int, rank: int, world: int,
               seg_len: Optional[int] = None) -> Shard:
    """Cut the full square operator (users first, then items) into this rank's two local operators."""
    ip = A.indptr.cpu().numpy()
    N = n_users + n_items
    ub = balanced_bounds(ip, 0, n_users, world)
    ib = balanced_bounds(ip, n_users, N, world) - n_users
    mu = max(1, int(np.diff(ub).max()))
    mi = max(1, int(np.diff(ib).max()))
    A_ui = _slice_rows(A, int(ub[rank]), int(ub[rank + 1]), n_users, ib, mi, world * mi, seg_len)
    A_iu = _slice_rows(A, n_users + int(ib[rank]), n_users + int(ib[rank + 1]), 0, ub, mu, world * mu, seg_len)
    return Shard(rank, world, n_users, n_items, ub, ib, mu, mi, A_ui, A_iu)


def pad_table(full: torch.Tensor, bounds: np.ndarray, pad: int) -> torch.Tensor:
    """[n, d] table in global row order -> [world*pad, d] padded layout (zeros in the gaps)."""
    world = len(bounds) - 1
    out = torch.zeros((world * pad, full.shape[1]), dtype=full.dtype, device=full.device)
    for q in range(world):
        a, b = int(bounds[q]), int(bounds[q + 1])
        out[q * pad:q * pad + (b - a)] = full[a:b]
    return out


LayerFn = Callable[..., None]


def _default_layer_fn(A, X, mode, Y=None, E0=None, acc=None, out=None, n_mean=1.0):
    from .ops import propagate_layer
    propagate_layer(A, X, mode, Y=Y, E0=E0, acc=acc, out=out, n_mean=n_mean)


class ShardedPropagation:
    """K-layer LightGCN propagation of a row-sharded graph (see module docstring)."""

    def __init__(self, shard: Shard, E0_user: torch.Tensor, E0_item: torch.Tensor, K: int,
                 group=None, layer_fn: Optional[LayerFn] = None):
        """E0_user / E0_item: the FULL layer-0 tables in global row order (replicated input, as every
        rank holds the embedding parameters); dtype f32 or bf16."""
        self.s = shard
        self.K = K
        self.group = group
        self.layer_fn = layer_fn or _default_layer_fn
        d = E0_user.shape[1]
        self.d = d
        dev, dt = E0_user.device, E0_user.dtype
        s = shard
        self.Xu = [pad_table(E0_user, s.user_bounds, s.mu)] + \
                  [torch.zeros((s.world * s.mu, d), dtype=dt, device=dev) for _ in range(2)]
        self.Xi = [pad_table(E0_item, s.item_bounds, s.mi)] + \
                  [torch.zeros((s.world * s.mi, d), dtype=dt, device=dev) for _ in range(2)]
        self.send_u = [torch.zeros((s.mu, d), dtype=dt, device=dev) for _ in range(2)]
        self.send_i = [torch.zeros((s.mi, d), dtype=dt, device=dev) for _ in range(2)]
        self.acc_u = torch.zeros((s.n_u_local, d), dtype=torch.float32, device=dev)
        self.acc_i = torch.zeros((s.n_i_local, d), dtype=torch.float32, device=dev)
        self.out_u = torch.zeros((s.n_u_local, d), dtype=torch.float32, device=dev)
        self.out_i = torch.zeros((s.n_i_local, d), dtype=torch.float32, device=dev)

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

    def _slab(self, table: torch.Tensor, pad: int, n_local: int) -> torch.Tensor:
        r = self.s.rank
        return table[r * pad:r * pad + n_local]

    def _gather(self, table: torch.Tensor, send: torch.Tensor, n_local: int):
        if self.s.world == 1:  # the single "gather" is a copy into the table
            table[:n_local].copy_(send[:n_local])  # (plumbing: a device memcpy)
            return None
        return dist.all_gather_into_tensor(table, send, group=self.group, async_op=True)

    def schedule(self) -> List[Tuple[str, int]]:
        """Issue order: alternate the two chains (U1, I1, I2, U2, U3, I3, ...)."""
        order = []
        for k in range(1, self.K + 1):
            pair = [("u", k), ("i", k)] if k % 2 == 1 else [("i", k), ("u", k)]
            order.extend(pair)
        return order

    def step(self) -> Tuple[torch.Tensor, torch.Tensor]:
        """One full propagation; returns this rank's (out_user, out_item) fp32 layer means."""
        s = self.s
        pending = {}  # (side, k) -> async work handle of the gather that publishes layer k
        for side, k in self.schedule():
            src_side = "i" if side == "u" else "u"
            h = pending.pop((src_side, k - 1), None)
            if h is not None:
                h.wait()
            mode = self._mode(k)
            if side == "u":
                A, X = s.A_ui, self.Xi[self._buf(k - 1)]
                Yt, send, n_loc = self.Xu[self._buf(k)], self.send_u[k & 1], s.n_u_local
                E0 = self._slab(self.Xu[0], s.mu, n_loc)
                acc, out = self.acc_u, self.out_u
            else:
                A, X = s.A_iu, self.Xu[self._buf(k - 1)]
                Yt, send, n_loc = self.Xi[self._buf(k)], self.send_i[k & 1], s.n_i_local
                E0 = self._slab(self.Xi[0], s.mi, n_loc)
                acc, out = self.acc_i, self.out_i
            Y = send[:n_loc] if k < self.K else None
            self.layer_fn(A, X, mode, Y=Y, E0=E0, acc=acc, out=out, n_mean=float(self.K + 1))
            if k < self.K:
                pending[(side, k)] = self._gather(Yt, send, n_loc)
        for h in pending.values():
            if h is not None:
                h.wait()
        return self.out_u, self.out_i

    def gather_outputs(self) -> Tuple[torch.Tensor, torch.Tensor]:
        """All-gather the sharded layer means into full [U, d] / [I, d] fp32 tables."""
        s = self.s
        outs = []
        for loc, bounds, pad in ((self.out_u, s.user_bounds, s.mu), (self.out_i, s.item_bounds, s.mi)):
            slab = torch.zeros((pad, self.d), dtype=torch.float32, device=loc.device)
            slab[:loc.shape[0]] = loc
            full = torch.empty((s.world * pad, self.d), dtype=torch.float32, device=loc.device)
            if s.world > 1:
                dist.all_gather_into_tensor(full, slab, group=self.group)
            else:
                full.copy_(slab)
            parts = [full[q * pad:q * pad + int(bounds[q + 1] - bounds[q])] for q in range(s.world)]
            outs.append(torch.cat(parts))
        return outs[0], outs[1]
