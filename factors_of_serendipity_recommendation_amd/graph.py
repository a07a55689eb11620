"""Normalized-adjacency CSR graphs in HBM and their SpMM launch plans.

Replaces the reference's host-side graph build (``Loader.getSparseGraph``,
lightGCN/LightGCN-PyTorch-master/code/dataloader.py:339-376, and ``Data.get_adj_mat``,
LightGCN-tf/utility/load_data.py:77-106): the edge list is uploaded once and the whole
``D^-1/2 A D^-1/2`` CSR is built on the GPU (``lgx_build_norm_adj``).

HBM layout of a ``CSRGraph`` (N = n_users + n_items rows; users first, then items, exactly the
row order of the reference's ``cat([users_emb, items_emb])`` at model.py:151):
    indptr  int64 [N+1]      indices int32 [nnz]      vals float32 [nnz]
plus the launch plan of ``make_plan`` (segment tables, int32) and an fp32 partial-sum scratch.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib

# Segment plans (tools/segprobe.py, one MI355X, SpMM layer time by seg_len and gathers in flight):
#  - graphs under 2^24 nnz (tables L2/MALL-resident): ~64 K segments of 32..128 nonzeros, run with
#    8 gathers in flight per lane (csrc/spmm.hip picks that for seg_len <= 128): Gowalla shape 37.8
#    -> 36.9 us, ML-1M 37.8 -> 35.8 us, Amazon-book shape 144.3 -> 126.6 us per layer;
#  - larger graphs: ~32 K segments of 64..8192 with 16 in flight (C4: 8192, 29.9 ms per layer against
#    30.7 at 2048 and 30.6 at 16384, tools/spmm_probe.py --phase).
_SMALL_NNZ = 1 << 24

# Column blocking of the item rows (lgx_csr cb_*): the item rows gather the user table, which at C4
# is 5.12 GB (f32) / 2.56 GB (bf16), far past the 256 MB Infinity Cache.  Cut into column ranges,
# each launch gathers one slice of the table, at the price of one pass over every item row per block
# (segment table, row bounds, partial CSR lines) and an f32 read + write of the carried row sums.
# tools/cb_probe.py (one MI355X, C4 PLAIN layer, profiles/r03_cb_probe.txt):
#   f32:  57.24 ms unblocked; 55.10 / 53.58 / 57.63 / 60.66 / 69.51 ms in 4 / 8 / 13 / 16 / 24 blocks
#   bf16: 28.94 ms unblocked; 28.95 / 29.03 / 34.25 ms in 4 / 8 / 13 blocks
# so tables of >= 4 GiB are cut into 640 MiB slices (f32 C4: 8 blocks) and smaller ones not at all.
_CB_TABLE_MIN = 4 << 30
_CB_SLICE_BYTES = 640 << 20


def choose_seg_len(nnz: int) -> int:
    """Segment length: long enough to amortise the fix-up, short enough that hub rows are split
    into >= the chip's group slots (power of two; see the table above)."""
    if nnz < _SMALL_NNZ:
        target, lo, hi = 65536, 32, 128
    else:
        target, lo, hi = 32768, 256, 8192
    want = max(1, nnz // target)
    s = lo
    while s < want and s < hi:
        s *= 2
    return s


@dataclass
class Plan:
    """Host-side (numpy) launch plan; see ``struct lgx_csr`` in include/lgx.h."""

    seg_row: np.ndarray
    seg_part: np.ndarray
    seg_slot: np.ndarray
    split_row: np.ndarray
    split_ptr: np.ndarray
    seg_len: int

    @property
    def n_partials(self) -> int:
        return int(self.split_ptr[-1]) if len(self.split_ptr) else 0


def make_plan(indptr: np.ndarray, seg_len: Optional[int] = None,
              phases: Optional[Sequence[Tuple[int, int]]] = None) -> Plan:
    """Cut every row into segments of <= seg_len nonzeros (every row, even an empty one, gets at
    least one segment because its epilogue must still run) and order them longest-first so that
    groups of one wave see similar trip counts and hub rows start early.

    phases: row ranges [r0, r1) that partition the rows, in launch order; each is ordered
    longest-first on its own.  For the bipartite adjacency, (items, users) keeps the gathers of
    one launch phase inside ONE table (item rows read the user table, user rows the item table),
    so the cache holds one working set at a time instead of both interleaved."""
    indptr = np.asarray(indptr, dtype=np.int64)
    lens = np.diff(indptr)
    nnz = int(indptr[-1]) if len(indptr) else 0
    if seg_len is None:
        seg_len = choose_seg_len(nnz)
    nseg = np.maximum(1, -(-lens // seg_len)).astype(np.int64)
    if phases is None:
        order = np.argsort(-lens, kind="stable")
    else:
        cover = sorted((int(a), int(b)) for a, b in phases)
        if (cover and (cover[0][0] != 0 or cover[-1][1] != len(lens))) or any(
                cover[j][1] != cover[j + 1][0] for j in range(len(cover) - 1)):
            raise ValueError(f"phases {list(phases)} do not partition rows [0, {len(lens)})")
        order = np.concatenate([int(a) + np.argsort(-lens[int(a):int(b)], kind="stable") for a, b in phases]
                               + [np.zeros(0, dtype=np.int64)])
    nseg_o = nseg[order]
    total = int(nseg_o.sum())
    if total >= 2**31:
        raise ValueError("too many row segments for int32 plan tables")
    seg_row = np.repeat(order, nseg_o).astype(np.int32)
    starts = np.cumsum(nseg_o) - nseg_o
    seg_part = (np.arange(total, dtype=np.int64) - np.repeat(starts, nseg_o)).astype(np.int32)
    split_mask = nseg_o > 1
    split_row = order[split_mask].astype(np.int32)
    split_counts = nseg_o[split_mask]
    split_ptr = np.zeros(len(split_row) + 1, dtype=np.int64)
    np.cumsum(split_counts, out=split_ptr[1:])
    slot_base = np.full(len(lens), -1, dtype=np.int64)
    slot_base[split_row] = split_ptr[:-1]
    seg_slot = np.where(nseg[seg_row] > 1, slot_base[seg_row] + seg_part, -1).astype(np.int32)
    return Plan(seg_row, seg_part, seg_slot, split_row, split_ptr.astype(np.int32), int(seg_len))


@dataclass
class CSRGraph:
    """A row block of the normalized adjacency resident in HBM, ready for ``lgx_propagate*``.

    ``n_rows`` output rows; column ids index a table of ``n_cols`` rows.  For the single-GPU
    operator n_rows == n_cols == n_users + n_items."""

    indptr: torch.Tensor
    indices: torch.Tensor
    vals: torch.Tensor
    n_rows: int
    n_cols: int
    n_users: int = 0
    n_items: int = 0
    plan: Optional[Plan] = None
    col_blocking: bool = True  # column-block the item rows when their gathered table is large
    col_block_min: int = _CB_TABLE_MIN      # (tests lower these to block small graphs)
    col_block_slice: int = _CB_SLICE_BYTES
    _dev_plan: dict = field(default_factory=dict, repr=False)

    @property
    def nnz(self) -> int:
        return int(self.indices.numel())

    @property
    def device(self) -> torch.device:
        return self.indptr.device

    def ensure_plan(self, seg_len: Optional[int] = None) -> "CSRGraph":
        if self.plan is None or (seg_len is not None and seg_len != self.plan.seg_len):
            self.plan = make_plan(self.indptr.cpu().numpy(), seg_len, self.phases())
            self._dev_plan.clear()
        if not self._dev_plan:
            dev = self.device
            p = self.plan
            self._dev_plan = {
                "seg_row": torch.from_numpy(p.seg_row).to(dev),
                "seg_part": torch.from_numpy(p.seg_part).to(dev),
                "seg_slot": torch.from_numpy(p.seg_slot).to(dev),
                "split_row": torch.from_numpy(p.split_row).to(dev),
                "split_ptr": torch.from_numpy(p.split_ptr).to(dev),
            }
        return self

    def phases(self) -> Optional[Tuple[Tuple[int, int], ...]]:
        """Launch phases of the full bipartite adjacency: user rows (gathering the item table),
        then item rows (gathering the user table).  One table per phase keeps the L2 / MALL
        working set to one table at a time: the C4 layer takes 41.8 ms phased against 44.1 ms
        with both kinds of rows interleaved longest-first (tools/spmm_probe.py --phase)."""
        U, I = self.n_users, self.n_items
        if U > 0 and I > 0 and self.n_rows == U + I == self.n_cols:
            return ((0, U), (U, U + I))
        return None

    def partials(self, d: int) -> Optional[torch.Tensor]:
        self.ensure_plan()
        n = self.plan.n_partials
        if n == 0:
            return None
        key = ("partials", d)
        t = self._dev_plan.get(key)
        if t is None:
            t = torch.empty((n, d), dtype=torch.float32, device=self.device)
            self._dev_plan[key] = t
        return t

    def col_block_count(self, d: int, elem_size: int) -> int:
        """Column blocks of the item rows for tables of d x elem_size-byte rows (0 = none): the
        square bipartite operator only, when the user table they gather is at least
        ``col_block_min`` bytes (4 GiB), its plan phased users-first, and every item row holding
        user columns only.  That last condition is what makes the item rows' (row, column) keys
        sorted, which ``col_blocks`` relies on: an operator with self-loops (the reference TF
        'norm' / plain adjacencies add the identity, load_data.py:142, LightGCN.py:457) keeps the
        one-launch layer.  The checks run once per graph and the count once per table shape."""
        if not self.col_blocking or self.phases() is None or self.n_users < 2:
            return 0
        table = self.n_users * d * elem_size
        if table < self.col_block_min:
            return 0
        key = ("cb_count", d, elem_size, self.col_block_min, self.col_block_slice)
        got = self._dev_plan.get(key)
        if got is not None:
            return got
        self.ensure_plan()
        nb = 0
        if self._users_first_plan() and self._item_rows_gather_users_only():
            nb = int(max(1, min(64, -(-table // self.col_block_slice), self.n_users)))
        self._dev_plan[key] = nb
        return nb

    def _users_first_plan(self) -> bool:
        """The plan's user-row segments and split rows form a prefix (phases users, then items)."""
        got = self._dev_plan.get("users_first")
        if got is None:
            p, U = self.plan, self.n_users
            nu, ns = int(np.count_nonzero(p.seg_row < U)), int(np.count_nonzero(p.split_row < U))
            got = bool((p.seg_row[:nu] < U).all() and (p.split_row[:ns] < U).all())
            self._dev_plan["users_first"] = got
        return got

    def _item_rows_gather_users_only(self) -> bool:
        """Every column of the item rows is a user id (< n_users), checked on the device."""
        got = self._dev_plan.get("items_users_only")
        if got is None:
            s0 = int(self.indptr[self.n_users].item())
            tail = self.indices[s0:]
            got = bool(tail.numel() == 0 or int(tail.max().item()) < self.n_users)
            self._dev_plan["items_users_only"] = got
        return got

    def col_blocks(self, nb: int) -> dict:
        """Block b of item row r covers the nonzeros [ptr[b, r], ptr[b + 1, r]) -- the columns
        (user ids) in [b U / nb, (b + 1) U / nb) -- with its own launch plan (global row ids).
        Built once per nb on the device: the (row, column) keys of the item rows are sorted, so
        every boundary is one searchsorted."""
        key = ("cb", nb)
        got = self._dev_plan.get(key)
        if got is not None:
            return got
        self.ensure_plan()
        U, I, dev = self.n_users, self.n_items, self.device
        ip = self.indptr
        s0 = int(ip[U].item())
        item_ptr = ip[U:U + I + 1]
        lens = torch.diff(item_ptr)
        rows = torch.repeat_interleave(torch.arange(I, device=dev, dtype=torch.int64), lens)
        keys = rows * U + self.indices[s0:].to(torch.int64)
        del rows
        cuts = (torch.arange(1, nb, device=dev, dtype=torch.int64) * U) // nb
        q = (torch.arange(I, device=dev, dtype=torch.int64)[None, :] * U + cuts[:, None]).reshape(-1)
        inner = (torch.searchsorted(keys, q) + s0).reshape(nb - 1, I)
        del keys, q
        ptr = torch.cat([item_ptr[:-1][None, :], inner, item_ptr[1:][None, :]]).contiguous()  # [nb + 1, I]
        blen = torch.diff(ptr, dim=0).cpu().numpy()
        plans, dplans = [], []
        for b in range(nb):
            ipb = np.zeros(I + 1, dtype=np.int64)
            np.cumsum(blen[b], out=ipb[1:])
            pb = make_plan(ipb, self.plan.seg_len)
            pb.seg_row = (pb.seg_row.astype(np.int64) + U).astype(np.int32)
            pb.split_row = (pb.split_row.astype(np.int64) + U).astype(np.int32)
            plans.append(pb)
            dplans.append({k: torch.from_numpy(getattr(pb, k)).to(dev)
                           for k in ("seg_row", "seg_part", "seg_slot", "split_row", "split_ptr")})
        # the unblocked rows (users) are the first phase of the full plan: a prefix of its segments,
        # split rows and partial slots
        p = self.plan
        got = {"ptr": ptr, "plans": plans, "dplans": dplans,
               "n_user_segs": int(np.count_nonzero(p.seg_row < U)),
               "n_user_split": int(np.count_nonzero(p.split_row < U))}
        self._dev_plan[key] = got
        return got

    def c_struct(self, d: int, elem_size: Optional[int] = None) -> _lib.LgxCSR:
        """``struct lgx_csr`` view (device pointers) for an embedding dim d; with the storage
        element size, the item rows are column-blocked when col_block_count says so."""
        self.ensure_plan()
        p, dp = self.plan, self._dev_plan
        part = self.partials(d)
        nb = self.col_block_count(d, elem_size) if elem_size else 0
        n_segs, n_split = len(p.seg_row), len(p.split_row)
        cb = (0, 0, None, None, None)
        if nb > 0:
            blk = self.col_blocks(nb)
            n_segs, n_split = blk["n_user_segs"], blk["n_user_split"]
            key = ("cb_struct", nb, d)
            keep = self._dev_plan.get(key)
            if keep is None:
                n_part = max(pb.n_partials for pb in blk["plans"])
                bpart = torch.empty((max(n_part, 1), d), dtype=torch.float32, device=self.device)
                carry = torch.empty((self.n_items, d), dtype=torch.float32, device=self.device)
                arr = (_lib.LgxPlan * nb)()
                for b, (pb, q) in enumerate(zip(blk["plans"], blk["dplans"])):
                    arr[b] = _lib.LgxPlan(q["seg_row"].data_ptr(), q["seg_part"].data_ptr(), q["seg_slot"].data_ptr(),
                                          len(pb.seg_row), pb.seg_len,
                                          q["split_row"].data_ptr() if len(pb.split_row) else None,
                                          q["split_ptr"].data_ptr(), len(pb.split_row), pb.n_partials,
                                          bpart.data_ptr() if pb.n_partials else None)
                keep = self._dev_plan[key] = (arr, bpart, carry)
            arr, _, carry = keep
            cb = (self.n_users, nb, blk["ptr"].data_ptr(), arr, carry.data_ptr())
        return _lib.LgxCSR(
            self.indptr.data_ptr(), self.indices.data_ptr(), self.vals.data_ptr(),
            self.n_rows, self.n_cols, self.nnz,
            dp["seg_row"].data_ptr(), dp["seg_part"].data_ptr(), dp["seg_slot"].data_ptr(),
            n_segs, p.seg_len,
            dp["split_row"].data_ptr() if n_split else None,
            dp["split_ptr"].data_ptr(),
            n_split, p.n_partials,
            part.data_ptr() if part is not None else None,
            *cb,
        )

    def to_sparse_coo(self) -> torch.Tensor:
        """The reference's graph object: a coalesced float32 torch sparse COO [N, N] on the same
        device (dataloader.py:331-337, 373-374)."""
        rows = torch.repeat_interleave(torch.arange(self.n_rows, device=self.device),
                                       torch.diff(self.indptr))
        idx = torch.stack([rows, self.indices.long()])
        return torch.sparse_coo_tensor(idx, self.vals, (self.n_rows, self.n_cols)).coalesce()

    def to_scipy(self):
        import scipy.sparse as sp
        return sp.csr_matrix((self.vals.cpu().numpy(), self.indices.cpu().numpy(),
                              self.indptr.cpu().numpy()), shape=(self.n_rows, self.n_cols))


def _stream_ptr(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_gpu(*tensors: torch.Tensor) -> None:
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError("factors_of_serendipity_recommendation_amd ops run on the GPU only "
                               f"(got a tensor on {t.device}); there is no CPU fallback")


def build_norm_adj(users, items, n_users: int, n_items: int, dedup: bool = False,
                   device="cuda", seg_len: Optional[int] = None) -> CSRGraph:
    """D^-1/2 A D^-1/2 of the bipartite graph on the GPU (``lgx_build_norm_adj``).

    dedup=False: duplicate (u,i) pairs are summed (PyTorch Loader, dataloader.py:288);
    dedup=True: they collapse to one edge (TF Data, load_data.py:61)."""
    device = torch.device(device)
    u = torch.as_tensor(users).to(device=device, dtype=torch.int32).contiguous()
    i = torch.as_tensor(items).to(device=device, dtype=torch.int32).contiguous()
    require_gpu(u, i)
    E = int(u.numel())
    if int(i.numel()) != E:
        raise ValueError("users and items must have the same length")
    if E:
        lo_u, hi_u = int(u.min()), int(u.max())
        lo_i, hi_i = int(i.min()), int(i.max())
        if lo_u < 0 or hi_u >= n_users or lo_i < 0 or hi_i >= n_items:
            raise ValueError("edge index out of range")
    N = n_users + n_items
    L = _lib.lib()
    ws = ctypes.c_size_t(0)
    _lib.check(L.lgx_build_norm_adj_workspace(E, n_users, n_items, ctypes.byref(ws)),
               "lgx_build_norm_adj_workspace")
    indptr = torch.empty(N + 1, dtype=torch.int64, device=device)
    indices = torch.empty(max(2 * E, 1), dtype=torch.int32, device=device)
    vals = torch.empty(max(2 * E, 1), dtype=torch.float32, device=device)
    work = torch.empty(max(ws.value, 1), dtype=torch.uint8, device=device)
    _lib.check(L.lgx_build_norm_adj(u.data_ptr(), i.data_ptr(), E, n_users, n_items, int(dedup),
                                    indptr.data_ptr(), indices.data_ptr(), vals.data_ptr(),
                                    work.data_ptr(), ws.value, _stream_ptr(device)),
               "lgx_build_norm_adj")
    del work
    nnz = int(indptr[-1].item())
    g = CSRGraph(indptr, indices[:nnz], vals[:nnz], N, N, n_users, n_items)
    g.ensure_plan(seg_len)
    return g


def from_csr_arrays(indptr, indices, vals, n_cols: Optional[int] = None, device="cuda",
                    n_users: int = 0, n_items: int = 0, seg_len: Optional[int] = None) -> CSRGraph:
    """Wrap existing CSR arrays (e.g. a loaded ``s_pre_adj_mat.npz``) as a device CSRGraph."""
    device = torch.device(device)
    ip = torch.as_tensor(np.asarray(indptr, dtype=np.int64) if not torch.is_tensor(indptr) else indptr)
    ip = ip.to(device=device, dtype=torch.int64).contiguous()
    ix = torch.as_tensor(indices).to(device=device, dtype=torch.int32).contiguous()
    vv = torch.as_tensor(vals).to(device=device, dtype=torch.float32).contiguous()
    require_gpu(ip)
    n_rows = ip.numel() - 1
    g = CSRGraph(ip, ix, vv, n_rows, n_cols if n_cols is not None else n_rows, n_users, n_items)
    g.ensure_plan(seg_len)
    return g


def from_sparse_coo(G: torch.Tensor, n_users: int = 0, n_items: int = 0,
                    seg_len: Optional[int] = None) -> CSRGraph:
    """Accept the reference's graph (a coalesced torch sparse COO, dataloader.py:373-374) and
    derive the CSR row pointer on the GPU (``lgx_csr_from_coo_rows``)."""
    if not G.is_sparse:
        raise TypeError("expected a torch sparse COO tensor")
    G = G.coalesce()
    require_gpu(G)
    idx = G.indices()
    rows = idx[0].contiguous()
    n_rows, n_cols = G.shape
    indptr = torch.empty(n_rows + 1, dtype=torch.int64, device=G.device)
    _lib.check(_lib.lib().lgx_csr_from_coo_rows(rows.data_ptr(), rows.numel(), n_rows, indptr.data_ptr(),
                                                _stream_ptr(G.device)), "lgx_csr_from_coo_rows")
    g = CSRGraph(indptr, idx[1].to(torch.int32).contiguous(), G.values().to(torch.float32).contiguous(),
                 n_rows, n_cols, n_users, n_items)
    g.ensure_plan(seg_len)
    return g
