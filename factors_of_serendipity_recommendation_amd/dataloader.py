"""Drop-in ``Loader`` (lightGCN/LightGCN-PyTorch-master/code/dataloader.py:223-408) whose
files are parsed and whose adjacency is built on the GPU.

Same file format (``uid item item ...`` per line in train.txt / test.txt), same sizes
(n_user = max uid + 1, m_item = max item + 1 over train AND test, :247-285), same attributes and
methods (n_users, m_items, trainDataSize, testDict, allPos, UserItemNet, getUserPosItems,
getUserItemFeedback, getSparseGraph).  ``getSparseGraph()`` still honours the
``s_pre_adj_mat.npz`` cache (:343, :367) and still returns a coalesced float32 torch sparse COO on
the device (:373-374); ``getCSRGraph()`` hands the HIP engine the CSR it was built from.

Nothing here loops over users or lines in Python, so a 10^8-edge train.txt loads in seconds:
  * the text is parsed by ``lgx_parse_lines_*`` into flat (line uid, line offsets, items) arrays
    that stay on the device; the adjacency is built from them without a host round trip;
  * ``allPos`` / ``getUserPosItems`` are views (``PosLists``) over one sorted, de-duplicated
    per-user CSR (what ``UserItemNet[u].nonzero()[1]`` returns, :299-317), built by one device sort;
  * ``testDict`` is a read-only mapping (``TestDict``) over a stable per-user grouping of the test
    pairs, keys in first-appearance order and items in file order (``__build_test``, :389-399);
  * ``UserItemNet`` (the scipy matrix, duplicates summed, :288) is built on first access only.
"""
from __future__ import annotations

import os
from collections.abc import Mapping, Sequence
from typing import List, Optional, Tuple

import numpy as np
import scipy.sparse as sp
import torch

from .graph import CSRGraph, build_norm_adj, from_csr_arrays

DEFAULT_CONFIG = {"A_split": False, "A_n_fold": 100}


def _flat_lines_host(path: str):
    """Host reader of the same grammar (dataloader.py:247-260) -> flat (uids, offsets, items)."""
    uids: List[int] = []
    lens: List[int] = []
    parts_all: List[np.ndarray] = []
    with open(path) as f:
        for line in f.readlines():
            if len(line) > 0:
                parts = line.strip("\n").split(" ")
                uids.append(int(parts[0]))
                row = np.asarray([int(i) for i in parts[1:]], dtype=np.int64)
                lens.append(len(row))
                parts_all.append(row)
    off = np.zeros(len(uids) + 1, dtype=np.int64)
    np.cumsum(np.asarray(lens, dtype=np.int64), out=off[1:])
    items = np.concatenate(parts_all) if parts_all else np.zeros(0, np.int64)
    return (torch.as_tensor(np.asarray(uids, dtype=np.int64)), torch.from_numpy(off), torch.from_numpy(items))


def read_flat(path: str, device) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """(line uid int64 [L], line offsets int64 [L+1], items int64 [P]) on ``device``; on a CUDA
    device the bytes are parsed by the GPU (``ops.read_interactions_device``)."""
    device = torch.device(device)
    if device.type == "cuda":
        from .ops import read_interactions_device
        lu, lp, it, _ = read_interactions_device(path, device)
        return lu.to(torch.int64), lp, it.to(torch.int64)
    return _flat_lines_host(path)


def read_interactions(path: str, device=None):
    """Parse one LightGCN txt file -> (uids, items-per-line lists) (dataloader.py:247-260)."""
    lu, lp, it = read_flat(path, device if device is not None else "cpu")
    lu, lp, it = lu.cpu().numpy(), lp.cpu().numpy(), it.cpu().numpy()
    return lu.tolist(), [it[lp[j]:lp[j + 1]] for j in range(len(lu))]


class PosLists(Sequence):
    """Per-user sorted unique item lists as one CSR (``indptr`` int64 [n+1], ``indices`` int32):
    ``lists[u]`` is what ``UserItemNet[u].nonzero()[1]`` returns (dataloader.py:404-408).  A view
    over a subset of users (``rows``) keeps the parent CSR; ``device_csr()`` packs the selected rows
    on the device without a Python loop, which ``ops.lists_to_device_csr`` uses."""

    def __init__(self, indptr: np.ndarray, indices: np.ndarray, dev_csr=None, rows: Optional[np.ndarray] = None):
        self.indptr, self.indices, self._dev, self.rows = indptr, indices, dev_csr, rows

    def __len__(self):
        return len(self.indptr) - 1 if self.rows is None else len(self.rows)

    def __getitem__(self, j):
        if isinstance(j, slice):
            return [self[t] for t in range(*j.indices(len(self)))]
        n = len(self)
        if j < 0:
            j += n
        if not 0 <= j < n:
            raise IndexError("PosLists index out of range")
        u = j if self.rows is None else int(self.rows[j])
        return self.indices[self.indptr[u]:self.indptr[u + 1]]

    def select(self, users) -> "PosLists":
        users = np.asarray(users, dtype=np.int64).reshape(-1)
        if self.rows is not None:
            users = self.rows[users]
        n = len(self.indptr) - 1
        if users.size and (users.min() < 0 or users.max() >= n):
            raise IndexError("user id out of range")
        return PosLists(self.indptr, self.indices, self._dev, users)

    def device_csr(self, device) -> Tuple[torch.Tensor, torch.Tensor]:
        device = torch.device(device)
        if self._dev is None or self._dev[0].device != device:
            self._dev = (torch.from_numpy(self.indptr).to(device), torch.from_numpy(self.indices).to(device))
        ip, ix = self._dev
        if self.rows is None:
            return ip, ix
        return gather_csr_rows(ip, ix, torch.from_numpy(self.rows).to(device))


def gather_csr_rows(indptr: torch.Tensor, indices: torch.Tensor, rows: torch.Tensor):
    """The CSR of the listed rows, in list order, on the CSR's device (no Python loop)."""
    start = indptr[rows]
    lens = indptr[rows + 1] - start
    ptr = torch.zeros(rows.numel() + 1, dtype=torch.int64, device=indptr.device)
    torch.cumsum(lens, 0, out=ptr[1:])
    total = int(ptr[-1])
    if total == 0:
        return ptr, torch.zeros(1, dtype=indices.dtype, device=indices.device)
    owner = torch.repeat_interleave(torch.arange(rows.numel(), device=indptr.device), lens)
    src = start[owner] + (torch.arange(total, device=indptr.device) - ptr[owner])
    return ptr, indices[src].contiguous()


class TestDict(Mapping):
    """Read-only ``{user: [items]}`` over grouped test pairs: keys in first-appearance order, each
    value the user's items in file order, as ``Loader.__build_test`` (dataloader.py:389-399)."""

    def __init__(self, users: np.ndarray, indptr: np.ndarray, items: np.ndarray):
        self._users, self._ptr, self._items = users, indptr, items
        self._pos = {}  # built on first lookup (one dict of ints, not of lists)

    def __len__(self):
        return len(self._users)

    def __iter__(self):
        return iter(self._users.tolist())

    def keys(self):
        return self._users.tolist()

    def __getitem__(self, u):
        if not self._pos:
            self._pos = dict(zip(self._users.tolist(), range(len(self._users))))
        j = self._pos[int(u)]
        return self._items[self._ptr[j]:self._ptr[j + 1]].tolist()

    def csr(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """(users, indptr, items) in key order."""
        return self._users, self._ptr, self._items


def _group_by_user(users: torch.Tensor, items: torch.Tensor):
    """Stable grouping of (user, item) pairs: (keys in first-appearance order, indptr, items)."""
    if users.numel() == 0:
        return np.zeros(0, np.int64), np.zeros(1, np.int64), np.zeros(0, np.int64)
    order = torch.sort(users, stable=True).indices
    su, si = users[order], items[order]
    keys, counts = torch.unique_consecutive(su, return_counts=True)
    ptr = torch.zeros(keys.numel() + 1, dtype=torch.int64, device=users.device)
    torch.cumsum(counts, 0, out=ptr[1:])
    first = order[ptr[:-1]]                      # first appearance of each key in file order
    kord = torch.argsort(first)
    lens = counts[kord]
    ptr2 = torch.zeros_like(ptr)
    torch.cumsum(lens, 0, out=ptr2[1:])
    # regroup the items so that the groups follow kord
    owner = torch.repeat_interleave(torch.arange(keys.numel(), device=users.device), lens)
    src = ptr[kord][owner] + (torch.arange(si.numel(), device=users.device) - ptr2[owner])
    return keys[kord].cpu().numpy(), ptr2.cpu().numpy(), si[src].cpu().numpy()


class Loader:
    """Dataset type for pytorch; includes the graph (GPU-built)."""

    def __init__(self, config: Optional[dict] = None, path: str = "../data/gowalla", device="cuda",
                 cache_adj: bool = True):
        config = dict(DEFAULT_CONFIG, **(config or {}))
        self.split = config["A_split"]
        self.folds = config["A_n_fold"]
        self.path = path
        self.device = torch.device(device)
        self.cache_adj = cache_adj
        tr_u, tr_p, tr_i = read_flat(os.path.join(path, "train.txt"), self.device)
        te_u, te_p, te_i = read_flat(os.path.join(path, "test.txt"), self.device)
        # one row per pair (the reference's trainUser / trainItem, :259-260)
        tr_pu = torch.repeat_interleave(tr_u, torch.diff(tr_p))
        te_pu = torch.repeat_interleave(te_u, torch.diff(te_p))
        maxes = [int(t.max()) for t in (tr_i, te_i) if t.numel()]
        umax = [int(t.max()) for t in (tr_u, te_u) if t.numel()]
        self.m_item = max(maxes + [0]) + 1
        self.n_user = max(umax + [0]) + 1
        self._train_pairs = (tr_pu, tr_i)            # device copies for the adjacency build
        self.trainUniqueUsers = tr_u.cpu().numpy()
        self.trainUser = tr_pu.cpu().numpy()
        self.trainItem = tr_i.cpu().numpy()
        self.testUniqueUsers = te_u.cpu().numpy()
        self.testUser = te_pu.cpu().numpy()
        self.testItem = te_i.cpu().numpy()
        self.traindataSize = int(len(self.trainItem))
        self.testDataSize = int(len(self.testItem))
        self.Graph = None
        self._csr: Optional[CSRGraph] = None
        self._uin = None
        # degrees with duplicates counted (sums of the reference's UserItemNet, :290-293)
        self.users_D = np.bincount(self.trainUser, minlength=self.n_user).astype(np.float64)
        self.users_D[self.users_D == 0.] = 1
        self.items_D = np.bincount(self.trainItem, minlength=self.m_item).astype(np.float64)
        self.items_D[self.items_D == 0.] = 1.
        self._allPos = self._build_pos(tr_pu, tr_i)
        self.__testDict = TestDict(*_group_by_user(te_pu, te_i))

    def _build_pos(self, users: torch.Tensor, items: torch.Tensor) -> PosLists:
        """Sorted unique items per user: one sort of the packed (user, item) keys."""
        keys = torch.unique(users * self.m_item + items)  # sorted, duplicates collapsed
        pu = keys // self.m_item
        ptr = torch.zeros(self.n_user + 1, dtype=torch.int64, device=keys.device)
        torch.cumsum(torch.bincount(pu, minlength=self.n_user), 0, out=ptr[1:])
        idx = (keys % self.m_item).to(torch.int32)
        dev = (ptr, idx) if keys.device.type == "cuda" else None
        return PosLists(ptr.cpu().numpy(), idx.cpu().numpy(), dev)

    @property
    def n_users(self):
        return self.n_user

    @property
    def m_items(self):
        return self.m_item

    @property
    def trainDataSize(self):
        return self.traindataSize

    @property
    def testDict(self):
        return self.__testDict

    @property
    def allPos(self):
        return self._allPos

    @property
    def UserItemNet(self):
        """(users, items) bipartite graph; duplicates summed as csr_matrix does (:288-289)."""
        if self._uin is None:
            self._uin = sp.csr_matrix((np.ones(len(self.trainUser)), (self.trainUser, self.trainItem)),
                                      shape=(self.n_user, self.m_item))
        return self._uin

    def getCSRGraph(self) -> CSRGraph:
        """The normalized adjacency as a device CSRGraph (built once)."""
        if self._csr is None:
            cache = os.path.join(self.path, "s_pre_adj_mat.npz")
            if self.cache_adj and os.path.exists(cache):
                A = sp.load_npz(cache).tocsr()
                A.sort_indices()
                self._csr = from_csr_arrays(A.indptr, A.indices, A.data.astype(np.float32), n_cols=A.shape[1],
                                            device=self.device, n_users=self.n_users, n_items=self.m_items)
            else:
                u, i = self._train_pairs
                self._csr = build_norm_adj(u, i, self.n_users, self.m_items, dedup=False, device=self.device)
                if self.cache_adj:
                    try:
                        sp.save_npz(cache, self._csr.to_scipy())
                    except OSError:
                        pass
        return self._csr

    def getSparseGraph(self):
        if self.Graph is None:
            G = self.getCSRGraph().to_sparse_coo()
            if self.split:
                N = G.shape[0]
                fold_len = N // self.folds
                bounds = [(f * fold_len, N if f == self.folds - 1 else (f + 1) * fold_len) for f in range(self.folds)]
                dense_rows = G.indices()[0]
                self.Graph = []
                for s, e in bounds:  # _split_A_hat (dataloader.py:319-329)
                    m = (dense_rows >= s) & (dense_rows < e)
                    idx = G.indices()[:, m].clone()
                    idx[0] -= s
                    self.Graph.append(torch.sparse_coo_tensor(idx, G.values()[m], (e - s, N)).coalesce())
            else:
                self.Graph = G
        return self.Graph

    def getUserItemFeedback(self, users, items):
        return np.array(self.UserItemNet[users, items]).astype("uint8").reshape((-1,))

    def getUserPosItems(self, users):
        """A ``PosLists`` view: ``[allPos[u] for u in users]`` without the per-user slicing."""
        return self._allPos.select(users)
