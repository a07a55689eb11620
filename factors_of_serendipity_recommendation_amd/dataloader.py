"""Drop-in ``Loader`` (lightGCN/LightGCN-PyTorch-master/code/dataloader.py:223-408) whose
adjacency is built on the GPU.

Same file format (``uid item item ...`` per line in train.txt / test.txt), same sizes
(n_user = max uid + 1, m_item = max item + 1 over train AND test, :247-285), same attributes and
methods (n_users, m_items, trainDataSize, testDict, allPos, UserItemNet, getUserPosItems,
getUserItemFeedback, getSparseGraph).  ``getSparseGraph()`` still honours the
``s_pre_adj_mat.npz`` cache (:343, :367) and still returns a coalesced float32 torch sparse COO on
the device (:373-374); ``getCSRGraph()`` hands the HIP engine the CSR it was built from.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import numpy as np
import scipy.sparse as sp
import torch

from .graph import CSRGraph, build_norm_adj, from_csr_arrays

DEFAULT_CONFIG = {"A_split": False, "A_n_fold": 100}


def read_interactions(path: str, device=None):
    """Parse one LightGCN txt file -> (uids, items-per-line lists) (dataloader.py:247-260).
    On a CUDA device the bytes are parsed by the GPU (``ops.read_interactions_device``)."""
    if device is not None and torch.device(device).type == "cuda":
        from .ops import read_interactions_device
        lu, lp, it, _ = read_interactions_device(path, device)
        lu, lp, it = lu.cpu().numpy(), lp.cpu().numpy(), it.cpu().numpy().astype(np.int64)
        return lu.tolist(), [it[lp[j]:lp[j + 1]] for j in range(len(lu))]
    uids: List[int] = []
    rows: List[np.ndarray] = []
    with open(path) as f:
        for line in f.readlines():
            if len(line) > 0:
                parts = line.strip("\n").split(" ")
                uids.append(int(parts[0]))
                rows.append(np.asarray([int(i) for i in parts[1:]], dtype=np.int64))
    return uids, rows


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
        tr_uids, tr_rows = read_interactions(os.path.join(path, "train.txt"), self.device)
        te_uids, te_rows = read_interactions(os.path.join(path, "test.txt"), self.device)
        self.trainUniqueUsers = np.asarray(tr_uids)
        self.trainUser = np.concatenate([np.full(len(r), u) for u, r in zip(tr_uids, tr_rows)]) if tr_rows else np.zeros(0, np.int64)
        self.trainItem = np.concatenate(tr_rows) if tr_rows else np.zeros(0, np.int64)
        self.testUniqueUsers = np.asarray(te_uids)
        self.testUser = np.concatenate([np.full(len(r), u) for u, r in zip(te_uids, te_rows)]) if te_rows else np.zeros(0, np.int64)
        self.testItem = np.concatenate(te_rows) if te_rows else np.zeros(0, np.int64)
        m_item = max([int(r.max()) for r in tr_rows + te_rows if len(r)] + [0])
        n_user = max(tr_uids + te_uids + [0])
        self.m_item = m_item + 1
        self.n_user = n_user + 1
        self.traindataSize = int(len(self.trainItem))
        self.testDataSize = int(len(self.testItem))
        self.Graph = None
        self._csr: Optional[CSRGraph] = None
        # (users, items) bipartite graph; duplicates summed as csr_matrix does (:288-289)
        self.UserItemNet = sp.csr_matrix((np.ones(len(self.trainUser)), (self.trainUser, self.trainItem)),
                                         shape=(self.n_user, self.m_item))
        self.users_D = np.array(self.UserItemNet.sum(axis=1)).squeeze()
        self.users_D[self.users_D == 0.] = 1
        self.items_D = np.array(self.UserItemNet.sum(axis=0)).squeeze()
        self.items_D[self.items_D == 0.] = 1.
        self._allPos = self.getUserPosItems(list(range(self.n_user)))
        self.__testDict = self.__build_test()

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
                self._csr = build_norm_adj(self.trainUser, self.trainItem, self.n_users, self.m_items,
                                           dedup=False, device=self.device)
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

    def __build_test(self) -> Dict[int, List[int]]:
        test_data: Dict[int, List[int]] = {}
        for i, item in enumerate(self.testItem):
            user = int(self.testUser[i])
            test_data.setdefault(user, []).append(int(item))
        return test_data

    def getUserItemFeedback(self, users, items):
        return np.array(self.UserItemNet[users, items]).astype("uint8").reshape((-1,))

    def getUserPosItems(self, users):
        return [self.UserItemNet[user].nonzero()[1] for user in users]
