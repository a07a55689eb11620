"""Drop-in ``LightGCN`` nn.Module whose propagation runs on the MI355X HIP engine.

Mirrors ``model.LightGCN`` (lightGCN/LightGCN-PyTorch-master/code/model.py:87-220): same
constructor ``(config, dataset)``, same config keys (latent_dim_rec, lightGCN_n_layers, keep_prob,
A_split, pretrain, dropout, user_emb/item_emb), same parameters ``embedding_user`` /
``embedding_item`` (so checkpoints load with ``strict=True``, code/main.py:29,34,93), same methods
``computer / getUsersRating / getEmbedding / bpr_loss / forward``.  ``self.Graph`` stays the
reference's torch sparse COO object (a plain attribute, not a buffer); the HIP engine works on the
CSR built from it (or handed over by our ``Loader.getCSRGraph``).

Differences, all documented in DESIGN.md:
  * computer() = one fused HIP propagation (lgx_propagate) instead of K torch.sparse.mm + stack +
    mean; its backward reuses the same propagation (A^ is symmetric, so (1/(K+1)) sum_k A^k is
    self-adjoint);
  * in eval mode the propagated tables are cached while the weights are unchanged (the reference
    recomputes the full K-layer propagation for every 100-user test batch, model.py:180);
  * getUsersRating returns sigmoid scores from the HIP MFMA kernel (not differentiable: the
    reference only calls it under torch.no_grad(), Procedure.py:109,127).
  * bpr_loss runs as two fused HIP kernels (lgx_bpr_loss_forward/backward) on f32 tables;
    bpr_loss_torch keeps the reference's torch-op form as the parity reference.
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import nn

from . import ops
from .graph import CSRGraph, from_csr_arrays, from_sparse_coo


class _Propagate(torch.autograd.Function):
    """out = mean_k A^k E0 ; dE0 = mean_k (A^T)^k dout  (A^T = A for the normalized adjacency)."""

    @staticmethod
    def forward(ctx, E0: torch.Tensor, A: CSRGraph, K: int, A_T: Optional[CSRGraph]):
        ctx.A_T = A_T if A_T is not None else A
        ctx.K = K
        return ops.propagate(A, E0, K)

    @staticmethod
    def backward(ctx, g: torch.Tensor):
        gE0 = ops.propagate(ctx.A_T, g.contiguous().to(torch.float32), ctx.K)
        return gE0, None, None, None


def propagate_autograd(E0: torch.Tensor, A: CSRGraph, K: int, A_T: Optional[CSRGraph] = None) -> torch.Tensor:
    return _Propagate.apply(E0, A, K, A_T)


class _BPRLoss(torch.autograd.Function):
    """bpr_loss (model.py:196-209) as two fused HIP kernels (csrc/bpr.hip): forward reads each
    triple's 3 propagated and 3 ego rows once; backward adds the row gradients into dense [N, d]
    tables -- the propagated one then flows into _Propagate.backward."""

    @staticmethod
    def forward(ctx, light, ego_user, ego_item, users, pos, neg):
        loss, reg, coef = ops.bpr_loss_forward(light, ego_user, ego_item, users, pos, neg)
        ctx.save_for_backward(light, ego_user, ego_item, users, pos, neg, coef)
        return loss, reg

    @staticmethod
    def backward(ctx, g_loss, g_reg):
        light, ego_user, ego_item, users, pos, neg, coef = ctx.saved_tensors
        z = torch.zeros((), dtype=torch.float32, device=light.device)
        g_light, g_user, g_item = ops.bpr_loss_backward(light, ego_user, ego_item, users, pos, neg, coef,
                                                        z if g_loss is None else g_loss,
                                                        z if g_reg is None else g_reg)
        return g_light, g_user, g_item, None, None, None


def _graph_to_csr(G, dataset, n_users: int, n_items: int) -> CSRGraph:
    if hasattr(dataset, "getCSRGraph"):
        return dataset.getCSRGraph()
    if isinstance(G, (list, tuple)):  # A_split folds (dataloader.py:319-329): stack the row blocks
        G = torch.cat([g.coalesce() for g in G], dim=0)
    if torch.is_tensor(G) and G.is_sparse:
        if not G.is_cuda:
            G = G.cuda()
        return from_sparse_coo(G, n_users, n_items)
    if hasattr(G, "tocsr"):  # a scipy matrix
        c = G.tocsr()
        c.sort_indices()
        return from_csr_arrays(c.indptr, c.indices, c.data, n_cols=c.shape[1], n_users=n_users, n_items=n_items)
    raise TypeError(f"unsupported graph object {type(G)}")


class BasicModel(nn.Module):
    def getUsersRating(self, users):
        raise NotImplementedError


class LightGCN(BasicModel):
    def __init__(self, config: dict, dataset):
        super().__init__()
        self.config = config
        self.dataset = dataset
        self.__init_weight()

    def __init_weight(self):
        self.num_users = self.dataset.n_users
        self.num_items = self.dataset.m_items
        self.latent_dim = self.config["latent_dim_rec"]
        self.n_layers = self.config["lightGCN_n_layers"]
        self.keep_prob = self.config.get("keep_prob", 0.6)
        self.A_split = self.config.get("A_split", False)
        self.embedding_user = nn.Embedding(num_embeddings=self.num_users, embedding_dim=self.latent_dim)
        self.embedding_item = nn.Embedding(num_embeddings=self.num_items, embedding_dim=self.latent_dim)
        if self.config.get("pretrain", 0) == 0:
            nn.init.normal_(self.embedding_user.weight, std=0.1)  # model.py:112-113
            nn.init.normal_(self.embedding_item.weight, std=0.1)
        else:
            self.embedding_user.weight.data.copy_(torch.as_tensor(self.config["user_emb"]))
            self.embedding_item.weight.data.copy_(torch.as_tensor(self.config["item_emb"]))
        self.f = nn.Sigmoid()
        self.Graph = self.dataset.getSparseGraph()
        self._csr: CSRGraph = _graph_to_csr(self.Graph, self.dataset, self.num_users, self.num_items)
        self._eval_cache = None

    # ------------------------------------------------------------------ edge dropout (model.py:125-143)
    def __dropout_x(self, keep_prob: float):
        """Same RNG draw as the reference: torch.rand(nnz) on the host generator, kept where
        rand + keep_prob >= 1 (model.py:129-130), kept values / keep_prob (:132)."""
        A = self._csr
        keep = (torch.rand(A.nnz) + keep_prob).int().bool().to(A.device)
        rows = torch.repeat_interleave(torch.arange(A.n_rows, device=A.device), torch.diff(A.indptr))[keep]
        cols = A.indices.long()[keep]
        vals = A.vals[keep] / keep_prob
        N = A.n_rows
        G = torch.sparse_coo_tensor(torch.stack([rows, cols]), vals, (N, N)).coalesce()
        GT = torch.sparse_coo_tensor(torch.stack([cols, rows]), vals, (N, N)).coalesce()
        return from_sparse_coo(G, A.n_users, A.n_items), from_sparse_coo(GT, A.n_users, A.n_items)

    def _light_out(self) -> torch.Tensor:
        """The propagated [U+I, d] table (model.py:145-177) on the HIP engine."""
        users_emb = self.embedding_user.weight
        items_emb = self.embedding_item.weight
        use_cache = (not self.training) and not torch.is_grad_enabled()
        key = (users_emb._version, items_emb._version, users_emb.data_ptr(), items_emb.data_ptr())
        if use_cache and self._eval_cache is not None and self._eval_cache[0] == key:
            return self._eval_cache[1]
        all_emb = torch.cat([users_emb, items_emb])
        if self.config.get("dropout", 0) and self.training:
            A, A_T = self.__dropout_x(self.keep_prob)
        else:
            A, A_T = self._csr, None
        light_out = propagate_autograd(all_emb, A, self.n_layers, A_T)
        if use_cache:
            self._eval_cache = (key, light_out)
        return light_out

    def computer(self):
        """propagate methods for lightGCN (model.py:145-177): (users, items) views of one table."""
        return torch.split(self._light_out(), [self.num_users, self.num_items])

    def getUsersRating(self, users):
        all_users, all_items = self.computer()
        return ops.score_dense(all_users.detach(), all_items.detach(), user_rows=users.long(), apply_sigmoid=True)

    def getEmbedding(self, users, pos_items, neg_items):
        all_users, all_items = self.computer()
        users_emb = all_users[users]
        pos_emb = all_items[pos_items]
        neg_emb = all_items[neg_items]
        users_emb_ego = self.embedding_user(users)
        pos_emb_ego = self.embedding_item(pos_items)
        neg_emb_ego = self.embedding_item(neg_items)
        return users_emb, pos_emb, neg_emb, users_emb_ego, pos_emb_ego, neg_emb_ego

    def bpr_loss(self, users, pos, neg):
        """model.py:196-209.  f32 tables go through the fused kernels (_BPRLoss); other dtypes
        through the reference's torch ops (bpr_loss_torch)."""
        w_u, w_i = self.embedding_user.weight, self.embedding_item.weight
        if not getattr(self, "_lgx_trusted_indices", False):
            # the reference's torch indexing raises on a bad id; the fused kernel would turn the
            # loss into NaN instead, so check the ranges here (one host sync).  BPR_train_original
            # skips this for its own sampler's draws, which are in range by construction.
            lim = torch.tensor([self.num_users, self.num_items, self.num_items], device=w_u.device)
            idx = [t.reshape(-1).long() for t in (users, pos, neg)]
            if idx[0].numel():
                lo = torch.stack([t.min() for t in idx])
                hi = torch.stack([t.max() for t in idx])
                if bool(((lo < 0) | (hi >= lim)).any()):
                    raise IndexError("bpr_loss: user / item index out of range")
        light = self._light_out()
        if light.dtype == w_u.dtype == w_i.dtype == torch.float32 and light.is_contiguous():
            return _BPRLoss.apply(light, w_u, w_i, users, pos, neg)
        return self.bpr_loss_torch(users, pos, neg)

    def bpr_loss_torch(self, users, pos, neg):
        """The reference's bpr_loss in torch ops (model.py:196-209), kept as the parity reference."""
        (users_emb, pos_emb, neg_emb, userEmb0, posEmb0, negEmb0) = self.getEmbedding(users.long(), pos.long(),
                                                                                      neg.long())
        reg_loss = (1 / 2) * (userEmb0.norm(2).pow(2) + posEmb0.norm(2).pow(2) +
                              negEmb0.norm(2).pow(2)) / float(len(users))
        pos_scores = torch.sum(torch.mul(users_emb, pos_emb), dim=1)
        neg_scores = torch.sum(torch.mul(users_emb, neg_emb), dim=1)
        loss = torch.mean(torch.nn.functional.softplus(neg_scores - pos_scores))
        return loss, reg_loss

    def forward(self, users, items):
        all_users, all_items = self.computer()
        users_emb = all_users[users]
        items_emb = all_items[items]
        return torch.sum(torch.mul(users_emb, items_emb), dim=1)


MODELS = {"lgn": LightGCN}  # register.MODELS (register.py:25-28); PureMF is out of scope
