"""MI355X-native LightGCN propagation + full-catalog scoring engine.

Drop-in for the hot path of csjwj2023/factors-of-serendipity-recommendation:
``model.LightGCN.computer()`` (K-layer normalized-adjacency SpMM + layer mean), the adjacency build
of ``Loader.getSparseGraph`` / ``Data.get_adj_mat``, full-catalog scoring + positive mask + top-k
(``Procedure.Test``, ``batch_test.test``, ``eval_score_matrix_foldout``) and the recommend.py
similarity calls.  Compute runs in hand-written gfx950 HIP kernels (liblgx.so, C ABI in
include/lgx.h); there is no CPU fallback.
"""
from . import _lib
from ._lib import build, version
from .graph import CSRGraph, build_norm_adj, from_csr_arrays, from_sparse_coo, make_plan
from .ops import (fill_normal, foldout_metrics, gather_scores, propagate, propagate_layer, score_dense,
                  score_topk, spmm, topk_rows)

__all__ = [
    "build", "version", "CSRGraph", "build_norm_adj", "from_csr_arrays", "from_sparse_coo", "make_plan",
    "propagate", "propagate_layer", "spmm", "score_dense", "score_topk", "topk_rows", "foldout_metrics",
    "gather_scores", "fill_normal",
]
