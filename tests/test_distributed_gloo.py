"""CPU: the N>1 propagation schedule (user shards; items by a chunked push whose partials are
exchanged per chunk and summed in rank order, users by pull from the all-gathered item table)
over a gloo process group, world sizes 2, 3, 4 and 8, against the
float64 oracle.  The SpMM and epilogue callables are the oracle (injected); the orchestration,
operators, padding and collectives are the product code of distributed.py."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from factors_of_serendipity_recommendation_amd import _lib
from factors_of_serendipity_recommendation_amd.distributed import ShardedPropagation, make_shard
from factors_of_serendipity_recommendation_amd.graph import CSRGraph
from oracle import oracle


def cpu_layer(A, X, mode, Y=None, E0=None, acc=None, out=None, n_mean=1.0):
    y = torch.from_numpy(oracle.spmm(A.indptr.numpy(), A.indices.numpy(), A.vals.numpy(),
                                     X.float().numpy())).float()
    if mode == _lib.LGX_LAYER_PARTIAL:
        out.copy_(y)
        return
    cpu_epilogue(y, mode, Y=Y, E0=E0, acc=acc, out=out, n_mean=n_mean)


def cpu_epilogue(y, mode, Y=None, E0=None, acc=None, out=None, n_mean=1.0):
    if mode in (_lib.LGX_LAYER_PLAIN, _lib.LGX_LAYER_FIRST, _lib.LGX_LAYER_MID):
        Y.copy_(y)
    if mode == _lib.LGX_LAYER_FIRST:
        acc.copy_(E0.float() + y)
    elif mode == _lib.LGX_LAYER_MID:
        acc.add_(y)
    elif mode == _lib.LGX_LAYER_LAST:
        out.copy_((acc + y) / n_mean)
    elif mode == _lib.LGX_LAYER_ONLY:
        out.copy_((E0.float() + y) / n_mean)


def cpu_stack(A, X, E0, prev, out, n_mean):
    y = torch.from_numpy(oracle.spmm(A.indptr.numpy(), A.indices.numpy(), A.vals.numpy(),
                                     X.float().numpy())).float()
    acc = E0.float().clone()
    for t in prev:
        acc += t.float()
    out.copy_((acc + y) / n_mean)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, K, result_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(42)
        U, I, E = 120, 90, 2500
        u = rng.integers(0, U, E).astype(np.int32)
        i = (rng.zipf(1.4, E) % I).astype(np.int32)
        ip, ix, iv = oracle.build_norm_adj(u, i, U, I, dedup=True)
        A = CSRGraph(torch.from_numpy(ip), torch.from_numpy(ix), torch.from_numpy(iv), U + I, U + I, U, I)
        E0 = torch.from_numpy((rng.standard_normal((U + I, 8)) * 0.1).astype(np.float32))
        shard = make_shard(A, U, I, rank, world, seg_len=16)
        prop = ShardedPropagation(shard, E0[:U], E0[U:], K, layer_fn=cpu_layer, epilogue_fn=cpu_epilogue,
                                  stack_fn=cpu_stack)
        prop.step()
        prop.step()  # a second step must give the same answer (buffers re-used)
        ou, oi = prop.gather_outputs()
        if rank == 0:
            ref = oracle.propagate(ip, ix, iv, E0.numpy(), K)
            result_q.put((np.abs(ou.numpy() - ref[:U]).max(), np.abs(oi.numpy() - ref[U:]).max(),
                          prop.schedule()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,K", [(2, 3), (2, 4), (3, 1), (2, 2), (4, 3), (8, 2)])
def test_sharded_propagation_gloo(world, K):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, K, q)) for r in range(world)]
    for p in procs:
        p.start()
    eu, ei, sched = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert eu < 1e-5 and ei < 1e-5, (eu, ei)
    assert len(sched) == 3 * K


def _chunk_worker(rank, world, port, K, result_q):
    """One graph, the same shard, propagated with 1 / 3 / 4 / 7 push chunks and from the rank's own
    user rows only: gathered outputs equal bit for bit (each row keeps its summation; the cross-rank sum runs in rank order); phases
    recorded for every step."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(7)
        U, I, E = 150, 97, 3000
        u = rng.integers(0, U, E).astype(np.int32)
        i = (rng.zipf(1.3, E) % I).astype(np.int32)
        ip, ix, iv = oracle.build_norm_adj(u, i, U, I, dedup=True)
        A = CSRGraph(torch.from_numpy(ip), torch.from_numpy(ix), torch.from_numpy(iv), U + I, U + I, U, I)
        E0 = torch.from_numpy((rng.standard_normal((U + I, 8)) * 0.1).astype(np.float32))
        shard = make_shard(A, U, I, rank, world, seg_len=16)
        outs, phases = [], None
        u0, u1 = int(shard.user_bounds[rank]), int(shard.user_bounds[rank + 1])
        for nc, local in ((1, False), (3, False), (4, False), (7, False), (4, True)):
            # the last pass hands the rank only its own user rows (the bench's layout)
            prop = ShardedPropagation(shard, E0[u0:u1] if local else E0[:U], E0[U:], K, layer_fn=cpu_layer,
                                      epilogue_fn=cpu_epilogue, stack_fn=cpu_stack, n_chunks=nc,
                                      local_user_rows=local)
            assert len(prop.push_chunks) == min(nc, shard.mi)
            prop.record_phases = nc == 4 and not local
            prop.step()
            prop.step()
            if prop.record_phases:
                phases = prop.phase_summary()
            ou, oi = prop.gather_outputs()
            outs.append(torch.cat([ou, oi]).numpy())
        if rank == 0:
            ref = oracle.propagate(ip, ix, iv, E0.numpy(), K)
            result_q.put(([bool(np.array_equal(outs[0], o)) for o in outs[1:]],
                          float(np.abs(outs[0] - ref).max()), phases))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_chunked_exchange_equals_unchunked_bit_for_bit(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_chunk_worker, args=(r, world, port, 3, q)) for r in range(world)]
    for p in procs:
        p.start()
    same, err, phases = q.get(timeout=180)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert all(same), same
    assert err < 1e-5
    for name in ("push", "allgather_wait", "pull", "exchange_wait", "reduce", "epilogue", "comm_exposed_ms"):
        assert name in phases and phases[name] >= 0.0, phases


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_from_edges_equals_cut_of_full_operator(world):
    """make_shard_from_edges (each rank builds only its rows from the sorted edge list) == make_shard
    on the full oracle-built operator, bit for bit: bounds, indptr, column ids, values, transposes."""
    from factors_of_serendipity_recommendation_amd.distributed import make_shard_from_edges
    rng = np.random.default_rng(3)
    U, I, E = 300, 200, 6000
    keys = np.unique(rng.integers(0, U, E) * I + (rng.zipf(1.3, E) % I))
    u, i = (keys // I).astype(np.int32), (keys % I).astype(np.int32)
    ip, ix, iv = oracle.build_norm_adj(u, i, U, I, dedup=True)
    A = CSRGraph(torch.from_numpy(ip), torch.from_numpy(ix), torch.from_numpy(iv), U + I, U + I, U, I)
    for rank in range(world):
        a = make_shard(A, U, I, rank, world, seg_len=16)
        b = make_shard_from_edges(torch.from_numpy(u), torch.from_numpy(i), U, I, rank, world, seg_len=16)
        assert np.array_equal(a.user_bounds, b.user_bounds) and a.mi == b.mi
        for x, y in ((a.A_pull, b.A_pull), (a.A_push, b.A_push)):
            assert torch.equal(x.indptr, y.indptr) and torch.equal(x.indices, y.indices)
            assert torch.equal(x.vals, y.vals)


def test_shard_from_edges_rejects_duplicate_or_unsorted_edges():
    from factors_of_serendipity_recommendation_amd.distributed import make_shard_from_edges
    u = torch.tensor([0, 0, 1, 2], dtype=torch.int32)
    for items in ([1, 1, 0, 3], [2, 1, 0, 3]):  # a repeated edge; items out of order within user 0
        with pytest.raises(ValueError):
            make_shard_from_edges(u, torch.tensor(items, dtype=torch.int32), 3, 4, 0, 1, seg_len=16)
    make_shard_from_edges(u, torch.tensor([1, 2, 0, 3], dtype=torch.int32), 3, 4, 0, 1, seg_len=16)
