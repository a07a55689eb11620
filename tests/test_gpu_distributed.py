"""GPU: the multi-GPU propagation schedule with the REAL HIP layer kernels.  The box has one GPU,
so the two ranks share cuda:0 and exchange over gloo (RCCL refuses two ranks on one device); a
world-1 RCCL group with the collectives forced on runs the chunked push's async all-to-alls
(summed in rank order by lgx_sum_slabs) and the item all-gather on the device; the 8-GPU RCCL run is the bench's job.  Checked against the
float64 oracle (fp32 tolerance)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, K, dtype_name, q, backend="gloo"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if backend == "nccl":
        torch.cuda.set_device(0)
        dist.init_process_group(backend, rank=rank, world_size=world, device_id=torch.device("cuda:0"))
    else:
        dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        from oracle import oracle
        import factors_of_serendipity_recommendation_amd as lgx
        from factors_of_serendipity_recommendation_amd.distributed import ShardedPropagation, make_shard
        dtype = torch.float32 if dtype_name == "f32" else torch.bfloat16
        rng = np.random.default_rng(5)
        U, I, E = 3000, 2000, 60000
        u = rng.integers(0, U, E).astype(np.int32)
        i = (rng.zipf(1.3, E) % I).astype(np.int32)
        A = lgx.build_norm_adj(u, i, U, I, dedup=True, device="cuda:0")
        E0 = (torch.from_numpy(rng.standard_normal((U + I, 64)).astype(np.float32)) * 0.1)
        if dtype == torch.bfloat16:
            E0 = E0.to(torch.bfloat16).float()
        shard = make_shard(A, U, I, rank, world, seg_len=64)
        outs = []
        u0, u1 = int(shard.user_bounds[rank]), int(shard.user_bounds[rank + 1])
        # one push launch, then 4 chunks each with its own exchange, then 4 chunks from this rank's
        # user rows only (the bench's layout: no replicated user table)
        for nc, local in ((1, False), (4, False), (4, True)):
            Eu = E0[u0:u1] if local else E0[:U]
            prop = ShardedPropagation(shard, Eu.cuda().to(dtype), E0[U:].cuda().to(dtype), K,
                                      force_collectives=backend == "nccl", n_chunks=nc, local_user_rows=local)
            if backend == "nccl":
                assert prop._collective and prop._a2a_native  # async all_to_all_single / all_gather_into_tensor
            prop.record_phases = True
            prop.step()
            prop.step()
            ph = prop.phase_summary()
            assert ph["push"] > 0 and ph["pull"] > 0 and ph["comm_exposed_ms"] >= 0, ph
            if not prop._a2a_native and prop._collective:  # gloo: host-synchronous exchanges, stamped apart
                assert ph["exchange_sync"] >= 0 and ph["comm_exposed_ms"] >= ph["exchange_sync"], ph
            ou, oi = prop.gather_outputs()
            outs.append((ou.clone(), oi.clone()))
        torch.cuda.synchronize()
        assert all(torch.equal(a, b) for a, b in zip(outs[0], outs[1])), "chunked layer differs from one launch"
        assert all(torch.equal(a, b) for a, b in zip(outs[1], outs[2])), "local user rows differ from the full table"
        if rank == 0:
            ref = oracle.propagate(A.indptr.cpu().numpy(), A.indices.cpu().numpy(), A.vals.cpu().numpy(),
                                   E0.numpy(), K)
            got = np.concatenate([ou.cpu().numpy(), oi.cpu().numpy()])
            err = np.abs(got - ref)
            rel = 1e-5 if dtype == torch.float32 else 2e-2
            tol = rel * np.abs(ref) + rel * np.sqrt(np.mean(ref ** 2))
            q.put((bool((err <= tol).all()), float(err.max())))
    except Exception as e:  # surface the failure to the parent
        if rank == 0:
            q.put((False, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,K,dt", [(2, 3, "f32"), (2, 4, "bf16"), (3, 2, "f32")])
def test_sharded_propagation_real_kernels(world, K, dt):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, K, dt, q)) for r in range(world)]
    for p in procs:
        p.start()
    ok, info = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
    assert ok, info
    assert all(p.exitcode == 0 for p in procs)


@pytest.mark.parametrize("K,dt", [(3, "f32"), (3, "bf16")])
def test_sharded_propagation_world1_rccl_forced_collectives(K, dt):
    """One rank, backend "nccl" (RCCL): the push chunks' all-to-alls and the item all-gather are
    issued as async RCCL collectives (the world>1 code path), not the world-1 copies."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(0, 1, _free_port(), K, dt, q, "nccl"))
    p.start()
    ok, info = q.get(timeout=300)
    p.join(timeout=120)
    assert ok, info
    assert p.exitcode == 0


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_fill_normal_rows_equal_rows_of_the_full_table(dt):
    """lgx_fill_normal_at (bench.py N>1: each rank fills only its own rows of E0): rows [r0, r1) of a
    table filled from offset r0 * d equal the same rows of the whole table, bit for bit, for odd
    offsets (the Box-Muller pairs straddle the cut) as well."""
    import factors_of_serendipity_recommendation_amd as lgx
    N, d = 10_001, 24
    full = lgx.fill_normal((N, d), 0.1, 2020, dtype=dt)
    for r0, r1 in ((0, 1), (1, 2), (3_333, 7_777), (N - 5, N)):
        part = lgx.fill_normal((r1 - r0, d), 0.1, 2020, dtype=dt, first=r0 * d)
        assert torch.equal(part, full[r0:r1]), (r0, r1)
    flat = lgx.fill_normal((7,), 0.1, 2020, dtype=dt, first=5)  # an odd element offset
    assert torch.equal(flat, full.view(-1)[5:12])
