"""Multi-process (world_size 2, gloo, CPU) tests of the sample-parallel
plumbing: partitioning, conditioning broadcast, ragged all-gather."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from chemeleon_amd.distributed import broadcast_conditioning, gather_states, partition


def test_partition_balances_edge_work():
    nat = [40] * 512
    for w in (1, 2, 4, 8):
        parts = partition(nat, w)
        assert parts[0][0] == 0 and parts[-1][1] == 512
        assert all(p[1] - p[0] == 512 // w for p in parts)
    g = torch.Generator().manual_seed(7)
    rag = torch.randint(1, 81, (2048,), generator=g).tolist()
    parts = partition(rag, 8)
    work = [sum(n * n for n in rag[a:b]) for a, b in parts]
    assert max(work) / min(work) < 1.02
    assert [p[1] for p in parts[:-1]] == [p[0] for p in parts[1:]]
    assert partition([5, 5, 5], 3) == [(0, 1), (1, 2), (2, 3)]
    with pytest.raises(ValueError, match="cannot be sharded"):
        partition([5, 5], 3)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        nat_global = [3, 5, 2, 7, 4]
        parts = partition(nat_global, world)
        g0, g1 = parts[rank]
        local = nat_global[g0:g1]
        n0 = sum(nat_global[:g0])
        N = sum(local)
        a = torch.arange(n0, n0 + N)
        x = torch.arange(n0, n0 + N, dtype=torch.float32)[:, None].repeat(1, 3)
        lat = torch.arange(g0, g1, dtype=torch.float32)[:, None, None].repeat(1, 3, 3)
        A, X, LT, nat = gather_states((a, x, lat), local)
        # with every rank's crystal list known up front: no size exchange, same result
        A2, X2, LT2, nat2 = gather_states((a, x, lat), local, natoms_all=[nat_global[r0:r1] for r0, r1 in parts])
        assert torch.equal(A, A2) and torch.equal(X, X2) and torch.equal(LT, LT2) and nat == nat2
        # fewer crystals than ranks: every rank raises before any collective (no rank hangs)
        from chemeleon_amd.distributed import sample_distributed
        try:
            sample_distributed(None, [4], cond=None, null=None)
            raised = False
        except ValueError:
            raised = True
        assert raised
        cond = torch.full((1, 4), float(rank == 0)) * 3.0
        null = torch.full((1, 4), float(rank == 0)) * 5.0
        c, n = broadcast_conditioning(cond, null)
        q.put((rank, A.tolist(), X[:, 0].tolist(), LT[:, 0, 0].tolist(), nat, c.tolist(), n.tolist()))
    finally:
        dist.destroy_process_group()


def test_two_rank_gather_and_broadcast():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, A, X, LT, nat, c, n in res:
        assert nat == [3, 5, 2, 7, 4]
        assert A == list(range(21)) and X == [float(i) for i in range(21)]
        assert LT == [0.0, 1.0, 2.0, 3.0, 4.0]
        assert c == [[3.0] * 4] and n == [[5.0] * 4]
