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
    from chemeleon_amd.distributed import NODE_COST
    work = [sum(n * n + NODE_COST * n for n in rag[a:b]) for a, b in parts]
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


class _StubModel:
    """Stands in for Chemeleon on the CPU: sample_states yields, for every t, states that encode the global
    node / crystal indices and t, so the gathered batch shows whether every rank's slice landed in place.
    It records the arguments the distributed sampler passed (global sizes, bases, the conditioning)."""

    text_guide = True
    hparams = {"text_dim": 4}
    device = torch.device("cpu")
    mask_lattice_matrix = torch.ones(3, 3, dtype=torch.bool)

    def __init__(self):
        self.calls = []

    def _conditioning(self, texts, B, cond, null):
        return cond.expand(B, -1).contiguous(), null.expand(B, -1).contiguous()

    def sample_states(self, natoms, texts, cond_scale, step_lr, *, noise, seed, text_embeds, null_text_embeds, clone,
                      node_base, graph_base, init, global_sizes, graph, t_stop=0, lanes=1):
        self.calls.append(dict(natoms=list(natoms), node_base=node_base, graph_base=graph_base,
                               global_sizes=global_sizes, cond=text_embeds.clone(), noise=noise, lanes=lanes))
        N, B = sum(natoms), len(natoms)
        for t in range(3, t_stop - 1, -1):
            a = torch.arange(node_base, node_base + N) * 10 + t
            x = torch.arange(node_base, node_base + N, dtype=torch.float32)[:, None].repeat(1, 3) + t
            lat = torch.arange(graph_base, graph_base + B, dtype=torch.float32)[:, None, None].repeat(1, 3, 3) + t
            yield t, a, x, lat


def _sampler_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from chemeleon_amd.distributed import sample_states_distributed
        nat = [3, 5, 2, 7, 4, 6]
        m = _StubModel()
        cond = torch.full((1, 4), 3.0) if rank == 0 else torch.zeros(1, 4)  # only rank 0 holds the encoder output
        null = torch.full((1, 4), 5.0) if rank == 0 else torch.zeros(1, 4)
        every = [(t, a.tolist(), x[:, 0].tolist(), lat[:, 0, 0].tolist())
                 for t, a, x, lat in sample_states_distributed(m, nat, None, noise="torch", text_embeds=cond,
                                                               null_text_embeds=null, every_step=True)]
        final = [t for t, *_ in sample_states_distributed(m, nat, None, noise="torch", text_embeds=cond,
                                                            null_text_embeds=null)]
        q.put((rank, every, final, m.calls[0]["global_sizes"], m.calls[0]["node_base"], m.calls[0]["graph_base"],
               m.calls[0]["cond"][:, 0].tolist()))
    finally:
        dist.destroy_process_group()


def test_distributed_sampler_gathers_the_whole_batch_on_every_rank():
    """sample_states_distributed (the path Chemeleon.sample() takes under a process group): every rank gets
    the whole batch in global order at every step (every_step=True) or only the final one; each rank samples
    its Σn²-balanced slice with the GLOBAL sizes and its node / crystal bases (the parity-mode noise slicing),
    and the conditioning held by rank 0 reaches every rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sampler_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    nat = [3, 5, 2, 7, 4, 6]
    parts = partition(nat, 2)
    for rank, every, final, gsz, nb, gb, cond in res:
        assert [t for t, *_ in every] == [3, 2, 1, 0] and final == [0]
        for t, a, x, lat in every:
            assert a == [i * 10 + t for i in range(sum(nat))]
            assert x == [float(i + t) for i in range(sum(nat))]
            assert lat == [float(g + t) for g in range(len(nat))]
        g0 = parts[rank][0]
        assert gsz == (sum(nat), len(nat)) and gb == g0 and nb == sum(nat[:g0])
        assert cond == [3.0] * (parts[rank][1] - g0)


def _error_worker(rank, world, port, q):
    """Rank 0 alone holds (mis-shaped) conditioning; an unsupported keyword; t_stop / lanes forwarded."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from chemeleon_amd.distributed import sample_states_distributed
        nat = [3, 5, 2, 7]
        m = _StubModel()
        out = {}
        bad = torch.full((3, 4), 1.0) if rank == 0 else None  # 3 rows for 4 crystals: only rank 0 can tell
        try:
            list(sample_states_distributed(m, nat, None, noise="torch", text_embeds=bad, null_text_embeds=bad))
            out["shape"] = "no error"
        except ValueError as e:
            out["shape"] = "ValueError" if "text_embeds has shape" in str(e) else repr(e)
        except RuntimeError as e:
            out["shape"] = "RuntimeError" if "rank 0 failed" in str(e) else repr(e)
        try:
            list(sample_states_distributed(m, nat, None, noise="torch", text_embeds=torch.ones(1, 4),
                                           null_text_embeds=torch.ones(1, 4), node_base=5))
            out["kw"] = "no error"
        except ValueError as e:
            out["kw"] = "ValueError" if "node_base" in str(e) else repr(e)
        ts = [t for t, *_ in sample_states_distributed(m, nat, None, noise="torch", text_embeds=torch.ones(1, 4),
                                                         null_text_embeds=torch.ones(1, 4), t_stop=2, lanes=2)]
        out["t_stop"] = ts
        out["lanes"] = m.calls[-1]["lanes"]
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_distributed_sampler_errors_reach_every_rank():
    """a conditioning error found on rank 0 (the only rank holding the vectors) raises on EVERY
    rank instead of leaving the others blocked in the broadcast; sample_states keywords the shards compute
    themselves are refused on every rank before any collective; t_stop and lanes are forwarded."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_error_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert res[0]["shape"] == "ValueError" and res[1]["shape"] == "RuntimeError"
    for r in (0, 1):
        assert res[r]["kw"] == "ValueError"
        assert res[r]["t_stop"] == [2]
        assert res[r]["lanes"] == 2
