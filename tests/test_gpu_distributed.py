"""Sample-parallel sampling end to end on the GPU: two ranks (sharing the one GPU of the test box,
gloo process group) run `chemeleon_amd.distributed` — Σn²-balanced partition, conditioning
broadcast from rank 0, noise independent of the rank count, ragged all-gather — and must return
exactly the single-process result:
* perf mode (device Philox noise keyed by global node / graph index), a short ragged run;
* parity mode (noise="torch", the reference's CPU RNG stream, every rank drawing the global tensors
  and keeping its rows) over configs[1] (64 x 20, T = 1000) against the reference's own trajectory
  (tests/golden/trajectory_64x20_T1000.npz): bit-identical to the single-process run and inside the
  same reference gate (tests/test_gpu_parity.py gate_64x20);
* Chemeleon.sample() under an initialised process group (the drop-in call reaching N ranks)."""

import os
import socket

import pytest
import torch

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a HIP device")]

NAT = [5, 9, 3, 12, 7, 4, 11]
T = 20


def _model(timesteps=T):
    from chemeleon_amd import Chemeleon
    from chemeleon_amd.config import default_config
    from chemeleon_amd.synthetic import synthetic_state_dict
    cfg = default_config()
    cfg["timesteps"] = timesteps
    torch.manual_seed(0)
    m = Chemeleon(cfg)
    m.decoder.load_state_dict(synthetic_state_dict(default_config()))
    return m.to("cuda:0").eval()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from chemeleon_amd.distributed import sample_distributed
    from chemeleon_amd.synthetic import synthetic_text_embeds
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        m = _model()
        cond, null = synthetic_text_embeds(512)
        if rank != 0:  # only rank 0 holds the text-encoder output; the broadcast must deliver it
            cond, null = torch.zeros_like(cond), torch.zeros_like(null)
        a, x, lat, nat = sample_distributed(m, NAT, cond.cuda(), null.cuda(), seed=3, noise="philox")
        q.put((rank, a.cpu().numpy(), x.cpu().numpy(), lat.cpu().numpy(), nat))  # (numpy: see _parity_worker)
    finally:
        dist.destroy_process_group()


def test_two_ranks_match_single_process():
    import torch.multiprocessing as mp
    from chemeleon_amd.distributed import sample_distributed
    from chemeleon_amd.synthetic import synthetic_text_embeds
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=150) for _ in range(2)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    cond, null = synthetic_text_embeds(512)
    a1, x1, l1, nat1 = sample_distributed(_model(), NAT, cond.cuda(), null.cuda(), seed=3, noise="philox")
    assert nat1 == NAT
    for rank, a, x, lat, nat in res:
        assert nat == NAT, rank
        assert torch.equal(torch.from_numpy(a), a1.cpu()), f"rank {rank}: atom types differ"
        assert torch.equal(torch.from_numpy(x), x1.cpu()), f"rank {rank}: coordinates differ"
        assert torch.equal(torch.from_numpy(lat), l1.cpu()), f"rank {rank}: lattices differ"


def _parity_worker(rank, world, port, q, want):
    import numpy as np
    import torch.distributed as dist
    from chemeleon_amd.distributed import sample_states_distributed
    from chemeleon_amd.synthetic import synthetic_text_embeds
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        m = _model(1000)
        cond, null = synthetic_text_embeds(512)
        if rank != 0:
            cond, null = torch.zeros_like(cond), torch.zeros_like(null)
        torch.manual_seed(42)  # every rank seeds its CPU generator as the single-process caller does
        got = {}
        for t, a, x, lat in sample_states_distributed(m, [20] * 64, None, 2.0, 1e-5, noise="torch",
                                                      text_embeds=cond.cuda(), null_text_embeds=null.cuda(),
                                                      every_step=want):
            if t in want:
                got[t] = [v.cpu().numpy().copy() for v in (a, x, lat)]
        # (numpy through the queue: a torch tensor travels as a shared fd that dies with this process)
        gen_state = torch.get_rng_state().numpy().copy()
        # the drop-in call: sample() notices the process group and shards by itself
        torch.manual_seed(7)
        atoms = m.sample(None, 5, 6, text_embeds=cond.cuda(), null_text_embeds=null.cuda())
        summary = [(at.get_atomic_numbers().tolist(), at.get_scaled_positions().tolist(), np.asarray(at.cell).tolist())
                   for at in atoms]
        q.put((rank, got, gen_state, summary))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_two_ranks_parity_mode_64x20_trajectory(golden):
    import numpy as np
    import torch.multiprocessing as mp
    from chemeleon_amd.synthetic import synthetic_text_embeds
    from tests.test_gpu_parity import gate_64x20
    g = golden("trajectory_64x20_T1000.npz")
    want = set(int(t) for t in g["t"])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_parity_worker, args=(r, 2, port, q, want)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=500) for _ in range(2)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    # the single-process run of the same call
    m = _model(1000)
    cond, null = synthetic_text_embeds(512)
    torch.manual_seed(42)
    one = {}
    for t, a, x, lat in m.sample_states([20] * 64, None, 2.0, 1e-5, noise="torch", text_embeds=cond.cuda(),
                                        null_text_embeds=null.cuda(), clone=False):
        if t in want:
            one[t] = [v.cpu().numpy().copy() for v in (a, x, lat)]
    gen_one = torch.get_rng_state()
    torch.manual_seed(7)
    atoms = m.sample(None, 5, 6, text_embeds=cond.cuda(), null_text_embeds=null.cuda())
    summary_one = [(at.get_atomic_numbers().tolist(), at.get_scaled_positions().tolist(), np.asarray(at.cell).tolist())
                   for at in atoms]
    for rank, got, gen_state, summary in res:
        assert sorted(got) == sorted(one), rank
        for t in sorted(one):
            for k, what in enumerate(("atom types", "coordinates", "lattices")):
                assert np.array_equal(got[t][k], one[t][k]), f"rank {rank}, t={t}: {what} differ from one process"
        assert np.array_equal(gen_state, gen_one.numpy()), f"rank {rank}: CPU generator ends elsewhere than in one process"
        assert summary == summary_one, f"rank {rank}: Chemeleon.sample() under 2 ranks differs from one process"
        gate_64x20(got, g, label=f"64x20 T=1000, 2 ranks (rank {rank})")
