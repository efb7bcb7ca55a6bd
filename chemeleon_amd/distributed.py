"""Sample-parallel sampling over one process per GPU (torch.distributed;
backend "nccl" is RCCL on ROCm, riding xGMI between MI355X GPUs).

Samples are independent (CSPNet never mixes crystals: cspnet.py:321 builds
edges inside a crystal only), so the path shards without any per-step
exchange:
  1. rank 0 computes the conditioning vectors once (the frozen text encoder)
     and broadcasts them (2 x [B, 512] fp32);
  2. every rank samples a contiguous range of crystals, balanced by work
     (sum of n^2 + NODE_COST * n: edges and atoms). The noise never
     depends on the number of ranks: in parity mode (noise="torch", the
     reference's CPU RNG stream) every rank advances the CPU generator
     over the global draws and keeps its own rows
     (chemeleon_amd.noise); in perf mode (noise="philox") device Philox noise
     is keyed by GLOBAL node / graph index;
  3. the finished structures are all-gathered (padded to the largest shard).
Chemeleon.sample() takes this path by itself when torch.distributed is
initialised over more than one rank.
The reference has no distributed sampler (its Lightning DDP is training only,
run.py:78-92); this module is the MI355X-native counterpart asked for by the
north star.
"""

from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


# per-atom cost of a crystal in units of one fc edge (n^2 edges, n atoms): the node-side work (FiLM, the per-node
# halves of edge layer 1, the node MLP: per-row GEMMs at small M) fitted on the eight ranks' shares of configs[4]
# run one by one on one MI355X (profiles/r6/share: ms per step = 7.66e-5 sum n^2 + 1.28e-3 sum n + c, ratio 16.7)
NODE_COST = 16


def partition(natoms: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """Contiguous [g0, g1) crystal ranges per rank with roughly equal work,
    sum of n^2 + NODE_COST * n (fc edges and atoms). Every rank gets at least
    one crystal; fewer crystals than ranks is an error."""
    natoms = [int(n) for n in natoms]
    G = len(natoms)
    if G < max(world, 1):
        raise ValueError(f"{G} crystals cannot be sharded over {world} ranks (one crystal at least per rank)")
    if world <= 1:
        return [(0, G)]
    w = [n * n + NODE_COST * n for n in natoms]
    total = float(sum(w))
    bounds, acc, g = [0], 0.0, 0
    for r in range(1, world):
        target = total * r / world
        # leave at least one crystal for each remaining rank
        limit = G - (world - r)
        while g < limit and (acc + w[g] <= target or g < bounds[-1] + 1):
            acc += w[g]
            g += 1
        bounds.append(g)
    bounds.append(G)
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


def broadcast_conditioning(cond: torch.Tensor, null: torch.Tensor, src: int = 0, group=None):
    """Rank `src` holds the text-encoder outputs; everyone receives them."""
    cond = cond.contiguous()
    null = null.contiguous()
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(cond, src, group=group)
        dist.broadcast(null, src, group=group)
    return cond, null


def gather_states(states: Tuple[torch.Tensor, torch.Tensor, torch.Tensor], natoms_local: Sequence[int],
                  group=None, natoms_all: Optional[Sequence[Sequence[int]]] = None
                  ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, List[int]]:
    """All-gather (atom_types [N_r], frac [N_r,3], lattices [B_r,3,3]) from
    every rank, padding to the largest shard. Returns the concatenated global
    tensors (rank order) and the global natoms list.

    natoms_all (every rank's crystal list, e.g. from `partition` of a global
    list all ranks hold) skips the size exchange: then the gather is exactly
    three collectives and no host synchronisation. Without it the sizes are
    exchanged first (two small all-gathers, one host read each)."""
    a, x, lat = states
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return a, x, lat, list(natoms_local)
    world = dist.get_world_size(group)
    dev = x.device
    if natoms_all is None:
        nl = torch.tensor([len(natoms_local)], device=dev, dtype=torch.long)
        counts = [torch.zeros_like(nl) for _ in range(world)]
        dist.all_gather(counts, nl, group=group)
        counts = torch.cat(counts).tolist()
        bmax = max(counts)
        nat = torch.zeros(bmax, device=dev, dtype=torch.long)
        nat[:len(natoms_local)] = torch.tensor(list(natoms_local), device=dev)
        nats = [torch.zeros_like(nat) for _ in range(world)]
        dist.all_gather(nats, nat, group=group)
        rows = torch.stack(nats).tolist()
        natoms_all = [rows[r][:counts[r]] for r in range(world)]
    natoms_all = [[int(n) for n in ns] for ns in natoms_all]
    if len(natoms_all) != world:
        raise ValueError("natoms_all must hold one crystal list per rank")
    counts = [len(ns) for ns in natoms_all]
    bmax = max(counts)
    nmax = max(sum(ns) for ns in natoms_all)

    def pad(t, rows):
        out = torch.zeros((rows,) + tuple(t.shape[1:]), device=dev, dtype=t.dtype)
        out[:t.shape[0]] = t
        return out

    res = []
    for t, rows in ((a, nmax), (x, nmax), (lat, bmax)):
        p = pad(t.contiguous(), rows)
        buf = [torch.empty_like(p) for _ in range(world)]
        dist.all_gather(buf, p, group=group)
        res.append(buf)
    A = torch.cat([res[0][r][:sum(natoms_all[r])] for r in range(world)])
    X = torch.cat([res[1][r][:sum(natoms_all[r])] for r in range(world)])
    LT = torch.cat([res[2][r][:counts[r]] for r in range(world)])
    return A, X, LT, [n for ns in natoms_all for n in ns]


def _world(group):
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def _shared_conditioning(model, texts, B, cond, null, group):
    """Conditioning vectors [B, text_dim] on every rank: the text encoder (or the given vectors) on
    rank 0 only, then one broadcast of each (the north star's "computed once on host and
    broadcast"). None for a model without text guidance.

    Rank 0 validates the given vectors and computes the conditioning first, then broadcasts a status
    flag: if it failed, EVERY rank raises (rank 0 its own error, the others a RuntimeError naming it),
    so no rank is left blocked in a broadcast that never comes (the other ranks may not hold the
    vectors at all: sample_distributed lets rank 0 alone pass them)."""
    if not model.text_guide:
        return None, None
    world, rank = _world(group)
    dev = model.device
    d = model.hparams["text_dim"]
    err = None
    c = torch.zeros(B, d, device=dev)
    n = torch.zeros(B, d, device=dev)
    if rank == 0 or world == 1:
        try:
            for name, v in (("text_embeds", cond), ("null_text_embeds", null)):
                if v is not None and (v.dim() != 2 or v.shape[0] not in (1, B) or v.shape[1] != d):
                    raise ValueError(f"{name} has shape {tuple(v.shape)}; expected [1 or {B}, {d}] for {B} crystals")
            c, n = model._conditioning(texts, B, cond, null)
        except Exception as e:  # noqa: BLE001 (re-raised below, after every rank has heard of it)
            err = e
    if world > 1:
        flag = torch.tensor([0 if err is None else 1], device=dev, dtype=torch.int32)
        dist.broadcast(flag, 0, group=group)
        if int(flag.item()):
            if err is not None:
                raise err
            raise RuntimeError("rank 0 failed to compute the text conditioning (see rank 0's error); every rank stops")
    elif err is not None:
        raise err
    return broadcast_conditioning(c, n, 0, group)


@torch.no_grad()
def sample_states_distributed(model, natoms: Sequence[int], texts=None, cond_scale: float = 2.0,
                              step_lr: float = 1e-5, *, noise: str = "torch", seed: int = 0, text_embeds=None,
                              null_text_embeds=None, group=None, init: Optional[Tuple] = None,
                              every_step=False, graph: Optional[bool] = None, t_stop: int = 0, lanes: int = 1,
                              clone: bool = False, **unsupported):
    """Reverse loop over a GLOBAL crystal list, sharded across the ranks of `group`: yields
    (t, atom_types, frac_coords, lattices) of the WHOLE batch on every rank, for every t
    (every_step=True, one all-gather per step: the stream / return_trajectory case), for the t in
    every_step (a collection of timesteps) and the final state, or only the final state t = 0
    (every_step=False: one all-gather at the end; nothing is exchanged inside the loop).

    noise="torch" (parity mode, the default of Chemeleon.sample): every rank advances the global CPU
    generator over the reference's global draws (chemeleon.py:348-349, 400-404, 418, 435, 455) and
    keeps its own rows, so the gathered result is bit-identical to the single-process run for any
    rank count, provided every rank seeded its generator the same way (torch.manual_seed(s) before
    the call, as for the reference). noise="philox": device noise keyed by (seed, t, global index);
    the initial noise comes from Generator(seed) at the global size.

    t_stop / lanes / clone act as in Chemeleon.sample_states (the final gather is at t = t_stop); the
    shard placement keywords of sample_states (node_base, graph_base, global_sizes) are computed here
    from the global list and refused if passed (ValueError on every rank, before any collective)."""
    if unsupported:
        raise ValueError(f"{sorted(unsupported)}: not accepted when sampling over ranks (the shard offsets and "
                         "global sizes are computed from the global crystal list)")
    world, rank = _world(group)
    natoms = [int(n) for n in natoms]
    # every rank holds the same list, so every rank raises here, before any collective
    if len(natoms) < world:
        raise ValueError(f"{len(natoms)} crystals cannot be sharded over {world} ranks (one crystal at least per rank)")
    if noise not in ("torch", "philox"):
        raise ValueError("noise must be 'torch' or 'philox'")
    ranges = partition(natoms, world)
    g0, g1 = ranges[rank]
    B, N = len(natoms), sum(natoms)
    cond, null = _shared_conditioning(model, texts, B, text_embeds, null_text_embeds, group)
    if cond is not None:
        cond, null = cond[g0:g1], null[g0:g1]
    node_base = sum(natoms[:g0])
    local = natoms[g0:g1]
    n1 = node_base + sum(local)
    if init is None and noise == "philox":  # global initial noise from one seeded CPU generator
        g = torch.Generator().manual_seed(seed)
        l0 = torch.randn(B, 3, 3, generator=g) * model.mask_lattice_matrix
        x0 = torch.randn(N, 3, generator=g)
        init = (l0, x0)
    if init is not None:
        l0, x0 = init
        if l0.shape[0] != B or x0.shape[0] != N:
            raise ValueError("init holds the global (l_T [B,3,3], x_T [N,3]) of the whole batch")
        init = (l0[g0:g1], x0[node_base:n1])
    natoms_all = [natoms[r0:r1] for r0, r1 in ranges]
    it = model.sample_states(local, None, cond_scale, step_lr, noise=noise, seed=seed, text_embeds=cond,
                             null_text_embeds=null, clone=False, node_base=node_base, graph_base=g0, init=init,
                             global_sizes=(N, B) if noise == "torch" else None, graph=graph, t_stop=t_stop,
                             lanes=lanes)
    want = None if isinstance(every_step, bool) else {int(t) for t in every_step}
    for t, a, x, lat in it:
        if t == t_stop or (every_step is True) or (want is not None and t in want):
            A_, X_, L_, _ = gather_states((a, x, lat), local, group, natoms_all=natoms_all)
            if clone and world == 1:  # (one rank: the gather hands back the sampler's own buffers)
                A_, X_, L_ = A_.clone(), X_.clone(), L_.clone()
            yield t, A_, X_, L_


@torch.no_grad()
def sample_distributed(model, natoms: Sequence[int], cond: torch.Tensor, null: torch.Tensor, cond_scale=2.0,
                       step_lr=1e-5, seed: int = 0, group=None, init: Optional[Tuple] = None, noise: str = "torch",
                       graph: Optional[bool] = None):
    """Sample `natoms` (global list) across all ranks; returns the global final
    state (atom_types, frac_coords, lattices, natoms) on every rank.
    `cond` / `null` are the [1 or B, text_dim] conditioning vectors held by
    rank 0 (broadcast here). noise as in sample_states_distributed."""
    last = None
    for last in sample_states_distributed(model, natoms, None, cond_scale, step_lr, noise=noise, seed=seed,
                                          text_embeds=cond, null_text_embeds=null, group=group, init=init,
                                          graph=graph):
        pass
    _, a, x, lat = last
    return a, x, lat, [int(n) for n in natoms]
