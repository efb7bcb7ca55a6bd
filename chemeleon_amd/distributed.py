"""Sample-parallel sampling over one process per GPU (torch.distributed;
backend "nccl" is RCCL on ROCm, riding xGMI between MI355X GPUs).

Samples are independent (CSPNet never mixes crystals: cspnet.py:321 builds
edges inside a crystal only), so the path shards without any per-step
exchange:
  1. rank 0 computes the conditioning vectors once (the frozen text encoder)
     and broadcasts them (2 x [B, 512] fp32);
  2. every rank samples a contiguous range of crystals, balanced by edge work
     (sum of n^2); device Philox noise is keyed by GLOBAL node / graph index,
     so the result does not depend on the number of ranks;
  3. the finished structures are all-gathered (padded to the largest shard).
The reference has no distributed sampler (its Lightning DDP is training only,
run.py:78-92); this module is the MI355X-native counterpart asked for by the
north star.
"""

from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


def partition(natoms: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """Contiguous [g0, g1) crystal ranges per rank with roughly equal sum of
    n^2 (the fc edge work). Every rank gets at least one crystal; fewer
    crystals than ranks is an error."""
    natoms = [int(n) for n in natoms]
    G = len(natoms)
    if G < max(world, 1):
        raise ValueError(f"{G} crystals cannot be sharded over {world} ranks (one crystal at least per rank)")
    if world <= 1:
        return [(0, G)]
    w = [n * n for n in natoms]
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


@torch.no_grad()
def sample_distributed(model, natoms: Sequence[int], cond: torch.Tensor, null: torch.Tensor, cond_scale=2.0,
                       step_lr=1e-5, seed: int = 0, group=None, init: Optional[Tuple] = None):
    """Sample `natoms` (global list) across all ranks; returns the global final
    state (atom_types, frac_coords, lattices, natoms) on every rank.
    `cond` / `null` are the [1 or B, text_dim] conditioning vectors held by
    rank 0 (broadcast here)."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    natoms = [int(n) for n in natoms]
    # every rank holds the same list, so every rank raises here, before any collective
    if len(natoms) < world:
        raise ValueError(f"{len(natoms)} crystals cannot be sharded over {world} ranks (one crystal at least per rank)")
    ranges = partition(natoms, world)
    g0, g1 = ranges[rank]
    cond, null = broadcast_conditioning(cond.to(model.device), null.to(model.device), 0, group)
    if cond.shape[0] == len(natoms):
        cond, null = cond[g0:g1], null[g0:g1]
    node_base = sum(natoms[:g0])
    if init is None:  # global initial noise from one seeded CPU generator, sliced per rank
        g = torch.Generator().manual_seed(seed)
        l0 = torch.randn(len(natoms), 3, 3, generator=g) * model.mask_lattice_matrix
        x0 = torch.randn(sum(natoms), 3, generator=g)
    else:
        l0, x0 = init
    local = natoms[g0:g1]
    last = None
    for last in model.sample_states(local, None, cond_scale, step_lr, noise="philox", seed=seed, text_embeds=cond,
                                    null_text_embeds=null, clone=False, node_base=node_base, graph_base=g0,
                                    init=(l0[g0:g1], x0[node_base:node_base + sum(local)])):
        pass
    return gather_states(last[1:], local, group, natoms_all=[natoms[r0:r1] for r0, r1 in ranges])
