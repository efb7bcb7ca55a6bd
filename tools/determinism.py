"""Run-to-run determinism of the sampling step (GPU box, repo root).

    python tools/determinism.py gpurun_out/det_a.npz [--n-samples 64]   # then again into det_b.npz
    python tools/lib_diff.py compare gpurun_out/det_a.npz gpurun_out/det_b.npz

In one process: the same reverse step (t = 500, Philox noise) repeated three times from the same state,
and one decoder pair call (cond / null) on that state repeated three times; prints whether the repeats
agree bit for bit and saves the first result of each for the cross-process comparison.
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from chemeleon_amd import Chemeleon
    from chemeleon_amd.config import default_config
    from chemeleon_amd.synthetic import synthetic_state_dict, synthetic_text_embeds

    p = argparse.ArgumentParser()
    p.add_argument("out")
    p.add_argument("--n-samples", type=int, default=64)
    p.add_argument("--n-atoms", type=int, default=40)
    a = p.parse_args()
    cfg = default_config()
    torch.manual_seed(0)  # (SigmaScheduler's sigmas_norm is a Monte-Carlo estimate drawn from the CPU generator)
    model = Chemeleon(cfg)
    model.decoder.load_state_dict(synthetic_state_dict(cfg))
    model = model.to("cuda:0").eval()
    cond, null = synthetic_text_embeds(cfg["text_dim"])
    natoms = [a.n_atoms] * a.n_samples
    B, N = len(natoms), sum(natoms)
    g = torch.Generator().manual_seed(600)
    at = torch.randint(0, 104, (N,), generator=g)
    x = torch.rand(N, 3, generator=g)
    lat = torch.randn(B, 3, 3, generator=g) * 3
    res = {}
    steps = []
    for _ in range(3):
        a1, x1, l1 = model.reverse_step(500, at, x, lat, natoms, 2.0, 1e-5, cond, null, noise=None, seed=11)
        steps.append((a1.cpu().numpy(), x1.cpu().numpy(), l1.cpu().numpy()))
    res["step_a"], res["step_x"], res["step_l"] = steps[0]
    same = [all(np.array_equal(u, v) for u, v in zip(steps[0], s)) for s in steps[1:]]
    print(f"step repeats bit-identical in-process: {same}")
    dev = "cuda:0"
    nat = torch.tensor(natoms)
    te = model.time_embed(torch.full((B,), 500, dtype=torch.long)).to(dev)
    outs = []
    for _ in range(3):
        o = model.decoder(atom_types=at.to(dev), frac_coords=x.to(dev), lattices=lat.to(dev), num_atoms=nat.to(dev),
                          node2graph=torch.arange(B).repeat_interleave(nat).to(dev), t=te,
                          text_embeds=cond.expand(B, -1).to(dev))
        outs.append([o.node_features.cpu().numpy(), o.atom_types_out.cpu().numpy(), o.coords_out.cpu().numpy(),
                     o.lattice_out.cpu().numpy()])
    for k, name in enumerate(("dec_h", "dec_types", "dec_coords", "dec_lattice")):
        if k:  # (node features stay out of the file: 84 MB at 512 x 40; compared in-process above)
            res[name] = outs[0][k]
    same = [all(np.array_equal(u, v) for u, v in zip(outs[0], s)) for s in outs[1:]]
    print(f"decoder repeats bit-identical in-process: {same}")
    np.savez(a.out, **res)
    print(f"saved {a.out}")


if __name__ == "__main__":
    main()
