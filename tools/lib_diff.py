"""Bit-identity of two library builds (A/B variants loaded with CHM_LIB), GPU box, repo root.

    CHM_LIB=abl/x/libchemeleon_hip.so python tools/lib_diff.py run gpurun_out/x.npz [--n-samples 512]
    python tools/lib_diff.py compare gpurun_out/a.npz gpurun_out/b.npz

`run` takes three reverse steps (t = 1000, 500, 2, Philox noise, seed 11) from one seeded random state
per t with synthetic weights and saves the states; `compare` requires them equal bit for bit.
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(out, n_samples, n_atoms, ts):
    import torch

    from chemeleon_amd import Chemeleon
    from chemeleon_amd.config import default_config
    from chemeleon_amd.synthetic import synthetic_state_dict, synthetic_text_embeds

    cfg = default_config()
    torch.manual_seed(0)  # (SigmaScheduler's sigmas_norm is a Monte-Carlo estimate drawn from the CPU generator)
    model = Chemeleon(cfg)
    model.decoder.load_state_dict(synthetic_state_dict(cfg))
    model = model.to("cuda:0").eval()
    cond, null = synthetic_text_embeds(cfg["text_dim"])
    natoms = [n_atoms] * n_samples
    B, N = len(natoms), sum(natoms)
    res = {}
    for t in ts:
        g = torch.Generator().manual_seed(100 + t)
        a = torch.randint(0, 104, (N,), generator=g)
        x = torch.rand(N, 3, generator=g)
        lat = torch.randn(B, 3, 3, generator=g) * 3
        a1, x1, l1 = model.reverse_step(t, a, x, lat, natoms, 2.0, 1e-5, cond, null, noise=None, seed=11)
        torch.cuda.synchronize()
        res[f"a{t}"], res[f"x{t}"], res[f"l{t}"] = a1.cpu().numpy(), x1.cpu().numpy(), l1.cpu().numpy()
    np.savez(out, **res)
    print(f"saved {out}: {n_samples}x{n_atoms}, t = {ts}, lib {os.environ.get('CHM_LIB', 'default')}")


def compare(fa, fb):
    a, b = np.load(fa), np.load(fb)
    bad = [k for k in a.files if not np.array_equal(a[k], b[k])]
    for k in bad:
        d = np.abs(a[k].astype(np.float64) - b[k].astype(np.float64))
        print(f"DIFF {k}: {int((d > 0).sum())} elements, max {d.max():.3e}")
    print("bit-identical" if not bad else f"{len(bad)} arrays differ")
    return 0 if not bad else 1


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("cmd", choices=["run", "compare"])
    p.add_argument("files", nargs="+")
    p.add_argument("--n-samples", type=int, default=512)
    p.add_argument("--n-atoms", type=int, default=40)
    p.add_argument("--t", type=int, nargs="+", default=[1000, 500, 2])
    a = p.parse_args()
    if a.cmd == "run":
        run(a.files[0], a.n_samples, a.n_atoms, a.t)
    else:
        sys.exit(compare(*a.files[:2]))
