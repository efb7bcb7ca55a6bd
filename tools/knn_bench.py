"""Throughput of the knn (radius-graph) edge mode: reverse steps of `Chemeleon.sample_states`
with CSPNet(edge_style="knn") (eager: the graph is rebuilt every decoder call), Philox noise,
synthetic weights, from a mid-trajectory state (t = 500: the pure-noise start has degenerate
lattices). Prints one JSON line per size. Usage: python tools/knn_bench.py [n_samples ...]"""

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from chemeleon_amd import Chemeleon, _lib  # noqa: E402
from chemeleon_amd.config import default_config  # noqa: E402
from chemeleon_amd.synthetic import synthetic_state_dict, synthetic_text_embeds  # noqa: E402


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [64, 512]
    cfg = default_config()
    cfg["edge_style"] = "knn"
    torch.manual_seed(0)
    m = Chemeleon(cfg)
    m.decoder.load_state_dict(synthetic_state_dict(default_config()))
    m = m.to("cuda").eval()
    cond, null = synthetic_text_embeds(512)
    for n in sizes:
        natoms = [40] * n
        N = 40 * n
        g = torch.Generator().manual_seed(3)
        a = torch.randint(1, 104, (N,), generator=g)
        x = torch.rand(N, 3, generator=g)
        diag = 6.0 + 2.0 * torch.rand(n, 3, generator=g)
        lat = (torch.diag_embed(diag) + 0.3 * (torch.rand(n, 3, 3, generator=g) - 0.5)) * m.mask_lattice_matrix
        steps, warm = 6, 2
        for k in range(warm + steps):
            if k == warm:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            a, x, lat = m.reverse_step(500 - k, a, x, lat, natoms, 2.0, 1e-5, cond, null, noise=None, seed=1)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        E = int(_lib.load().chm_batch_num_edges(m.decoder.hip_batch(natoms, max_pairs=2).handle))
        print(json.dumps({"mode": "knn", "n_samples": n, "n_atoms": 40, "ms_per_step": dt * 1e3,
                          "structures_per_sec": n / (1000 * dt), "edges_last_call": E,
                          "fc_edges_same_batch": 1600 * n}))


if __name__ == "__main__":
    main()
