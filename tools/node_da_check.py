"""One reverse step at 512x40 and a ragged batch with fixed noise; writes the outputs to argv[1]
(run once with CHM_NODE_DA=1 and once without, then compare: the DA node GEMM must be bit-identical)."""
import sys
import torch
sys.path.insert(0, ".")
from tests.test_gpu_parity import _model
from chemeleon_amd.synthetic import synthetic_text_embeds

cn = synthetic_text_embeds(512)
m = _model(1000)
out = {}
for tag, nat in (("512x40", [40] * 512), ("ragged", torch.randint(1, 81, (300,), generator=torch.Generator().manual_seed(3)).tolist())):
    B, N = len(nat), sum(nat)
    g = torch.Generator().manual_seed(4)
    a0 = torch.randint(0, 100, (N,), generator=g); x0 = torch.rand(N, 3, generator=g)
    l0 = torch.eye(3).expand(B, 3, 3) * 4.0 + 0.3 * torch.randn(B, 3, 3, generator=g)
    nz = (torch.rand((N, 104), generator=g), torch.randn(B, 3, 3, generator=g), torch.randn(N, 3, generator=g),
          torch.randn(N, 3, generator=g))
    out[tag] = [t.cpu() for t in m.reverse_step(500, a0, x0, l0, nat, 2.0, 1e-5, cn[0], cn[1], noise=nz)]
torch.save(out, sys.argv[1])
if len(sys.argv) > 2:
    ref = torch.load(sys.argv[2], weights_only=True)
    for k in out:
        for u, v in zip(out[k], ref[k]):
            assert torch.equal(u, v), f"{k}: outputs differ"
    print("bit-identical")
