import torch, sys
sys.path.insert(0, '.')
from tests.test_gpu_parity import _model
from chemeleon_amd.synthetic import synthetic_text_embeds
cn = synthetic_text_embeds(512)
nat = [40] * 64
B, N = len(nat), sum(nat)
g = torch.Generator().manual_seed(12)
a0 = torch.randint(0, 100, (N,), generator=g); x0 = torch.rand(N, 3, generator=g)
l0 = torch.eye(3).expand(B, 3, 3) * 4.0 + 0.3 * torch.randn(B, 3, 3, generator=g)
nz = (torch.rand((N, 104), generator=g), torch.randn(B, 3, 3, generator=g), torch.randn(N, 3, generator=g), torch.randn(N, 3, generator=g))
m = _model(1000)
outs = []
for layer, lag in ((0, 10), (1, 10), (1, 1), (0, 10)):
    m.decoder.set_option("edge_layer", layer); m.decoder.set_option("edge_lag", lag)
    o = [t.cpu() for t in m.reverse_step(500, a0, x0, l0, nat, 2.0, 1e-5, cn[0], cn[1], noise=nz)]
    outs.append(o)
    print(layer, lag, [float(t.float().abs().max()) for t in o], flush=True)
for k in (1, 2, 3):
    print(k, [torch.equal(u, v) for u, v in zip(outs[0], outs[k])], [float((u.float()-v.float()).abs().max()) for u, v in zip(outs[0], outs[k])])
