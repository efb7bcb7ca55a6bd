"""One-line summary of a bench.py JSON line (last line of the given log)."""
import json
import sys

line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
j = json.loads(line)
r = j["roofline"]
l2 = j.get("edge_layer2") or {}
l1 = j.get("edge_layer1") or {}


def f(v, fmt):
    return format(v, fmt) if isinstance(v, (int, float)) else "-"


print(f"{j['value']:.3f} {j['unit']}  {j['ms_per_step']:.2f} ms/step  "
      f"dominant {f(r['avg_ms'], '.3f')} ms ({f(r['frac'], '.3f')})  "
      f"L2 {f(l2.get('avg_ms'), '.3f')} ms  L1 {f(l1.get('avg_ms'), '.3f')} ms  "
      f"path {j['path']['tflops']:.0f} TF")
extra = []
if r.get("mfma_busy") is not None:
    extra.append(f"MFMA busy {r['mfma_busy']:.3f}")
if r.get("traffic"):
    extra.append(f"traffic {r['traffic'] / 1e9:.2f} GB/launch"
                 + (f" ({r['traffic'] / r['traffic_algorithmic']:.2f}x alg)" if r.get("traffic_algorithmic") else ""))
if "edge_repairs" in j:
    extra.append(f"repairs {j['edge_repairs']}")
if "per_rank_ms_per_step" in j:
    extra.append(f"n_gpus {j['n_gpus']} ranks {j['per_rank_ms_per_step']['min']:.2f}-{j['per_rank_ms_per_step']['max']:.2f} ms")
if extra:
    print("  " + "  ".join(extra))
