"""One-line summary of a bench.py JSON line (last line of the given log)."""
import json
import sys

line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
j = json.loads(line)
print(f"{j['value']:.3f} {j['unit']}  {j['ms_per_step']:.2f} ms/step  "
      f"L2 {j['roofline']['avg_ms']:.3f} ms ({j['roofline']['frac']:.3f})  "
      f"L1 {j['edge_layer1']['avg_ms']:.3f} ms ({j['edge_layer1']['frac']:.3f})  "
      f"path {j['path']['tflops']:.0f} TF")
