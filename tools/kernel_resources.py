"""Per-kernel registers / scratch / spills of a HIP source (hipcc -Rpass-analysis=kernel-resource-usage).
Usage: python tools/kernel_resources.py chemeleon_amd/csrc/edge16.hip [name filter]"""
import re
import subprocess
import sys

src = __import__("os").path.abspath(sys.argv[1])
filt = sys.argv[2] if len(sys.argv) > 2 else ""
r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o", "/tmp/_kr.o",
                    "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True, cwd="/tmp")
cur, rows = None, []
for line in r.stderr.splitlines():
    m = re.search(r"remark: +([A-Za-z /\[\]]+): (.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for c in rows:
    if filt in c["name"]:
        print(f"{c['name'][:60]:60s} VGPR {c.get('VGPRs'):>4} AGPR {c.get('AGPRs'):>3} SGPR {c.get('TotalSGPRs'):>4} "
              f"scratch {c.get('ScratchSize [bytes/lane]'):>4} spill s/v {c.get('SGPRs Spill')}/{c.get('VGPRs Spill')}")
