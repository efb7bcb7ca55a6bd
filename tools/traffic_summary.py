"""Per-launch HBM traffic per kernel from the two PMC passes of tools/pmc_traffic.sh
(FETCH_SIZE x2 per the gfx950 correction + WRITE_SIZE; chemeleon_amd/pmc.py), with the box it ran on.
Usage: python tools/traffic_summary.py gpurun_out/traffic > profiles/rN/traffic.json
(run on the GPU box, so that `box` names the machine the counters came from)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from chemeleon_amd.pmc import box_id, traffic  # noqa: E402


def main(path):
    json.dump({"note": "FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, bytes per launch, averaged",
               "box": box_id(), "kernels": traffic(path + "/fetch", path + "/write")}, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
