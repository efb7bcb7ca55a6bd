"""HBM traffic per kernel launch from rocprofv3 PMC passes (bench.py's in-run `roofline.traffic`,
tools/traffic_summary.py).

Counters as /opt/skills/guides/MI355X_MICROARCH.md prescribes for gfx950: FETCH_SIZE and WRITE_SIZE
(KiB) in two separate `rocprofv3 --pmc` passes (FETCH_SIZE uses 3 TCC counters, WRITE_SIZE 2: one
pass holds at most 4); FETCH_SIZE reports half the bytes of wide coalesced streaming reads on
gfx950, so it is doubled. Measurement tooling only: nothing on the sampling path imports this."""

import collections
import csv
import glob
import os
import socket


def per_kernel(path, counter):
    """{kernel name: [bytes per dispatch]} of `counter` from every *counter_collection.csv under path."""
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        per_dispatch = collections.defaultdict(float)
        names = {}
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] != counter:
                    continue
                per_dispatch[r["Dispatch_Id"]] += float(r["Counter_Value"])
                names[r["Dispatch_Id"]] = r["Kernel_Name"]
        for d, v in per_dispatch.items():
            vals[names[d]].append(v * 1024.0)
    return vals


def traffic(fetch_dir, write_dir):
    """{kernel: {launches, read_bytes (FETCH_SIZE x2), write_bytes, bytes_per_launch}} averaged per launch."""
    fetch = per_kernel(fetch_dir, "FETCH_SIZE")
    write = per_kernel(write_dir, "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, []), write.get(k, [])
        if not f and not w:
            continue
        fb = 2.0 * sum(f) / len(f) if f else None
        wb = sum(w) / len(w) if w else None
        out[k] = {"launches": max(len(f), len(w)), "read_bytes": fb, "write_bytes": wb,
                  "bytes_per_launch": (fb or 0.0) + (wb or 0.0)}
    return out


def box_id(device_uuid=None):
    """Which machine / GPU a measurement came from: host name, the measured device's UUID (when the
    caller knows it) and the unique ids of the node's GPUs (sysfs), so figures from different boxes
    are not mixed."""
    ids = []
    for f in sorted(glob.glob("/sys/class/drm/card*/device/unique_id")):
        try:
            with open(f) as fh:
                v = fh.read().strip()
            if v and v not in ids:
                ids.append(v)
        except OSError:
            pass
    out = {"host": socket.gethostname(), "node_gpu_unique_ids": ids[:8]}
    if device_uuid:
        out["device_uuid"] = str(device_uuid)
    return out
