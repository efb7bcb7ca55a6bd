#!/usr/bin/env python3
"""Benchmark of the Chemeleon reverse-diffusion sampling path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Metric (BASELINE.json): structures/sec of a 1000-step sample at n_atoms=40,
n_samples=512 in total, at 1/2/4/8 GPUs (strong scaling: the 512 samples are
split across ranks, 512/N each, contiguous ranges; samples are independent so
there is no collective in the timed region).

A "step" = one reverse-diffusion timestep over the rank's whole batch: the
predictor classifier-free-guidance decoder pair, the D3PM / lattice / VE
updates, the corrector pair and the Langevin update (chm_sample_step), with
the state resident in HBM and device (Philox) noise. Every timestep has the
same shapes, so structures/sec = n_samples / (T * seconds_per_step), T = 1000.
Weights: the seeded synthetic recipe of the real architecture (hidden 512,
6 layers, 128 frequencies, fc edges); conditioning: seeded vectors broadcast
from rank 0 (RCCL), standing in for the frozen text encoder's output.

One JSON line is printed by rank 0, including:
  roofline     — the dominant kernel (edge message GEMM) against fp32 MFMA peak,
                 timed live with HIP events on its launch stream;
  msgpass      — the message-passing aggregation kernel against HBM peak;
  cpu_baseline — the CPU oracle (a restatement of the reference PyTorch CPU
                 path) timed on this host on a bounded sample (rank 0, N=1).
"""

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

T_STEPS = 1000
MFMA_F32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: dense fp32 MFMA (= vector) peak
MFMA_BF16_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA peak (spec)
# bf16x3 arithmetic: six bf16 MFMA products per fp32-accurate product, so the
# ceiling for fp32-equivalent flops on the bf16 pipe is 2.5 PF / 6
BF16X3_PEAK_TFLOPS = MFMA_BF16_PEAK_TFLOPS / 6
HBM_PEAK_GBS = 8000.0         # MI355X_MICROARCH.md: HBM3E spec peak
H, FD, L, A = 512, 768, 6, 104


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--n-samples", type=int, default=512, help="total samples across all ranks")
    p.add_argument("--n-atoms", type=int, default=40)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-samples", type=int, default=64)
    p.add_argument("--cpu-steps", type=int, default=3)
    p.add_argument("--no-api-legs", action="store_true",
                   help="skip the legs that time Chemeleon.sample() end to end (1000 steps, perf mode) and the "
                        "parity-mode (noise='torch') step")
    p.add_argument("--no-graph", action="store_true", help="launch every kernel eagerly instead of replaying a "
                   "captured HIP graph of the reverse step")
    p.add_argument("--lanes", type=int, default=1, help="concurrent sample groups per GPU, each on its own stream "
                   "inside the captured step graph (their GEMM epilogues then overlap each other's matrix work)")
    p.add_argument("--math", choices=["split16", "bf16x3", "f32"], default="split16",
                   help="decoder GEMM arithmetic (both fp32-accurate; see include/chemeleon_hip.h)")
    p.add_argument("--ragged", action="store_true",
                   help="SURVEY C4 workload: natoms = randint(1, 81, generator seed 7) per sample (use with "
                        "--n-samples 2048), ranks split by sum of n^2; not the headline metric")
    p.add_argument("--no-traffic", action="store_true",
                   help="skip the in-run HBM traffic measurement of the dominant kernel (two rocprofv3 --pmc passes "
                        "over a 2-step eager probe; roofline.traffic then falls back to the committed profile)")
    p.add_argument("--noise", choices=["philox", "torch"], default="philox",
                   help="philox: device noise keyed by global index (the headline); torch: parity mode, the "
                        "reference's CPU RNG stream drawn on every rank at the global size, each rank uploading its "
                        "rows before every replay of the captured step (chemeleon_amd.noise)")
    p.add_argument("--share", type=int, default=1, metavar="N",
                   help="profiling: run, on this one GPU, the share of rank --share-rank of an N-rank job (the "
                        "sharding of sample(): contiguous ranges balanced by sum of n^2); value then counts that "
                        "share's structures")
    p.add_argument("--share-rank", type=int, default=0)
    p.add_argument("--traffic-probe", action="store_true", help=argparse.SUPPRESS)  # (the PMC passes' workload)
    return p.parse_args()


def edge_layer_bytes(natoms, P=2, pairs=None):
    """Algorithmic HBM bytes of one k_edge16_layer launch (both edge layers of a CSP layer, split16):
    F read once (E x 768 fp16 hi/lo), S written and read once per conditioning (E x 512 fp16 hi/lo +
    one packed exponent word per row), the P / Q node halves read, agg written, the split weights
    D (512 x 768) and W2 (512 x 512) read once."""
    E = sum(n * n for n in natoms)
    N = sum(natoms)
    pairs = edge_pairs_on() if pairs is None else pairs
    f = (sum(n * (n + 1) // 2 for n in natoms) if pairs else E) * FD * 4  # (on pairs: one feature row per pair)
    s = P * E * (H * 4 + 4)
    return f + 2 * s + P * N * 2 * H * 4 + P * N * H * 4 + (H * FD + H * H) * 4


def message_layer_bytes(natoms, P=2):
    """Algorithmic HBM bytes of one edge-layer-2 launch (k_edge16<EPI_SEGMEAN>: S.W2^T + SiLU + fused
    scatter_mean, both conditionings): S read once (E x 512 fp16 hi/lo + one packed exponent word per
    row, per conditioning), agg written, the split weight W2 (512 x 512) read once."""
    E = sum(n * n for n in natoms)
    N = sum(natoms)
    return P * E * (H * 4 + 4) + P * N * H * 4 + H * H * 4


def edge_pairs_on():
    """Edge layer 1 on unordered pairs (option edge_pairs, the library default; CHM_EDGE_PAIRS=0 turns it off)."""
    return os.environ.get("CHM_EDGE_PAIRS", "1") != "0"


EDGE_PAIRS_LAYER_DEFAULT = "1"  # (the library's default of option edge_pairs_layer)


def pairs_layer_kernel():
    """The one-grid kernel of both edge layers on pairs (option edge_pairs_layer, 0 = two launches)."""
    mode = os.environ.get("CHM_EDGE_PAIRS_LAYER", EDGE_PAIRS_LAYER_DEFAULT)
    return None if mode == "0" else "k_edge16_pairs_grid"


def decoder_pair_flops(natoms, P=2, share_fourier=True, pairs=None):
    """Algorithmic fp32 flops of one decoder call pair as implemented
    (SURVEY.md §8(d) factorised formula, with the Fourier projection shared
    by the cond/null pair; with edge layer 1 on pairs, the Fourier projection
    once per unordered pair i <= j: sum n(n+1)/2 rows instead of sum n^2)."""
    E = sum(n * n for n in natoms)
    Ep = sum(n * (n + 1) // 2 for n in natoms)
    N = sum(natoms)
    B = len(natoms)
    pairs = edge_pairs_on() if pairs is None else pairs
    edge = L * ((1 if share_fourier else P) * 2 * FD * H * (Ep if pairs else E) + E * P * 2 * H * H)
    node = P * N * L * (4 * H * H + 2 * (2 * H * H + H * H) + 2 * H * H)
    heads = P * N * 2 * H * 107 + P * B * 2 * 640 * 2 * H
    return edge + node + heads


def host_cores():
    """CPU cores this process may use: the affinity mask, capped by the cgroup CPU quota (a GPU
    box shows all of the machine's CPUs in os.cpu_count() but grants one GPU's share), and by the
    physical core count when SMT siblings are visible (lscpu's cores x sockets)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    how = f"affinity {n}"
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            q = max(1, int(int(quota) // int(period)))
            if q < n:
                n, how = q, how + f", cgroup quota {q}"
    except (OSError, ValueError):
        pass
    try:
        import subprocess
        info = dict(line.split(":", 1) for line in subprocess.run(["lscpu"], capture_output=True, text=True,
                                                                  timeout=10).stdout.splitlines() if ":" in line)
        phys = int(info["Core(s) per socket"]) * int(info["Socket(s)"])
        if phys < n:
            n, how = phys, how + f", physical cores {phys}"
    except Exception:  # noqa: BLE001
        pass
    return n, how


def cpu_baseline(n_samples, n_atoms, steps):
    """Time the oracle (CPU restatement of the reference path) on this host."""
    from chemeleon_amd.config import default_config
    from chemeleon_amd.synthetic import synthetic_state_dict, synthetic_text_embeds
    from oracle import chemeleon_oracle as O
    threads, how = host_cores()
    torch.set_num_threads(threads)
    cfg = default_config()
    torch.manual_seed(0)
    m = O.OracleModel(cfg, synthetic_state_dict(cfg))
    cond, null = synthetic_text_embeds(512)
    nat = torch.tensor([n_atoms] * n_samples)
    B, N = n_samples, n_samples * n_atoms
    n2g = torch.arange(B).repeat_interleave(nat)
    g = torch.Generator().manual_seed(1)
    a = torch.zeros(N, dtype=torch.long)
    x = torch.rand(N, 3, generator=g)
    lat = torch.randn(B, 3, 3, generator=g) * O.LATTICE_MASK
    c, nl = cond.expand(B, -1), null.expand(B, -1)
    with torch.no_grad():
        nz = m.draw_noise(T_STEPS, N, B)
        m.step(T_STEPS, a, x, lat, nat, n2g, c, nl, nz)  # warm-up
        t0 = time.perf_counter()
        for k in range(steps):
            t = T_STEPS - 1 - k
            nz = m.draw_noise(t, N, B)
            a, x, lat, _ = m.step(t, a, x, lat, nat, n2g, c, nl, nz)
        dt = (time.perf_counter() - t0) / steps
    return {"value": n_samples / (dt * T_STEPS), "unit": "structures/sec", "cores": threads, "kind": "port",
            "sample": f"oracle (torch CPU restatement of the reference path) {n_samples}x{n_atoms} atoms, "
                      f"{steps} timed reverse steps after 1 warm-up, {dt:.2f} s/step, extrapolated x{T_STEPS}; "
                      f"{threads} torch threads ({how})",
            "s_per_step": dt}


def api_legs(model, n_samples, n_atoms, cond, null, seed, headline):
    """What a drop-in caller gets (reference chemeleon.py:469-490): Chemeleon.sample() end to end
    in perf mode (one captured HIP graph replayed per timestep, device Philox noise), including
    graph capture, the final device->host copy and get_atoms; the same call in the default
    parity mode (noise='torch': the reference's CPU RNG stream drawn on the host every step and
    copied in before each replay of the captured step) over 30 steps; and parity mode's eager
    per-step cost (graph=False, the round-1 path)."""
    out = {}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    atoms = model.sample(None, n_atoms, n_samples, 2.0, 1e-5, noise="philox", seed=seed, text_embeds=cond,
                         null_text_embeds=null)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert len(atoms) == n_samples
    out["sample_philox_graph"] = {"value": n_samples / dt, "unit": "structures/sec", "seconds": dt,
                                  "ratio_to_headline": (n_samples / dt) / headline,
                                  "call": f"Chemeleon.sample(n_atoms={n_atoms}, n_samples={n_samples}, "
                                          "noise='philox') incl. graph capture and get_atoms"}
    for key, graph, steps, note in (
            ("torch_noise_graph_step", True, 30, "noise='torch' (parity mode, the default of sample()): host RNG "
                                                 "draw into pinned buffers, copy, replay of the captured step"),
            ("torch_noise_step", False, 3, "noise='torch' with graph=False: host RNG draw + upload per step, eager "
                                           "launches")):
        it = model.sample_states([n_atoms] * n_samples, None, 2.0, 1e-5, noise="torch", text_embeds=cond,
                                 null_text_embeds=null, clone=False, graph=graph)
        next(it)
        next(it)  # warm-up step (and graph capture)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            next(it)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
        it.close()
        out[key] = {"ms_per_step": ms, "structures_per_sec": n_samples / (ms * 1e-3 * T_STEPS), "steps": steps,
                    "note": note}
    return out


def _stored_traffic(kernel_key):
    """HBM bytes per launch of the dominant kernel from the newest committed PMC profile
    (tools/pmc_traffic.sh -> tools/traffic_summary.py -> profiles/<round>/traffic.json), with the box
    that profile ran on: the fallback when the in-run passes are skipped or fail."""
    here = os.path.dirname(os.path.abspath(__file__))
    pdir = os.path.join(here, "profiles")
    for rnd in sorted(os.listdir(pdir), reverse=True) if os.path.isdir(pdir) else []:
        f = os.path.join(pdir, rnd, "traffic.json")
        if os.path.isfile(f):
            try:
                d = json.load(open(f))
                for name, v in d["kernels"].items():
                    if kernel_key in name:
                        return v["bytes_per_launch"], {"source": f"profiles/{rnd}/traffic.json ({name})",
                                                       "box": d.get("box", "not recorded (an earlier box)")}
            except Exception:  # noqa: BLE001
                return None, None
    return None, None


def _run_pmc_pass(counter, outdir, argv, limit_s):
    """One `rocprofv3 --pmc <counter>` pass over this script in probe mode, as a child process (the
    profiler preloads its library into the probe; this process is not re-exec'd), killed with its
    process group at `limit_s`."""
    import shutil
    import signal
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    cmd = [prof, "--pmc"] + counter.split() + ["-d", outdir, "-o", counter.split()[0].lower(), "--output-format",
                                                "csv", "--", sys.executable, os.path.abspath(__file__),
                                                "--traffic-probe"] + argv
    env = dict(os.environ, TMPDIR="/tmp")
    log = open(os.path.join(outdir + ".log"), "w")
    p = subprocess.Popen(cmd, cwd="/tmp", env=env, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    try:
        rc = p.wait(timeout=limit_s)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        p.wait()
        rc = "timeout"
    log.close()
    return rc


def measure_traffic(args, kernel_key, limit_s=240):
    """roofline.traffic measured on this box: FETCH_SIZE and WRITE_SIZE in two rocprofv3 --pmc passes
    (MI355X_MICROARCH.md: separate passes, FETCH_SIZE x2 on gfx950) over a probe that runs the same
    workload eagerly for 2 reverse steps; bytes per launch of the dominant kernel."""
    import tempfile
    from chemeleon_amd.pmc import box_id, traffic
    root = tempfile.mkdtemp(prefix="chm_pmc_", dir="/tmp")
    argv = ["--n-samples", str(args.n_samples), "--n-atoms", str(args.n_atoms), "--math", args.math,
            "--seed", str(args.seed)]
    t0 = time.perf_counter()
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        rc = _run_pmc_pass(counter, os.path.join(root, counter.lower()), argv, limit_s)
        if rc != 0:
            return None, {"error": f"rocprofv3 --pmc {counter} pass exited with {rc}",
                          "log": os.path.join(root, counter.lower() + ".log")}
    ks = traffic(os.path.join(root, "fetch_size"), os.path.join(root, "write_size"))
    for name, v in ks.items():
        if kernel_key in name and v["read_bytes"] is not None and v["write_bytes"] is not None:
            src = {"source": f"measured in this run: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over a 2-step eager "
                             f"probe of the same workload ({name}, {v['launches']} launches)",
                   "read_bytes": v["read_bytes"], "write_bytes": v["write_bytes"],
                   "box": box_id(getattr(torch.cuda.get_device_properties(0), "uuid", None))}
            # a third pass: MFMA busy share of the dominant kernel (SQ_VALU_MFMA_BUSY_CYCLES over all SIMDs
            # against GRBM_GUI_ACTIVE, the sum over the 8 XCDs of their active cycles: 1024 SIMDs x GRBM / 8)
            d = os.path.join(root, "mfma")
            if _run_pmc_pass("SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE", d, argv, limit_s) == 0:
                from chemeleon_amd.pmc import per_kernel
                busy = [x for k, xs in per_kernel(d, "SQ_VALU_MFMA_BUSY_CYCLES").items() if kernel_key in k for x in xs]
                act = [x for k, xs in per_kernel(d, "GRBM_GUI_ACTIVE").items() if kernel_key in k for x in xs]
                if busy and act and sum(act) > 0:  # (per_kernel scales by 1024 for KiB counters: cancels here)
                    src["mfma_busy"] = sum(busy) / (1024.0 * sum(act) / 8.0)
            src["seconds"] = time.perf_counter() - t0
            return v["bytes_per_launch"], src
    return None, {"error": f"no {kernel_key} dispatch in the PMC output", "dir": root}


def traffic_probe(args):
    """The PMC passes' workload: this rank's batch, two eager reverse steps (no graph, no timing)."""
    from chemeleon_amd import Chemeleon
    from chemeleon_amd.config import default_config
    from chemeleon_amd.synthetic import synthetic_state_dict, synthetic_text_embeds
    dev = torch.device("cuda", 0)
    cfg = default_config()
    torch.manual_seed(0)
    model = Chemeleon(cfg)
    model.decoder.load_state_dict(synthetic_state_dict(cfg))
    model = model.to(dev).eval()
    model.decoder.set_math(args.math)
    cond, null = synthetic_text_embeds(512)
    it = model.sample_states([args.n_atoms] * args.n_samples, None, 2.0, 1e-5, noise="philox", seed=args.seed,
                             text_embeds=cond.to(dev), null_text_embeds=null.to(dev), clone=False, t_stop=998,
                             graph=False)
    for _ in it:
        pass
    torch.cuda.synchronize()


def launch_plan(gpus, env, device_count):
    """What `bench.py --gpus N` does in this process, decided before anything touches the GPU.

    * ("run", None): this process is a rank (WORLD_SIZE set by a launcher, equal to N) or N == 1;
    * ("spawn", N): N > 1 and no launcher: start N ranks as a child `torch.distributed.run` and
      forward its output (this process never initialises HIP, so nothing is exec'd from a GPU process);
    * ("refuse", why): inconsistent requests that would otherwise measure the wrong thing — a
      launcher's WORLD_SIZE different from --gpus, or more RCCL ranks than visible GPUs (gloo
      rehearsals, CHM_DIST_BACKEND=gloo, may share one GPU between ranks)."""
    if gpus < 1:
        return "refuse", f"--gpus {gpus}: need at least one GPU"
    world = env.get("WORLD_SIZE")
    if world is not None:
        if int(world) != gpus:
            return "refuse", f"--gpus {gpus} but the launcher's WORLD_SIZE is {world}"
        return "run", None
    if gpus == 1:
        return "run", None
    backend = env.get("CHM_DIST_BACKEND", "nccl")
    if backend == "nccl" and device_count < gpus:
        return "refuse", (f"--gpus {gpus} asks for {gpus} RCCL ranks, one per GPU, but {device_count} GPU(s) are "
                          "visible (CHM_DIST_BACKEND=gloo rehearses the multi-rank path on fewer GPUs)")
    return "spawn", gpus


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n, argv):
    """Run this script as N ranks under torch.distributed.run (one process per GPU, rendezvous on
    127.0.0.1) and return its exit code; rank 0 prints the JSON line, which passes through."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    print(f"bench.py: no launcher found, starting {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=env).returncode


def main():
    args = parse()
    plan, why = launch_plan(args.gpus, os.environ, torch.cuda.device_count())
    if plan == "refuse":
        raise SystemExit(f"bench.py: {why}")
    if plan == "spawn":
        raise SystemExit(spawn_ranks(why, sys.argv[1:]))
    if args.traffic_probe:
        traffic_probe(args)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # One process per GPU. The device is LOCAL_RANK modulo the visible GPUs (the identity on an
    # 8-GPU node); CHM_DIST_BACKEND=gloo rehearses the same path with several ranks sharing one GPU.
    # The two backends differ only in init_process_group.
    backend = os.environ.get("CHM_DIST_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from chemeleon_amd import Chemeleon, _lib
    from chemeleon_amd.config import default_config
    from chemeleon_amd.synthetic import synthetic_state_dict, synthetic_text_embeds

    # shard: contiguous sample ranges, 512/N each (ragged: balanced by sum of n^2)
    from chemeleon_amd.distributed import partition
    total = args.n_samples
    if args.ragged:
        all_nat = torch.randint(1, 81, (total,), generator=torch.Generator().manual_seed(7)).tolist()
    else:
        all_nat = [args.n_atoms] * total
    ranges = partition(all_nat, world)
    share_of = None
    if args.share > 1:  # (profiling one rank's share of a larger job on this GPU)
        if world > 1 or not 0 <= args.share_rank < args.share:
            raise SystemExit("bench.py: --share runs one rank's share on ONE process (0 <= --share-rank < --share)")
        r0, r1 = partition(all_nat, args.share)[args.share_rank]
        share_of = (args.share_rank, args.share, total)
        all_nat = all_nat[r0:r1]
        total = len(all_nat)
        ranges = [(0, total)]
    per = [b - a for a, b in ranges]
    g0 = ranges[rank][0]
    natoms = all_nat[ranges[rank][0]:ranges[rank][1]]
    node_base = sum(all_nat[:g0])
    # initial noise of the whole job from one seeded generator, sliced per rank (with the
    # global-index Philox keys the result is then independent of the rank count)
    gen = torch.Generator().manual_seed(args.seed)
    mask = torch.tensor([[1, 0, 1], [1, 1, 1], [0, 0, 1]]).bool()
    l_init = torch.randn(total, 3, 3, generator=gen) * mask
    x_init = torch.randn(sum(all_nat), 3, generator=gen)
    init = (l_init[g0:g0 + len(natoms)], x_init[node_base:node_base + sum(natoms)])

    cfg = default_config()
    torch.manual_seed(0)
    model = Chemeleon(cfg)
    model.decoder.load_state_dict(synthetic_state_dict(cfg))
    model = model.to(dev).eval()
    cond, null = synthetic_text_embeds(512)
    cond, null = cond.to(dev), null.to(dev)
    if dist is not None:  # text embedding computed once on rank 0, broadcast over RCCL
        dist.broadcast(cond, 0)
        dist.broadcast(null, 0)

    model.decoder.set_math(args.math)
    draw_ms = draw_ms_8 = None
    if args.noise == "torch":
        # parity mode: every rank seeds the CPU generator alike and draws the whole job's tensors (initial
        # state and per-step noise), keeping its rows; the per-step host draw of this rank's share, timed alone
        from chemeleon_amd.noise import StepNoise
        sn = StepNoise(sum(all_nat), total, A, node_base, node_base + sum(natoms), g0, g0 + len(natoms))
        bufs = tuple(torch.empty(sh).pin_memory() for sh in sn.local_shapes)
        sn.draw(out=bufs)
        t0 = time.perf_counter()
        for _ in range(10):
            sn.draw(out=bufs)
        draw_ms = (time.perf_counter() - t0) / 10 * 1e3
        # and what one rank of an 8-rank run of this job draws per step (its rows of the global tensors)
        r8 = partition(all_nat, 8)[0] if len(all_nat) >= 8 else (0, len(all_nat))
        sn8 = StepNoise(sum(all_nat), total, A, 0, sum(all_nat[r8[0]:r8[1]]), r8[0], r8[1])
        bufs8 = tuple(torch.empty(sh).pin_memory() for sh in sn8.local_shapes)
        sn8.draw(out=bufs8)
        t0 = time.perf_counter()
        for _ in range(10):
            sn8.draw(out=bufs8)
        draw_ms_8 = (time.perf_counter() - t0) / 10 * 1e3
        torch.manual_seed(args.seed)
        it = model.sample_states(natoms, None, 2.0, 1e-5, noise="torch", text_embeds=cond, null_text_embeds=null,
                                 clone=False, node_base=node_base, graph_base=g0,
                                 global_sizes=(sum(all_nat), total), graph=not args.no_graph)
    else:
        it = model.sample_states(natoms, None, 2.0, 1e-5, noise="philox", seed=args.seed, text_embeds=cond,
                                 null_text_embeds=null, clone=False, node_base=node_base, graph_base=g0, init=init,
                                 graph=not args.no_graph, lanes=args.lanes)
    next(it)  # initial state
    _lib.prof_events(reset=True)  # edge-kernel health counters (wait timeouts, repairs) from here on
    # per-kernel HIP-event instrumentation (eager launches only; graph captures are not instrumented)
    _lib.check(_lib.load().chm_prof_reset(), "prof_reset")
    _lib.check(_lib.load().chm_prof_enable(1), "prof_enable")
    for _ in range(args.warmup):
        next(it)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        state = next(it)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if not args.no_graph:
        # the timed steps replayed a captured graph: time the kernels with HIP events in an
        # instrumented eager pass of 2 reverse steps on the same shapes, right after the timed region
        _lib.check(_lib.load().chm_prof_reset(), "prof_reset")
        it2 = model.sample_states(natoms, None, 2.0, 1e-5, noise="philox", seed=args.seed, text_embeds=cond,
                                  null_text_embeds=null, clone=False, node_base=node_base, graph_base=g0,
                                  init=init, t_stop=998, graph=False)
        for _ in it2:
            pass
        torch.cuda.synchronize()
    # the dominant kernel: both edge layers in one grid (k_edge16_layer, the default on fc batches) or,
    # when that is off, the edge message GEMM; with the one-grid kernel on, a second eager pass times the
    # two layers as separate launches for context
    nlay, ms_lay = _lib.prof_read(_lib.K_EDGE_LAYER)
    ndec, ms_dec = _lib.prof_read(_lib.K_DECODER)
    if nlay:
        _lib.check(_lib.load().chm_prof_reset(), "prof_reset")
        model.decoder.set_option("edge_layer", 0)
        it3 = model.sample_states(natoms, None, 2.0, 1e-5, noise="philox", seed=args.seed, text_embeds=cond,
                                  null_text_embeds=null, clone=False, node_base=node_base, graph_base=g0,
                                  init=init, t_stop=998, graph=False)
        for _ in it3:
            pass
        torch.cuda.synchronize()
        model.decoder.set_option("edge_layer", 1)
    _lib.check(_lib.load().chm_prof_enable(0), "prof_disable")
    torch.cuda.synchronize()
    events = _lib.prof_events()
    per_rank = [elapsed]
    if dist is not None:
        tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        every = [torch.zeros_like(tt) for _ in range(world)]
        dist.all_gather(every, tt)
        per_rank = [float(v.item()) for v in every]
        elapsed = max(per_rank)
        ev = torch.tensor([events[k] for k in _lib.EVENT_NAMES], device=dev, dtype=torch.float64)
        dist.all_reduce(ev)  # (summed over ranks)
        events = {k: int(v) for k, v in zip(_lib.EVENT_NAMES, ev.tolist())}
        # finished structures -> every rank (the all-gather of the sampler; outside the timed region)
        from chemeleon_amd.distributed import gather_states
        gather_states(state[1:], natoms, natoms_all=[all_nat[a:b] for a, b in ranges])

    s_per_step = elapsed / args.steps
    value = total / (s_per_step * T_STEPS)

    # live per-kernel timing (HIP events on the launch stream)
    nmsg, ms_msg = _lib.prof_read(_lib.K_EDGE_MESSAGE)
    nfou, ms_fou = _lib.prof_read(_lib.K_EDGE_FOURIER)
    E = sum(n * n for n in natoms)
    N = sum(natoms)
    msg_flops = 2.0 * (2 * E) * H * H  # one launch covers both conditionings
    msg_tflops = msg_flops / (ms_msg / nmsg * 1e-3) / 1e12 if nmsg else None
    seg_bytes = 2.0 * (E * H * 4 + N * H * 4)
    step_flops = 2 * decoder_pair_flops(natoms)
    math = model.decoder.get_math()
    Ep = sum(n * (n + 1) // 2 for n in natoms)
    fou_flops = 2.0 * (Ep if edge_pairs_on() else E) * 768 * H  # edge layer 1: D.f once for both conditionings
    # (on pairs: once per unordered pair, k_edge16_pairs)
    fou_tflops = fou_flops / (ms_fou / nfou * 1e-3) / 1e12 if nfou else None
    msg_kernel = ((pairs_layer_kernel() or "k_edge16_pairs") if edge_pairs_on() else "k_edge16_layer") if nlay \
        else "k_edge16<2"
    traffic, traffic_src = None, "not collected for the ragged workload" if args.ragged else "not collected"
    if math == "split16" and not args.ragged:
        if rank == 0 and world == 1 and not args.no_traffic:
            try:
                traffic, traffic_src = measure_traffic(args, msg_kernel)
            except Exception as e:  # noqa: BLE001
                traffic, traffic_src = None, {"error": repr(e)}
        if traffic is None and (args.n_samples, args.n_atoms, world) == (512, 40, 1):  # (the stored profile's shape)
            failed = traffic_src
            traffic, traffic_src = _stored_traffic(msg_kernel)
            if traffic_src is not None:
                traffic_src["in_run"] = failed if not args.no_traffic and world == 1 else "skipped"
    lay_flops = fou_flops + msg_flops
    lay_tflops = lay_flops / (ms_lay / nlay * 1e-3) / 1e12 if nlay else None
    # fp32-equivalent ceilings: bf16x3 = 2.5 PF / 6 products; split16 edge GEMMs = 2.5 PF (fp16 dense
    # = bf16 rate) / 3 products; f32 = the fp32 MFMA peak
    peak = {"bf16x3": BF16X3_PEAK_TFLOPS, "split16": MFMA_BF16_PEAK_TFLOPS / 3}.get(math, MFMA_F32_PEAK_TFLOPS)

    # standalone message-passing aggregation kernel (chm_segment_mean) on the
    # bench batch's edge layout, [2, E, 512] fp32 messages (HIP events)
    seg_gbs = seg_ms = None
    try:
        b = model.decoder.hip_batch(natoms, 2)
        msg = torch.empty(2, b.num_edges, H, device=dev).normal_()
        agg = torch.empty(2, b.num_nodes, H, device=dev)
        L_ = _lib.load()
        st = _lib.stream_handle(dev)
        for _ in range(2):
            _lib.check(L_.chm_segment_mean(b.handle, 2, _lib.ptr(msg), msg.numel(), _lib.ptr(agg), agg.numel(), st), "segment_mean")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            _lib.check(L_.chm_segment_mean(b.handle, 2, _lib.ptr(msg), msg.numel(), _lib.ptr(agg), agg.numel(), st), "segment_mean")
        e1.record()
        torch.cuda.synchronize()
        seg_ms = e0.elapsed_time(e1) / 10
        seg_gbs = seg_bytes / (seg_ms * 1e-3) / 1e9
        del msg, agg
    except Exception as e:  # noqa: BLE001
        print("segment_mean microbench failed:", repr(e), file=sys.stderr)

    out = {
        "metric": ("structures/sec (1000-step sample, n_atoms=40)" if not args.ragged else
                   "structures/sec (1000-step sample, natoms = randint(1, 81), SURVEY C4)"),
        "value": value,
        "unit": "structures/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": s_per_step * 1e3,
        "per_rank_ms_per_step": {"min": min(per_rank) / args.steps * 1e3, "max": max(per_rank) / args.steps * 1e3},
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": {"f32": "f32", "bf16x3": "f32 (bf16x3-split MFMA, fp32 accumulate)",
                  "split16": "f32 (fp16x2-split edge and node GEMMs with power-of-two row scales, fp32 accumulate)"}[math],
        "data": "synthetic (seeded random-init weights of the real architecture; seeded conditioning vectors)",
        "config": {"workload": f"sample n_samples={total} (x{per[rank]}/GPU) "
                               f"n_atoms={'randint(1,81) seed 7' if args.ragged else args.n_atoms}, "
                               f"T={T_STEPS}; step = one reverse timestep (4 decoder calls)",
                   "n_samples": total, "n_atoms": "ragged 1-80" if args.ragged else args.n_atoms,
                   "timesteps": T_STEPS,
                   "parallelism": f"sample-sharded x{world}",
                   "noise": ("philox (device)" if args.noise == "philox" else
                             "torch (parity mode: the reference's CPU RNG stream at the global size on every rank, "
                             "this rank's rows uploaded before each replay)"),
                   "launch": "eager" if args.no_graph else f"hip graph replay per step, {args.lanes} stream lane(s)",
                   "share": (None if share_of is None else
                             f"rank {share_of[0]}'s share of a {share_of[1]}-rank job of {share_of[2]} crystals "
                             f"({total} crystals, {sum(all_nat)} atoms, {sum(n * n for n in all_nat)} edges), run alone "
                             "on one GPU; value counts this share's structures")},
        "roofline": {"bound": "mfma",
                     "timing": ("HIP events on the launch stream, eager pass of 2 steps after the timed graph replays"
                                if not args.no_graph else "HIP events on the launch stream over warm-up + timed steps"),
                     "kernel": {"split16": ((f"both edge layers of a CSP layer in one grid, layer 1 on "
                                             f"unordered pairs ({msg_kernel}: D.f once per pair i <= j, both "
                                             "directions' S = SiLU(U +- V + P + Q); S.W2^T + SiLU + fused "
                                             "scatter_mean; 16x16x32 MFMA), both conditionings, incl. its two repair "
                                             "launches (no-ops unless a check fails)") if edge_pairs_on() else
                                            ("both edge layers of a CSP layer in one grid (k_edge16_layer: D.f + P_i + "
                                             "Q_j + SiLU -> S, S.W2^T + SiLU + fused scatter_mean; 16x16x32 MFMA), "
                                             "both conditionings, incl. its two repair launches (no-ops unless a "
                                             "check fails)")) if nlay else
                                           (f"edge message GEMM + fused scatter_mean ({msg_kernel}, EPI_SEGMEAN, "
                                            "16x16x32 MFMA), both conditionings"),
                                "bf16x3": "edge message GEMM + fused scatter_mean (k_gemm3_big<EPI_SEGMEAN>), "
                                          "both conditionings",
                                "f32": "edge message GEMM (k_gemm, S.W2^T + SiLU, both conditionings)"}[math],
                     "achieved": lay_tflops if nlay else msg_tflops, "peak": peak, "unit": "TFLOP/s",
                     "frac": ((lay_tflops if nlay else msg_tflops) / peak) if (lay_tflops or msg_tflops) else None,
                     "traffic": traffic,
                     "traffic_source": traffic_src,
                     "mfma_busy": (traffic_src.get("mfma_busy") if isinstance(traffic_src, dict) else None),
                     "mfma_busy_note": "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs), in-run PMC "
                                       "pass over the same probe as traffic",
                     "traffic_algorithmic": (edge_layer_bytes(natoms) if nlay else message_layer_bytes(natoms)),
                     "peak_note": {"bf16x3": "fp32-equivalent flops; bf16 dense MFMA 2.5 PF / 6 products",
                                   "split16": "fp32-equivalent flops (3 fp16 MFMA products each); fp16 dense MFMA "
                                           "2.5 PF / 3 products",
                                   "f32": "fp32 MFMA dense peak"}[math],
                     "flops_per_launch": lay_flops if nlay else msg_flops, "launches": nlay or nmsg,
                     "avg_ms": (ms_lay / nlay) if nlay else (ms_msg / nmsg if nmsg else None)},
        "msgpass": {"bound": "hbm", "kernel": "k_segment_mean (standalone scatter_mean, chm_segment_mean)",
                    "achieved": seg_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": (seg_gbs / HBM_PEAK_GBS) if seg_gbs else None, "bytes_per_launch": seg_bytes,
                    "avg_ms": seg_ms,
                    "note": ("in the sampler the aggregation is fused into the message GEMM epilogue; this is the "
                             "standalone kernel on the same [2,E,512] shape" if math != "f32" else
                             "the kernel as launched by the sampler")},
        "edge_layer2": {"kernel": "edge layer 2 alone (k_edge16<2>: S.W2^T + SiLU + fused scatter_mean), both "
                                  "conditionings" + (" (second eager pass, two launches per layer)" if nlay else ""),
                        "achieved": msg_tflops, "peak": peak, "unit": "TFLOP/s",
                        "frac": (msg_tflops / peak) if msg_tflops else None, "flops_per_launch": msg_flops,
                        "avg_ms": ms_msg / nmsg if nmsg else None},
        "edge_layer1": {"kernel": ("edge layer 1 on unordered pairs (k_edge16_pairs: D.f once per pair i <= j, both "
                                   "directions' S = SiLU(U +- V + P + Q) written split), both conditionings"
                                   if edge_pairs_on() else
                                   "edge layer 1 (D.f + P_i + Q_j + SiLU, S written split), both conditionings"),
                        "achieved": fou_tflops, "peak": peak, "unit": "TFLOP/s",
                        "frac": (fou_tflops / peak) if fou_tflops else None, "flops_per_launch": fou_flops,
                        "avg_ms": ms_fou / nfou if nfou else None},
        "path": {"tflops": step_flops / s_per_step / 1e12, "mfma_frac": step_flops / s_per_step / 1e12 / peak,
                 "math": math, "flops_per_step_per_gpu": step_flops,
                 "edge_fourier_avg_ms": ms_fou / nfou if nfou else None,
                 "decoder_pair_avg_ms": ms_dec / ndec if ndec else None},
        "noise_host_draw_ms": draw_ms,
        "noise_host_draw_ms_8rank_share": draw_ms_8,
        "edge_repairs": events["layer_repairs"] + events["tail_repairs"],
        "edge_events": dict(events, note="device counters over warm-up, timed and eager passes (chm_prof_events): "
                                         "repairs recompute a layer whose intra-grid check failed; 0 = none ran"),
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_api_legs and not args.ragged:
        try:
            out["api"] = api_legs(model, total, args.n_atoms, cond, null, args.seed, value)
        except Exception as e:  # noqa: BLE001
            out["api"] = {"error": repr(e)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(args.cpu_samples, args.n_atoms, args.cpu_steps)
        except Exception as e:  # noqa: BLE001
            out["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
