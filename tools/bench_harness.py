"""Process launch, rendezvous and timing shared by bench.py and tools/bench_configs.py.

bench.py contract: `python bench.py --gpus N ...` runs N ranks (one process per GPU).  Under torchrun the
environment (WORLD_SIZE / RANK / LOCAL_RANK / MASTER_*) says so; started by hand with --gpus N > 1 and no
WORLD_SIZE, `launch()` starts `python -m torch.distributed.run --nproc-per-node N` on the same command line
as a child process (this process never touches the GPU) and exits with its status.

Timing: W warmup steps, an untimed settle period, then barrier + device synchronize, K timed steps, device
synchronize + barrier; each rank's wall time is gathered, the slowest rank's time is the job's time.
"""
import os
import socket
import subprocess
import sys
import time

import numpy as np


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def needs_launch(gpus):
    return gpus is not None and gpus > 1 and "WORLD_SIZE" not in os.environ


def launch(gpus, script, argv):
    """Run `script argv` as `gpus` torchrun ranks (child process); returns its exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", script] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def world_from_env(gpus):
    """(world, rank, local_rank); refuses a --gpus that disagrees with the launcher's WORLD_SIZE."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if gpus is not None and gpus != world:
        raise SystemExit(f"bench: --gpus {gpus} but the launcher started WORLD_SIZE={world} ranks")
    return world, rank, local


def init(world, local, backend):
    """Process group for world > 1 (RCCL over xGMI for the GPU workloads, gloo for the CPU self-test)."""
    if world == 1:
        return None
    import torch
    import torch.distributed as dist
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group("gloo")
    seen = dist.get_world_size()
    if seen != world:
        raise SystemExit(f"bench: process group has {seen} ranks, WORLD_SIZE says {world}")
    return dist


def shard(total_or_per_rank, rank, world, scaling):
    """(begin, count) of this rank's contiguous slice.  weak: every rank owns `per_rank` units of the global
    batch [0, world*per_rank); strong: the fixed total is split as evenly as possible."""
    if scaling == "weak":
        return rank * total_or_per_rank, total_or_per_rank
    base, extra = divmod(total_or_per_rank, world)
    begin = rank * base + min(rank, extra)
    return begin, base + (1 if rank < extra else 0)


def timed(step, args, dist, stream=None, gpu=True):
    """Returns (elapsed_s of the slowest rank, mean kernel ms (HIP events on `stream`; slowest rank),
    per-rank elapsed list, untimed settle steps)."""
    sync = (lambda: __import__("torch").cuda.synchronize()) if gpu else (lambda: None)
    for _ in range(args.warmup):
        step()
    sync()
    settle = 0
    tw = time.perf_counter()
    while time.perf_counter() - tw < args.settle_s:
        for _ in range(10):
            step()
        settle += 10
        sync()
    ev = None
    if gpu:
        import torch
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if dist:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for k in range(args.steps):
        if ev:
            ev[k][0].record(stream)
        step()
        if ev:
            ev[k][1].record(stream)
    sync()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev])) if ev else elapsed * 1e3 / max(args.steps, 1)
    per_rank = [elapsed]
    if dist:
        import torch
        dev = torch.device("cuda", torch.cuda.current_device()) if gpu else torch.device("cpu")
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        allt = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(allt, t)
        per_rank = [float(x[0]) for x in allt]
        elapsed = max(per_rank)
        kern_ms = max(float(x[1]) for x in allt)
    return elapsed, kern_ms, per_rank, settle


def graph_reps(steps, cap=20):
    """R = the largest divisor of K (= steps) not above `cap`: K/R replays of an R-launch graph time exactly K steps."""
    return max(r for r in range(1, min(cap, max(steps, 1)) + 1) if steps % r == 0)


def capture(launch, reps):
    """A HIP graph of `reps` calls of launch(stream), captured on a side stream after one warm-up call (first-use
    host work happens outside the capture)."""
    import torch
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        launch(side)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s = torch.cuda.current_stream()
        for _ in range(reps):
            launch(s)
    torch.cuda.synchronize()
    return g


def cpu_topology():
    """(affinity threads, physical cores among them, SMT threads per core, cgroup CPU quota or None, model)."""
    aff = sorted(os.sched_getaffinity(0))
    cores, model = set(), ""
    cur = {}
    try:
        with open("/proc/cpuinfo") as f:
            for line in list(f) + ["\n"]:
                if not line.strip():
                    if cur.get("processor") is not None and int(cur["processor"]) in aff:
                        cores.add((cur.get("physical id", "0"), cur.get("core id", cur["processor"])))
                    cur = {}
                    continue
                k, _, v = line.partition(":")
                cur[k.strip()] = v.strip()
                if k.strip() == "model name" and not model:
                    model = v.strip()
    except OSError:
        pass
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()
            if q != "max":
                quota = float(q) / float(p)
    except (OSError, ValueError):
        pass
    phys = len(cores) or len(aff)
    return len(aff), phys, max(1, len(aff) // phys), quota, model
