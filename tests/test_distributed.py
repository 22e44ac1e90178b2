"""Multi-process path on CPU (gloo, world_size 2): sharding + cross-rank reduction.

The GPU bench shards a global batch by contiguous index ranges, regenerates each shard from
(seed, global index) and reduces only scalars.  Here the same partitioning runs with the oracle
as the per-rank compute on the CPU, and the all-reduced checksum must equal the single-process one.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from bbm_amd.shard import shard_range, weak_range

N_GLOBAL = 20_011
SEED = 77


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _checksum(begin, end):
    from tests import oracle_util as ou
    din = ou.dirgen_numpy(SEED, 0, begin, end - begin, mode=1)
    dout = ou.dirgen_numpy(SEED, 1, begin, end - begin, mode=1)
    r = ou.port_eval_pdf("CookTorrance", [0.5, 0.5, 0.5, 0.2, 1.5], din, dout)
    r = np.where(np.isfinite(r), r, 0.0)
    return np.array([r[:3].astype(np.float64).sum(), r[3].astype(np.float64).sum(), float(end - begin)])


def _worker(rank, world, port, out_q, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if mode == "strong":
        b, e = shard_range(N_GLOBAL, rank, world)
    else:
        b, e = weak_range(N_GLOBAL // world, rank)
    t = torch.tensor(_checksum(b, e), dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    mx = torch.tensor([float(rank)], dtype=torch.float64)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)      # bench.py's max-over-ranks timing reduction
    if rank == 0:
        out_q.put((t.numpy().tolist(), float(mx[0])))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_ranges_partition():
    for n in (0, 1, 7, 100, 20_011):
        for w in (1, 2, 3, 8):
            r = [shard_range(n, k, w) for k in range(w)]
            assert r[0][0] == 0 and r[-1][1] == n
            assert all(r[k][1] == r[k + 1][0] for k in range(w - 1))
            assert max(e - b for b, e in r) - min(e - b for b, e in r) <= 1
    assert weak_range(10, 3) == (30, 40)
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


@pytest.mark.parametrize("mode", ["strong", "weak"])
def test_two_rank_gloo_reduction_matches_single_process(mode):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    res, mx = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = N_GLOBAL if mode == "strong" else (N_GLOBAL // world) * world
    ref = _checksum(0, n)
    np.testing.assert_allclose(res, ref, rtol=1e-12)
    assert mx == world - 1
