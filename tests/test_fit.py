"""Fitting path, host side (CPU only: no kernel runs).

* the batched compass (bbm_amd.fit.Compass) reproduces the reference's compass search
  (include/optimizer/compass.h:82-140) step for step when scored with the reference's own loss
  values: identical parameter vectors (bit for bit) and losses after every step;
* the golden fixtures themselves are the reference's (re-checked against the live shim when present);
* sharding of the sample grid and the cross-rank reduction (gloo, world size 2): every rank takes
  the same compass decisions as a single process.
"""
import os

import numpy as np
import pytest

from tests import oracle_util as ou

META_FIT, FIT = ou.golden_fit()


def _model(name, params=None):
    import bbm_amd
    m = bbm_amd.BsdfModel(name)
    if params is not None:
        m.set_parameter_values(params)
    return m


def test_golden_fit_fixtures_are_the_references():
    """Regenerating a few fixture values with the live reference shim gives identical numbers."""
    if ou.ref() is None:
        pytest.skip("reference shim not built")
    for key, total in list(META_FIT["loss"].items())[:4]:
        name, grid, kind = key.rsplit("_", 2)
        kind = int(kind.replace("loss", ""))
        got = ou.ref_loss_total(name, FIT[f"{name}_fitted"], FIT[f"{name}_reference"], META_FIT["grids"][grid], kind)
        assert got == np.float32(total), key


@pytest.mark.parametrize("ci", range(len(META_FIT["compass"])))
def test_compass_matches_reference_trajectory(ci):
    """Host compass logic + the reference's loss values == the reference compass, bit for bit."""
    if ou.ref() is None:
        pytest.skip("reference shim not built")
    from bbm_amd import fit
    run = META_FIT["compass"][ci]
    name, grid = run["model"], META_FIT["grids"][run["grid"]]
    model = _model(name)
    loss = ou.RefTotalLoss(model, FIT[f"{name}_reference"], grid, run["loss"])
    opt = fit.Compass(loss, model)
    assert len(opt.idx) == run["nopt"]
    assert opt.loss_value == np.float32(run["loss0"])
    ref_params, ref_loss = FIT[f"compass{ci}_params"], FIT[f"compass{ci}_loss"]
    for t in range(run["steps"]):
        e = opt.step()
        np.testing.assert_array_equal(model.parameter_values(fit.ALL), ref_params[t], err_msg=f"step {t}")
        assert e == ref_loss[t], f"step {t}: {e} vs {ref_loss[t]}"
    # one batched scoring call per step (plus the initial loss), instead of 2P serial loss passes
    assert loss.calls == run["steps"] + 1


def test_shard_ranges_partition_the_grid():
    from bbm_amd.fit import shard_range
    for total in (0, 1, 7, 1_458_000):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(e - b for b, e in spans) - min(e - b for b, e in spans) <= 1


class _OracleShardLoss:
    """SampledLoss with the GPU launch replaced by the reference's per-sample losses on this rank's
    shard of a golden grid (double sums); the cross-rank reduction is SampledLoss's own."""

    def __init__(self, fitted, reference, grid_name, loss_kind, dist):
        from bbm_amd import fit
        import torch
        self.fitted, self.reference, self.loss_kind, self.dist = fitted, reference, loss_kind, dist
        d = FIT[f"{grid_name}_dirs"]
        self.total = d.shape[1]
        rank, world = (dist.get_rank(), dist.get_world_size()) if dist else (0, 1)
        b, e = fit.shard_range(self.total, rank, world)
        self.din, self.dout = d[:3, b:e], d[3:, b:e]
        self._torch = torch
        self.probe_sums = fit.SampledLoss.probe_sums.__get__(self)
        self.probe_losses = fit.SampledLoss.probe_losses.__get__(self)
        self.__call__ = fit.SampledLoss.__call__.__get__(self)

    def update(self):
        pass

    def local_sums(self, probes):
        s = [np.sum(ou.ref_pair_losses(self.fitted.name, p, self.reference, self.din, self.dout, self.loss_kind),
                    dtype=np.float64) for p in np.asarray(probes, np.float32)]
        return self._torch.tensor(s, dtype=self._torch.float64)

    def __call__(self, params=None):
        p = self.fitted._params if params is None else params
        return float(self.probe_losses(np.asarray(p, np.float32)[None])[0])


def _trajectory(loss, model, steps):
    from bbm_amd import fit
    opt = fit.Compass(loss, model)
    out = []
    for _ in range(steps):
        opt.step()
        out.append(model.parameter_values(fit.ALL).copy())
    return np.stack(out)


def _dist_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        name = "Aggregate<Lambertian,CookTorrance>"
        model = _model(name)
        loss = _OracleShardLoss(model, FIT[f"{name}_reference"], "grid0", 3, dist)
        q.put((rank, _trajectory(loss, model, 6)))
    finally:
        dist.destroy_process_group()


def test_sharded_compass_two_ranks_gloo():
    """World size 2 (gloo): each rank scores its half of the grid, the sums are all-reduced, and both
    ranks follow the single-process trajectory."""
    if ou.ref() is None:
        pytest.skip("reference shim not built")
    import multiprocessing as mp
    import socket
    name = "Aggregate<Lambertian,CookTorrance>"
    model = _model(name)
    single = _trajectory(_OracleShardLoss(model, FIT[f"{name}_reference"], "grid0", 3, None), model, 6)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dist_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    import queue
    import time
    t0 = time.time()
    while len(res) < len(procs):
        try:
            r, v = q.get(timeout=2)
            res[r] = v
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            assert not dead, f"a rank died (exit codes {dead})"
            assert time.time() - t0 < 300, "ranks did not finish"

    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    np.testing.assert_array_equal(res[0], res[1])
    np.testing.assert_array_equal(res[0], single)


def _pairs_dist_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    from bbm_amd import fit
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 5 + 3 * rank                                  # ranks hold different numbers of their own pairs
        d = torch.zeros((3, n), dtype=torch.float32)
        loss = fit.SampledLoss(_model("Aggregate<Lambertian,CookTorrance>"), torch.zeros((3, n)), "standardLog",
                               pairs=(d, d), dist=dist)
        # stand-in for the device launch: every local sample contributes 1 to each probe's sum
        loss.local_sums = lambda probes: torch.full((len(probes),), float(n), dtype=torch.float64)
        q.put((rank, loss.total, loss.begin, loss.n, loss.probe_losses(np.zeros((2, 4), np.float32)).tolist()))
    finally:
        dist.destroy_process_group()


def test_own_pairs_two_ranks_gloo():
    """SampledLoss(pairs=..., dist=...) with world size 2 (gloo): each rank's own pairs are its part of the grid, so
    total is the sum of the ranks' counts, begin the lower ranks' count, and the mean loss divides the all-reduced
    sums by that total (a mean of 1 per sample stays 1)."""
    import multiprocessing as mp
    import queue
    import socket
    import time
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_pairs_dist_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res, t0 = {}, time.time()
    while len(res) < len(procs):
        try:
            r = q.get(timeout=2)
            res[r[0]] = r[1:]
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            assert not dead, f"a rank died (exit codes {dead})"
            assert time.time() - t0 < 300, "ranks did not finish"
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][:3] == (13, 0, 5) and res[1][:3] == (13, 5, 8)
    assert res[0][3] == res[1][3] == [1.0, 1.0]
