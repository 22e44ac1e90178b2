"""checkBsdf on the GPU (bbm_amd.check): host logic on the CPU (no GPU needed).

* the counter-based draws restated in numpy: range, 24-bit grid, shard slices;
* gamma_q (P value of the chi-square test) against the reference's util/gamma.h;
* merging per-shard accumulators (sums, first-max) and a world-size-2 gloo gather of them;
* option parsing / CLI behaviour of bin/checkBsdf.cpp:420-479;
* the CPU oracle of the statistics is sane on models with known answers (Lambertian reflectance =
  albedo, pdf integrals, chi-square P values), so the GPU tests compare against a meaningful checker.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from bbm_amd import check
from tests import check_oracle as co
from tests import oracle_util as ou

needs_ref = pytest.mark.skipif(ou.ref() is None, reason="reference shim (oracle/_ref) not built")


def test_draws_are_24bit_uniforms_and_shard_consistent():
    u = co.draws(co.REFLECTANCE, 5489, 0, 0, 0, 100_000)
    assert u.dtype == np.float32 and u.shape == (2, 100_000)
    assert u.min() >= 0 and u.max() < 1
    assert np.all((u * 16777216.0) == np.floor(u * 16777216.0))
    assert abs(u.mean() - 0.5) < 5e-3
    part = co.draws(co.REFLECTANCE, 5489, 0, 0, 40_000, 10)
    np.testing.assert_array_equal(part, u[:, 40_000:40_010])
    # streams are independent across slot / draw / test / seed
    others = [co.draws(co.REFLECTANCE, 5489, 1, 0, 0, 1000), co.draws(co.REFLECTANCE, 5489, 0, 1, 0, 1000),
              co.draws(co.PDF, 5489, 0, 0, 0, 1000), co.draws(co.REFLECTANCE, 1, 0, 0, 0, 1000)]
    for o in others:
        assert abs(np.corrcoef(o[0], u[0, :1000])[0, 1]) < 0.1


@needs_ref
@pytest.mark.parametrize("a,x", [(0.5, 0.1), (0.5, 3.0), (4.5, 2.0), (4.5, 9.0), (9.5, 12.0), (30.0, 25.0),
                                 (95.0, 110.0), (95.0, 60.0), (2.0, 0.0), (1.0, 1e-3)])
def test_gamma_q_matches_reference(a, x):
    want = co.gamma_q(a, x)
    got = check.gamma_q(a, x)
    assert abs(got - want) <= 2e-5 * max(abs(want), 1e-6) + 1e-7, (got, want)


def test_merge_acc_sums_and_first_maximum():
    a = np.zeros((2, check.ACC))
    b = np.zeros((2, check.ACC))
    a[:, :8] = 1.0
    b[:, :8] = 2.0
    a[0, 8:10] = (5.0, 10)
    b[0, 8:10] = (5.0, 3)      # tie: lower sample index wins
    a[1, 8:10] = (7.0, 1)
    b[1, 8:10] = (6.0, 0)
    a[:, 10:12] = (-1.0, 1.8e19)
    b[:, 10:12] = (2.0, 99)
    m = check.merge_acc([a, b])
    assert np.all(m[:, :8] == 3.0)
    assert tuple(m[0, 8:10]) == (5.0, 3) and tuple(m[1, 8:10]) == (7.0, 1)
    assert tuple(m[0, 10:12]) == (2.0, 99)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gather_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    acc = np.zeros((3, check.ACC))
    acc[:, :8] = rank + 1
    acc[:, 8] = [rank, 1 - rank, 4.0]
    acc[:, 9] = [10 + rank, 20 + rank, 30 + rank]
    acc[:, 10:12] = (-1.0, 1.8e19)
    merged = check._gather_acc(acc, dist)
    counts = check._sum_counts(np.full((2, 4), rank + 1, np.int64), dist)
    q.put((rank, merged, counts))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_gather_merges_like_one_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, merged, counts in res:
        assert np.all(merged[:, :8] == 3.0)
        assert merged[0, 8] == 1.0 and merged[0, 9] == 11      # rank 1 holds the larger max
        assert merged[1, 8] == 1.0 and merged[1, 9] == 20      # rank 0 holds it
        assert merged[2, 8] == 4.0 and merged[2, 9] == 30      # tie: lower index
        assert np.all(counts == 3)


def test_options_and_cli_errors(capsys):
    assert check.parse_options(["test=pdf", "samples=10", "sampleSphere"]) == \
        {"test": "pdf", "samples": "10", "sampleSphere": "true"}
    assert check.main([]) == -1
    assert check.main(["bsdfmodel=Lambertian()"]) == -1
    assert check.main(["test=nonsense"]) == 0
    assert check.main(["test=pdf", "bogus=1"]) == 0
    out = capsys.readouterr().out
    assert "ERROR: no test specified." in out and "Unrecognized test: 'nonsense'" in out
    assert "ERROR: invalid keywords: ['bogus']." in out


def test_chi2_statistic():
    pdf = np.array([0.25, 0.25, 0.25, 0.25, 0.0])
    counts = np.array([260, 240, 250, 250, 0])
    c2, df = check.chi2(pdf, counts, 1000)
    assert df == 3 and abs(c2 - (100 + 100) / 250) < 1e-12


def test_reflectance_outs_follow_reference_formula():
    o = check.reflectance_outs(4)
    assert o.dtype == np.float32 and o.shape == (3, 4)
    np.testing.assert_allclose(o[2], np.cos(np.arange(4) * np.pi / 8), atol=1e-7)
    assert np.all(o[1] == 0)


@needs_ref
def test_oracle_statistics_are_sane():
    lam = [0.5, 0.5, 0.5]
    # Lambertian: MC reflectance -> albedo (sphere sampling and importance sampling)
    e = co.reflectance("Lambertian", lam, [0, 0, 1], 200_000, 5489, 0, importance=False)
    assert abs(e[0] / 200_000 - 0.5) < 0.01
    e = co.reflectance("Lambertian", lam, [0, 0, 1], 50_000, 5489, 0, importance=True)
    assert abs(e[0] / 50_000 - 0.5) < 1e-3
    # reciprocity of a reciprocal model: round-off only
    s, h, k = co.symmetry("Lambertian", lam, 10_000, 5489, co.RECIPROCITY)
    assert s.max() == 0.0 and h == 0.0
    # pdfInt: Lambertian integrates to 1 over the sphere
    t = co.trial_dirs(co.PDFINT, 5489, 2)
    v = co.pdf_int("Lambertian", lam, t[:, 0], 200_000, 5489, 0) / 200_000
    assert abs(v - 1.0) < 0.02
    # chi-square: cosine sampling against its own pdf is accepted
    t = co.trial_dirs(co.SAMPLE_COUNT, 5489, 1)
    th, ph = 5, 8
    pdf = co.sample_pdf("Lambertian", lam, t[:, 0], 0, th * ph, 512, 5489, th, ph) / 512
    cnt = co.sample_count("Lambertian", lam, t[:, 0], 0, 20_000, 5489, th, ph)
    c2, df = check.chi2(pdf, cnt, 20_000)
    assert check.gamma_q((df - 1) / 2, c2 / 2) > 1e-3
