"""The reference's RUNTIME aggregate on the GPU: bbm::aggregatebsdf (include/bbm/aggregatebsdf.h:40-190), what
fromString<bsdf_ptr> / bsdf_import -- and so checkBsdf, plotBsdf and the Mitsuba plugin -- build from
"Aggregate(...)" (bsdf_string_convert.h:59).  Its eval / reflectance are left folds from 0, its pdf adds
w_k pdf_k / sum term by term, and it returns no sample where the weights sum to <= eps; aggregatemodel (the
template type) right-folds, divides the inner product once and samples anyway.  bbm_amd.fromString gives both the
fused Aggregate(Lambertian, X) kernels (BBM_HIP_RUNTIME_AGGREGATE) and the composed path (BBM_HIP_AGGREGATE_BSDF
nodes) these semantics; the reference side is the reference's own bsdf_ptr / aggregatebsdf objects built from the
same tree (oracle/ref_runtime.cpp), in floatRGB (per-lane bar and proofs of tests/test_gpu_parity.py) and
doubleRGB (the f64 bar of tests/test_gpu_f64.py)."""
import numpy as np
import pytest

from tests import oracle_util as ou
from tests import test_gpu_parity as tp
from tests import test_gpu_f64 as tf

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

INP = ou.golden_inputs()
# (string, tree) -- a fused two-child form, a three-child composed one, a nested one with a fused child
STRINGS = {
    "fused_ct": "Aggregate(Lambertian(albedo = [0.2, 0.3, 0.4]), CookTorrance(albedo = [0.6, 0.5, 0.4], roughness = 0.25, eta = 1.6))",
    "fused_bagher": None,      # filled from fits/bagher_sgd.fit (alum-bronze) below
    "three": "Aggregate(Lambertian(albedo = [0.2, 0.3, 0.4]), CookTorrance(roughness = 0.3), GGX(roughness = 0.15))",
    "nested": "Aggregate(Aggregate(Lambertian(albedo = [0.25, 0.25, 0.25]), Ward(roughness = [0.2, 0.3])), "
              "Aggregate(Lambertian(albedo = [0.1, 0.2, 0.1]), GGX(roughness = 0.2)), OrenNayar)",
}


@pytest.fixture(scope="module")
def bbm():
    import bbm_amd
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    torch.cuda.set_device(0)
    if ou.ref() is None:
        pytest.skip("oracle/_ref not built")
    import json
    import os
    with open(os.path.join(ou.ROOT, "tests", "golden", "fits.json")) as f:
        rows = json.load(f)["bagher_sgd.fit"]
    STRINGS["fused_bagher"] = next(r[1] for r in rows if r[0] == "alum-bronze")
    return bbm_amd


def tree_of(m):
    """The oracle tree (oracle_util.runtime_tree) of a bbm_amd model built by fromString."""
    import bbm_amd
    if isinstance(m, bbm_amd.AggregateModel):
        assert m.runtime
        return ("Aggregate", [tree_of(c) for c in m._children])
    if m.name.startswith("Aggregate<"):
        assert m.runtime
        return ou.runtime_fit_tree(m.name, m.parameter_values())
    return (m.name, m.parameter_values())


def _claimed(tree, sout, sxi):
    """Lanes where aggregatebsdf::sample (aggregatebsdf.h:122-137) hands xi to some child, recursively: x = xi0 * sum
    is claimed by the last child k with 0 <= x - (w_0 + .. + w_{k-1}) <= w_k, all in float32 as the reference does.
    Elsewhere (xi0 outside [0, 1], or the running residual rounding past the last weight) the reference's BsdfSample
    keeps its uninitialised direction and flag -- indeterminate, like the sum <= eps bail-out."""
    f = np.float32
    if tree[0] != "Aggregate":
        return np.ones(sout.shape[1], bool)
    w = []
    for k in tree[1]:
        r = ou.ref_runtime_reflectance(k, sout)
        w.append((r[0] + r[1]) + r[2])
    total = f(0)
    for wk in w:
        total = total + wk
    x = sxi[0].astype(f) * total
    claimed = np.zeros(sout.shape[1], bool)
    nxs = np.zeros(sout.shape[1], f)
    pick = np.full(sout.shape[1], -1)
    for i, wk in enumerate(w):
        m = (x >= 0) & (x <= wk)
        with np.errstate(divide="ignore", invalid="ignore"):
            nx = np.where(wk > np.finfo(f).eps, x / wk, f(0)).astype(f)
        pick = np.where(m, i, pick)
        nxs = np.where(m, nx, nxs)
        x = (x - wk).astype(f)
    for i, k in enumerate(tree[1]):
        lanes = pick == i
        if lanes.any():
            sub = _claimed(k, sout[:, lanes], np.stack([nxs[lanes], sxi[1][lanes]]))
            claimed[np.nonzero(lanes)[0][sub]] = True
    return claimed


def _batches(bbm):
    n = 1 << 20
    out = [(INP["pin"], INP["pout"])]
    for mi, mo in ((0, 0), (0, 1)):
        out.append((bbm.fill_directions(0xBB5EED, 0, 0, n, mode=mi).cpu().numpy(),
                    bbm.fill_directions(0xBB5EED, 1, 0, n, mode=mo).cpu().numpy()))
    return out


def test_fromstring_builds_runtime_aggregates(bbm):
    m = bbm.fromString(STRINGS["fused_ct"])
    assert isinstance(m, bbm.BsdfModel) and m.runtime and m.name == "Aggregate<Lambertian,CookTorrance>"
    assert not bbm.Aggregate(bbm.Lambertian(), bbm.CookTorrance()).runtime
    m = bbm.fromString(STRINGS["nested"])
    assert isinstance(m, bbm.AggregateModel) and m.runtime
    assert m._children[0].runtime and m._children[1].runtime and m._children[1].name == "Aggregate<Lambertian,GGX>"


@pytest.mark.parametrize("key", ["fused_ct", "fused_bagher", "three", "nested"])
def test_runtime_eval_pdf_reflectance_vs_reference(bbm, key):
    m = bbm.fromString(STRINGS[key])
    tree = tree_of(m)
    stats = {}
    for bi, (din, dout) in enumerate(_batches(bbm)):
        got = tp._gpu_evalpdf(m, din, dout)
        ref = ou.ref_runtime_eval_pdf(tree, din, dout)
        provers = [tp._input_ulps_prover(lambda a, b: ou.ref_runtime_eval_pdf(tree, a, b), [din, dout], got),
                   tp._libm_prover(lambda a, b: ou.ref_runtime_eval_pdf(tree, a, b, nthreads=1), [din, dout], got)]
        stats[f"batch{bi}"] = tp.check_lanes(got, ref, f"runtime {key} batch{bi}", provers, model=m.name)
    sout = INP["sout"]
    refl = m.reflectance(tp._dev(sout)).cpu().numpy()
    tp.check_lanes(refl, ou.ref_runtime_reflectance(tree, sout), f"runtime {key} reflectance",
                   [tp._input_ulps_prover(lambda o: ou.ref_runtime_reflectance(tree, o), [sout], refl)], model=m.name)
    tp._report(f"runtime_{key}", stats)


@pytest.mark.parametrize("key", ["fused_ct", "three", "nested"])
def test_runtime_sample_vs_reference(bbm, key):
    """Flags identical; directions within the bar (or reproduced by the reference at xi moved by <= 2 float steps);
    the sample's pdf against the reference's runtime pdf at the GPU's direction.  Lanes where the weights sum to
    <= eps, or whose xi0 no child claims (_claimed), get no sample from the reference (an indeterminate BsdfSample):
    there the GPU must return direction 0 and flag None."""
    m = bbm.fromString(STRINGS[key])
    tree = tree_of(m)
    n = 1 << 18
    out = bbm.fill_directions(0xBB5EED, 2, 0, n, mode=1).cpu().numpy()
    xi = torch.rand((2, n), generator=torch.Generator(device="cuda").manual_seed(7), device="cuda").cpu().numpy()
    for sout, sxi in ((INP["sout"], INP["sxi"]), (out, xi)):
        got, flag = tp._gpu_sample(m, sout, sxi)
        ref, rflag = ou.ref_runtime_sample(tree, sout, sxi)
        w = ou.ref_runtime_reflectance(tree, sout)
        wsum = ((np.float32(0) + w[0]) + w[1]) + w[2]
        live = wsum > np.finfo(np.float32).eps
        assert np.all(flag[~live] == 0) and np.all(got[:, ~live] == 0)
        unclaimed = live & ~_claimed(tree, sout, sxi)
        assert np.all(flag[unclaimed] == 0) and np.all(got[:3, unclaimed] == 0), f"{key}: unclaimed lanes"
        live &= ~unclaimed
        assert np.array_equal(flag[live].astype(np.uint32), rflag[live]), f"{key}: flags"
        dok = tp._dir_ok(got[:3, live], ref[:3, live])
        bad = np.nonzero(live)[0][~dok]
        if bad.size:
            def ref_dir(o, x):
                d, _ = ou.ref_runtime_sample(tree, o, x)
                return d[:3]
            p = ou.explained_by_input_ulps(ref_dir, [sout[:, bad], sxi[:, bad]], got[:3, bad], k=2)
            assert p.all(), f"{key}: {int((~p).sum())} sample directions outside the bar, lanes {bad[~p][:4]}"
        lanes = np.nonzero(live & (flag != 0))[0]
        pref = ou.ref_runtime_eval_pdf(tree, got[:3, lanes], sout[:, lanes])[3:]
        tp.check_lanes(got[3:, lanes], pref, f"runtime {key} sample pdf",
                       [tp._input_ulps_prover(lambda a, b: ou.ref_runtime_eval_pdf(tree, a, b)[3:],
                                              [got[:3, lanes], sout[:, lanes]], got[3:, lanes])], model=m.name)


@pytest.mark.parametrize("key", ["fused_ct", "three", "nested"])
def test_runtime_f64_vs_reference(bbm, key):
    """doubleRGB: the same strings' models on float64 tensors (fused runtime kernels and composed
    BBM_HIP_AGGREGATE_BSDF nodes in f64) against the reference's doubleRGB aggregatebsdf."""
    m = bbm.fromString(STRINGS[key])
    tree = tree_of(m)
    n = 1 << 20
    din = bbm.fill_directions(0xBB5EED, 0, 0, n, mode=0).cpu().numpy()
    dout = bbm.fill_directions(0xBB5EED, 1, 0, n, mode=1).cpu().numpy()
    got = tf._gpu(m, din, dout)
    ref = ou.ref_runtime_eval_pdf(tree, din.astype(np.float64), dout.astype(np.float64), f64=True)
    tf._check(got, ref, f"runtime {key} f64",
              lambda a, b: ou.ref_runtime_eval_pdf(tree, a, b, f64=True), [din.astype(np.float64), dout.astype(np.float64)])


def test_runtime_differs_from_aggregatemodel_where_the_reference_does(bbm):
    """The two semantics are not interchangeable: on the three-child string the reference's aggregatebsdf and
    aggregatemodel differ in the last bit of eval or pdf on many lanes, and the GPU follows each one exactly as
    often as the oracle of that kind (checked lane by lane above); here: the runtime model is not the template one."""
    m = bbm.fromString(STRINGS["three"])
    kids = [bbm.BsdfModel(c.name) for c in m._children]
    for k, c in zip(kids, m._children):
        k.set_parameter_values(c.parameter_values())
    t = bbm.Aggregate(*kids)
    assert isinstance(t, bbm.AggregateModel) and not t.runtime
    din, dout = INP["pin"], INP["pout"]
    a, b = tp._gpu_evalpdf(m, din, dout), tp._gpu_evalpdf(t, din, dout)
    ra = ou.ref_runtime_eval_pdf(tree_of(m), din, dout)
    assert np.mean(a == ra) >= np.mean(b == ra)
