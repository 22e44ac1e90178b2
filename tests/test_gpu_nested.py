"""Nested aggregates on the GPU: aggregatemodel<aggregatemodel<...>, ...> (aggregatemodel_base takes any bsdfmodel
child, include/bsdfmodel/aggregatemodel.h:22, another aggregate included) through the composed path
(bbm_hip_aggregate_* with BBM_HIP_AGGREGATE children, bbm_amd.AggregateModel of AggregateModels), against the
reference's own nested aggregate types instantiated in oracle/_ref (ref_fit.cpp: nested1_t .. nested3_t), in
floatRGB (per-lane bar and proofs of tests/test_gpu_parity.py) and doubleRGB (the f64 bar of test_gpu_f64.py); plus
the flat composed aggregates in doubleRGB (bbm_hip_aggregate_*_f64)."""
import numpy as np
import pytest

from tests import oracle_util as ou
from tests import test_gpu_parity as tp
from tests import test_gpu_f64 as tf

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

INP = ou.golden_inputs()
NESTED = ["Aggregate<Aggregate<Lambertian,Ward>,GGX>", "Aggregate<Aggregate<Lambertian,CookTorrance>,Ward>",
          "Aggregate<GGX,Aggregate<Phong,Aggregate<Ward,OrenNayar>>>"]
FLAT_F64 = ["Aggregate<CookTorrance,GGX>", "Aggregate<Lambertian,CookTorrance,GGX>"]


@pytest.fixture(scope="module")
def bbm():
    import bbm_amd
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    torch.cuda.set_device(0)
    return bbm_amd


def parse_key(key):
    """'Aggregate<A,Aggregate<B,C>>' -> ('Aggregate', [A, ('Aggregate', [B, C])])."""
    def node(i):
        j = i
        while j < len(key) and key[j] not in "<,>":
            j += 1
        name = key[i:j]
        if j < len(key) and key[j] == "<":
            kids, j = [], j + 1
            while True:
                k, j = node(j)
                kids.append(k)
                if key[j] == ",":
                    j += 1
                    continue
                return (name, kids), j + 1
        return name, j
    t, end = node(0)
    assert end == len(key), key
    return t


def build(bbm, key, params):
    """The model of `key` with the flat parameter vector `params` (leaves in base-class order), composed through
    bbm.Aggregate exactly as fromString would (a fused Aggregate(Lambertian, X) stays fused)."""
    params = np.asarray(params, np.float32)
    pos = [0]

    def make(t):
        if isinstance(t, str):
            m = bbm.BsdfModel(t)
            n = m.parameter_values().size
            m.set_parameter_values(params[pos[0]:pos[0] + n])
            pos[0] += n
            return m
        return bbm.Aggregate(*[make(k) for k in t[1]])
    m = make(parse_key(key))
    assert pos[0] == params.size
    return m


def param_sets(key):
    p0 = np.asarray(ou.ref_default_params(key), np.float32)
    return [p0, (p0 * np.float32(0.875)).astype(np.float32)]


def test_nested_models_are_nested(bbm):
    m = build(bbm, NESTED[0], param_sets(NESTED[0])[0])
    assert isinstance(m, bbm.AggregateModel) and isinstance(m._children[0], bbm.AggregateModel)
    m = build(bbm, NESTED[1], param_sets(NESTED[1])[0])
    assert isinstance(m._children[0], bbm.BsdfModel) and m._children[0].name == "Aggregate<Lambertian,CookTorrance>"
    m = build(bbm, NESTED[2], param_sets(NESTED[2])[0])
    assert isinstance(m._children[1]._children[1], bbm.AggregateModel)


@pytest.mark.parametrize("key", NESTED)
def test_nested_eval_pdf_reflectance_vs_reference(bbm, key):
    n = 1 << 20
    batches = [(INP["pin"], INP["pout"])]
    for mi, mo in ((0, 1), (0, 0)):
        batches.append((bbm.fill_directions(0xBB5EED, 0, 0, n, mode=mi).cpu().numpy(),
                        bbm.fill_directions(0xBB5EED, 1, 0, n, mode=mo).cpu().numpy()))
    stats = {}
    for si, params in enumerate(param_sets(key)):
        m = build(bbm, key, params)
        for bi, (din, dout) in enumerate(batches):
            got = tp._gpu_evalpdf(m, din, dout)
            ref = ou.oracle_eval_pdf(key, params, din, dout, nthreads=8)
            stats[f"[{si}] batch{bi}"] = tp.check_lanes(got, ref, f"{key}[{si}] batch{bi}",
                                                        tp._evalpdf_provers(bbm, key, params, din, dout, got))
        refl = m.reflectance(tp._dev(INP["sout"])).cpu().numpy()
        tp.check_lanes(refl, ou.ref_reflectance(key, params, INP["sout"]), f"{key}[{si}] reflectance",
                       [tp._input_ulps_prover(lambda o, p=params: ou.ref_reflectance(key, p, o), [INP["sout"]], refl)])
    tp._report("nested_" + key.replace("<", "_").replace(">", "").replace(",", "_"), stats)


@pytest.mark.parametrize("key", NESTED)
def test_nested_sample_vs_reference(bbm, key):
    n = 1 << 18
    out = bbm.fill_directions(0xBB5EED, 2, 0, n, mode=1)
    xi = torch.rand((2, n), generator=torch.Generator(device="cuda").manual_seed(5), device="cuda")
    for sout, sxi in ((INP["sout"], INP["sxi"]), (out.cpu().numpy(), xi.cpu().numpy())):
        for params in param_sets(key):
            m = build(bbm, key, params)
            got, flag = tp._gpu_sample(m, sout, sxi)
            ref, rflag = ou.oracle_sample(key, params, sout, sxi, nthreads=8)
            tp._check_samples(bbm, key, params, sout, sxi, got, flag, ref, rflag, key)


@pytest.mark.parametrize("key", NESTED + FLAT_F64)
def test_composed_f64_vs_reference(bbm, key):
    """doubleRGB composed aggregates (bbm_hip_aggregate_*_f64), flat and nested, against the reference's doubleRGB
    aggregate of the same type: eval / pdf on 1M pairs, reflectance, sample."""
    n = 1 << 20
    din = bbm.fill_directions(0xBB5EED, 0, 0, n, mode=0).cpu().numpy()
    dout = bbm.fill_directions(0xBB5EED, 1, 0, n, mode=1).cpu().numpy()
    params = param_sets(key)[1]
    if key in FLAT_F64:
        kids = key[len("Aggregate<"):-1].split(",")
        ms, k = [], 0
        for nm in kids:
            c = bbm.BsdfModel(nm)
            c.set_parameter_values(params[k:k + c._params.size])
            k += c._params.size
            ms.append(c)
        m = bbm.Aggregate(*ms, fused=False)
    else:
        m = build(bbm, key, params)
    assert isinstance(m, bbm.AggregateModel) and m.has_f64()
    got = tf._gpu(m, din, dout)
    ref = ou.ref_eval_pdf_double(key, params, din, dout, nthreads=8)
    st = tf._check(got, ref, f"{key} f64", lambda a, b: ou.ref_eval_pdf_double(key, params, a, b, nthreads=8),
                   [din, dout])
    refl = m.reflectance(tf._d(INP["sout"])).cpu().numpy()
    rref = ou.ref_reflectance_double(key, params, INP["sout"])
    tf._check(refl, rref, f"{key} f64 reflectance")
    s = m.sample(tf._d(INP["sout"]), tf._d(INP["sxi"]))
    torch.cuda.synchronize()
    sdir, spdf, sflag = ou.ref_sample_double(key, params, INP["sout"], INP["sxi"], nthreads=8)
    assert np.array_equal(s.flag.cpu().numpy().astype(np.uint32), np.asarray(sflag).astype(np.uint32))
    d = s.direction.cpu().numpy()
    assert np.nanmax(np.abs(d - sdir)) <= 1e-9, np.nanmax(np.abs(d - sdir))
    tf._check(s.pdf.cpu().numpy()[None], spdf[None], f"{key} f64 sample pdf")
    tf._report("composed_" + key.replace("<", "_").replace(">", "").replace(",", "_"), st)


def test_nested_scratch_stays_bounded(bbm):
    """The scratch pool serves nested composed calls and returns its idle blocks on trim."""
    key = NESTED[2]
    m = build(bbm, key, param_sets(key)[0])
    din = bbm.fill_directions(3, 0, 0, 1 << 20, mode=1)
    dout = bbm.fill_directions(3, 1, 0, 1 << 20, mode=1)
    for _ in range(3):
        m.eval_pdf(din, dout)
    torch.cuda.synchronize()
    held = bbm.scratch_bytes()
    assert held > 0
    freed = bbm.scratch_trim()
    assert freed == held and bbm.scratch_bytes() == 0
    rgb, pdf = m.eval_pdf(din, dout)          # the pool refills on demand
    torch.cuda.synchronize()
    assert torch.isfinite(pdf).all()
