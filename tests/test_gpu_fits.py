"""Every published material on the GPU: each line of each fits/*.fit (1 302 fitted Aggregate(Lambertian, X)
materials, tests/golden/fits.json) parsed by bbm_amd.fromString and evaluated on the golden direction set
(1 024 hemisphere + 256 sphere pairs + 33 edge cases) through its fused kernel, against the reference itself
(oracle/_ref: what the reference's bsdf_import builds from that line -- the runtime aggregatebsdf of bsdf_ptrs to
lambertian and X at those parameters, oracle/ref_runtime.cpp) -- eval + pdf and reflectance, under the per-lane
gate and proofs of tests/test_gpu_parity.py.  fromString gives the fused kernel the runtime aggregate's semantics
(BBM_HIP_RUNTIME_AGGREGATE): its pdf adds w_k pdf_k / sum term by term where aggregatemodel divides the inner
product.  The golden fixtures pin 3-4
parameter sets per model; this is the parameter space the library is actually used with."""
import json
import os

import numpy as np
import pytest

from tests import oracle_util as ou
from tests import test_gpu_parity as tp

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

INP = ou.golden_inputs()
with open(os.path.join(ou.ROOT, "tests", "golden", "fits.json")) as f:
    FITS = json.load(f)


@pytest.fixture(scope="module")
def bbm():
    import bbm_amd
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    torch.cuda.set_device(0)
    return bbm_amd


@pytest.mark.parametrize("fname", sorted(FITS))
def test_every_published_material_matches_reference(bbm, fname):
    if ou.ref() is None:
        pytest.skip("oracle/_ref not built")
    stats = {}
    pin, pout, sout = INP["pin"], INP["pout"], INP["sout"]
    n_mat = 0
    for mat, s, key, params in FITS[fname]:
        if params is None:          # a line the reference itself rejects (value beyond the float range)
            continue
        m = bbm.fromString(s)
        assert m.name == key, (fname, mat)
        p = np.asarray(params, np.float32)
        np.testing.assert_array_equal(m.parameter_values(), p)
        assert m.runtime, (fname, mat)
        tree = ou.runtime_fit_tree(key, p)
        got = tp._gpu_evalpdf(m, pin, pout)
        ref = ou.ref_runtime_eval_pdf(tree, pin, pout)
        provers = [tp._input_ulps_prover(lambda a, b: ou.ref_runtime_eval_pdf(tree, a, b), [pin, pout], got),
                   tp._libm_prover(lambda a, b: ou.ref_runtime_eval_pdf(tree, a, b, nthreads=1), [pin, pout], got)]
        st = tp.check_lanes(got, ref, f"{fname}:{mat} eval+pdf", provers, model=key)
        refl = m.reflectance(tp._dev(sout)).cpu().numpy()
        rr = ou.ref_runtime_reflectance(tree, sout)
        tp.check_lanes(refl, rr, f"{fname}:{mat} reflectance",
                       [tp._input_ulps_prover(lambda o: ou.ref_runtime_reflectance(tree, o), [sout], refl)], model=key)
        stats[mat] = {k: st[k] for k in ("max_rel_normal", "max_rel_proven", "frac_bit_exact", "lanes_outside_bar",
                                         "proven_by")}
        n_mat += 1
    assert n_mat == sum(1 for x in FITS[fname] if x[3] is not None)
    tp._report("fits_" + fname.replace(".fit", ""), {
        "materials": n_mat, "lanes": n_mat * pin.shape[1],
        "max_rel_normal": max(v["max_rel_normal"] for v in stats.values()),
        "lanes_outside_bar": sum(v["lanes_outside_bar"] for v in stats.values()),
        "min_frac_bit_exact": min(v["frac_bit_exact"] for v in stats.values()),
        "per_material": stats})
