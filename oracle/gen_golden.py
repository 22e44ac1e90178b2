#!/usr/bin/env python3
"""oracle/gen_golden.py -- TEST INFRASTRUCTURE ONLY: writes the golden vectors in tests/golden/.

Drives the reference's own implementation (oracle/_ref/libbbm_ref.so, built by `make -C oracle ref`
from /root/reference/include + backbone/native, see oracle/ref_harness.cpp) on a fixed, seeded
set of direction pairs and parameter sets, and stores inputs + outputs as small .npz fixtures.
Only the fixtures are committed; the reference never travels to the GPU box.

What is pinned, per model (tests/golden/<Model>.npz):
  * eval (RGB) + pdf, floatRGB, component=All, unit=Radiance, for every parameter set
    (defaults, a published fit where one exists in /root/reference/fits, two seeded random sets);
  * eval + pdf for component Diffuse / Specular and unit Importance (defaults) -> mask semantics;
  * eval + pdf in doubleRGB (defaults) -> floatRGB-vs-doubleRGB spread, for reporting;
  * sample(out, xi) -> direction, pdf, flag (floatRGB) for every parameter set;
  * reflectance(out) (defaults).
Shared inputs and per-model metadata (defaults, bounds, toString) live in inputs.npz / models.json.

Run:  python oracle/gen_golden.py   (needs /root/reference; takes a few seconds)
"""
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
OUT = os.path.join(ROOT, "tests", "golden")
SEED = 0xBB5EED

# bsdf_flag (include/bbm/bsdf_flag.h:21-27) and unit_t (include/bbm/unit.h:20-24)
FLAG_NONE, FLAG_DIFFUSE, FLAG_SPECULAR, FLAG_ALL = 0, 1, 2, 3
UNIT_RADIANCE, UNIT_IMPORTANCE = 0, 1

# Published fits used as one parameter set (file:line in /root/reference/fits); params are the
# flat parameter_values() vector in attribute order.
FITS = {
    # fits/low_cooktorrance_E1.fit:3 alum-bronze (LowCookTorrance == CookTorrance composition)
    "CookTorrance": [0.05872, 0.04367, 0.05223, 0.017044, 1.46492],
    "LowCookTorrance": [0.05872, 0.04367, 0.05223, 0.017044, 1.46492],
    # fits/ngan_cooktorrance.fit:3 blue-acrylic (attribute order albedo, roughness, eta)
    "NganCookTorrance": [0.0291, 0.0193, 0.0118, 0.0137, 0.117],
    # fits/low_cooktorrance_E1.fit:3 alum-bronze diffuse part
    "Lambertian": [0.1063, 0.0816, 0.0557],
}


FIT_FILES = {   # Aggregate(Lambertian, X) -> the published fit used as the 'fit' parameter set (first entry)
    "Aggregate<Lambertian,Bagher>": "bagher_sgd.fit",
    "Aggregate<Lambertian,CookTorrance>": "low_cooktorrance_E1.fit",
    "Aggregate<Lambertian,LowCookTorrance>": "low_cooktorrance_E1.fit",
    "Aggregate<Lambertian,LowAshikhminShirley>": "low_ashikhminshirley_E1.fit",
    "Aggregate<Lambertian,LowMicrofacetFit>": "low_lowmicrofacet_E2.fit",
    "Aggregate<Lambertian,LowSmooth>": "low_lowsmooth_E2.fit",
    "Aggregate<Lambertian,NganAshikhminShirley>": "ngan_ashikhminshirley.fit",
    "Aggregate<Lambertian,NganBlinnPhong>": "ngan_blinnphong.fit",
    "Aggregate<Lambertian,NganCookTorrance>": "ngan_cooktorrance.fit",
    "Aggregate<Lambertian,NganLafortune>": "ngan_lafortune.fit",
    "Aggregate<Lambertian,NganWard>": "ngan_ward.fit",
    "Aggregate<Lambertian,NganWardDuer>": "ngan_wardduer.fit",
    "Aggregate<Lambertian,NganHe>": "ngan_he.fit",
}


def fit_params(name):
    """Parameter vector of the first material of the model's published fit file (fits/*.fit, `name =
    Aggregate(...)`), parsed with the host mirror's fromString (attribute layout of bbm_amd/models.py)."""
    sys.path.insert(0, ROOT)
    from bbm_amd import models as bm
    from bbm_amd.backbone import _parse_value, _tokenize
    path = os.path.join("/root/reference/fits", FIT_FILES[name])
    line = next(l for l in open(path) if "=" in l and not l.lstrip().startswith("#"))
    tok = _tokenize(line.split("=", 1)[1])
    # Aggregate ( Child ( attr = v , ... ) , Child ( ... ) )
    out, i = [], 2
    for child in bm.AGGREGATES[name]:
        layout = bm.ATTRIBUTES[child]
        vals = {}
        i += 2
        while tok[i] != ")":
            attr = tok[i]
            v, i = _parse_value(tok, i + 2)
            vals[attr] = np.asarray(v, np.float32).reshape(-1)
            if tok[i] == ",":
                i += 1
        i += 1
        if tok[i] == ",":
            i += 1
        return_vals = []
        for attr, shape in layout:
            n = bm.attr_size(shape)
            v = vals.get(attr)
            if v is None:
                return None          # attribute missing from the file: no 'fit' set
            return_vals.append(np.repeat(v, n) if v.size == 1 and n > 1 else v)
        out.append(np.concatenate(return_vals))
    return np.concatenate(out).astype(np.float32)


def golden_file(name):
    """tests/golden file of a model: Aggregate<Lambertian,X> -> Aggregate_Lambertian_X.npz"""
    return name.replace("<", "_").replace(",", "_").replace(">", "") + ".npz"


def load_ref():
    path = os.path.join(HERE, "_ref", "libbbm_ref.so")
    if not os.path.exists(path):
        sys.exit("oracle/_ref/libbbm_ref.so missing: run `make -C oracle ref` first")
    lib = ctypes.CDLL(path)
    lib.bbmref_model_name.restype = ctypes.c_char_p
    return lib


def fptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def sph(z, phi):
    s = np.sqrt(np.maximum(1.0 - z * z, 0.0))
    return np.stack([s * np.cos(phi), s * np.sin(phi), z]).astype(np.float32)


def make_pairs(rng):
    """(3,N) in / out directions: upper-hemisphere pairs, full-sphere pairs, edge cases."""
    na, nb = 1024, 256
    ins = [sph(rng.random(na), 2 * np.pi * rng.random(na))]
    outs = [sph(rng.random(na), 2 * np.pi * rng.random(na))]
    ins.append(sph(2 * rng.random(nb) - 1, 2 * np.pi * rng.random(nb)))
    outs.append(sph(2 * rng.random(nb) - 1, 2 * np.pi * rng.random(nb)))

    def n(v):
        v = np.asarray(v, np.float64)
        return v / np.linalg.norm(v)

    e_in, e_out = [], []
    zn = [0, 0, 1]
    edge = [
        (zn, zn),                                  # normal incidence
        (n([0.3, 0.1, 0.9]), n([-0.2, 0.05, 0.8])),  # survey spot value
        (n([0.5, 0.2, 0.6]), n([0.5, 0.2, 0.6])),    # in == out
        (n([0.5, 0.2, 0.6]), n([-0.5, -0.2, 0.6])),  # in == reflect(out): h == n
        (n([0.3, 0.0, 0.7]), n([-0.3, 0.001, 0.7])),  # near specular
        (n([1, 0, 1e-4]), n([-1, 0, 1e-4])),        # both grazing
        (n([1, 0, 1e-4]), zn),                      # one grazing
        ([1, 0, 0], zn),                            # z(in) == 0 exactly
        (zn, [0, 1, 0]),                            # z(out) == 0 exactly
        (n([0.2, 0.3, -0.5]), zn),                  # below horizon
        (zn, n([0.2, 0.3, -0.5])),
        (n([0.2, 0.3, -0.5]), n([-0.1, 0.3, -0.5])),  # both below
        (n([0.9, 0.0, 0.1]), n([-0.9, 0.0, 0.1])),  # grazing specular
        (n([0.9, 0.0, 0.1]), n([0.9, 0.0, 0.1])),   # grazing retro
        (n([0.0, 0.7, 0.7]), n([0.7, 0.0, 0.7])),   # 90 deg azimuth
        (n([1e-4, 0, 1]), n([-1e-4, 0, 1])),        # near-normal, tiny xy
        (n([0.6, 0.6, 0.1]), n([0.1, -0.9, 0.3])),
        ([0.0, 0.0, 1.0], n([0.0, 1e-3, 1.0])),
    ]
    for a, b in edge:
        e_in.append(np.asarray(a, np.float32))
        e_out.append(np.asarray(b, np.float32))
    # deterministic grid of near-normal / grazing elevations
    for zi in (1e-3, 0.05, 0.5, 0.999, 0.99999):
        for zo in (1e-3, 0.3, 0.9999):
            e_in.append(np.asarray(n([np.sqrt(1 - zi * zi), 0.0, zi]), np.float32))
            e_out.append(np.asarray(n([-np.sqrt(1 - zo * zo) * 0.8, np.sqrt(1 - zo * zo) * 0.6, zo]), np.float32))
    ins.append(np.stack(e_in, axis=1))
    outs.append(np.stack(e_out, axis=1))
    return np.ascontiguousarray(np.concatenate(ins, 1)), np.ascontiguousarray(np.concatenate(outs, 1))


def make_samples(rng):
    ma, mb = 512, 128
    outs = [sph(rng.random(ma), 2 * np.pi * rng.random(ma)), sph(2 * rng.random(mb) - 1, 2 * np.pi * rng.random(mb))]
    xis = [rng.random((2, ma)).astype(np.float32), rng.random((2, mb)).astype(np.float32)]
    # edge xi: boundaries, out of range (masked), and edge outs
    ex = [(0, 0), (1, 1), (0, 1), (1, 0), (0.5, 0.5), (1e-7, 0.5), (0.9999999, 0.5), (-0.1, 0.5), (0.5, 1.1), (0.25, 0.75)]
    eo = [[0, 0, 1], [0.6, 0.0, 0.8], [0.999, 0.0, 0.0447], [0.0, 0.0, -1.0], [0.3, 0.4, 0.8660254]]
    e_out, e_xi = [], []
    for o in eo:
        for x in ex:
            v = np.asarray(o, np.float64)
            e_out.append((v / np.linalg.norm(v)).astype(np.float32))
            e_xi.append(np.asarray(x, np.float32))
    outs.append(np.stack(e_out, 1))
    xis.append(np.stack(e_xi, 1))
    return np.ascontiguousarray(np.concatenate(outs, 1)), np.ascontiguousarray(np.concatenate(xis, 1))


def param_sets(name, defaults, lo, hi, rng):
    sets = [("default", np.asarray(defaults, np.float32))]
    if name in FITS:
        sets.append(("fit", np.asarray(FITS[name], np.float32)))
    elif name in FIT_FILES:
        fp = fit_params(name)
        if fp is not None:
            sets.append(("fit", fp))
    for k in range(2):
        p = []
        for d, a, b in zip(defaults, lo, hi):
            if b > 1e30 or a < -1e30:       # unbounded: scatter around the default
                p.append(d * np.exp(rng.uniform(-1.0, 1.0)) if d != 0 else rng.uniform(0.1, 2.0))
            else:
                p.append(rng.uniform(a + 0.05 * (b - a), b))
        sets.append((f"random{k}", np.asarray(p, np.float32)))
    return sets


def main():
    lib = load_ref()
    rng = np.random.default_rng(SEED)
    pin, pout = make_pairs(rng)
    sout, sxi = make_samples(rng)
    N, M = pin.shape[1], sout.shape[1]
    os.makedirs(OUT, exist_ok=True)
    np.savez_compressed(os.path.join(OUT, "inputs.npz"), pin=pin, pout=pout, sout=sout, sxi=sxi,
                        seed=np.uint64(SEED))

    meta = {"seed": SEED, "n_pairs": N, "n_samples": M,
            "generator": "oracle/gen_golden.py via oracle/_ref/libbbm_ref.so (reference headers, native backbone)",
            "flags": "g++ -std=c++20 -O2 -march=x86-64-v3 -ffp-contract=off", "models": {}}
    buf = (ctypes.c_float * 64)()
    sbuf = ctypes.create_string_buffer(4096)
    for i in range(lib.bbmref_num_models()):
        bname = lib.bbmref_model_name(i)
        name = bname.decode()
        k = lib.bbmref_default_params(bname, buf, 64)
        defaults = [float(buf[j]) for j in range(k)]
        lib.bbmref_param_bounds(bname, 0, buf, 64)
        lo = [float(buf[j]) for j in range(k)]
        lib.bbmref_param_bounds(bname, 1, buf, 64)
        hi = [float(buf[j]) for j in range(k)]
        sets = param_sets(name, defaults, lo, hi, np.random.default_rng(SEED + i + 1))
        arrays = {}
        strings = []
        for si, (tag, p) in enumerate(sets):
            lib.bbmref_to_string(bname, fptr(p), k, sbuf, 4096)
            strings.append(sbuf.value.decode())
            arrays[f"params{si}"] = p
            ev = np.zeros((4, N), np.float32)
            lib.bbmref_eval_pdf(bname, fptr(p), k, ctypes.c_size_t(N), fptr(pin[0]), fptr(pin[1]), fptr(pin[2]),
                                fptr(pout[0]), fptr(pout[1]), fptr(pout[2]), FLAG_ALL, UNIT_RADIANCE, 3,
                                fptr(ev[0]), fptr(ev[1]), fptr(ev[2]), fptr(ev[3]), 1)
            arrays[f"evalpdf{si}"] = ev
            so = np.zeros((4, M), np.float32)
            sf = np.zeros(M, np.uint32)
            lib.bbmref_sample(bname, fptr(p), k, ctypes.c_size_t(M), fptr(sout[0]), fptr(sout[1]), fptr(sout[2]),
                              fptr(sxi[0]), fptr(sxi[1]), FLAG_ALL, UNIT_RADIANCE,
                              fptr(so[0]), fptr(so[1]), fptr(so[2]), fptr(so[3]), fptr(sf), 1)
            arrays[f"sample{si}"] = so
            arrays[f"sflag{si}"] = sf.astype(np.uint8)
            rf = np.zeros((3, M), np.float32)
            lib.bbmref_reflectance(bname, fptr(p), k, ctypes.c_size_t(M), fptr(sout[0]), fptr(sout[1]), fptr(sout[2]),
                                   FLAG_ALL, UNIT_RADIANCE, fptr(rf[0]), fptr(rf[1]), fptr(rf[2]))
            arrays[f"reflectance{si}"] = rf
        p = sets[0][1]
        for tag, comp, unit in (("diffuse", FLAG_DIFFUSE, UNIT_RADIANCE), ("specular", FLAG_SPECULAR, UNIT_RADIANCE),
                                ("importance", FLAG_ALL, UNIT_IMPORTANCE)):
            ev = np.zeros((4, N), np.float32)
            lib.bbmref_eval_pdf(bname, fptr(p), k, ctypes.c_size_t(N), fptr(pin[0]), fptr(pin[1]), fptr(pin[2]),
                                fptr(pout[0]), fptr(pout[1]), fptr(pout[2]), comp, unit, 3,
                                fptr(ev[0]), fptr(ev[1]), fptr(ev[2]), fptr(ev[3]), 1)
            arrays[f"evalpdf_{tag}"] = ev
        evd = np.zeros((4, N), np.float64)
        lib.bbmref_eval_pdf_double(bname, fptr(p), k, ctypes.c_size_t(N), fptr(pin[0]), fptr(pin[1]), fptr(pin[2]),
                                   fptr(pout[0]), fptr(pout[1]), fptr(pout[2]), FLAG_ALL, UNIT_RADIANCE, 3,
                                   fptr(evd[0]), fptr(evd[1]), fptr(evd[2]), fptr(evd[3]), 1)
        arrays["evalpdf_double"] = evd
        rf = np.zeros((3, M), np.float32)
        lib.bbmref_reflectance(bname, fptr(p), k, ctypes.c_size_t(M), fptr(sout[0]), fptr(sout[1]), fptr(sout[2]),
                               FLAG_ALL, UNIT_RADIANCE, fptr(rf[0]), fptr(rf[1]), fptr(rf[2]))
        arrays["reflectance"] = rf
        for tag, comp in (("diffuse", FLAG_DIFFUSE), ("specular", FLAG_SPECULAR)):
            rf = np.zeros((3, M), np.float32)
            lib.bbmref_reflectance(bname, fptr(p), k, ctypes.c_size_t(M), fptr(sout[0]), fptr(sout[1]), fptr(sout[2]),
                                   comp, UNIT_RADIANCE, fptr(rf[0]), fptr(rf[1]), fptr(rf[2]))
            arrays[f"reflectance_{tag}"] = rf
        abuf = (ctypes.c_uint32 * 64)()
        ka = lib.bbmref_param_attrs(bname, abuf, 64)
        attrs = [int(abuf[j]) for j in range(ka)]
        np.savez_compressed(os.path.join(OUT, golden_file(name)), **arrays)
        meta["models"][name] = {"nparams": k, "defaults": defaults, "lower": lo, "upper": hi,
                                "sets": [t for t, _ in sets], "strings": strings, "attrs": attrs}
        print(f"{name:24s} k={k:2d} sets={len(sets)}")
    with open(os.path.join(OUT, "models.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
