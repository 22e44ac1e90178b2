#!/usr/bin/env python3
"""oracle/gen_fit_golden.py -- TEST INFRASTRUCTURE ONLY: golden vectors for the fitting path
(tests/golden/fit.npz + fit.json), from the reference's own implementation (oracle/_ref, ref_fit.cpp).

Pinned:
  * spherical_linearizer index -> (in, out) for three grids (include/linearizer/spherical_linearizer.h:63-101);
  * sampledlossfunction per-sample losses and the reference's serial float total
    (include/bbm/sampledlossfunction.h:62-87) for every sample loss (include/loss/*.h), two fitted
    models against published fits used as synthetic "measured" references;
  * compass search trajectories (include/optimizer/compass.h:82-140): parameters and loss after
    every step.
The MERL grid (merl_linearizer) has no forward-map fixture: the reference's forward map does not
compile (see ref_fit.cpp); tests pin ours through the reference's inverse map instead.

Run:  python oracle/gen_fit_golden.py   (needs oracle/_ref/libbbm_ref.so)
"""
import ctypes
import json
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
from gen_golden import fit_params, fptr, load_ref  # noqa: E402

F32 = np.float32
HEMI = [float(F32(2 * math.pi)), float(F32(0.5 * math.pi))]

# (name, samples_in, samples_out, start_in, end_in, start_out, end_out) -- (phi, theta)
GRIDS = [
    ("grid0", (8, 5), (6, 4), (0, 0), HEMI, (0, 0), HEMI),
    # lowLog's default layout: theta_out only (cosine_weighted_log.h:83-84), phi_out fixed at 0..2pi
    ("grid1", (12, 7), (1, 9), (0, 0), HEMI, (0, 0), [float(F32(2 * math.pi)), HEMI[1]]),
    ("grid2", (5, 4), (7, 3), (0.1, 0.05), (3.0, 1.4), (0.2, 0.1), (6.0, 1.5)),
]

LOSS_MODELS = [
    # (fitted model, fitted params: defaults, reference params: published fit)
    "Aggregate<Lambertian,Bagher>",
    "Aggregate<Lambertian,CookTorrance>",
]

COMPASS_RUNS = [
    # (model, grid, loss kind, steps)
    ("Aggregate<Lambertian,CookTorrance>", "grid0", 3, 30),
    ("Aggregate<Lambertian,CookTorrance>", "grid2", 0, 20),
    ("Aggregate<Lambertian,Bagher>", "grid0", 3, 8),
]


def desc(g):
    _, si, so, a, b, c, d = g
    s_in = np.asarray(si, np.uint64)
    s_out = np.asarray(so, np.uint64)
    rng = np.asarray(list(a) + list(b) + list(c) + list(d), np.float32)
    return s_in, s_out, rng


def main():
    lib = load_ref()
    lib.bbmref_linearizer_size.restype = ctypes.c_int64
    buf = (ctypes.c_float * 64)()
    arrays, meta = {}, {"grids": {}, "loss": {}, "compass": []}
    for g in GRIDS:
        s_in, s_out, rng = desc(g)
        n = lib.bbmref_linearizer_size(0, fptr(s_in), fptr(s_out), fptr(rng))
        d = np.zeros((6, n), np.float32)
        assert lib.bbmref_linearize(0, fptr(s_in), fptr(s_out), fptr(rng), ctypes.c_uint64(0), ctypes.c_size_t(n),
                                    *[fptr(d[k]) for k in range(6)]) == 0
        arrays[f"{g[0]}_dirs"] = d
        meta["grids"][g[0]] = {"samples_in": list(g[1]), "samples_out": list(g[2]), "start_in": list(map(float, g[3])),
                               "end_in": list(map(float, g[4])), "start_out": list(map(float, g[5])),
                               "end_out": list(map(float, g[6])), "size": int(n)}
    for name in LOSS_MODELS:
        k = lib.bbmref_default_params(name.encode(), buf, 64)
        fitted = np.array(buf[:k], np.float32)
        ref = fit_params(name)
        arrays[f"{name}_fitted"] = fitted
        arrays[f"{name}_reference"] = ref
        for g in GRIDS[:2]:
            s_in, s_out, rng = desc(g)
            n = meta["grids"][g[0]]["size"]
            for kind in range(6):
                per = np.zeros(n, np.float32)
                tot = np.zeros(1, np.float32)
                assert lib.bbmref_loss(name.encode(), fptr(fitted), fptr(ref), k, 0, fptr(s_in), fptr(s_out), fptr(rng),
                                       kind, fptr(per), fptr(tot), 8) == n
                arrays[f"{name}_{g[0]}_loss{kind}"] = per
                meta["loss"][f"{name}_{g[0]}_loss{kind}"] = float(tot[0])
    for ci, (name, gname, kind, steps) in enumerate(COMPASS_RUNS):
        g = next(x for x in GRIDS if x[0] == gname)
        s_in, s_out, rng = desc(g)
        k = lib.bbmref_default_params(name.encode(), buf, 64)
        init = np.array(buf[:k], np.float32)
        ref = fit_params(name)
        params = np.zeros((steps, k), np.float32)
        losses = np.zeros(steps, np.float32)
        loss0 = np.zeros(1, np.float32)
        P = lib.bbmref_compass(name.encode(), fptr(init), fptr(ref), k, 0, fptr(s_in), fptr(s_out), fptr(rng), kind,
                               steps, fptr(params), fptr(losses), fptr(loss0))
        arrays[f"compass{ci}_params"] = params.reshape(-1)[:steps * P].reshape(steps, P)   # packed steps x P
        arrays[f"compass{ci}_loss"] = losses
        meta["compass"].append({"model": name, "grid": gname, "loss": kind, "steps": steps, "nopt": int(P),
                                "loss0": float(loss0[0])})
        print(f"compass {name} {gname} loss={kind}: {loss0[0]:.6g} -> {losses[-1]:.6g} ({steps} steps, P={P})")
    out = os.path.join(ROOT, "tests", "golden")
    np.savez_compressed(os.path.join(out, "fit.npz"), **arrays)
    with open(os.path.join(out, "fit.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
