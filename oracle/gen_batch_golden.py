#!/usr/bin/env python3
"""oracle/gen_batch_golden.py -- TEST INFRASTRUCTURE ONLY: golden vectors for bbm::batch (include/bbm/batch.h:27-92),
from the reference's own implementation (oracle/_ref, ref_fit.cpp: bbmref_batch_indices / bbmref_batch_loss).

Pinned (tests/golden/batch.json):
  * the indices bbm::batch draws through bbm::rng<Size_t> (backbone/native/include/backbone/random.h:40-66:
    std::mt19937_64 + std::uniform_int_distribution<Size_t> over [0, samples()]) after construction and after each
    update(), for three seeds and two sample counts (a fit grid and the MERL grid);
  * batch::operator()(idx) -- the per-sample losses of the batch's drawn samples -- on fit grid0 for the two fitted
    models of tests/golden/fit.npz (fitted = defaults, reference = a published fit), standardLog.

Run:  python oracle/gen_batch_golden.py   (needs oracle/_ref/libbbm_ref.so)
"""
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
from tests import oracle_util as ou  # noqa: E402

SEEDS = [5489, 1, 0xBB5EED]
SAMPLES = [960, 90 * 90 * 180]
BATCH, UPDATES = 64, 3
LOSS_RUNS = [("Aggregate<Lambertian,CookTorrance>", 7, 128, 2), ("Aggregate<Lambertian,Bagher>", 11, 96, 2)]


def main():
    meta_fit, fit = ou.golden_fit()
    out = {"indices": [], "losses": []}
    for seed in SEEDS:
        for n in SAMPLES:
            idx = ou.ref_batch_indices(seed, n, BATCH, UPDATES)
            out["indices"].append({"seed": seed, "samples": n, "batchsize": BATCH, "updates": UPDATES,
                                   "index": [int(v) for v in idx.ravel()]})
    for name, seed, bs, upd in LOSS_RUNS:
        per = ou.ref_batch_losses(name, fit[f"{name}_fitted"], fit[f"{name}_reference"], meta_fit["grids"]["grid0"], 3,
                                  seed, bs, upd)
        out["losses"].append({"model": name, "grid": "grid0", "loss": 3, "seed": seed, "batchsize": bs, "updates": upd,
                              "per_sample": [float(v) for v in per.ravel()]})
    with open(os.path.join(ROOT, "tests", "golden", "batch.json"), "w") as f:
        json.dump(out, f, indent=0)
    print("wrote tests/golden/batch.json")


if __name__ == "__main__":
    main()
