"""Diagnostics (round 6): the He family's parts -- D per channel (lib_ab/hediag1), (sigma, S, G) (hediag2) and
(F red, F green, 1 / (pi z z)) (hediag3) -- at the 90 sampler backscatter directions, for each golden parameter set,
written as hex floats to gpurun_out/he_parts_<variant>.json.  Run once per variant library:
    BBM_HIP_LIB=bbm_amd/lib_ab/hediag1/libbbm_hip.so python tools/dbg_he_parts.py hediag1"""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import bbm_amd  # noqa: E402
from tests import oracle_util as ou  # noqa: E402

torch.cuda.set_device(0)
d = ou.sampler_backscatter_dirs().astype(np.float32)
out = {}
for name in ("He", "HeWestin", "HeHolzschuch"):
    g = ou.golden_model(name)
    for si in range(3):
        m = bbm_amd.BsdfModel(name)
        m.set_parameter_values(g[f"params{si}"])
        t = torch.from_numpy(d).cuda()
        rgb, _ = m.eval_pdf(t, t)
        out[f"{name}_{si}"] = [[float(x).hex() for x in row] for row in rgb.cpu().numpy().T]
json.dump(out, open(f"gpurun_out/he_parts_{sys.argv[1]}.json", "w"))
print("done", sys.argv[1])
