"""Diagnostics: the He family's parts -- D per channel (BBM_HIP_HE_DIAG=1), (sigma, S, G) (=2) and (F red, F green,
1 / (pi z z)) (=3), from diagnostics builds of the library -- plus the shipped library's eval, for each golden parameter
set, written as hex floats to gpurun_out/he_parts_<variant>.json, at the 90 sampler backscatter directions (default)
or at 4096 random (upper hemisphere, upper hemisphere) pairs (argument `pairs`, the pairs saved alongside):
    BBM_HIP_LIB=bbm_amd/lib_ab/hediag1/libbbm_hip.so python tools/dbg_he_parts.py hediag1 [pairs]
Round 6 used it to pin every part against the reference (profiles/r06_oracle_slp.txt)."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import bbm_amd  # noqa: E402
from tests import oracle_util as ou  # noqa: E402

torch.cuda.set_device(0)
pairs = len(sys.argv) > 2 and sys.argv[2] == "pairs"
if pairs:
    din = ou.dirgen_numpy(0xBB5EED, 0, 0, 4096, mode=0)
    dout = ou.dirgen_numpy(0xBB5EED, 1, 0, 4096, mode=0)
else:
    din = dout = ou.sampler_backscatter_dirs().astype(np.float32)
out = {"pairs": [[float(x).hex() for x in col] for col in np.concatenate([din, dout]).T]}
for name in ("He", "HeWestin", "HeHolzschuch"):
    g = ou.golden_model(name)
    for si in range(3):
        m = bbm_amd.BsdfModel(name)
        m.set_parameter_values(g[f"params{si}"])
        rgb, _ = m.eval_pdf(torch.from_numpy(np.ascontiguousarray(din)).cuda(), torch.from_numpy(np.ascontiguousarray(dout)).cuda())
        out[f"{name}_{si}"] = [[float(x).hex() for x in row] for row in rgb.cpu().numpy().T]
json.dump(out, open(f"gpurun_out/he_parts_{sys.argv[1]}{'_pairs' if pairs else ''}.json", "w"))
print("done", sys.argv[1])
