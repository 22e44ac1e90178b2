"""The He family's 90 backscatter evaluations (the sampler CDF's inputs, ndf/sampler.h:143-181) on the GPU against
the reference, per golden parameter set: how many differ and by how many ulps.  Writes gpurun_out/dbg_he_cdf.json."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import bbm_amd  # noqa: E402
from tests import oracle_util as ou  # noqa: E402

torch.cuda.set_device(0)
meta = ou.golden_meta()
d = ou.sampler_backscatter_dirs().astype(np.float32)
out = {}
for name in ("He", "HeWestin", "HeHolzschuch", "NganHe"):
    g = ou.golden_model(name)
    for si in range(len(meta["models"][name]["sets"])):
        params = g[f"params{si}"]
        m = bbm_amd.BsdfModel(name)
        m.set_parameter_values(params)
        t = torch.from_numpy(d).cuda()
        rgb, _ = m.eval_pdf(t, t)
        got = rgb.cpu().numpy()
        ref = ou.oracle_eval_pdf(name, params, d, d, nthreads=4)[:3]
        u = ou.ulp_diff(got, ref)
        bad = np.nonzero(np.any(u > 0, axis=0))[0]
        out[f"{name}[{si}]"] = {"differ": int(bad.size), "max_ulp": int(u.max()), "bins": bad.tolist()[:20],
                                "got": got[:, bad[:4]].T.tolist(), "ref": ref[:, bad[:4]].T.tolist()}
        print(name, si, out[f"{name}[{si}]"], flush=True)
json.dump(out, open("gpurun_out/dbg_he_cdf.json", "w"), indent=1)
