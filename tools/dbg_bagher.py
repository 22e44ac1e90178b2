"""Dump the Bagher lanes farthest from the reference (1M-pair parity batches) to gpurun_out/dbg_bagher.npz."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
import bbm_amd  # noqa: E402
from tests import oracle_util as ou  # noqa: E402

torch.cuda.set_device(0)
meta = ou.golden_meta()
n = 1 << 20
res = {}
for name in sys.argv[1:]:
    g = ou.golden_model(name)
    for mode_out in (1, 0):
        din = bbm_amd.fill_directions(0xBB5EED, 0, 0, n, mode=0)
        dout = bbm_amd.fill_directions(0xBB5EED, 1, 0, n, mode=mode_out)
        hin, hout = din.cpu().numpy(), dout.cpu().numpy()
        for si in range(len(meta["models"][name]["sets"])):
            m = bbm_amd.BsdfModel(name)
            m.set_parameter_values(g[f"params{si}"])
            rgb, pdf = m.eval_pdf(din, dout)
            got = torch.cat([rgb, pdf[None]]).cpu().numpy()
            ref = ou.oracle_eval_pdf(name, g[f"params{si}"], hin, hout, nthreads=16)
            rel = np.abs(got.astype(np.float64) - ref) / np.maximum(np.abs(ref), 1e-38)
            rel[np.abs(ref) < np.finfo(np.float32).tiny] = 0
            lane = rel.max(0)
            worst = np.argsort(-lane)[:16]
            tag = f"{name}_{si}_0{mode_out}"
            res[tag + "_lanes"] = worst
            res[tag + "_in"] = hin[:, worst]
            res[tag + "_out"] = hout[:, worst]
            res[tag + "_got"] = got[:, worst]
            res[tag + "_ref"] = ref[:, worst]
            res[tag + "_params"] = g[f"params{si}"]
            print(tag, "bit_exact", float(np.mean(ou.ulp_diff(got, ref) == 0)), "outside", int((lane > 1e-5).sum()),
                  "worst", lane[worst[:4]].tolist(), flush=True)
np.savez("gpurun_out/dbg_bagher.npz", **res)
