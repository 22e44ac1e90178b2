"""Quick parity of the loaded library (BBM_HIP_LIB selects an A/B build) against the reference on 1M-pair batches:
per model and golden parameter set, bit-identical fraction, lanes outside the 1e-5 bar (no per-lane proofs) and max
relative error over normal reference values.   python tools/quick_parity.py Bagher "Aggregate<Lambertian,Bagher>" """
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import bbm_amd  # noqa: E402
from tests import oracle_util as ou  # noqa: E402


def main(names):
    torch.cuda.set_device(0)
    meta = ou.golden_meta()
    n = 1 << 20
    out = {}
    for mode_out in (1, 0):
        din = bbm_amd.fill_directions(0xBB5EED, 0, 0, n, mode=0)
        dout = bbm_amd.fill_directions(0xBB5EED, 1, 0, n, mode=mode_out)
        hin, hout = din.cpu().numpy(), dout.cpu().numpy()
        for name in names:
            g = ou.golden_model(name)
            for si in range(len(meta["models"][name]["sets"])):
                m = bbm_amd.BsdfModel(name)
                m.set_parameter_values(g[f"params{si}"])
                rgb, pdf = m.eval_pdf(din, dout)
                got = torch.cat([rgb, pdf[None]]).cpu().numpy()
                ref = ou.oracle_eval_pdf(name, g[f"params{si}"], hin, hout, nthreads=16)
                exact = float(np.mean(ou.ulp_diff(got, ref) == 0))
                normal = np.abs(ref) >= np.finfo(np.float32).tiny
                rel = np.abs(got.astype(np.float64) - ref) / np.maximum(np.abs(ref), 1e-38)
                out[f"{name}[{si}] 0{mode_out}"] = {"bit_exact": exact, "outside_1e-5": int(np.sum(rel[normal] > 1e-5)),
                                                    "max_rel": float(rel[normal].max())}
                print(name, si, mode_out, out[f"{name}[{si}] 0{mode_out}"], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1:])
