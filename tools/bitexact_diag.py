"""Where the GPU's results differ from the reference's in the last bit (diagnostics, GPU box): for one model and
parameter set on config 2's input distribution (hemisphere x hemisphere, 1M pairs), every output value that is not
bit-identical to the reference's, with its inputs, per output channel, and whether the reference value is subnormal.

    python tools/bitexact_diag.py CookTorrance 0 [--out gpurun_out/bitexact_CookTorrance_0.npz]

Test infrastructure: the oracle is the checker only.
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tests import oracle_util as ou  # noqa: E402
import bbm_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("model")
    ap.add_argument("set", type=int)
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    din = bbm_amd.fill_directions(0xBB5EED, 0, 0, a.n, mode=0).cpu().numpy()
    dout = bbm_amd.fill_directions(0xBB5EED, 1, 0, a.n, mode=0).cpu().numpy()
    params = ou.golden_model(a.model)[f"params{a.set}"]
    m = bbm_amd.BsdfModel(a.model)
    m.set_parameter_values(params)
    rgb, pdf = m.eval_pdf(torch.from_numpy(din).cuda(), torch.from_numpy(dout).cuda())
    torch.cuda.synchronize()
    got = np.concatenate([rgb.cpu().numpy(), pdf.cpu().numpy()[None]], 0)
    ref = ou.oracle_eval_pdf(a.model, params, din, dout, nthreads=8)
    ulp = ou.ulp_diff(got, ref)
    diff = ulp != 0
    sub = (np.abs(ref) < ou.FLT_MIN) & (ref != 0)
    print(f"{a.model}[{a.set}]: {diff.sum()} of {diff.size} values not bit-exact "
          f"(frac_bit_exact {1 - diff.mean():.6f}); per output {diff.sum(1).tolist()}; "
          f"with subnormal reference {int((diff & sub).sum())}; lanes {int(diff.any(0).sum())}")
    for k, nm in enumerate("rgbp"):
        d = diff[k]
        if d.any():
            print(f"  {nm}: {int(d.sum())} values, ulps histogram {np.bincount(np.minimum(ulp[k][d], 9)).tolist()}, "
                  f"subnormal ref {int((d & sub[k]).sum())}")
    lanes = np.nonzero(diff.any(0))[0]
    out = a.out or os.path.join(ROOT, "gpurun_out", f"bitexact_{a.model}_{a.set}.npz")
    np.savez_compressed(out, lanes=lanes, din=din[:, lanes], dout=dout[:, lanes], got=got[:, lanes], ref=ref[:, lanes],
                        params=np.asarray(params, np.float32))


if __name__ == "__main__":
    main()
