"""GPU diagnostics for adapter_check findings: composed-aggregate reflectance channels and HeWestin pdf zeros."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bbm_amd
from tests import oracle_util as ou

torch.cuda.set_device(0)
rng = np.random.default_rng(3)


def sphere(n):
    z = (2 * rng.random(n) - 1).astype(np.float32)
    ph = (2 * np.pi * rng.random(n)).astype(np.float32)
    s = np.sqrt(np.maximum(1 - z * z, 0)).astype(np.float32)
    return np.stack([s * np.cos(ph), s * np.sin(ph), z]).astype(np.float32)


n = 262144
out = sphere(n)
dout = torch.from_numpy(out).cuda()
ct, ggx = bbm_amd.CookTorrance(), bbm_amd.GGX()
agg = bbm_amd.Aggregate(ct, ggx, fused=False)
for rep in range(3):
    r = agg.reflectance(dout).cpu().numpy()
    a = ct.reflectance(dout).cpu().numpy()
    b = ggx.reflectance(dout).cpu().numpy()
    s = (a + b).astype(np.float32)
    bad = np.nonzero(np.any(r != s, axis=0))[0]
    print("composed reflectance rep", rep, "lanes != a+b:", bad.size, "per channel:", [(r[c] != s[c]).sum() for c in range(3)],
          "first", bad[:8])
    ref = ou.ref_reflectance("Aggregate<CookTorrance,GGX>", np.concatenate([ct.parameter_values(), ggx.parameter_values()]), out)
    print("   vs reference: lanes outside bar", (~ou.parity_ok(r, ref)).any(0).sum())

# HeWestin pdf on sphere pairs, compaction path vs scalar path
he = bbm_amd.BsdfModel("HeWestin")
din = sphere(65536)
dout2 = sphere(65536)
rgb, pdf = he.eval_pdf(torch.from_numpy(din).cuda(), torch.from_numpy(dout2).cuda())
pdf = pdf.cpu().numpy()
ref = ou.oracle_eval_pdf("HeWestin", he.parameter_values(), din, dout2, nthreads=8)
live = (din[2] > 0) & (dout2[2] > 0)
print("HeWestin pdf: live", live.sum(), "gpu pdf==0 & ref>0:", ((pdf == 0) & (ref[3] > 0)).sum(),
      "eval outside bar:", (~ou.parity_ok(rgb.cpu().numpy(), ref[:3])).any(0).sum())
# the CDF: backscatter evals
hb = ou.sampler_backscatter_dirs()
g = he.eval_pdf(torch.from_numpy(hb).cuda(), torch.from_numpy(hb).cuda())[0].cpu().numpy()
rb = ou.oracle_eval_pdf("HeWestin", he.parameter_values(), hb, hb, nthreads=1)[:3]
print("backscatter eval outside bar:", (~ou.parity_ok(g, rb)).any(0).sum(), "gpu zeros", (g == 0).all(0).sum(), "ref zeros", (rb == 0).all(0).sum())
# single pair path (n=1, scalar kernel) for the first few zero lanes
z = np.nonzero((pdf == 0) & (ref[3] > 0))[0][:4]
for i in z:
    a1 = torch.from_numpy(np.ascontiguousarray(din[:, i:i + 1])).cuda()
    b1 = torch.from_numpy(np.ascontiguousarray(dout2[:, i:i + 1])).cuda()
    print("lane", i, "batch pdf", pdf[i], "single pdf", float(he.eval_pdf(a1, b1)[1][0]), "ref", ref[3][i])
