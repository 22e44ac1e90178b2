"""Dump one sample lane of the large-batch sample test (inputs + GPU output) for CPU-side analysis."""
import sys
import numpy as np
import torch
import bbm_amd as bbm

name, lane = sys.argv[1], int(sys.argv[2])
n = 1 << 20
out = bbm.fill_directions(0xBB5EED, 2, 0, n, mode=1)
xi = torch.rand((2, n), generator=torch.Generator(device="cuda").manual_seed(5), device="cuda")
m = bbm.BsdfModel(name)
s = m.sample(out, xi)
torch.cuda.synchronize()
sl = slice(lane, lane + 1)
o = out[:, sl].contiguous()
res = {"out": o.cpu().numpy(), "xi": xi[:, sl].cpu().numpy(), "dir": s.direction[:, sl].cpu().numpy(),
       "pdf": s.pdf[sl].cpu().numpy(), "params": np.asarray(m.parameter_values(), np.float32)}
# GPU directions over a sweep of xi0 around the lane's value
ks = np.arange(-200, 201)
x0 = float(res["xi"][0, 0])
sweep_xi = torch.tensor(np.stack([np.float32(x0) * (1 + ks * 1e-7), np.full(ks.size, res["xi"][1, 0])]).astype(np.float32),
                        device="cuda")
so = o.expand(3, ks.size).contiguous()
ss = m.sample(so, sweep_xi)
torch.cuda.synchronize()
res["sweep_xi"] = sweep_xi.cpu().numpy()
res["sweep_dir"] = ss.direction.cpu().numpy()
np.savez(f"gpurun_out/diag_{name}_{lane}.npz", **res)
print({k: v.ravel()[:6] for k, v in res.items() if k != "sweep_dir" and k != "sweep_xi"})
