import sys, os, numpy as np, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import bbm_amd as bbm
from tests import oracle_util as ou
n = 1 << 16
din = bbm.fill_directions(7, 0, 0, n, mode=1); dout = bbm.fill_directions(7, 1, 0, n, mode=1)
for rep in range(3):
    lam, child = bbm.Lambertian(albedo=[0.2, 0.3, 0.4]), bbm.BsdfModel("NganHe")
    fused = bbm.Aggregate(lam, child); composed = bbm.Aggregate(lam, child, fused=False)
    fr, fp = fused.eval_pdf(din, dout); cr, cp = composed.eval_pdf(din, dout)
    ch, chp = child.eval_pdf(din, dout)
    torch.cuda.synchronize()
    d = (fr != cr).any(0).nonzero().flatten().cpu().numpy()
    print("rep", rep, "differing lanes", d.size, d[:8])
    if d.size:
        i = d[:4]
        print(" fused", fr[:, i].cpu().numpy().T.tolist()); print(" comp ", cr[:, i].cpu().numpy().T.tolist())
        print(" child", ch[:, i].cpu().numpy().T.tolist())
        p = np.asarray(child.parameter_values() if hasattr(child, "parameter_values") else [], np.float32)
        print(" in", din[:, i].cpu().numpy().T.tolist(), "out", dout[:, i].cpu().numpy().T.tolist())
