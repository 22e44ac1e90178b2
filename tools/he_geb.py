import sys, numpy as np, torch
sys.path.insert(0, ".")
import bbm_amd
torch.cuda.set_device(0)
n = 1 << 20
din = bbm_amd.fill_directions(0xBB5EED, 0, 0, n, mode=0)
dout = bbm_amd.fill_directions(0xBB5EED, 1, 0, n, mode=0)
for name in sys.argv[1:]:
    m = bbm_amd.BsdfModel(name)
    rgb, _ = m.eval_pdf(din, dout, mode=1)
    torch.cuda.synchronize()
    a = rgb.cpu().numpy()
    np.savez_compressed(f"gpurun_out/he_geb_{name}.npz", terms=a[0].astype(np.int16), g=a[1], eb=a[2])
    print(name, a[0].mean(), flush=True)
