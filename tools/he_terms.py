"""He-family series lengths on the GPU (diagnostics): with a library built -DBBM_HIP_HE_COUNT_TERMS
(tools/build_variant.sh heterms -DBBM_HIP_HE_COUNT_TERMS) the compaction kernel's eval returns, per pair, the number
of series terms run and the two-phase length key instead of the BSDF value.  From those this prints, for config 3's
inputs (hemisphere pairs, all live), the mean terms per pair and the mean wave-max terms per pair for
  * consecutive waves (the one-phase kernel),
  * waves of the two-phase kernel (each 256-job chunk counting-sorted by the key),
  * waves sorted by the true term count (a perfect key) -- and the resulting lane utilisation of the series.
   BBM_HIP_LIB=bbm_amd/lib_ab/heterms/libbbm_hip.so python tools/he_terms.py He HeWestin NganHe
"""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import bbm_amd  # noqa: E402


def wave_max(t, order, chunk=256):
    t = t[: len(t) // chunk * chunk]
    out = np.empty_like(t)
    for c0 in range(0, len(t), chunk):
        blk = t[c0:c0 + chunk][order(c0)]
        w = blk.reshape(-1, 64).max(1)
        out[c0:c0 + chunk] = np.repeat(w, 64)
    return out


def main(models, n=1 << 20, seed=0xBB5EED):
    din = bbm_amd.fill_directions(seed, 0, 0, n, mode=0)
    dout = bbm_amd.fill_directions(seed, 1, 0, n, mode=0)
    res = {}
    for name in models:
        m = bbm_amd.BsdfModel(name)
        rgb, _ = m.eval_pdf(din, dout, mode=1)
        torch.cuda.synchronize()
        terms = rgb[0].cpu().numpy().astype(np.int64)
        key = rgb[1].cpu().numpy().astype(np.int64)
        n2 = len(terms) // 256 * 256
        terms, key = terms[:n2], key[:n2]
        unsorted = wave_max(terms, lambda c0: np.arange(256))
        keyed = wave_max(terms, lambda c0: np.argsort(key[c0:c0 + 256], kind="stable"))
        perfect = wave_max(terms, lambda c0: np.argsort(terms[c0:c0 + 256], kind="stable"))
        mean = float(terms.mean())
        res[name] = {"pairs": int(n2), "mean_terms": mean,
                     "wave_max_consecutive": float(unsorted.mean()), "wave_max_keyed": float(keyed.mean()),
                     "wave_max_perfect_256": float(perfect.mean()),
                     "lane_util_consecutive": mean / float(unsorted.mean()),
                     "lane_util_keyed": mean / float(keyed.mean()),
                     "lane_util_perfect_256": mean / float(perfect.mean()),
                     "terms_hist": np.bincount(terms, minlength=65).tolist()}
        print(name, {k: round(v, 3) for k, v in res[name].items() if isinstance(v, float)}, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    torch.cuda.set_device(0)
    main(sys.argv[1:] or ["He", "HeWestin", "NganHe"])
