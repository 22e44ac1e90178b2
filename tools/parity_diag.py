"""Parity diagnostics (GPU box): every lane outside the strict per-lane bar (tests/oracle_util.parity_ok),
for every model x parameter set on the golden inputs and on 1M-pair batches, with its inputs, so the
cause can be studied offline against the reference (oracle/_ref) in the build container.

    python tools/parity_diag.py [--n 1048576] [--models A,B] [--out gpurun_out/parity_diag.npz]

Writes <out> (violating lanes: model, set, batch, lane, in xyz, out xyz, got[4], ref[4]) and a JSON summary
next to it (per model/set: lanes checked, violations, subnormal-reference lanes, max rel error over normal
reference values).  Test infrastructure: uses the oracle only as the checker.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tests import oracle_util as ou  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--models", default="")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "parity_diag.npz"))
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--max-keep", type=int, default=2000, help="violating lanes kept per (model, set, batch)")
    args = ap.parse_args()
    import bbm_amd
    torch.cuda.set_device(0)
    meta, inp = ou.golden_meta(), ou.golden_inputs()
    names = [m for m in bbm_amd.model_names() if m in meta["models"] and m in ou.oracle_models()]
    if args.models:
        names = [m for m in names if m in args.models.split(",")]
    n = args.n
    batches = {"golden": (inp["pin"], inp["pout"])}
    for tag, mi, mo in (("hemi_sphere", 0, 1), ("hemi_hemi", 0, 0)):
        din = bbm_amd.fill_directions(0xBB5EED, 0, 0, n, mode=mi).cpu().numpy()
        dout = bbm_amd.fill_directions(0xBB5EED, 1, 0, n, mode=mo).cpu().numpy()
        batches[tag] = (din, dout)
    # the He-family samplers' CDF is built from 90 backscatter evaluations eval(h, h) at theta = (i/90)^2 pi/2,
    # phi = 0 (ndf/sampler.h:143-181): a mismatch there moves every pdf, so those pairs are checked as well
    th = ((np.arange(90) / 90.0) ** 2 * (np.pi / 2)).astype(np.float32).astype(np.float64)
    hb = np.stack([np.sin(th), np.zeros_like(th), np.cos(th)]).astype(np.float32)
    batches["backscatter"] = (hb, hb)
    rows, summary = [], {}
    t0 = time.time()
    for name in names:
        g = ou.golden_model(name)
        for si in range(len(meta["models"][name]["sets"])):
            params = g[f"params{si}"]
            m = bbm_amd.BsdfModel(name)
            m.set_parameter_values(params)
            for btag, (din, dout) in batches.items():
                rgb, pdf = m.eval_pdf(torch.from_numpy(np.ascontiguousarray(din)).cuda(),
                                      torch.from_numpy(np.ascontiguousarray(dout)).cuda())
                torch.cuda.synchronize()
                got = np.concatenate([rgb.cpu().numpy(), pdf.cpu().numpy()[None]], 0)
                ref = ou.oracle_eval_pdf(name, params, din, dout, nthreads=args.threads)
                ok = ou.parity_ok(got, ref)
                bad_lane = np.nonzero(~ok.all(0))[0]
                sub = (np.abs(ref) < ou.FLT_MIN) & (ref != 0)
                key = f"{name}[{si}]/{btag}"
                expl = np.zeros(bad_lane.size, bool)
                if bad_lane.size:
                    expl = ou.explained_by_input_ulps(
                        lambda a, b: ou.oracle_eval_pdf(name, params, a, b, nthreads=args.threads),
                        [din[:, bad_lane], dout[:, bad_lane]], got[:, bad_lane])
                summary[key] = {"lanes": int(got.shape[1]), "bad_lanes": int(bad_lane.size),
                                "bad_values": int((~ok).sum()),
                                "explained_by_2ulp_inputs": int(expl.sum()),
                                "subnormal_ref_values": int(sub.sum()),
                                "flushed_to_zero": int((sub & (got == 0)).sum()),
                                "max_rel_normal": ou.max_rel_normal(got, ref),
                                "frac_bit_exact": float(np.mean(ou.ulp_diff(got, ref) == 0)),
                                "max_ulp": int(ou.ulp_diff(got, ref).max())}
                for lane, e in list(zip(bad_lane, expl))[:args.max_keep]:
                    rows.append((name, si, btag, int(lane), din[:, lane], dout[:, lane], got[:, lane], ref[:, lane], e))
                if bad_lane.size:
                    print(key, summary[key], flush=True)
        print(f"{name} done ({time.time() - t0:.0f} s)", flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    np.savez_compressed(args.out,
                        model=np.array([r[0] for r in rows]), set=np.array([r[1] for r in rows], np.int32),
                        batch=np.array([r[2] for r in rows]), lane=np.array([r[3] for r in rows], np.int64),
                        din=np.array([r[4] for r in rows], np.float32).reshape(-1, 3),
                        dout=np.array([r[5] for r in rows], np.float32).reshape(-1, 3),
                        got=np.array([r[6] for r in rows], np.float32).reshape(-1, 4),
                        ref=np.array([r[7] for r in rows], np.float32).reshape(-1, 4),
                        explained=np.array([r[8] for r in rows], bool))
    with open(args.out.replace(".npz", ".json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(f"{len(rows)} violating lanes kept; summary -> {args.out.replace('.npz', '.json')}")


if __name__ == "__main__":
    main()
