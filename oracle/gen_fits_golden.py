"""TEST INFRASTRUCTURE ONLY.  Writes tests/golden/fits.json: every material of every published fit file
(/root/reference/fits/*.fit, `name = Aggregate(Lambertian(...), X(...))`) with the parameter vector the
reference's own bbm::fromString gives for its model string (oracle/_ref: bbmref_from_string; All | Dependent
attributes in declaration order).  tests/test_fits.py parses the same strings with bbm_amd.fromString and
requires the identical vectors and the kernel each maps to.

    python oracle/gen_fits_golden.py        (needs /root/reference and oracle/_ref/libbbm_ref.so)
"""
import ctypes
import glob
import json
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
FITS = "/root/reference/fits"


def model_key(s):
    """Registry key of a model string: Aggregate(A(...), B(...)) -> Aggregate<A,B>, X(...) -> X."""
    s = s.strip()
    head = re.match(r"([A-Za-z_]\w*)\s*\(", s).group(1)
    if head != "Aggregate":
        return head
    inner = s[s.index("(") + 1:s.rindex(")")]
    kids, depth, start = [], 0, 0
    for i, ch in enumerate(inner):
        if ch in "([":
            depth += 1
        elif ch in ")]":
            depth -= 1
        elif ch == "," and depth == 0:
            kids.append(inner[start:i])
            start = i + 1
    kids.append(inner[start:])
    return "Aggregate<" + ",".join(model_key(k) for k in kids) + ">"


def main():
    lib = ctypes.CDLL(os.path.join(HERE, "_ref", "libbbm_ref.so"))
    buf = (ctypes.c_float * 128)()
    out = {}
    for path in sorted(glob.glob(os.path.join(FITS, "*.fit"))):
        rows = []
        for line in open(path):
            line = line.strip()
            if not line or line.startswith("#") or "=" not in line:
                continue
            material, model = (x.strip() for x in line.split("=", 1))
            key = model_key(model)
            k = lib.bbmref_from_string(key.encode(), model.encode(), buf, 128)
            if k == -2:
                raise SystemExit(f"oracle has no model {key} ({os.path.basename(path)}: {material})")
            # k == -1: the reference's fromString throws (e.g. a value beyond the float range): recorded as None
            rows.append([material, model, key, [float(buf[i]) for i in range(k)] if k >= 0 else None])
        out[os.path.basename(path)] = rows
        print(f"{os.path.basename(path)}: {len(rows)} materials, {sum(r[3] is None for r in rows)} rejected by the reference")
    with open(os.path.join(ROOT, "tests", "golden", "fits.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))


if __name__ == "__main__":
    main()
