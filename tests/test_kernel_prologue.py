"""Every __global__ kernel of the library fills the LDS tables (math_tables_init()) before it constructs a model or
evaluates anything (CPU-only source check).

The glibc restatements (bbm_amd/csrc/math.hpp: expf / logf / powf and everything built on them) read their tables
from LDS copies that each kernel fills in its prologue; a kernel that skipped it would read uninitialised LDS.  Only
plain loads may come first (k_eval_pdf_v4 issues its first quad's loads ahead of the prologue).  The only exemption is
runtime.hip, which does not include the device math layer (its gather kernel uses no table)."""
import glob
import os
import re

from tests import oracle_util as ou

KERNEL = re.compile(r"__global__[^;{]*?\)\s*\{", re.S)
# what may not precede the prologue: a model, an evaluation, a table function, a call into the device math
BEFORE_INIT = re.compile(r"\bModel\s+\w+\s*[({]|\bm\.|model_|_glibc|eval(?!_prefetch|_pipeline)|sample|reflectance|loss")
EXEMPT = {"runtime.hip"}


def test_every_kernel_fills_the_lds_tables_first():
    src = sorted(glob.glob(os.path.join(ou.ROOT, "bbm_amd", "csrc", "*.hip")) +
                 glob.glob(os.path.join(ou.ROOT, "bbm_amd", "csrc", "*.hpp")))
    kernels, missing = 0, []
    for f in src:
        if os.path.basename(f) in EXEMPT:
            continue
        s = open(f).read()
        for m in KERNEL.finditer(s):
            kernels += 1
            body = s[m.end():]
            k = body.find("math_tables_init();")
            nxt = KERNEL.search(body)
            head = re.sub(r"//[^\n]*", "", body[:max(k, 0)])          # code before the prologue, comments dropped
            if k < 0 or (nxt is not None and k > nxt.start()) or BEFORE_INIT.search(head) \
                    or head.count("{") != head.count("}"):           # at the kernel's top level
                line = s[:m.start()].count("\n") + 1
                missing.append(f"{os.path.basename(f)}:{line}")
    assert kernels >= 40
    assert not missing, f"kernels without math_tables_init() ahead of any evaluation: {missing}"


def test_runtime_unit_uses_no_table():
    s = open(os.path.join(ou.ROOT, "bbm_amd", "csrc", "runtime.hip")).read()
    assert "math.hpp" not in s and "expf_glibc" not in s and "powf_glibc" not in s
