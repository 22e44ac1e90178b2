"""Static instruction counts of kernels in a device assembly file (hipcc --cuda-device-only -S):
   python tools/isa_count.py /tmp/f64.s 'k_eval_pdf_f64.*Bagher.*Li2ELb1'
prints, per matching kernel: instructions, VALU, f64 VALU, transcendental, branches, VGPRs, spill stores."""
import re
import sys


def kernels(path):
    s = open(path).read()
    for m in re.finditer(r'^(_Z\w+):\s*;', s, re.M):
        start = m.end()
        end = s.find('.Lfunc_end', start)
        yield m.group(1), s[start:end], s


def main():
    path, pat = sys.argv[1], re.compile(sys.argv[2])
    for name, body, s in kernels(path):
        if not pat.search(name):
            continue
        ins = [l.strip().split()[0] for l in body.split('\n')
               if l.strip() and not l.strip().startswith(('.', ';')) and not l.strip().endswith(':')]
        valu = [i for i in ins if i.startswith('v_')]
        f64 = [i for i in valu if 'f64' in i]
        trans = [i for i in valu if re.match(r'v_(exp|log|rcp|rsq|sqrt|sin|cos)_', i)]
        br = [i for i in ins if i.startswith('s_cbranch')]
        meta = re.search(r'\.name:\s+' + re.escape(name) + r'\s.*?\.vgpr_count:\s+(\d+)', s, re.S)
        spill = sum(1 for i in ins if i.startswith('scratch_store') or i.startswith('buffer_store'))
        print(f"{len(ins):6d} ins {len(valu):6d} valu {len(f64):5d} f64 {len(trans):4d} trans {len(br):3d} br "
              f"vgpr {meta.group(1) if meta else '?':>4} spill {spill:3d}  {name[:110]}")


if __name__ == "__main__":
    main()
