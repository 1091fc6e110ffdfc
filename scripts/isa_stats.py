#!/usr/bin/env python3
"""Static instruction mix of every path_kernel instance in a hipcc -S listing
(profiling aid): total / VALU / f64 VALU / transcendental / SALU / LDS / VMEM
counts, VGPRs, spills and LDS. usage: isa_stats.py listing.s [more.s ...]"""
import re
import sys

TRANS = ("v_rcp", "v_rsq", "v_sqrt", "v_exp", "v_log", "v_sin", "v_cos")


def kernels(txt):
    for m in re.finditer(r"\n(_Z\S*path_kernel\S*):[^\n]*\n(.*?)\n\.Lfunc_end", txt, re.S):
        yield m.group(1), m.group(2)


def meta(txt, name):
    m = re.search(r"\.amdhsa_kernel " + re.escape(name) + r"\n(.*?)\.end_amdhsa_kernel", txt, re.S)
    d = {}
    if m:
        for k in ("amdhsa_next_free_vgpr", "amdhsa_group_segment_fixed_size", "amdhsa_private_segment_fixed_size"):
            mm = re.search(r"\." + k + r" (\d+)", m.group(1))
            if mm:
                d[k.replace("amdhsa_", "")] = int(mm.group(1))
    return d


for f in sys.argv[1:]:
    txt = open(f).read()
    for name, body in kernels(txt):
        ops = [l.split()[0] for l in body.split("\n") if l.startswith("\t") and l.strip() and l.strip()[0] not in ".;"]
        c = dict(total=len(ops), valu=sum(o.startswith("v_") for o in ops),
                 f64=sum(o.startswith("v_") and "f64" in o for o in ops),
                 trans=sum(o.startswith(TRANS) for o in ops), salu=sum(o.startswith("s_") for o in ops),
                 lds=sum(o.startswith("ds_") for o in ops),
                 vmem=sum(o.startswith(("global_", "buffer_", "flat_", "scratch_")) for o in ops))
        c.update(meta(txt, name))
        short = re.sub(r"_ZN12_GLOBAL__N_111path_kernelI(.*)EEvNS_7KParamsE", r"\1", name)
        print(f, short, c)
