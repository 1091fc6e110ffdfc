#!/usr/bin/env python3
"""Per-kernel ISA hashes of the product build (gfx950 device code of
ipt_kernels.hip + ipt_post.hip), to show that a source clean-up (removing
dead A/B switches, diagnostics) leaves every kernel instruction-for-
instruction unchanged.

usage: isa_hash.py OUT.json [extra hipcc flags...]
Compiles with __graft_entry__.HIPCC_FLAGS (device only, -S), splits the
assembly per function and hashes its instruction lines (comments, labels'
numbering and metadata directives dropped).
"""
import hashlib
import json
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import __graft_entry__ as ge  # noqa: E402

out_json = sys.argv[1]
extra = sys.argv[2:]
flags = [f for f in ge.HIPCC_FLAGS if f not in ("-shared", "-fPIC")]
hashes = {}
with tempfile.TemporaryDirectory() as td:
    for src in ("ipt_kernels.hip", "ipt_post.hip"):
        s = Path(td) / (src + ".s")
        subprocess.run([ge._hipcc(), *flags, *extra, "--cuda-device-only", "-S", "-o", str(s),
                        str(ge.SRC / src)], check=True)
        fn = None
        body = []
        for line in open(s):
            m = re.match(r"^([A-Za-z_.$][\w.$]*):\s*(;.*)?$", line)
            if m and not m.group(1).startswith(".L"):
                fn, body = m.group(1), []
                continue
            if fn and line.startswith(".Lfunc_end"):
                hashes[fn] = hashlib.sha256("".join(body).encode()).hexdigest()[:16]
                fn = None
                continue
            if fn:
                t = line.split(";", 1)[0].rstrip()
                if not t.strip() or t.lstrip().startswith("."):
                    continue
                t = re.sub(r"\.LBB\d+_\d+", ".LBB", t)
                body.append(t + "\n")
json.dump(hashes, open(out_json, "w"), indent=1, sort_keys=True)
print(f"{len(hashes)} functions -> {out_json}")
