#!/usr/bin/env python3
"""Exhaustive device checks of the short reciprocal / division candidates
(ipt_math_selfcheck fn 17-20, include/ipt_capi.h): prints the mismatch
counts over all 2^32 bit patterns. Profiling aid; the same checks run as
tests/test_gpu_parity.py::test_fast_math_exhaustive."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from ipt_amd import capi

ctx = capi.Context(0)
for fn, what in ((17, "rcp, 1 correction == div_inrange_(1, x)"), (18, "rcp, 2 corrections == div_inrange_(1, x)"),
                 (19, "a/b, 1 quotient correction == IEEE, division pairs"),
                 (20, "a/b, 1 quotient correction == IEEE, near-all-ones divisors")):
    bad, first = ctx.math_selfcheck(fn)
    print(f"fn {fn} ({what}): {bad} mismatches of 2^32, first {first:#x}", flush=True)
