#!/usr/bin/env python3
"""One line per variant bench JSON: Mpaths/s (+ per-path events when counted)."""
import json, sys
v, f = sys.argv[1], sys.argv[2]
d = json.load(open(f))
ev = {k: round(x, 2) for k, x in (d.get("events_per_path") or {}).items()
      if k in ("traced_rays", "iterations", "sphere_frames", "skipped")}
print("variant", v, round(d["value"], 2), "Mpaths/s", ev if ev else "")
