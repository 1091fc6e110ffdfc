#!/usr/bin/env python3
"""Per-dispatch SQ counter summary of path_kernel (or the kernel PMC_KERNEL
names) from rocprofv3 CSV dirs."""
import csv, glob, os, sys, json
name = os.environ.get("PMC_KERNEL", "path_kernel")
res = {}
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/*counter_collection.csv"):
        per = {}
        for r in csv.DictReader(open(f)):
            if name not in r["Kernel_Name"]:
                continue
            per.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
            per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
        for k, v in per.items():
            vals = sorted(v.values())
            res[k] = vals[len(vals) // 2]
print(json.dumps(res, indent=1))
