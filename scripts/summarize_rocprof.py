#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output into profiles/<tag>_<cfg>_summary.json and
profiles/pmc_latest_<cfg>.json (read by bench.py for `traffic` / `occupancy`).

usage: summarize_rocprof.py TAG CFG BENCH_JSON STATS_DIR PMC_DIR [PMC_DIR...]

STATS_DIR: a `rocprofv3 --kernel-trace --stats` run; each PMC_DIR: one
`rocprofv3 --pmc ... --kernel-trace` pass of the same bench command (one
counter group per pass, MI355X_MICROARCH.md "rocprofv3 PMC slots").
Per kernel and dispatch, a counter's rows (its dimension instances) are
summed; the summary holds the mean over dispatches.

Derived for path_kernel:
* HBM bytes per launch = (FETCH_SIZE + WRITE_SIZE) KiB x 1024. FETCH_SIZE is
  not doubled: the guide's 2x correction is for wide coalesced streams; the
  path kernel's reads are 4-16 B gathers and scalar loads (uncalibrated
  widths, left as measured). The accumulate kernel's 4 B/lane coalesced
  stream gets the correction, reported separately.
* occupancy = mean resident waves per SIMD = SQ_WAVE_CYCLES (quad-cycles,
  summed over all waves) x 4 / (GRBM_GUI_ACTIVE / 8 XCDs x 256 CUs x 4 SIMDs)
  (GRBM_GUI_ACTIVE is the sum over the 8 XCDs of the cycles the GPU was busy;
  MI355X_MICROARCH.md "DVFS give-back", "s_memtime tick vs SQ PMC units");
  also the effective clock GRBM_GUI_ACTIVE / 8 / kernel time.
"""
import csv
import glob
import json
import shutil
import sys
from pathlib import Path

tag, cfg_name, bench_json, stats_dir, *pmc_dirs = sys.argv[1:]
out = Path("profiles")
out.mkdir(exist_ok=True)
N_XCD, N_SIMD = 8, 256 * 4


def short(name):
    for k in ("path_kernel", "accumulate_kernel", "raygen_kernel"):
        if k in name:
            return k
    return name[:40]


stats = {}
for f in glob.glob(f"{stats_dir}/**/*kernel_stats.csv", recursive=True):
    shutil.copy(f, out / f"{tag}_{cfg_name}_kernel_stats.csv")
    for r in csv.DictReader(open(f)):
        stats[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                                   "pct": float(r["Percentage"])}
pmc = {}
durations = {}
for d in pmc_dirs:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        per = {}
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            per.setdefault((k, r["Counter_Name"]), {}).setdefault(r["Dispatch_Id"], 0.0)
            per[(k, r["Counter_Name"])][r["Dispatch_Id"]] += float(r["Counter_Value"])
        for (k, cn), disp in per.items():
            vals = list(disp.values())
            pmc.setdefault(k, {})[cn] = sum(vals) / len(vals)
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            durations.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e9)

bench = json.loads(open(bench_json).read().strip().splitlines()[-1])
cfg = bench["config"]
paths_per_launch = cfg["width"] * cfg["height"] * cfg["spp_per_step"]
summary = {"tag": tag, "config_name": cfg_name, "kernel_stats": stats, "pmc": pmc, "config": cfg,
           "paths_per_launch": paths_per_launch, "bench_value": bench.get("value")}
pk = pmc.get("path_kernel", {})
if "FETCH_SIZE" in pk and "WRITE_SIZE" in pk:
    b = (pk["FETCH_SIZE"] + pk["WRITE_SIZE"]) * 1024
    summary["path_kernel_hbm_bytes_per_launch"] = b
    summary["path_kernel_hbm_bytes_per_path"] = b / paths_per_launch
# DRAM share of the fabric traffic (TCC_EA0_RDREQ_DRAM / TCC_EA0_RDREQ: the
# L2's memory-side read requests "destined for DRAM (MC)"; likewise writes).
# The Infinity Cache sits on the memory side of that interface, so its hits
# may still be counted as DRAM-destined: an upper bound on HBM bytes.
if "TCC_EA0_RDREQ_sum" in pk and "TCC_EA0_RDREQ_DRAM_sum" in pk and "FETCH_SIZE" in pk:
    rd_share = pk["TCC_EA0_RDREQ_DRAM_sum"] / max(pk["TCC_EA0_RDREQ_sum"], 1.0)
    wr_share = 1.0
    if "TCC_EA0_WRREQ_sum" in pk and "TCC_EA0_WRREQ_DRAM_sum" in pk:
        wr_share = pk["TCC_EA0_WRREQ_DRAM_sum"] / max(pk["TCC_EA0_WRREQ_sum"], 1.0)
    # reads weighted by request size (64 B, or 32 B for the TCC_EA0_RDREQ_32B
    # share, assumed the same among the DRAM-destined requests) rather than a
    # request-count ratio applied to FETCH_SIZE; writes keep WRITE_SIZE's share
    n32 = pk.get("TCC_EA0_RDREQ_32B_sum", 0.0)
    f32 = n32 / max(pk["TCC_EA0_RDREQ_sum"], 1.0)
    rd_bytes = pk["TCC_EA0_RDREQ_DRAM_sum"] * (64.0 * (1.0 - f32) + 32.0 * f32)
    dram = rd_bytes + pk.get("WRITE_SIZE", 0.0) * wr_share * 1024
    summary["path_kernel_dram_bytes_per_launch"] = dram
    summary["path_kernel_dram_bytes_per_path"] = dram / paths_per_launch
    summary["path_kernel_dram"] = {
        "read_requests": pk["TCC_EA0_RDREQ_sum"], "read_requests_dram": pk["TCC_EA0_RDREQ_DRAM_sum"],
        "read_dram_share": rd_share, "write_dram_share": wr_share,
        "read_requests_32B": pk.get("TCC_EA0_RDREQ_32B_sum"),
        "dram_credit_stall_cycles": pk.get("TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum"),
        "read_32B_share": f32,
        "source": ("RDREQ_DRAM x (64 B x (1 - 32B share) + 32 B x 32B share) + WRITE_SIZE x 1024 x WRREQ_DRAM/"
                   "WRREQ; the Infinity Cache is memory-side, so DRAM-destined requests include its hits: an "
                   "UPPER BOUND on HBM bytes (gfx950 tags every memory-side request DRAM-destined here)"),
    }
if "SQ_WAVE_CYCLES" in pk and "GRBM_GUI_ACTIVE" in pk:
    busy = pk["GRBM_GUI_ACTIVE"] / N_XCD  # GPU-busy cycles of the dispatch
    summary["path_kernel_occupancy"] = {
        "waves_per_simd": pk["SQ_WAVE_CYCLES"] * 4 / (busy * N_SIMD),
        "max_waves_per_simd_by_launch_bounds": None,
        "source": "SQ_WAVE_CYCLES x 4 / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)",
    }
    if "SQ_WAVES" in pk:
        summary["path_kernel_occupancy"]["waves_launched"] = pk["SQ_WAVES"]
    if durations.get("path_kernel"):
        t = sum(durations["path_kernel"]) / len(durations["path_kernel"])
        summary["path_kernel_occupancy"]["effective_clock_GHz"] = busy / t / 1e9
for key in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY",
            "TCC_HIT_sum", "TCC_MISS_sum", "TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_DRAM_sum",
            "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum"):
    if key in pk:
        summary.setdefault("path_kernel_per_path", {})[key] = pk[key] / paths_per_launch
ak = pmc.get("accumulate_kernel", {})
if "FETCH_SIZE" in ak and "WRITE_SIZE" in ak:
    summary["accumulate_hbm_bytes_per_launch_corrected"] = (2 * ak["FETCH_SIZE"] + ak["WRITE_SIZE"]) * 1024
json.dump(summary, open(out / f"{tag}_{cfg_name}_summary.json", "w"), indent=1)
json.dump(summary, open(out / f"pmc_latest_{cfg_name}.json", "w"), indent=1)
print(json.dumps({k: summary.get(k) for k in ("tag", "config_name", "path_kernel_hbm_bytes_per_path",
                                              "path_kernel_dram_bytes_per_path",
                                              "path_kernel_occupancy", "path_kernel_per_path")}, indent=1))
