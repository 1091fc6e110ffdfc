# Power and clock of the GPU while the C2 bench runs (rocm-smi sampled every
# 2 s in the background), plus the effective shader clock from GRBM_GUI_ACTIVE
# (sum over the 8 XCDs) / 8 / kernel time of one profiled step.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 5 30 rocm-smi -M -P -g > gpurun_out/smi_idle.txt 2>&1
( for i in $(seq 1 20); do rocm-smi -P -g --showmetrics >> gpurun_out/smi_load.txt 2>&1; sleep 2; done ) &
SMI=$!
timeout -k 10 200 python bench.py --steps 200 --warmup 5 --cpu-seconds 0 --no-counters > gpurun_out/power_bench.json 2> gpurun_out/power_bench.err; rc=$?
wait $SMI
[ $rc -eq 0 ] || { tail -3 gpurun_out/power_bench.err; exit $rc; }
timeout -k 10 200 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d gpurun_out/grbm -o g -- python bench.py --steps 1 --warmup 0 --cpu-seconds 0 --no-counters > gpurun_out/grbm.json 2> gpurun_out/grbm.err || { tail -3 gpurun_out/grbm.err; exit 1; }
python - <<'PY'
import csv, glob, json
d = json.load(open("gpurun_out/power_bench.json")); print("bench", round(d["value"], 2), d["unit"])
k = {}
for r in csv.DictReader(open(glob.glob("gpurun_out/grbm/*kernel_trace.csv")[0])):
    k[r["Dispatch_Id"]] = (r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
for r in csv.DictReader(open(glob.glob("gpurun_out/grbm/*counter_collection.csv")[0])):
    if "path_kernel" in r["Kernel_Name"] and r["Counter_Name"] == "GRBM_GUI_ACTIVE":
        t = k.get(r["Dispatch_Id"], (None, None))[1]
        print("path_kernel GRBM_GUI_ACTIVE", r["Counter_Value"], "time_s", t, "eff GHz", float(r["Counter_Value"]) / 8 / t / 1e9 if t else None)
PY
grep -i -E "power|sclk|Socket" gpurun_out/smi_idle.txt | head -8
grep -i -E "Average Graphics Package Power|Current Socket Graphics Package Power|sclk|current_gfxclk|average_gfx_activity|average_socket_power|throttle" gpurun_out/smi_load.txt | sort | uniq -c | sort -rn | head -30
