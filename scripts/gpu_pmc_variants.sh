# PMC counters of the C2 path kernel per library variant ($VARIANTS, as
# scripts/gpu_variants.sh; "default" = the product build), per path.
# PASSES: ';'-separated passes of ','-separated counters (one rocprofv3 run each).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
PASSES=${PASSES:-"SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_ACTIVE_INST_ANY,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_INST_ANY,SQ_WAIT_ANY"}
for v in ${VARIANTS:-default}; do
  if [ "$v" = default ]; then L=ipt_amd/lib/libipt_hip.so; else L=ipt_amd/lib/abl/libipt_$v.so; fi
  i=0
  IFS=';' read -ra PS <<< "$PASSES"
  for pass in "${PS[@]}"; do
    i=$((i+1))
    c=$(echo "$pass" | tr ',' ' ')
    IPT_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmcv_${v}_$i -o p -- python bench.py --steps 1 --warmup 0 --cpu-seconds 0 --no-counters > gpurun_out/pmcv_${v}_$i.json 2>gpurun_out/pmcv_${v}_$i.err || { echo "pmc $v pass $i failed"; tail -3 gpurun_out/pmcv_${v}_$i.err; exit 1; }
  done
  python scripts/pmc_sq.py gpurun_out/pmcv_${v}_* > gpurun_out/pmcv_$v.txt
  python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open(f"gpurun_out/pmcv_{v}.txt").read())
paths = 1024 * 1024 * 32
print(v, {k: round(x / paths, 2) for k, x in sorted(d.items())})
PY
done
