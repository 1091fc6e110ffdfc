#!/usr/bin/env bash
# One parametrised GPU job (replaces the single-use round launchers): each
# argument is a step, run in order, each under its own time limit; the job
# stops at the first failing step (no GPU step runs after a failure).
#
#   bash scripts/gpu_job.sh STEP [STEP ...]
#
#   tests[=K_EXPR]        pytest -m gpu (optionally -k K_EXPR)    -> gpurun_out/pytest_gpu.log
#   smoke                 __graft_entry__.smoke()
#   bench=CFG[:STEPS]     bench.py --config CFG (default steps)   -> gpurun_out/bench_CFG.json
#   ab=V1,V2,...@CFG[:N]  A/B of library variants (ipt_amd/lib/abl/libipt_V.so, `default` =
#                         the product library), N rounds of V1..Vk in turn, 2 bench steps each
#   sq=CFG,CFG            SQ / cache counter passes (TAG env)     -> gpurun_out/sq_TAG_CFG_summary.json
#   profile=CFG,CFG       rocprof stats + PMC traffic passes + bench lines (TAG env)
#   phases=CFG,CFG        IPT_PROF / IPT_STAMP builds' phase profiles (scripts/prof_phases.sh first)
#   ubench                VALU / packed-f32 issue microbenchmark (scripts/ubench_valu)
#   gather                dependent-gather latency by table size (scripts/ubench_gather)
#   gate[=LIBS]           the tail-overlap gate under rocprofv3 (scripts/gpu_gate_trace.sh; FORCE env)
#
# usage (gpurun): /usr/local/graft/bin/gpurun --timeout 900 -- 'bash scripts/gpu_job.sh tests=async bench=c2'
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-latest}

line() {  # one-line summary of a bench JSON line
  python3 - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
print(sys.argv[1], round(d["value"], 3), d["unit"], "ms/step", round(d["ms_per_step"], 1),
      "valu_frac", (r.get("valu") or {}).get("frac"), "hbm_frac", r.get("frac"))
PY
}

step() {
  local s=$1 k=${1%%=*} v=
  [ "$k" != "$s" ] && v=${s#*=}
  echo "== $s"
  case $k in
    tests)
      local sel=()
      [ -n "$v" ] && sel=(-k "$v")
      timeout -k 10 1100 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread "${sel[@]}" \
        > gpurun_out/pytest_gpu.log 2>&1; local rc=$?
      grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -2
      [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL|Timeout" gpurun_out/pytest_gpu.log | head -20; return $rc; } ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)
      local c=${v%%:*} n=
      [ "$c" != "$v" ] && n="--steps ${v#*:}"
      timeout -k 10 600 python3 bench.py --config "$c" $n --cpu-seconds 0 > "gpurun_out/bench_$c.json" \
        2> "gpurun_out/bench_$c.err" || { tail -5 "gpurun_out/bench_$c.err"; return 1; }
      line "gpurun_out/bench_$c.json" ;;
    ab)
      local vs=${v%%@*} rest=${v#*@} c n
      c=${rest%%:*}; n=1; [ "$c" != "$rest" ] && n=${rest#*:}
      for r in $(seq 1 "$n"); do
        for var in ${vs//,/ }; do
          local L=ipt_amd/lib/abl/libipt_$var.so
          [ "$var" = default ] && L=ipt_amd/lib/libipt_hip.so
          IPT_ABI_COMPAT=1 IPT_LIB_PATH=$L timeout -k 10 300 python3 bench.py --config "$c" --steps 2 --warmup 1 \
            --cpu-seconds 0 --no-counters > "gpurun_out/ab_${var}_${c}_$r.json" 2> "gpurun_out/ab_${var}_${c}_$r.err" \
            || { echo "variant $var failed"; tail -3 "gpurun_out/ab_${var}_${c}_$r.err"; return 1; }
          line "gpurun_out/ab_${var}_${c}_$r.json"
        done
      done ;;
    sq)
      TAG=$TAG CFGS="${v//,/ }" bash scripts/gpu_pmc_sq.sh ;;
    profile)
      TAG=$TAG CFGS="${v//,/ }" bash scripts/gpu_profile.sh ;;
    phases)
      CONFIGS="${v//,/ }" bash scripts/gpu_prof_phases.sh ;;
    gather)
      timeout -k 10 300 ./scripts/ubench_gather > gpurun_out/ubench_gather.jsonl && cat gpurun_out/ubench_gather.jsonl ;;
    gate)
      LIBS="${v//,/ }" FORCE=${FORCE:-0} bash scripts/gpu_gate_trace.sh ;;
    ubench)
      timeout -k 10 300 ./scripts/ubench_valu > gpurun_out/ubench_valu.jsonl && cat gpurun_out/ubench_valu.jsonl ;;
    *) echo "unknown step $s"; return 2 ;;
  esac
}

for s in "$@"; do
  step "$s" || { echo "step $s failed"; exit 1; }
done
