#!/usr/bin/env bash
# The tail-overlap gate under rocprofv3: a chunked synchronous
# render (tests/chunked_probe.py, IPT_TEST_CHUNK_UNITS) traced kernel by kernel
# with each library in LIBS (ipt_amd/lib/abl/libipt_<v>.so, `default` = the
# product library): which kernels run (a stream wait on ordinary memory runs as
# a ROCclr wait kernel, on signal memory as a CP packet), and, with FORCE=1, the
# product library's pool gate kept under counter collection (--pmc; the
# round-4 hang) -- that step last, under its own KILL timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp IPT_TEST_CHUNK_UNITS=3000 IPT_ABI_COMPAT=1
for v in ${LIBS:-oldgate default}; do
  L=ipt_amd/lib/abl/libipt_$v.so
  [ "$v" = default ] && L=ipt_amd/lib/libipt_hip.so
  rm -rf "gpurun_out/gate_$v"
  IPT_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/gate_$v" \
    -o run -- python3 tests/chunked_probe.py > "gpurun_out/gate_$v.log" 2>&1 || { echo "trace $v failed"; tail -5 "gpurun_out/gate_$v.log"; exit 1; }
  grep -h "chunked render" "gpurun_out/gate_$v.log"
  f=$(find "gpurun_out/gate_$v" -name "*kernel_stats.csv" | head -1)
  echo "== $v kernels:"; cut -d, -f1-3 "$f"
done
if [ "${FORCE:-0}" = 1 ]; then
  rm -rf gpurun_out/gate_force
  IPT_FORCE_POOL_GATE=1 timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES --kernel-trace --output-format csv \
    -d gpurun_out/gate_force -o run -- python3 tests/chunked_probe.py > gpurun_out/gate_force.log 2>&1
  echo "forced pool gate under --pmc: exit $?"; grep -h "chunked render" gpurun_out/gate_force.log
fi
