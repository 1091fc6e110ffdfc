cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { echo bench failed; tail -20 gpurun_out/bench1.err; exit 1; }
cat gpurun_out/bench1.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 4 --cpu-seconds 0 --no-counters > gpurun_out/prof_bench.json 2> gpurun_out/prof.err || { echo rocprof failed; tail -20 gpurun_out/prof.err; exit 1; }
find gpurun_out/prof -name "*stats*" | head
