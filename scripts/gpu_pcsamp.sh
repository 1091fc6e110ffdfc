# PC sampling of the C2 bench (profiling only)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > gpurun_out/rocprof_list.txt 2>&1; echo "list rc=$?"
grep -i -A12 "pc sampl\|pc_sampl" gpurun_out/rocprof_list.txt | head -40
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${METHOD:-stochastic} --pc-sampling-unit ${UNIT:-cycles} --pc-sampling-interval ${INTERVAL:-1048576} --output-format csv -d gpurun_out/pcs -o pcs -- python bench.py --steps 1 --warmup 0 --cpu-seconds 0 --no-counters > gpurun_out/pcs_bench.json 2> gpurun_out/pcs.err; echo "pcs rc=$?"
tail -5 gpurun_out/pcs.err
find gpurun_out/pcs -type f | head; du -sh gpurun_out/pcs
