cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu2.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu2.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r1 -o bench -- python bench.py --steps 4 --cpu-seconds 0 --no-counters > gpurun_out/prof_r1_bench.json 2> gpurun_out/prof_r1.err || { echo "rocprof stats failed"; tail gpurun_out/prof_r1.err; exit 1; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o fetch -- python bench.py --steps 2 --cpu-seconds 0 --no-counters > gpurun_out/pmc_fetch.json 2> gpurun_out/pmc_fetch.err || { echo "pmc fetch failed"; tail gpurun_out/pmc_fetch.err; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o write -- python bench.py --steps 2 --cpu-seconds 0 --no-counters > gpurun_out/pmc_write.json 2> gpurun_out/pmc_write.err || { echo "pmc write failed"; tail gpurun_out/pmc_write.err; exit 1; }
find gpurun_out/prof_r1 gpurun_out/pmc_fetch gpurun_out/pmc_write -type f | head -30
