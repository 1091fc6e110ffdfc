cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/pmc_list.txt 2>&1
grep -E "^\s*(SQ_|TCC_EA|GRBM)" gpurun_out/pmc_list.txt | head -5
wc -l gpurun_out/pmc_list.txt
