# per-phase lane utilisation (IPT_PROF) and step-segment shares (IPT_STAMP) for $CONFIGS
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in ${CONFIGS:-c2}; do
  for v in prof stamp; do
    IPT_LIB_PATH=ipt_amd/lib/abl/libipt_$v.so timeout -k 10 300 python scripts/prof_phases.py $c > gpurun_out/prof_${v}_$c.txt 2>&1 || { echo "$v $c failed"; tail -5 gpurun_out/prof_${v}_$c.txt; exit 1; }
    echo "== $v $c"; cat gpurun_out/prof_${v}_$c.txt
  done
done
