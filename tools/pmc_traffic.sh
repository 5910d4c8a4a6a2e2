# HBM traffic evidence: FETCH_SIZE / WRITE_SIZE per kernel (separate
# --pmc passes) and a kernel trace of the C2 headline, C3, C4 and C5 decodes
# of this tree.  Outputs: $OUT (default gpurun_out/pmc/) (summaries: <wl>_traffic.json).
set -o pipefail
out=${OUT:-gpurun_out/pmc}
mkdir -p $out
commit=${COMMIT:-unknown}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {  # tag counter cmd...
  local tag=$1 ctr=$2; shift 2
  timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d $out/$tag -o p -- "$@" > $out/$tag.log 2>&1 || { echo "pmc $tag failed"; tail -5 $out/$tag.log; exit 1; }
  echo "done $tag"
}
for wl in ${WLS:-c2 c2h c3 c4 c5}; do
  run ${wl}_f FETCH_SIZE python3 tools/wlbench.py $wl 3 1 $out/${wl}_bytes.json
  run ${wl}_w WRITE_SIZE python3 tools/wlbench.py $wl 3 1 $out/${wl}_bytes_w.json
  python3 tools/pmc_summary.py $wl $(ls $out/${wl}_f/*counter_collection.csv) $(ls $out/${wl}_w/*counter_collection.csv) $out/${wl}_bytes.json $out/${wl}_traffic.json $commit || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt_$wl -o k -- python3 tools/wlbench.py $wl 10 3 $out/${wl}_bytes_k.json > $out/kt_$wl.log 2>&1 || { echo "trace $wl failed"; exit 1; }
  python3 tools/prof_summary.py trace $(ls $out/kt_$wl/*kernel_trace.csv) 10 $out/${wl}_kernels.json > /dev/null || exit 1
  tail -1 $out/kt_$wl.log
done
ls $out
