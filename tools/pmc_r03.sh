# Round-3 HBM traffic evidence: FETCH_SIZE / WRITE_SIZE per kernel (separate
# --pmc passes) for the calibration kernels (tools/calib_fetch.hip) and the
# C2 headline, C3, C4 and C5 decodes of this tree.  Outputs: gpurun_out/r03pmc/.
set -o pipefail
out=gpurun_out/r03pmc
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {  # tag counter cmd...
  local tag=$1 ctr=$2; shift 2
  timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d $out/$tag -o p -- "$@" > $out/$tag.log 2>&1 || { echo "pmc $tag failed"; tail -5 $out/$tag.log; exit 1; }
  echo "done $tag"
}
run cal_f FETCH_SIZE tools/calib_fetch
run cal_w WRITE_SIZE tools/calib_fetch
python3 tools/prof_summary.py pmc $(ls $out/cal_f/*counter_collection.csv) $(ls $out/cal_w/*counter_collection.csv) $out/calib.json > /dev/null || exit 1
C2="python3 bench.py --no-cpu --no-b12 --no-hard --no-c3 --no-c4 --no-c5 --no-encode --no-file --steps 6 --warmup 1"
run c2_f FETCH_SIZE $C2
run c2_w WRITE_SIZE $C2
python3 tools/prof_summary.py pmc $(ls $out/c2_f/*counter_collection.csv) $(ls $out/c2_w/*counter_collection.csv) $out/c2.json > /dev/null || exit 1
for wl in c4 c3 c5; do
  run ${wl}_f FETCH_SIZE python3 tools/wlbench.py $wl 3 1
  run ${wl}_w WRITE_SIZE python3 tools/wlbench.py $wl 3 1
  python3 tools/prof_summary.py pmc $(ls $out/${wl}_f/*counter_collection.csv) $(ls $out/${wl}_w/*counter_collection.csv) $out/$wl.json > /dev/null || exit 1
done
ls $out
