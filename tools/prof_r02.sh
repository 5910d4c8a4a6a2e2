# Round-2 profiles: per-workload kernel traces (C3, C4, C5 alone via
# tools/wlbench.py) and FETCH/WRITE PMC passes for the C3 and C4 kernels
# (k_inflate, k_bin_*, k_list_levels ...).  Summaries land in gpurun_out/prof_r02/.
set -o pipefail
out=gpurun_out/prof_r02
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for wl in c3 c4 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt_$wl -o k -- python3 tools/wlbench.py $wl 10 3 > $out/kt_$wl.log 2>&1 || { echo "trace $wl failed"; tail -5 $out/kt_$wl.log; exit 1; }
  python3 tools/prof_summary.py trace $(ls $out/kt_$wl/*kernel_trace.csv) 10 $out/${wl}_kernels.json > /dev/null || exit 1
  tail -1 $out/kt_$wl.log
done
for wl in c3 c4; do
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pf_$wl -o f -- python3 tools/wlbench.py $wl 3 1 > $out/pf_$wl.log 2>&1 || { echo "pmc fetch $wl failed"; tail -5 $out/pf_$wl.log; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pw_$wl -o w -- python3 tools/wlbench.py $wl 3 1 > $out/pw_$wl.log 2>&1 || { echo "pmc write $wl failed"; tail -5 $out/pw_$wl.log; exit 1; }
  python3 tools/prof_summary.py pmc $(ls $out/pf_$wl/*counter_collection.csv) $(ls $out/pw_$wl/*counter_collection.csv) $out/${wl}_pmc.json > /dev/null || exit 1
done
ls $out/*.json
