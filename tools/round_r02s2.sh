# End-of-session evidence (round 2): the bench line, a rocprofv3 kernel trace
# of the bench's headline workload (C2) and per-workload kernel splits + PMC
# FETCH/WRITE bytes for C4 (the list walk).  Outputs under gpurun_out/r02s2/.
set -o pipefail
out=gpurun_out/r02s2
mkdir -p $out
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -5 $out/bench.err; exit 1; }
tail -c 600 $out/bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt_c2 -o k -- python3 bench.py --no-cpu --no-b12 --no-hard --no-c3 --no-c4 --no-c5 --no-encode --no-file --steps 20 > $out/kt_c2.log 2>&1 || { echo "c2 trace failed"; exit 1; }
grep -h "decode_staged" $out/kt_c2/*kernel_stats.csv | cut -c1-160
for wl in c4 c5 c3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt_$wl -o k -- python3 tools/wlbench.py $wl 10 3 > $out/kt_$wl.log 2>&1 || { echo "trace $wl failed"; tail -5 $out/kt_$wl.log; exit 1; }
  python3 tools/prof_summary.py trace $(ls $out/kt_$wl/*kernel_trace.csv) 10 $out/${wl}_kernels.json > /dev/null || exit 1
  tail -1 $out/kt_$wl.log
done
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pf_c4 -o f -- python3 tools/wlbench.py c4 3 1 > $out/pf_c4.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pw_c4 -o w -- python3 tools/wlbench.py c4 3 1 > $out/pw_c4.log 2>&1 || { echo "pmc write failed"; exit 1; }
python3 tools/prof_summary.py pmc $(ls $out/pf_c4/*counter_collection.csv) $(ls $out/pw_c4/*counter_collection.csv) $out/c4_pmc.json > /dev/null || exit 1
ls $out
