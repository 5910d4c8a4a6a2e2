# Round-end check: every GPU test, smoke, the bench line, rocprof kernel stats of the headline workload.
set -o pipefail
out=gpurun_out/final
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests failed"; tail -20 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -5 $out/bench.err; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt_c2 -o k -- python3 bench.py --no-cpu --no-b12 --no-hard --no-c3 --no-c4 --no-c5 --no-encode --no-file --steps 20 > $out/kt_c2.log 2>&1 || { echo "trace failed"; exit 1; }
grep -h "decode_staged" $out/kt_c2/*kernel_stats.csv | cut -c1-120
