# Round-3 full check: every GPU test, smoke, the bench line, then the PMC
# traffic passes and kernel traces of tools/pmc_r03.sh.  Stops at the first
# failing step.  Outputs under gpurun_out/<tag>/.
set -o pipefail
tag=${1:-r03}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -5 $out/bench.err; exit 1; }
cat $out/bench.json
[ -n "$NO_PMC" ] && exit 0
bash tools/pmc_r03.sh
