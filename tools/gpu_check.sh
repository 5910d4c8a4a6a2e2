# GPU check: parity tests (one process), smoke, default bench.  Each step has
# its own time limit; the script stops at the first failure.
set -o pipefail
tag=${1:-r}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${tag}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/${tag}_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/${tag}_bench.json; tail -3 gpurun_out/${tag}_bench.err; exit $rc
