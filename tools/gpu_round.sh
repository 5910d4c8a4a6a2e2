# Full GPU check: parity tests, smoke, bench, rocprof kernel trace of the bench.
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r}
timeout -k 10 400 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/${tag}_tests.log 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/${tag}_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1; echo "smoke rc=$?"; tail -1 gpurun_out/${tag}_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { echo "bench failed"; tail -5 gpurun_out/${tag}_bench.err; exit 1; }
cat gpurun_out/${tag}_bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o mix -- python bench.py --no-cpu --no-b12 --steps 20 > gpurun_out/${tag}_prof.log 2>&1; echo "prof rc=$?"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof_b12 -o b12 -- python tools/kbench.py 100000000 b12 > gpurun_out/${tag}_prof_b12.log 2>&1; echo "prof b12 rc=$?"
grep -h decode gpurun_out/${tag}_prof/*kernel_stats.csv gpurun_out/${tag}_prof_b12/*kernel_stats.csv | cut -c1-200
