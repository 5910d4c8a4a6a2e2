# rocprofv3 runs for the bench's decode kernel: kernel trace + stats of the
# exact bench command, then two PMC passes (FETCH_SIZE, WRITE_SIZE).
set -o pipefail
tag=${1:-r01}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_kt -o bench -- python3 bench.py --no-cpu > gpurun_out/${tag}_kt.json 2> gpurun_out/${tag}_kt.err || { echo "kt failed"; tail -5 gpurun_out/${tag}_kt.err; exit 1; }
cat gpurun_out/${tag}_kt.json
grep -h decode gpurun_out/${tag}_kt/bench_kernel_stats.csv | cut -c1-200
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${tag}_pf -o f -- python3 bench.py --no-cpu --no-b12 --no-hard --no-c3 --no-c4 --no-c5 --steps 5 --warmup 2 > gpurun_out/${tag}_pf.log 2>&1 || { echo "pmc fetch failed"; tail -5 gpurun_out/${tag}_pf.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${tag}_pw -o w -- python3 bench.py --no-cpu --no-b12 --no-hard --no-c3 --no-c4 --no-c5 --steps 5 --warmup 2 > gpurun_out/${tag}_pw.log 2>&1 || { echo "pmc write failed"; tail -5 gpurun_out/${tag}_pw.log; exit 1; }
ls gpurun_out/${tag}_pf gpurun_out/${tag}_pw
python3 tools/prof_split.py gpurun_out/${tag}_kt/bench_kernel_trace.csv 3 20 gpurun_out/${tag}_kernel_summary.json
