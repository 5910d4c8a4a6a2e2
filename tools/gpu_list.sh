# List parity tests + C4 kernel profile (one GPU call).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_list.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/list.log 2>&1
rc=$?; tail -3 gpurun_out/list.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4prof -o c4 -- python3 tools/c4bench.py > gpurun_out/c4prof.log 2>&1
rc=$?; grep -v "^[EW]20" gpurun_out/c4prof.log | tail -3; grep sbk gpurun_out/c4prof/c4_kernel_stats.csv | cut -c1-120; exit $rc
