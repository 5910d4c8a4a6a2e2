# Run a subset of the GPU tests in one process (args: tag, pytest selection).
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread "$@" > gpurun_out/${tag}.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -30 gpurun_out/${tag}.log; exit $rc
