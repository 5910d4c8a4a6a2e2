# C4 levels walk: step mode vs page mode (SB_LIST_PAGE), kernel times under rocprof
set -o pipefail
bash tools/gpu_tests.sh lst tests/test_gpu_list.py -m gpu --timeout 120 || exit 1
SB_LIST_PAGE=1 bash tools/gpu_tests.sh lstp tests/test_gpu_list.py tests/test_gpu_shard.py -m gpu --timeout 120 || exit 1
bash tools/kprof.sh c4s python3 tools/c4bench.py | grep -E "list|staged" | tail -4
grep ok= gpurun_out/kp_c4s.log
SB_LIST_PAGE=1 bash tools/kprof.sh c4p python3 tools/c4bench.py | grep -E "list|staged" | tail -4
grep ok= gpurun_out/kp_c4p.log
