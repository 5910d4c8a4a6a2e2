# C4 iteration: List / nested GPU tests, per-kernel trace of the C4 decode, SQ counters of the levels walk.
set -o pipefail
bash tools/gpu_tests.sh lst tests/test_gpu_list.py tests/test_gpu_nested.py tests/test_gpu_shard.py tests/test_gpu_abi_calls.py -m gpu --timeout 120 || exit 1
bash tools/kprof.sh c4 python3 tools/c4bench.py || exit 1
grep ok= gpurun_out/kp_c4.log
ROWS=50000000 bash tools/pmc_list.sh > /dev/null || exit 1
python3 - <<'PY'
import csv, glob, collections
for d in ["pmcl1", "pmcl2"]:
    f = glob.glob(f"gpurun_out/{d}/**/*counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:30]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        if "list_" in k:
            print(k, {c: round(sum(x) / len(x)) for c, x in v.items()})
PY
