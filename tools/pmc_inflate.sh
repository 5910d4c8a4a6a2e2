# SQ counters of k_inflate per dispatch for tools/c3bench.py (F64 dispatches first, then Utf8).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH --output-format csv -d gpurun_out/pmci -o p -- python3 tools/c3bench.py ${1:-10000000} > gpurun_out/pmci.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/pmci/**/*counter_collection.csv", recursive=True)
agg = collections.defaultdict(dict)
for r in csv.DictReader(open(f[0])):
    if "inflate" in r["Kernel_Name"]:
        agg[int(r["Dispatch_Id"])][r["Counter_Name"]] = agg[int(r["Dispatch_Id"])].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
for d in sorted(agg):
    print(d, {c: round(v) for c, v in sorted(agg[d].items())})
PY
