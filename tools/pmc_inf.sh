# SQ counters of k_inflate on the C3 columns (tools/c3bench.py, 10M rows),
# two passes of 8 SQ counters; summary per dispatch.
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/pmci$i -o p -- python3 $R/tools/c3bench.py ${1:-10000000} > $R/gpurun_out/pmci$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/pmci$i.log; exit 1; }
done
cd $R && python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(dict)
for i in (1, 2):
    f = glob.glob(f"gpurun_out/pmci{i}/**/*counter_collection.csv", recursive=True)
    for r in csv.DictReader(open(f[0])):
        if "k_inflate" in r["Kernel_Name"]:
            agg[(i, int(r["Dispatch_Id"]))][r["Counter_Name"]] = agg[(i, int(r["Dispatch_Id"]))].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
for k in sorted(agg):
    print(k, {c: round(v) for c, v in sorted(agg[k].items())})
PY
