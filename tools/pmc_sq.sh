# SQ counters of one kernel under a python workload, two passes of 8 SQ counters:
#   bash tools/pmc_sq.sh <kernel substring> <script.py> [args...]
# per-dispatch totals printed (last 4 dispatches).
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
kern=$1; script=$2; shift 2
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/pmcsq$i -o p -- python3 $R/$script "$@" > $R/gpurun_out/pmcsq$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/pmcsq$i.log; exit 1; }
done
cd $R && python3 - "$kern" <<'PY'
import csv, glob, collections, sys
agg = collections.defaultdict(dict)
for i in (1, 2):
    f = glob.glob(f"gpurun_out/pmcsq{i}/**/*counter_collection.csv", recursive=True)
    for r in csv.DictReader(open(f[0])):
        if sys.argv[1] in r["Kernel_Name"]:
            k = (i, int(r["Dispatch_Id"]))
            agg[k][r["Counter_Name"]] = agg[k].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
for i in (1, 2):
    for k in sorted(x for x in agg if x[0] == i)[-4:]:
        print(k, {c: round(v) for c, v in sorted(agg[k].items())})
PY
