# k_inflate instruction counters per decode-kernel variant: bash tools/pmc_variants.sh "v1 v2 ..." [rows]
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in $1; do
  PA_AMD_LIB=pa_amd/variants/libsb_$v.so timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/pmcv_$v -o p -- python3 tools/c3bench.py ${2:-10000000} > gpurun_out/pmcv_$v.log 2>&1 || exit 1
  python3 - "$v" <<'PY'
import csv, glob, collections, sys
v = sys.argv[1]
f = glob.glob(f"gpurun_out/pmcv_{v}/**/*counter_collection.csv", recursive=True)
agg = collections.defaultdict(dict)
for r in csv.DictReader(open(f[0])):
    if "inflate" in r["Kernel_Name"]:
        d = agg[int(r["Dispatch_Id"])]
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0) + float(r["Counter_Value"])
ds = sorted(agg)
for name, d in (("f64", ds[1]), ("utf8", ds[-1])):
    print(v, name, {c[8:]: round(x / 1e6, 1) for c, x in sorted(agg[d].items())})
PY
done
