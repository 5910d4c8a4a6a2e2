# SQ counters of the C3 LZ4 decoders (k_inflate): two passes of 8 SQ counters.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/pmc3a -o p -- python3 tools/c3bench.py 10000000 > gpurun_out/pmc3a.log 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmc3b -o p -- python3 tools/c3bench.py 10000000 > gpurun_out/pmc3b.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
for d in ("gpurun_out/pmc3a", "gpurun_out/pmc3b"):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"][:40]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[(k, r["Counter_Name"])] += 1
    for k, v in agg.items():
        if "inflate" in k or "bin_" in k:
            print(d, k, {c: round(x) for c, x in v.items()})
PY
