# usage: bash tools/c4ab.sh "variant ...": k_list_levels per decode-kernel variant (rocprof kernel trace)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in $1; do
  PA_AMD_LIB=pa_amd/variants/libsb_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c4ab_$v -o k -- python3 tools/c4bench.py > gpurun_out/c4ab_$v.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/c4ab_$v.log; exit 1; }
  python3 - "$v" <<'PY'
import csv, glob, sys
v = sys.argv[1]
f = glob.glob(f"gpurun_out/c4ab_{v}/**/*kernel_trace.csv", recursive=True)[0]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(f)) if "k_list_levels" in r["Kernel_Name"]]
print(v, "k_list_levels us:", round(sum(d[-5:]) / 5, 1))
PY
done
