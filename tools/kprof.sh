# Per-kernel durations (last dispatches) of a command under rocprofv3: bash tools/kprof.sh tag cmd...
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kp_$tag -o k -- "$@" > gpurun_out/kp_$tag.log 2>&1 || exit 1
python3 - "$tag" <<'PY'
import csv, glob, sys
tag = sys.argv[1]
f = glob.glob(f"gpurun_out/kp_{tag}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
for r in rows[-int(40):]:
    print(r["Kernel_Name"][:70], round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, 1))
PY
