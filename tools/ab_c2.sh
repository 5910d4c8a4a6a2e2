# A/B of the C2 headline kernel between library variants (pa_amd/variants/libsb_<v>.so), alternating.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for v in $VARIANTS; do
  PA_AMD_LIB=pa_amd/variants/libsb_$v.so timeout -k 10 200 python bench.py --no-cpu --no-b12 --no-hard --no-c3 --no-c4 --no-c5 --no-encode --no-file --steps 40 > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo "$v failed"; tail -3 gpurun_out/ab_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$v', d['value'],d['roofline']['frac'],d['roofline']['kernel_ms'])"
done
done
