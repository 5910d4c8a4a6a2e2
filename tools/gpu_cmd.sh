for L in pa_amd/variants/libsb_prio0.so pa_amd/variants/libsb_prio3.so pa_amd/variants/libsb_prio0.so pa_amd/variants/libsb_prio3.so; do
for m in torch own; do
PA_AMD_LIB=$L SB_BENCH_STREAMS=$m timeout -k 10 300 python bench.py --no-cpu --no-b12 --no-hard --no-c4 --no-encode --no-file --steps 10 > gpurun_out/pr.json 2>/dev/null || exit 1
python -c "
import json; d=json.loads(open('gpurun_out/pr.json').read().strip().splitlines()[-1])
print('$L $m', 'c3', d['c3_f64_utf8_lz4_nullable']['ms_per_step'], 'c5', d['c5_mixed_64col']['ms_per_step'])"
done; done
