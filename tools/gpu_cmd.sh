for v in lvcur acc4k st2k both lvcur acc4k; do
PA_AMD_LIB=$GRAFT_REPO_ROOT/pa_amd/variants/libsb_$v.so bash tools/gpu_r04.sh prof lv_$v tools/c4bench.py > /dev/null || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/lv_${v}_kernels.json'))
x={k[:40]:v['avg_us'] for k,v in d.items() if 'list_levels' in k or 'decode_staged' in k}
print('$v', x)"
grep ms/step gpurun_out/lv_${v}_kt.log
done
