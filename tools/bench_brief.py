"""One line per workload of a bench.py JSON line: python tools/bench_brief.py <bench.json>"""
import json
import sys


def main():
    d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    print("c2", d["value"], "GB/s", d["ms_per_step"], "ms wall", d["roofline"]["kernel_ms"], "ms kernel, frac",
          d["roofline"]["frac"])
    for k in ("c2_hard_mix", "bitpack_b12"):
        print(k, d[k]["decoded_GBps"], "GB/s", d[k]["kernel_ms"], "ms kernel")
    for k in ("c3_f64_utf8_lz4_nullable", "c4_list_int32_nested", "c5_mixed_64col"):
        x = d[k]
        print(k, x["ms_per_step"], "ms wall", x["kernel_ms_per_step"], "ms kernel, frac", x["roofline_frac"],
              "wall frac", x["roofline_frac_wall"])
    e = d.get("encode_gpu", {})
    for k, v in e.items():
        if "input_GBps" in v:
            print("encode", k, v["input_GBps"], "GB/s")
    c5 = d["c5_mixed_64col"]
    print("encode c5", c5.get("encode_gpu_GBps"), "GB/s")


if __name__ == "__main__":
    main()
