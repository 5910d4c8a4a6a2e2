"""Publish one PMC run (tools/pmc_traffic.sh output directory) into profiles/:
python tools/publish_traffic.py <gpurun_out/r03pmc> <tag>.

Writes profiles/<tag>_pmc_traffic.json -- one entry per bench.py workload
key (bench.load_traffic reads it), each with the commit the run measured,
per-step fetch / write / HBM bytes, the algorithmic bytes and
traffic_over_algorithmic, and the per-kernel split -- and copies each
workload's rocprofv3 kernel statistics (<tag>_<wl>_rocprof_kernel_stats.csv)
and kernel-time summary (<tag>_<wl>_kernels.json)."""
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH_KEYS = {"c2": "c2_int32_adaptive_bitpack_dict", "c2h": "c2_hard_mix", "c3": "c3_f64_utf8_lz4_nullable",
              "c4": "c4_list_int32_nested", "c5": "c5_mixed_64col"}


def main():
    src, tag = sys.argv[1], sys.argv[2]
    prof = os.path.join(ROOT, "profiles")
    out = {}
    for wl, key in BENCH_KEYS.items():
        p = os.path.join(src, f"{wl}_traffic.json")
        if not os.path.exists(p):
            continue
        t = json.load(open(p))
        st = t["step"]
        out[key] = {"commit": t["commit"], "round": t["round"], "source": f"profiles/{tag}_pmc_traffic.json",
                    "window": t.get("window"), "correction": t["correction"],
                    "hbm_bytes_per_step": st["hbm_bytes"], "fetch_bytes_per_step": st["fetch_bytes"],
                    "write_bytes_per_step": st["write_bytes"],
                    "algorithmic_bytes_per_step": t["algorithmic_bytes_per_step"],
                    "traffic_over_algorithmic": st["traffic_over_algorithmic"],
                    "kernels": {k: v for k, v in t["kernels"].items()
                                if v["fetch_bytes_per_step"] + v["write_bytes_per_step"] >= 1 << 20}}
        stats = os.path.join(src, f"kt_{wl}", "k_kernel_stats.csv")
        if os.path.exists(stats):
            shutil.copy(stats, os.path.join(prof, f"{tag}_{wl}_rocprof_kernel_stats.csv"))
        kj = os.path.join(src, f"{wl}_kernels.json")
        if os.path.exists(kj):
            shutil.copy(kj, os.path.join(prof, f"{tag}_{wl}_kernels.json"))
    json.dump(out, open(os.path.join(prof, f"{tag}_pmc_traffic.json"), "w"), indent=1)
    for k, v in out.items():
        print(k, v["commit"], v["traffic_over_algorithmic"])


if __name__ == "__main__":
    main()
