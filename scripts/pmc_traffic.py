"""HBM traffic per launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; separate runs).

usage: python scripts/pmc_traffic.py FETCH_DIR WRITE_DIR OUT_JSON [B T]
FETCH_SIZE / WRITE_SIZE are kilobytes per dispatch; gfx950 FETCH_SIZE counts half the bytes of wide
(16 B/lane) coalesced reads (MI355X_MICROARCH.md, HBM section), so it is doubled here.  Writes
{"shape": {"B", "T"}, "kernels": {kernel-short-name: {"fetch_bytes", "write_bytes", "hbm_bytes",
"dispatches"}}} averaged per launch (bench.py reads the traffic of the shape it runs).""" 
import csv
import json
import sys
from collections import defaultdict

SHORT = {"attn_bwd_roles_kernel": "attn_bwd_roles", "gemm_lnx_fwd_kernel": "gemm_lnx_fwd",
         "gemm_lnx_bwd_kernel": "gemm_lnx_bwd", "gemm_lnx64_kernel": "gemm_lnx_small",
         "attn_bwd_kv_dma_kernel": "attn_bwd_dkdv", "attn_bwd_kv_kernel": "attn_bwd_dkdv",
         "attn_bwd_q_dma_kernel": "attn_bwd_dq", "attn_fwd_dma_kernel": "attn_fwd", "attn_fwd_pp_kernel": "attn_fwd",
         "attn_fwd32_kernel": "attn_fwd", "wgrad8_grouped_kernel": "wgrad_grouped", "concat_kernel": "concat",
         "wgrad_grouped_kernel": "wgrad_grouped", "gemm8_kernel": "gemm8", "colsum_batched_kernel": "colsum_batched", "attn_bwd_q_kernel": "attn_bwd_dq", "attn_fwd_kernel": "attn_fwd",
         "gemm_bf16_dma_kernel": "gemm_bf16", "ln_bwd_kernel": "ln_bwd", "ln_fwd_kernel": "ln_fwd",
         "splitk_reduce_kernel": "splitk_reduce", "adam_kernel": "adam"}


def load(d, counter):
    per = defaultdict(dict)
    with open(f"{d}/run_counter_collection.csv") as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            name = next((v for k, v in SHORT.items() if k in row["Kernel_Name"]), None)
            if name:
                per[name][row["Dispatch_Id"]] = per[name].get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
    return {k: (sum(v.values()) / len(v), len(v)) for k, v in per.items()}


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        fb = fetch.get(k, (0.0, 0))[0] * 1024 * 2
        wb = write.get(k, (0.0, 0))[0] * 1024
        out[k] = {"fetch_bytes": fb, "write_bytes": wb, "hbm_bytes": fb + wb,
                  "dispatches": max(fetch.get(k, (0, 0))[1], write.get(k, (0, 0))[1])}
    doc = {"kernels": out}
    if len(sys.argv) > 5:
        doc = {"shape": {"B": int(sys.argv[4]), "T": int(sys.argv[5])}, "kernels": out}
    with open(sys.argv[3], "w") as f:
        json.dump(doc, f, indent=1)
    for k, v in out.items():
        print(f"{k:16s} {v['hbm_bytes'] / 1e6:10.1f} MB/launch (fetch {v['fetch_bytes'] / 1e6:.1f}, "
              f"write {v['write_bytes'] / 1e6:.1f}) n={v['dispatches']}")


if __name__ == "__main__":
    main()
