"""Summarise SQ counter passes (profiles/counters.sh output) into
profiles/sq_counters.json, which bench.py reads for roofline.sq_counters.

    python profiles/sq_summary.py <counters dir> <stage> <tag>

mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8):
GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS notes)
and SQ_VALU_MFMA_BUSY_CYCLES counts SIMD cycles. Only the stage's main kernel
(the largest average duration among the matching dispatches) is kept.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNELS = {"news_fused": "fused_news_kernel", "qkv_news": "proj_qkv_kernel<false",
           "qkv_user": "proj_qkv_kernel<true", "user_fused": "fused_user_kernel",
           "qkv_news_staged": "gemm_x6_kernel"}


def main():
    # (several stages may be read from one pass over the whole forward)
    d, stage, tag = sys.argv[1], sys.argv[2], sys.argv[3]
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("void ", "").replace("nrms::(anonymous namespace)::", "").split("(")[0]
            if KERNELS[stage] in k:
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    # the main pass dispatches many more MFMAs than any helper launch
    name = max(acc, key=lambda k: max(acc[k].get("SQ_INSTS_MFMA", [0])))
    cs = {c: sorted(v)[len(v) // 2] for c, v in acc[name].items()}   # median over dispatches
    busy = cs["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cs["GRBM_GUI_ACTIVE"] / 8)
    res = {"kernel": name, "mfma_busy": round(busy, 4),
           "valu_per_mfma": round(cs["SQ_INSTS_VALU"] / cs["SQ_INSTS_MFMA"], 3),
           "lds_bank_conflict_cycles": cs.get("SQ_LDS_BANK_CONFLICT"),
           "counters": cs, "source": f"profiles/{tag}_{stage}_sq_counters.txt"}
    here = os.path.dirname(os.path.abspath(__file__))
    with open(os.path.join(here, f"{tag}_{stage}_sq_counters.txt"), "w") as fh:   # (the cited source)
        fh.write(name + "\n")
        for c in sorted(acc[name]):
            fh.write(f"  {c:<32s}{cs[c]:>20.1f}  (n={len(acc[name][c])})\n")
    path = os.path.join(here, "sq_counters.json")
    try:
        allr = json.load(open(path))
    except (OSError, ValueError):
        allr = {}
    allr[stage] = res
    json.dump(allr, open(path, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "counters"}))


if __name__ == "__main__":
    main()
