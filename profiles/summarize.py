"""Summarise a profiles/run_profile.sh output directory into tracked files.

    python profiles/summarize.py gpurun_out/prof_r01 r01

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats, copied verbatim),
profiles/<tag>_summary.md (per-stage avg duration from the kernel trace,
per-launch HBM traffic from the PMC passes) and profiles/pmc_traffic.json
(per-stage hbm_bytes_per_launch read by bench.py).

Traffic correction (MI355X_MICROARCH.md §HBM): on gfx950 FETCH_SIZE reports
half the bytes of a wide coalesced streaming read, so read bytes are taken as
2 x FETCH_SIZE x 1024; WRITE_SIZE x 1024 is exact for 16-B streaming stores.
Both include Infinity-Cache hits (memory-side request counters).
"""
import csv
import re
import json
import os
import shutil
import sys
from collections import defaultdict

HERE = os.path.dirname(os.path.abspath(__file__))


def stage_of(name, grid_threads, wg):
    """Map (kernel, grid) of the bench workload (B=1024, V=70976) to a stage."""
    blocks = grid_threads // max(wg, 1)
    if "proj_x6_kernel<true" in name or "proj_qkv_kernel<true" in name:   # row-list mode: the UserEncoder after dedupe
        return "qkv_user"
    if "proj_x6_kernel<false" in name or "proj_qkv_kernel<false" in name:
        return "qkv_news"
    if "proj_x6_pack" in name:
        return "pack_qkv"
    if "forward_pack" in name:
        return "pack_all"
    if "pack_additive_b" in name:
        return "pack_add_news"
    if "pack_user_b" in name:
        return "pack_add_user"
    if "classify_groups" in name or "classify_titles" in name:
        return "classify"
    if "broadcast_padding" in name:
        return "broadcast"
    if "user_row_list" in name:
        return "user_row_list"
    if "gemm_xwt_f32_kernel<12, false>" in name or "gemm_x6" in name:
        return "qkv_user" if blocks in (2000, 4000) else "qkv_news"   # M = 51,200: 128- or 64-row tiles
    if "gemm_xwt_f32_kernel<13" in name:
        return "addscore_news" if blocks > 400 else "addscore_user"
    if "mhsa_rawexp_kernel<20" in name:
        return "mhsa_news"
    if "mhsa_rawexp_kernel<50" in name:
        return "mhsa_user"
    if "additive_pool_kernel" in name:
        return "pool_news" if blocks > 256 else "pool_user"
    if "score_kernel" in name:
        return "score"
    if "user_order_kernel" in name:   # the UserEncoder's dispatch order (LPT), part of its stage
        return "user_order"
    if "fused_user" in name:
        return "user_fused"
    if "fused_news" in name:   # the EXACT recheck launch (<MODE, true, ..>) is its own line
        m = re.search(r"fused_news_kernel<\d+, (true|false)", name)
        return "news_recheck" if m and m.group(1) == "true" else "news_fused"
    if "gather_rows_kernel" in name:
        return "gather"
    return None


def read_rows(path):
    with open(path) as f:
        rows = list(csv.DictReader(f))
    for r in rows:  # kernel-trace CSVs split grid / workgroup sizes per axis
        if "Grid_Size" not in r:
            r["Grid_Size"] = r["Grid_Size_X"]
            r["Workgroup_Size"] = r["Workgroup_Size_X"]
    return rows


def main(src, tag):
    import glob
    trace = [r for p in sorted(glob.glob(os.path.join(src, "trace", "*_kernel_trace.csv")))
             for r in read_rows(p)]
    dur = defaultdict(list)
    kname = {}
    for r in trace:
        st = stage_of(r["Kernel_Name"], int(r["Grid_Size"]), int(r["Workgroup_Size"]))
        if st:
            dur[st].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            kname[st] = r["Kernel_Name"]

    def counters(sub, cname):
        acc = defaultdict(list)
        rows = [r for p in sorted(glob.glob(os.path.join(src, sub, "*_counter_collection.csv")))
                for r in read_rows(p)]
        for r in rows:
            if r["Counter_Name"] != cname:
                continue
            st = stage_of(r["Kernel_Name"], int(r["Grid_Size"]), int(r["Workgroup_Size"]))
            if st:
                acc[st].append(float(r["Counter_Value"]))
        return acc

    fetch = counters("fetch", "FETCH_SIZE")
    write = counters("write", "WRITE_SIZE")
    traffic = {}
    lines = [f"# rocprofv3 summary `{tag}` (bench.py workload, B=1024, folded projection)", "",
             "| stage | kernel | launches | avg us | FETCH_SIZE KB/launch | WRITE_SIZE KB/launch | HBM bytes/launch (2xFETCH+WRITE) |",
             "|---|---|---|---|---|---|---|"]
    for st in sorted(dur, key=lambda s: -sum(dur[s]) / len(dur[s])):
        avg_us = sum(dur[st]) / len(dur[st]) / 1e3
        f = sum(fetch[st]) / len(fetch[st]) if fetch.get(st) else None
        w = sum(write[st]) / len(write[st]) if write.get(st) else None
        hbm = None if f is None or w is None else int((2 * f + w) * 1024)
        short = kname[st].replace("void ", "").replace("nrms::(anonymous namespace)::", "")
        short = short.split("(")[0]
        traffic[st] = {"kernel": short, "avg_duration_us": round(avg_us, 2),
                       "fetch_kb": f, "write_kb": w, "hbm_bytes_per_launch": hbm}
        lines.append(f"| {st} | `{short}` | {len(dur[st])} | {avg_us:.1f} | "
                     f"{'' if f is None else f'{f:.0f}'} | {'' if w is None else f'{w:.0f}'} | "
                     f"{'' if hbm is None else hbm} |")
    with open(os.path.join(HERE, f"{tag}_summary.md"), "w") as fo:
        fo.write("\n".join(lines) + "\n")
    with open(os.path.join(HERE, "pmc_traffic.json"), "w") as fo:
        json.dump(traffic, fo, indent=1)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                os.path.join(HERE, f"{tag}_kernel_stats.csv"))
    g = os.path.join(src, "trace", "gather_kernel_stats.csv")
    if os.path.exists(g):
        shutil.copy(g, os.path.join(HERE, f"{tag}_gather_kernel_stats.csv"))
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
