"""Reduce rocprofv3 FETCH_SIZE / WRITE_SIZE passes to bytes per launch.

FETCH_SIZE and WRITE_SIZE are reported in KiB.  On gfx950 FETCH_SIZE counts
wide coalesced streaming reads at half their bytes (MI355X_MICROARCH.md,
"HBM"), so it is doubled; WRITE_SIZE is exact for streaming stores.
Usage: python tools/pmc_reduce.py TAG CONFIG  (after tools/pmc.sh)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# kernel symbol -> name used by the library's in-process profiler (bench.py)
NAMES = [("hpair_kernel", "stage_a_h"), ("stage_a_kernel", "stage_a"), ("stage_b_kernel", "stage_b"),
         ("pair_final_kernel", "pair_bwd_L4_final"), ("pair_final2_kernel", "pair_bwd_L4_final"),
         ("vfwd_kernel", "vfwd"), ("cost_h_kernel", "cost_h"), ("cost_h2_kernel", "cost_h"),
         ("cost_h_global_kernel", "cost_h"), ("cost_ck_kernel", "cost_ck"), ("vstrip_kernel", "vstrip"),
         ("sky_words_kernel", "sky_words"),
         ("census_kernel", "census"), ("lr_kernel", "lr"), ("lr_cm_kernel", "lr"), ("sweep_kernel<7", "sweep_L8_acc"),
         ("sweep_split_kernel<7", "sweep_L8_acc"),
         ("median_fill_kernel", "post_median"), ("cc_local_kernel", "post_cc_local"),
         ("cc_merge_kernel", "post_cc_merge"), ("cc_count_kernel", "post_cc_count"),
         ("cc_apply_kernel", "post_cc_apply"), ("pf_prep_kernel", "post_prep"),
         ("lk_refine_kernel", "lk_refine"), ("sky_columns_kernel", "sky_columns"),
         ("sky_gray_kernel", "sky_gray"), ("bm_wta_kernel", "bm_wta"),
         # joint two-view launches (K64)
         ("stage_a2_kernel", "stage_a"), ("stage_b2_kernel", "stage_b"), ("sweep2_kernel<7", "sweep_L8_acc")]


def short(name):
    # the forward bands' diagonal stage A launches (template ROLES 1)
    key = "stage_a_kernel<"
    if key in name:
        args = name[name.index(key) + len(key):].split(">")[0].split(", ")
        if len(args) == 4 and args[3] == "1":
            return "stage_a_d"
        if len(args) == 4 and args[2] == "true":
            return "stage_a_hp"
    # the banded schedule's stage kernels (template flag HP / HROWS)
    for key, flag, val in (("stage_a_kernel<", "true", "stage_a_hp"), ("stage_b_kernel<", "false", "stage_b_d2")):
        if key in name:
            args = name[name.index(key) + len(key):].split(">")[0].split(", ")
            if len(args) == 3 and args[2] == flag:
                return val
    # the slanted passes, and vfwd writing the whole L3 volume (template L3OUT)
    if "slant_kernel<" in name:
        return "slant_up" if name.split("slant_kernel<")[1].startswith("true") else "slant_down"
    # (vfwd2_kernel<V, FULL, WIN, PF, L3OUT>: both views in one launch)
    if "vfwd2_kernel<" in name:
        args = name[name.index("vfwd2_kernel<") + len("vfwd2_kernel<"):].split(">")[0].split(", ")
        return "vfwd_l3" if len(args) >= 5 and args[4] == "true" else "vfwd"
    if "vfwd_kernel<" in name:
        args = name[name.index("vfwd_kernel<") + len("vfwd_kernel<"):].split(">")[0].split(", ")
        if len(args) >= 6 and args[5] == "true":
            return "vfwd_l3"
    for key, val in NAMES:
        if key in name:
            return val
    return None


def per_launch(tag, counter):
    files = glob.glob(os.path.join(ROOT, "gpurun_out", f"{tag}_pmc_{counter}", "**",
                                   "*counter_collection.csv"), recursive=True)
    acc = defaultdict(list)
    for f in files:
        for row in csv.DictReader(open(f)):
            k = short(row.get("Kernel_Name", ""))
            if k and row.get("Counter_Name") == counter:
                acc[k].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    tag, cfg = sys.argv[1], sys.argv[2]
    fetch = per_launch(tag, "FETCH_SIZE")
    write = per_launch(tag, "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        rd = 2.0 * fetch.get(k, 0.0) * 1024.0
        wr = write.get(k, 0.0) * 1024.0
        out[k] = {"read_bytes": rd, "write_bytes": wr, "bytes": rd + wr}
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    data = {}
    if os.path.exists(path):
        data = json.load(open(path))
    data[cfg] = {k: v["bytes"] for k, v in out.items()}
    data.setdefault("_detail", {})[cfg] = out
    sys.path.insert(0, ROOT)
    from bench import source_sha
    # the run tag, the commit the tree was taken from (GIT_SHA, passed in by
    # the caller: the GPU box has no .git) and the hash of the library's
    # sources, which bench.py compares with the code it runs
    data.setdefault("_tags", {})[cfg] = {"tag": tag, "git": os.environ.get("GIT_SHA", "unknown"),
                                         "src_sha": source_sha()}
    data["_source"] = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes (per config in "
                       "_tags: run tag, git commit, sha of the library sources); FETCH_SIZE "
                       "doubled (gfx950), KiB -> bytes; per-launch means; memory-side bytes "
                       "(Infinity Cache hits included, MI355X_MICROARCH.md 'HBM')")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    json.dump(data, open(path, "w"), indent=1, sort_keys=True)
    for k, v in out.items():
        print(f"  {k:22s} read {v['read_bytes']/1e6:9.1f} MB  write {v['write_bytes']/1e6:9.1f} MB")


if __name__ == "__main__":
    main()
