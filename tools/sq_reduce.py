"""Per-kernel averages of the SQ / GRBM passes of tools/sq_pass.sh.

SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles summed over
waves (MI355X_MICROARCH.md, "Per-instruction cycle constants"); the table
gives each as a share of SQ_WAVE_CYCLES, VALU and SALU instructions per
launch, and the effective clock GRBM_GUI_ACTIVE / 8 / kernel time.
Usage: python tools/sq_reduce.py TAG
"""
import csv
import glob
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from pmc_reduce import short  # noqa: E402


def main(tag):
    vals = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> [per dispatch]
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(ROOT, "gpurun_out", f"{tag}_sq_*", "**",
                                   "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        meta = {}
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = short(row["Kernel_Name"]) or row["Kernel_Name"][:40]
                key = (row["Dispatch_Id"], name, row["Counter_Name"])
                per[key] += float(row["Counter_Value"])
                meta[(row["Dispatch_Id"], name)] = (int(row["End_Timestamp"]) -
                                                    int(row["Start_Timestamp"]))
        for (disp, name, ctr), v in per.items():
            vals[name][ctr].append(v)
        for (disp, name), t in meta.items():
            dur[name].append(t)
    print(f"{'kernel':22s} {'us':>8s} {'wait%':>6s} {'inst%':>6s} {'act%':>6s} {'valu%':>6s} "
          f"{'VALU/launch':>12s} {'SALU/launch':>12s} {'GHz':>5s}")
    for name in sorted(vals, key=lambda n: -sum(dur[n]) / max(1, len(dur[n]))):
        c = {k: sum(v) / len(v) for k, v in vals[name].items()}
        us = sum(dur[name]) / len(dur[name]) / 1e3
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        ghz = c.get("GRBM_GUI_ACTIVE", 0) / 8 / (us * 1e3) if "GRBM_GUI_ACTIVE" in c else 0
        print(f"{name:22s} {us:8.1f} {100 * c.get('SQ_WAIT_ANY', 0) / wc:6.1f} "
              f"{100 * c.get('SQ_WAIT_INST_ANY', 0) / wc:6.1f} "
              f"{100 * c.get('SQ_ACTIVE_INST_ANY', 0) / wc:6.1f} "
              f"{100 * c.get('SQ_ACTIVE_INST_VALU', 0) / wc:6.1f} "
              f"{c.get('SQ_INSTS_VALU', 0):12.0f} {c.get('SQ_INSTS_SALU', 0):12.0f} {ghz:5.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
