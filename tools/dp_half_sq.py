"""Per-dispatch SQ table of tools/dp_half_sq.sh: for each kernel (chain1 =
one chain per wave, chain2 = two chains per wave) and chain count, the VALU
and SALU instructions, issue quad-cycles (SQ_ACTIVE_INST_ANY, summed over
waves) and wave quad-cycles per chain step.  Dispatches are matched across
the counter passes by their order (the probe launches the same sequence).
Usage: python tools/dp_half_sq.py TAG"""
import csv
import glob
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NSTEPS = 4096


def main(tag):
    rows = defaultdict(dict)  # (pass, dispatch) -> counters
    info = {}
    for k in range(2):
        for f in glob.glob(os.path.join(ROOT, "gpurun_out", f"{tag}_dpsq_{k}", "**",
                                       "*counter_collection.csv"), recursive=True):
            per = defaultdict(lambda: defaultdict(float))
            for r in csv.DictReader(open(f)):
                d = int(r["Dispatch_Id"])
                per[d][r["Counter_Name"]] += float(r["Counter_Value"])
                name = "chain2" if "chain2" in r["Kernel_Name"] else "chain1"
                grid = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
                info[(k, d)] = (name, grid)
            for d, c in per.items():
                rows[(k, d)].update(c)
    seq = {k: sorted(d for (kk, d) in rows if kk == k) for k in range(2)}
    print(f"{'kernel':8} {'chains':>7} {'waves/SIMD':>10} {'VALU/step':>10} {'SALU/step':>10} "
          f"{'issue qc/step':>13} {'wave qc/step':>12} {'busy qc/step':>12}")
    for i, d0 in enumerate(seq[0]):
        name, grid = info[(0, d0)]
        c = rows[(0, d0)]
        waves = grid // 64
        chains = waves * (2 if name == "chain2" else 1)
        if waves in (64, 128):   # the bit-exactness launches (128 chains)
            continue
        steps = chains * NSTEPS
        print(f"{name:8} {chains:7d} {waves / 1024:10.2f} {c['SQ_INSTS_VALU'] / steps:10.2f} "
              f"{c['SQ_INSTS_SALU'] / steps:10.2f} {c['SQ_ACTIVE_INST_ANY'] / steps:13.2f} "
              f"{c['SQ_WAVE_CYCLES'] / steps:12.2f} {c['SQ_BUSY_CYCLES'] / steps:12.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
