"""Reduce tools/timer_check.sh: for the slanted passes and the dominant
kernels, the library's event averages (bench.py's profile pass) in the
traced run against rocprofv3's durations of exactly those launches (the last
`steps` launches of each kernel in the trace), and the untraced runs' event
averages before and after.  Usage: python tools/timer_check.py TAG"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from pmc_reduce import short  # noqa: E402


def line(path):
    with open(path) as fh:
        return json.loads([x for x in fh.read().splitlines() if x.startswith("{")][-1])


def main(tag):
    g = os.path.join(ROOT, "gpurun_out")
    tr = line(os.path.join(g, f"{tag}_tc_traced.json"))
    u1 = line(os.path.join(g, f"{tag}_tc_untraced1.json"))
    u2 = line(os.path.join(g, f"{tag}_tc_untraced2.json"))
    steps = tr["steps"]
    f = glob.glob(os.path.join(g, f"{tag}_tc_trace", "**", "*kernel_trace.csv"), recursive=True)[0]
    durs = {}
    with open(f) as fh:
        for r in csv.DictReader(fh):
            durs.setdefault(short(r["Kernel_Name"]) or r["Kernel_Name"][:40], []).append(
                (int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    print(f"config {tr['config']['width']}x{tr['config']['height']} D={tr['config']['max_disp']}: "
          f"ms/step untraced {u1['ms_per_step']} / {u2['ms_per_step']}, traced {tr['ms_per_step']}")
    print(f"{'kernel':22} {'events(traced)':>14} {'rocprof same launches':>22} {'diff':>7} "
          f"{'events untraced 1 / 2':>22}")
    for name in sorted(tr["kernels"], key=lambda k: -tr["kernels"][k]["share_per_step_ms"])[:8]:
        ev = tr["kernels"][name]["avg_us"]
        n = tr["kernels"][name]["launches"]
        rp = None
        for k, v in durs.items():
            if k == name and len(v) >= n:
                last = sorted(v)[-n:]
                rp = sum(e - s for s, e in last) / n / 1e3
        a = u1["kernels"].get(name, {}).get("avg_us")
        b = u2["kernels"].get(name, {}).get("avg_us")
        d = f"{(ev / rp - 1) * 100:+.2f}%" if rp else "n/a"
        print(f"{name:22} {ev:14.1f} {rp if rp is None else round(rp, 1)!s:>22} {d:>7} {a!s:>10} / {b!s:<10}")


if __name__ == "__main__":
    main(sys.argv[1])
