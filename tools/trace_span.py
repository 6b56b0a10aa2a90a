"""Wall time of the slanted schedule's concurrent region from a rocprofv3
kernel trace: per frame, the span from the first start to the last end of the
top-down slanted pass (slant_kernel<false, ...>) and the H pair (hpair_kernel)
that runs beside it on a second stream -- what bench.py reports as
`slant_down_hpair` (fork to join, HIP events).
Usage: python tools/trace_span.py DIR/run_kernel_trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows),
            key=lambda x: x[0])
down = [e for e in ev if "slant_kernel<false" in e[2]]
hp = [e for e in ev if "hpair_kernel" in e[2]]
spans = []
for d in down:
    # the H pair launched with this top-down pass: the one whose interval overlaps it
    mate = [x for x in hp if x[0] < d[1] and x[1] > d[0]]
    if mate:
        spans.append((max(d[1], mate[0][1]) - min(d[0], mate[0][0])) / 1e3)
if spans:
    print(f"frames {len(spans)}  slant_down+hpair span: mean {sum(spans) / len(spans):.1f} us  "
          f"min {min(spans):.1f}  max {max(spans):.1f}")
    print(f"  slant_down alone: mean {sum((d[1] - d[0]) / 1e3 for d in down) / len(down):.1f} us; "
          f"hpair alone: mean {sum((x[1] - x[0]) / 1e3 for x in hp) / len(hp):.1f} us")
else:
    print("no concurrent slant_down / hpair launches in this trace")
