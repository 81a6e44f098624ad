"""Per-kernel mean duration and mean gap before each kernel (previous kernel's
end to this kernel's start) from rocprofv3 kernel-trace CSVs, for the wavefront
step's kernels (one directory per run)."""
import csv
import glob
import sys
from collections import defaultdict


def summary(d):
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    rows = list(csv.DictReader(open(f[0])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur, gap = defaultdict(list), defaultdict(list)
    prev_end = None
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:60]
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        dur[name].append(e - s)
        if prev_end is not None and 0 <= s - prev_end < 200_000:
            gap[name].append(s - prev_end)
        prev_end = e
    print(d)
    for k in sorted(dur, key=lambda k: -sum(dur[k])):
        g = gap.get(k, [])
        print(f"  {k:60s} n={len(dur[k]):4d} dur {sum(dur[k]) / len(dur[k]) / 1e3:9.2f} us"
              f"  gap before {sum(g) / max(len(g), 1) / 1e3:7.2f} us")


for d in sys.argv[1:]:
    summary(d)
