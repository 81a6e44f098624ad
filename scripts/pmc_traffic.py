"""Per-launch HBM traffic of one kernel instantiation from two rocprofv3 --pmc
passes (FETCH_SIZE, WRITE_SIZE; KB per dispatch).  gfx950 FETCH_SIZE counts
128-B reads at 64 B (MI355X_MICROARCH.md "HBM"), so it is doubled.

    python scripts/pmc_traffic.py <fetch_dir> <write_dir> <kernel_full> <short> <n> <nnz> <hw> <out.json>

kernel_full: the instantiation as bench.py names it (e.g.
"k_fused_pp16<14,2376,3,2,false>"), matched exactly against the demangled
Kernel_Name (spaces, "void", "lz::" and the argument list ignored).  The summary
records it with the sha256 of the kernel's source file and the commit (env
LZ_COMMIT), so bench.py refuses it once the kernel changes.
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import _norm, source_sha  # noqa: E402

fd, wd, kfull, short, n, nnz, hw, out = sys.argv[1:9]


def mean(d, counter):
    v, names = [], set()
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if _norm(r["Kernel_Name"]) == _norm(kfull) and r["Counter_Name"] == counter:
                v.append(float(r["Counter_Value"]))
                names.add(r["Kernel_Name"].split("(")[0])
    if not v:
        sys.exit(f"{kfull}: no {counter} dispatches in {d}")
    return sum(v) / len(v), len(v), sorted(names)


fetch_kb, nf, names = mean(fd, "FETCH_SIZE")
write_kb, nw, _ = mean(wd, "WRITE_SIZE")
res = {"kernel": short, "kernel_full": kfull, "kernel_names": names,
       "source_sha": source_sha(kfull), "commit": os.environ.get("LZ_COMMIT", "unknown"),
       "workload": {"n": int(n), "nnz": int(nnz), "halfwidth": int(hw)},
       "dispatches": {"fetch": nf, "write": nw},
       "FETCH_SIZE_KB": fetch_kb, "WRITE_SIZE_KB": write_kb,
       "read_bytes": 2 * fetch_kb * 1024, "write_bytes": write_kb * 1024,
       "hbm_bytes_per_launch": int(2 * fetch_kb * 1024 + write_kb * 1024),
       "note": "read = 2 x FETCH_SIZE (gfx950 tallies 128-B requests at 64 B); separate --pmc passes"}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
