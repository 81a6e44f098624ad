"""Per-launch HBM traffic of one kernel instantiation from two rocprofv3 --pmc
passes (FETCH_SIZE, WRITE_SIZE; KB per dispatch).  gfx950 FETCH_SIZE counts
128-B reads at 64 B (MI355X_MICROARCH.md "HBM"), so it is doubled.

    python scripts/pmc_traffic.py <fetch_dir> <write_dir> <kernel_full> <short> <n> <nnz> <hw> <out.json> [first]

first (k_wf16 of the default shape): the instantiation of a solve's first launch (XO = 1,
beta_0's Gram), summarised as hbm_bytes_first_launch; without it the first launches are
told apart from the steady ones of the same instantiation by their writes.

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
kfirst = sys.argv[9] if len(sys.argv) > 9 else None


def values(d, counter, kname=None):
    kname = kname or kfull
    v, names = [], set()
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if _norm(r["Kernel_Name"]) == _norm(kname) and r["Counter_Name"] == counter:
                v.append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
                names.add(r["Kernel_Name"].split("(")[0])
    if not v:
        sys.exit(f"{kname}: no {counter} dispatches in {d}")
    return [x for _, x in sorted(v)], sorted(names)


fv, names = values(fd, "FETCH_SIZE")
wv, _ = values(wd, "WRITE_SIZE")
first = None
if kfirst:
    f1, _ = values(fd, "FETCH_SIZE", kfirst)
    w1, _ = values(wd, "WRITE_SIZE", kfirst)
    first = int((2 * sum(f1) / len(f1) + sum(w1) / len(w1)) * 1024)
elif short == "k_wf16" and len(fv) == len(wv):
    # the wavefront kernel's first launch of a solve is pass 1 only (it writes
    # Y alone, half the others' writes): steady-state launches summarised
    # apart, the two passes' dispatches paired in launch order
    top = max(wv)
    keep = [i for i, w in enumerate(wv) if w > 0.75 * top]
    rest = [i for i in range(len(wv)) if i not in keep]
    if rest:
        first = int(sum(2 * fv[i] * 1024 + wv[i] * 1024 for i in rest) / len(rest))
    fv, wv = [fv[i] for i in keep], [wv[i] for i in keep]
fetch_kb, nf = sum(fv) / len(fv), len(fv)
write_kb, nw = sum(wv) / len(wv), len(wv)
res = {"kernel": short, "kernel_full": kfull, "kernel_names": names,
       "source_sha": source_sha(kfull), "commit": os.environ.get("LZ_COMMIT", "unknown"),
       "workload": {"n": int(n), "nnz": int(nnz), "halfwidth": int(hw)},
       "dispatches": {"fetch": nf, "write": nw},
       "FETCH_SIZE_KB": fetch_kb, "WRITE_SIZE_KB": write_kb,
       "read_bytes": 2 * fetch_kb * 1024, "write_bytes": write_kb * 1024,
       "hbm_bytes_per_launch": int(2 * fetch_kb * 1024 + write_kb * 1024),
       "note": "read = 2 x FETCH_SIZE (gfx950 tallies 128-B requests at 64 B); separate --pmc passes"}
if first is not None:
    res["hbm_bytes_first_launch"] = first
    res["note"] += ("; k_wf16: hbm_bytes_per_launch over the steady-state launches (pass 2 + pass 1), "
                    "hbm_bytes_first_launch over each solve's pass-1-only first launch")
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
