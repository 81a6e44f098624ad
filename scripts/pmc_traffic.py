"""Per-launch HBM traffic of one kernel from two rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE; KB per dispatch).  gfx950 FETCH_SIZE counts 128-B reads
at 64 B (MI355X_MICROARCH.md "HBM"), so it is doubled.

    python scripts/pmc_traffic.py <fetch_dir> <write_dir> <kernel> <n> <nnz> <hw> <out.json>
"""
import csv, glob, json, sys

fd, wd, kern, n, nnz, hw, out = sys.argv[1:8]


def mean(d, counter):
    v = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"] and r["Counter_Name"] == counter:
                v.append(float(r["Counter_Value"]))
    return sum(v) / len(v), len(v)


fetch_kb, nf = mean(fd, "FETCH_SIZE")
write_kb, nw = mean(wd, "WRITE_SIZE")
res = {"kernel": kern, "workload": {"n": int(n), "nnz": int(nnz), "halfwidth": int(hw)},
       "dispatches": {"fetch": nf, "write": nw},
       "FETCH_SIZE_KB": fetch_kb, "WRITE_SIZE_KB": write_kb,
       "read_bytes": 2 * fetch_kb * 1024, "write_bytes": write_kb * 1024,
       "hbm_bytes_per_launch": int(2 * fetch_kb * 1024 + write_kb * 1024),
       "note": "read = 2 x FETCH_SIZE (gfx950 tallies 128-B requests at 64 B); separate --pmc passes"}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
