"""Summarise rocprofv3 --pmc csv passes: mean per dispatch of a kernel."""
import collections, csv, glob, json, sys
root, pat = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/p*/*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(json.dumps({k: sum(v) / len(v) for k, v in sorted(agg.items())}, indent=0))
