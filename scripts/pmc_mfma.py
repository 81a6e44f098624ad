"""MFMA utilisation of the dense-step kernels from one rocprofv3 --pmc pass
(SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_VALU_MFMA_{F64,F32}, ..._MOPS_*, GRBM_GUI_ACTIVE).

    python scripts/pmc_mfma.py <pmc_dir> <tag> <n> <nnz> <hw> [kernel_full ...]

Writes profiles/<tag>_pmc_mfma_<short>.json for every kernel instantiation given
(as bench.py names it, e.g. "k_fused_update16<true,8,false>"; matched exactly
against the demangled name), stamped with the sha256 of the kernel's source file
and the commit (env LZ_COMMIT): bench.py refuses a summary of another source.
  MfmaUtil_pct = 100 * MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs)
  (GRBM_GUI_ACTIVE is summed over the 8 XCDs; MFMA_BUSY_CYCLES over all SIMDs)
  mfma_flop_per_launch = 512 * MOPS (a MOP is 512 FLOP: v_mfma_f64_16x16x4f64 = 4
  MOPS = 2048 FLOP, v_mfma_f32_32x32x2_f32 = 8 MOPS = 4096 FLOP).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import _norm, source_sha  # noqa: E402

d, tag, n, nnz, hw = sys.argv[1:6]
kernels = sys.argv[6:] or ["k_fused_pp16<14,2376,3,2,false>", "k_fused_update16<true,8,false>"]
rows = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        key = (r["Kernel_Name"], r["Dispatch_Id"])
        rows[key][r["Counter_Name"]] = float(r["Counter_Value"])
        rows[key]["_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for k in kernels:
    disp = [v for (name, _), v in rows.items() if _norm(name) == _norm(k)]
    full = sorted({name.split("(")[0] for (name, _) in rows if _norm(name) == _norm(k)})
    short = k.split("<")[0]
    if not disp:
        print(f"{k}: no dispatches")
        continue
    avg = {c: sum(x[c] for x in disp) / len(disp) for c in disp[0] if all(c in x for x in disp)}
    # per-dispatch MFMA MOPs: the launches of the largest count are a solve's
    # steady-state ones (a wavefront solve's first launch is pass 1 only)
    mops_d = [x.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0) + x.get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0.0) for x in disp]
    top = max(mops_d)
    steady = [x for x, mo in zip(disp, mops_d) if mo >= 0.999 * top]
    busy, grbm = avg.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0), avg.get("GRBM_GUI_ACTIVE", 0.0)
    mops = avg.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0) + avg.get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0.0)
    cyc = grbm / 8.0
    res = {"kernel": short, "kernel_full": k, "kernel_names": full, "dispatches": len(disp),
           "source_sha": source_sha(k), "commit": os.environ.get("LZ_COMMIT", "unknown"),
           "workload": {"n": int(n), "nnz": int(nnz), "halfwidth": int(hw)},
           "counters_avg_per_launch": avg,
           "MfmaUtil_pct": round(100.0 * busy / (cyc * 1024), 3) if cyc else None,
           "mfma_flop_per_launch": int(512 * mops),
           "mfma_flop_per_steady_launch": int(512 * top),
           "dispatch_mix": {"dispatches": len(disp), "steady": len(steady),
                            "mfma_flop_per_dispatch": sorted({int(512 * mo) for mo in mops_d})},
           "MfmaUtil_pct_steady": round(100.0 * sum(x.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for x in steady) /
                                        (sum(x.get("GRBM_GUI_ACTIVE", 0.0) for x in steady) / 8.0 * 1024), 3)
           if steady and all("GRBM_GUI_ACTIVE" in x for x in steady) else None,
           "effective_clock_GHz": round(cyc / avg["_ns"], 3) if avg.get("_ns") else None,
           "achieved_TFLOPs_profiled": round(512 * mops / avg["_ns"] / 1e3, 3) if avg.get("_ns") else None,
           "note": "one --pmc pass (no tracing); MfmaUtil = MFMA busy cycles / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs); "
                   "profiled clocks run below unprofiled ones"}
    out = os.path.join(root, "profiles", f"{tag}_pmc_mfma_{short}.json")
    json.dump(res, open(out, "w"), indent=1)
    print(out, res["MfmaUtil_pct"], res["mfma_flop_per_launch"], res["effective_clock_GHz"])
