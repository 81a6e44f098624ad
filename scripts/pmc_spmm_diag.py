"""The plain SpMM's counters, as it runs (C3) and with every input made
L2-resident by the in-kernel diagnostic (LZ_SPMM_DIAG=64): per-dispatch means of
the k_spmm_seg main instantiation from scripts/pmc_cmd.sh's passes, and the
derived rates (per-CU fractions of the kernel's cycles; GRBM_GUI_ACTIVE sums the
8 XCDs, the TA / TCP counters sum the 256 CUs).

    python scripts/pmc_spmm_diag.py <pmc_dir_normal> <pmc_dir_diag> <out.json>
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import _norm, source_sha  # noqa: E402

KFULL = "k_spmm_seg<double,16,48,768,false,0,false,false>"


def means(d):
    agg = defaultdict(list)
    for f in sorted(glob.glob(f"{d}/p*/*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if _norm(r["Kernel_Name"]) == _norm(KFULL):
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    if not agg:
        sys.exit(f"no {KFULL} dispatches in {d}")
    return {k: sum(v) / len(v) for k, v in sorted(agg.items())}


def derived(c):
    cyc = c["GRBM_GUI_ACTIVE"] / 8  # per XCD (= per CU) cycles of the dispatch
    cu = 256 * cyc
    return {
        "kernel_cycles": round(cyc),
        "TA_busy_frac": round(c["TA_TA_BUSY_sum"] / cu, 3),
        "TCP_pending_stall_frac": round(c["TCP_PENDING_STALL_CYCLES_sum"] / cu, 3),
        "L1_L2_read_latency_cycles": round(c["TCP_TCC_READ_REQ_LATENCY_sum"] / c["TCP_TCC_READ_REQ_sum"], 1),
        "L1_L2_read_requests": round(c["TCP_TCC_READ_REQ_sum"]),
        "L1_L2_read_req_per_clk_per_CU": round(c["TCP_TCC_READ_REQ_sum"] / cu, 4),
        "outstanding_reads_per_CU": round(c["TCP_TCC_READ_REQ_LATENCY_sum"] / cu, 1),
        "vmem_read_insts": round(c["SQ_INSTS_VMEM_RD"]),
        "vmem_write_insts": round(c["SQ_INSTS_VMEM_WR"]),
        "valu_insts": round(c["SQ_INSTS_VALU"]),
        "lds_insts": round(c["SQ_INSTS_LDS"]),
        "TA_busy_cycles_per_vmem_inst": round(c["TA_TA_BUSY_sum"] / (c["SQ_INSTS_VMEM_RD"] + c["SQ_INSTS_VMEM_WR"]), 1),
    }


nd, dd, out = sys.argv[1:4]
cn, cd = means(nd), means(dd)
rec = {
    "kernel_full": KFULL,
    "source_sha": source_sha("k_spmm_seg"),
    "commit": os.environ.get("LZ_COMMIT"),
    "workload": {"n": 10_000_000, "nnz": 100_000_182, "halfwidth": 4096, "b": 16, "dtype": "f64"},
    "what": "plain SpMM at C3 as it runs, and with LZ_SPMM_DIAG=64 (tile t stages tile t mod 64's CSR run: "
            "same instruction stream, every row pointer, CSR entry and X row an L2 hit); one --pmc pass per group "
            "(scripts/pmc_cmd.sh), means over the profiled dispatches",
    "normal": {"derived": derived(cn), "counters": cn},
    "all_l2_diag": {"derived": derived(cd), "counters": cd},
}
json.dump(rec, open(out, "w"), indent=1)
print(json.dumps({"normal": rec["normal"]["derived"], "all_l2_diag": rec["all_l2_diag"]["derived"]}, indent=1))
