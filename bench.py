"""Benchmark: block-Lanczos iterations/sec + SpMM achieved HBM GB/s vs peak
(BASELINE.json metric), n = 10M, nnz = 1e8, b = 16, fp64, on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c4]

A "step" is one block-Lanczos iteration (fused SpMM pass + alpha finish +
update pass + beta sqrtm) over the whole synthetic operator, inputs resident in
HBM.

--config c3 (default): BASELINE config C3.  N = 1: n = 1e7, nnz = 1e8, half
  width 4096 on one GPU.  N > 1 (launched by torch.distributed.run): weak
  scaling -- every rank owns a 10M-row slab of an N*10M-row banded operator,
  row-partitioned; each iteration exchanges only the Krylov-block rows other
  ranks reference (RCCL grouped send/recv, `--exchange halo`, default) or
  all-gathers the block (`--exchange allgather`); `value` counts
  slab-iterations/s summed over ranks.
--config c4: BASELINE config C4, strong scaling -- n = 4e7 rows in total,
  25 nnz/row (nnz = 1e9), half width 2^16, split over the N ranks.
At N > 1 (either config) the line reports the `--exchange` form (halo by
default) as `value` and times the other form (the north star's RCCL
all-gather) beside it on the same partition (extra.other_exchange).
`--gpus N` runs N ranks: under torch.distributed.run as given (WORLD_SIZE
must equal N, else the run fails), or, with WORLD_SIZE unset and N > 1, by
starting `python -m torch.distributed.run --nproc-per-node N ... bench.py`
as a child process before anything touches the GPU and relaying its line.

After the timed region the run checks itself: the device error word must be
0 (no persistent kernel abandoned a bounded spin) and, on one GPU, the first
steps' alpha / beta / row probe / Ritz values must match the CPU oracle run on
the same operator and start block (the same call times the CPU baseline).
rank 0 prints one JSON line on stdout (native libraries' own stdout output is
routed to stderr).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_MFMA_PEAK_TFS = 78.6  # v_mfma_f64_16x16x4f64: 32 FLOP/clk/SIMD x 1024 SIMDs x 2.4 GHz
RITZ_TOL = 1e-10  # BASELINE.json north star: Ritz values within 1e-10 of the reference
SPMM_ALL_L2_MS = 0.770  # the plain SpMM's all-L2 diagnostic at C3, round 6 (profiles/r06l_spmm_l2_ceiling.log)
# What plain streaming kernels reach on this hardware (scripts/gprobe/stream_probe.hip, 2 GiB arrays,
# 16-B accesses, best of its shapes and cache policies; one box, round 6): the practical HBM ceilings
# per read:write mix, beside the 8 TB/s nominal peak the roofline fractions are quoted against
STREAM_GBS = {"read": 6590.0, "write": 4940.0, "copy": 4970.0, "r2w1": 5040.0, "r3w2": 4880.0, "r3w3": 4750.0}
STREAM_SRC = "profiles/r06ac_stream_probe.log (scripts/gprobe/stream_probe.hip)"


def stream_ceiling(achieved_gbs, mix):
    """The achieved rate against the streaming probe's rate for the same read:write mix."""
    return {"mix": mix, "GBs": STREAM_GBS[mix], "frac": round(achieved_gbs / STREAM_GBS[mix], 4), "source": STREAM_SRC}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def spmm_bytes(n, nnz, b, sv=8):
    """Reference's A + 2B model + row_ptr: z(s_v+4) + (n+1)8 + 2 n b s_v."""
    return nnz * (sv + 4) + (n + 1) * 8 + 2 * n * b * sv


def col_bytes(n, hw):
    """Bytes per stored column index in the fused passes: 2 when every column is
    within int16 reach of its 16-row strip (col16_plan; banded operators with
    half-width < 32752 below 2^24 rows, LZ_PASS1_C16 not 0), else 4."""
    c16 = os.environ.get("LZ_PASS1_C16", "1") != "0" and hw + 15 <= 32767 and n < (1 << 24)
    return 2 if c16 else 4


def fused_pass_bytes(n, nnz, b, sv=8, cb=4):
    """Algorithmic bytes of one fused pass-1 launch (Q-free iteration): A (cb-byte
    columns), the Krylov block W_j read once, W_{j-1} read, W' written."""
    return nnz * (sv + cb) + (n + 1) * 8 + 3 * n * b * sv


def wf_bytes(n, nnz, b, launches, sv=8, cb=2):
    """Algorithmic bytes of `launches` wavefront-step launches of one solve
    (lz_wf.hip): the first is pass 1 only (A, B gathered once, Y written), each
    later one A + 5 n b s (Y_j, V_{j-1}, V_j read; V_{j+1}, Y_{j+1} written)."""
    a = nnz * (sv + cb) + (n + 1) * 8
    nb = n * b * sv
    return (a + 2 * nb) + max(launches - 1, 0) * (a + 5 * nb)


# MFMA work of the dense step per row (b = 16, v_mfma_f64_16x16x4f64 = 2048 FLOP):
# pass 1 epilogue, per 16-row strip: Q_j = W_j beta^-1 (4), W' = Y beta^-1 -
# W_{j-1} P1 (8), slab Q_j^T W' (4) = 16 MFMAs; pass 2: W'' = W' - W_j P2 (4),
# slab W''^T W'' (4) = 8 MFMAs.
PASS1_MFMA_FLOP_PER_ROW = 16 * 2048 // 16
PASS2_MFMA_FLOP_PER_ROW = 8 * 2048 // 16


def wf_kernel(n, hw, nnz=None, one_gpu=True):
    """(full name, PMC short name) of the wavefront-step kernel (lz_wf.hip wf_step16):
    <consumers, stage entries, stages, loaders, updaters, strip slots - 1, 16-bit columns,
    SW = false (the all-gather save-V_j form runs only at N > 1), GEN, XO = 0> -- GEN
    false for the one-GPU solve's launches of the default shapes (the specialised form,
    round 5); XO 1 is the default shape's first launch of a solve (beta_0's Gram, its own
    instantiation: wf_first_kernel), XO 2 the post-call state launch, not a step."""
    c16 = col_bytes(n, hw) == 2
    sh = os.environ.get("LZ_WF_SHAPE", "111")
    tf = 'true' if c16 else 'false'
    gen = 'false' if one_gpu else 'true'
    if nnz is not None and nnz > 10.2 * n:  # the wide shape (C4's density)
        return f"k_wf16<10,4400,2,1,{3 if c16 else 2},1,{tf},false,{gen},0>", "k_wf16"
    if sh not in ("10", "11", "12"):  # default: 1 loader + 11 consumers + 4 updaters
        return f"k_wf16<11,{11 * 16 * 11},3,1,4,1,{tf},false,{gen},0>", "k_wf16"
    nc = int(sh)
    du = {10: 2 if c16 else 1, 11: 2, 12: 3 if c16 else 2}[nc]
    return f"k_wf16<{nc},{nc * 16 * 11},3,2,{14 - nc},{du},{tf},false,true,0>", "k_wf16"


def wf_first_kernel(name):
    """The first launch of a solve for the default shape: the same kernel with XO = 1
    (None for the other shapes, whose first launch is the step kernel itself)."""
    return name[:-2] + "1>" if name.startswith("k_wf16<11,") and name.endswith(",0>") else None


# MFMA work of the wavefront step per row: updaters 12 (V_{j+1}) + 4 (G) + 4 (S2),
# consumers 4 (S1) per 16-row strip (lz_wf.hip: 20 mfma16 per updater strip, 4 per
# consumer strip); a solve's first launch is pass 1 only (the consumers' 4)
WF_MFMA_FLOP_PER_ROW = 24 * 2048 // 16
WF_MFMA_FLOP_PER_ROW_FIRST = 4 * 2048 // 16


def wf_mfma_flop(n, launches):
    """MFMA FLOP of one wavefront solve of `launches` launches (the first pass 1 only)."""
    return (WF_MFMA_FLOP_PER_ROW_FIRST + max(launches - 1, 0) * WF_MFMA_FLOP_PER_ROW) * n


def fused_kernel(nnz, n):
    """(full name, PMC short name) of the pass-1 kernel lz_fused.hip launches (b = 16 fp64)."""
    wide = nnz > 10.2 * n
    win = n >= (1 << 24)
    shape = "10,4400,2,2" if wide else "14,2376,3,2"
    return f"k_fused_pp16<{shape},{'true' if win else 'false'}>", "k_fused_pp16"


PASS2_KERNEL = "k_fused_update16<true,8,false>"  # the single-GPU pass 2 (lz_fused.hip fused_update16)


def spmm_kernel(nnz, n):
    """The plain SpMM kernel lz_csr_spmm launches for b = 16 fp64 (lz_spmm.hip launch_spmm_rm)."""
    cap = 1536 if nnz > 13.0 * n else 768
    win = n >= (1 << 24)
    return f"k_spmm_seg<double,16,48,{cap},{'true' if win else 'false'},0,false,false,false>"


# the source file of each profiled kernel: a committed counter file is used only
# while that file is byte-identical to the one profiled (profiles record its sha256)
KERNEL_SRC = {"k_wf16": "lz_wf.hip", "k_vl_spmv_win": "lz_fused.hip", "k_fused_pp16": "lz_fused.hip", "k_fused_update16": "lz_fused.hip", "k_spmm_seg": "lz_spmm.hip",
              "k_fused_el32": "lz_fused32.hip", "k_fused_ub32": "lz_fused32.hip", "k_gram16_f64": "lz_dense.hip",
              "k_gram32_f32": "lz_dense.hip"}
CSRC = os.path.join(ROOT, "gpu-implementation-of-signle-and-block-lanczos_amd", "csrc")


def source_sha(kernel):
    import hashlib
    f = next((v for k, v in KERNEL_SRC.items() if kernel.startswith(k)), None)
    if not f:
        return None
    return hashlib.sha256(open(os.path.join(CSRC, f), "rb").read()).hexdigest()[:16]


def _norm(name):
    return name.replace(" ", "").replace("lz::", "").replace("void", "").split("(")[0]


def pmc_record(kind, kernel, n, nnz, hw, kernel_full=None, nnz_tol=0.0):
    """A committed rocprofv3 PMC summary (profiles/*_pmc_<kind>_<kernel>.json or,
    kind "", profiles/*_pmc_<kernel>.json) of this bench's workload, newest first.
    Refused (None, reason) unless it names the kernel instantiation this run
    launches (kernel_full) and was taken on the current source of that kernel.
    nnz_tol > 0 (a distributed rank): a summary of the same rows and half width
    whose nnz is within that fraction (the per-rank share run by --config c4rank,
    whose columns stop at the share) is taken, and the source says so."""
    pat = f"*_pmc_{kind + '_' if kind else ''}{kernel}.json"
    reason = "no committed counter file for this workload"
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", pat)), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        w = d.get("workload", {})
        wn = w.get("nnz") or 0
        if not (w.get("n") == n and w.get("halfwidth") == hw and abs(wn - nnz) <= nnz_tol * nnz):
            continue
        rel = os.path.relpath(f, ROOT)
        if wn != nnz:
            rel += f" (the per-rank share: nnz {wn} against this rank's {nnz})"
        if _norm(d.get("kernel_full", "")) != _norm(kernel_full or kernel):
            reason = f"{rel}: kernel {d.get('kernel_full')!r} is not the launched {kernel_full!r}"
            continue
        if d.get("source_sha") is None or d.get("source_sha") != source_sha(kernel):
            reason = f"{rel}: taken on another source of {KERNEL_SRC.get(kernel, '?')} (stale)"
            continue
        return d, rel
    return None, reason


def pmc_traffic(kernel, n, nnz, hw, kernel_full=None):
    """HBM bytes per launch of `kernel` from the committed PMC summary (separate
    FETCH_SIZE / WRITE_SIZE passes, FETCH_SIZE doubled per MI355X_MICROARCH.md's
    gfx950 note; scripts/pmc_traffic.py).  (None, reason) unless taken on this
    workload, this kernel instantiation and this source."""
    d, src = pmc_record("", kernel, n, nnz, hw, kernel_full)
    return (d.get("hbm_bytes_per_launch"), src) if d else (None, src)


def host_cpu():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_stats(t_each, unit_per_s=1.0):
    """best / mean / worst rate of per-iteration wall times (the first one warms up)."""
    s = np.asarray(t_each[1:] if len(t_each) > 1 else t_each, dtype=float)
    return {"value": round(unit_per_s / float(s.min()), 4), "mean": round(unit_per_s / float(s.mean()), 4),
            "worst": round(unit_per_s / float(s.max()), 4), "samples": int(s.size)}


def compare_run(lz, m, b, got, ref, tol_rel, ritz_tol):
    """alpha / beta / q / Ritz of the first m steps against the oracle's."""
    al, be, q = got
    ao, bo, qo = ref
    al, be = np.asarray(al[:m], np.float64), np.asarray(be[:m + 1], np.float64)
    ao, bo = np.asarray(ao, np.float64), np.asarray(bo, np.float64)
    scale = max(1.0, float(np.abs(ao).max()), float(np.abs(bo[:m]).max()))
    r_gpu = lz.ritz_values(m, b, al, be)
    r_cpu = lz.ritz_values(m, b, ao, bo)
    res = {"steps_checked": m, "max_dalpha_rel": float(np.max(np.abs(al - ao)) / scale),
           "max_dbeta_rel": float(np.max(np.abs(be[:m] - bo[:m])) / scale),
           "max_dritz": float(np.max(np.abs(r_gpu - r_cpu))), "tol_rel": tol_rel, "ritz_tol": ritz_tol}
    if q is not None:
        res["max_dq"] = float(np.max(np.abs(np.asarray(q[: qo.size], np.float64) - qo)))
    res["ok"] = bool(res["max_dalpha_rel"] <= tol_rel and res["max_dbeta_rel"] <= tol_rel
                     and res["max_dritz"] <= ritz_tol)
    return res


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=["c3", "c4", "c4rank"], default="c3",
                    help="c4rank: one rank's share of C4 on one GPU (n = 5M of 40M, 25 nnz/row, half "
                         "width 2^16): the per-GPU step of the 8-GPU north-star configuration")
    ap.add_argument("--n", type=int, default=None, help="c3: rows per GPU (1e7); c4: rows in total (4e7)")
    ap.add_argument("--nnz-per-row", type=float, default=None)
    ap.add_argument("--halfwidth", type=int, default=None)
    ap.add_argument("--b", type=int, default=16)
    ap.add_argument("--unfused", action="store_true")
    ap.add_argument("--cpu-iters", type=int, default=None,
                    help="oracle iterations after the start-up step; the first is a warm-up, the "
                         "CPU baseline is the best of the rest (BASELINE.md 3: best of 5; c3 default 6, "
                         "c4 default 2: BASELINE.md reports the C4 CPU baseline at C3 scale only)")
    ap.add_argument("--no-cpu-baseline", action="store_true",
                    help="N = 1: skip the oracle legs (CPU baselines + parity); N > 1 always checks parity")
    ap.add_argument("--parity-steps", type=int, default=3, help="N > 1: steps checked against the oracle")
    ap.add_argument("--spmm-reps", type=int, default=20)
    ap.add_argument("--c2-steps", type=int, default=None, help="single-vector Lanczos steps at BASELINE config 1 (0: skip)")
    ap.add_argument("--c5-steps", type=int, default=None, help="block-32 fp32 power-law steps at BASELINE config 4 (0: skip)")
    ap.add_argument("--rand-steps", type=int, default=None,
                    help="block-Lanczos steps on the C3 uniform-random-column stress operator (0: skip)")
    ap.add_argument("--exchange", choices=["halo", "allgather"], default="halo",
                    help="multi-GPU Krylov-block exchange (N > 1, or with --dist at N = 1)")
    ap.add_argument("--no-second-exchange", action="store_true",
                    help="N > 1: do not time the other exchange form beside the headline one")
    ap.add_argument("--dist", action="store_true",
                    help="run the distributed entry point even at N = 1 (rehearsal of the N > 1 path)")
    args = ap.parse_args()
    c4 = args.config in ("c4", "c4rank")
    for k, v3, v4 in (("n", 10_000_000, 40_000_000), ("nnz_per_row", 10.0, 25.0), ("halfwidth", 4096, 1 << 16),
                      ("c2_steps", 200, 0), ("c5_steps", 10, 0), ("rand_steps", 10, 0), ("cpu_iters", 6, 2)):
        if getattr(args, k) is None:
            setattr(args, k, v4 if c4 else v3)
    if args.config == "c4rank" and args.n == 40_000_000:
        args.n = 5_000_000
    return args


def world_plan(gpus: int, env) -> str:
    """What `bench.py --gpus N` does in this environment, decided before anything
    touches the GPU: "run" (this process is the job, or one rank of it: WORLD_SIZE
    unset and N = 1, or WORLD_SIZE == N) or "launch" (WORLD_SIZE unset and N > 1:
    start N local ranks under torch.distributed.run as a child process).  A
    WORLD_SIZE that disagrees with --gpus is an error: a line for another N than
    the one asked for is never printed."""
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus {gpus}: at least 1")
    w = env.get("WORLD_SIZE")
    if w is None or w == "":
        return "launch" if gpus > 1 else "run"
    if int(w) != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={w}: refusing to report a {w}-rank run "
                         f"as {gpus} GPUs")
    return "run"


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def launch_cmd(argv, gpus: int, port: int):
    """The torch.distributed.run command that starts `gpus` ranks of this script
    with the same arguments (one process per GPU, rendezvous on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def relay(cmd, out=None) -> int:
    """Run cmd as a child process (this process has not touched the GPU, and
    never execs); its stderr passes through, its stdout -- rank 0's one JSON
    line -- is copied to ours.  Returns the child's exit status."""
    import subprocess
    out = out or sys.stdout
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=None, text=True)
    if p.stdout:
        out.write(p.stdout)
        out.flush()
    return p.returncode


def main():
    args = parse_args()
    if args.config == "c4rank" and args.gpus != 1:
        raise SystemExit("--config c4rank runs one rank's share on ONE GPU (the 8-GPU run is --config c4)")
    if world_plan(args.gpus, os.environ) == "launch":
        log(f"bench.py: --gpus {args.gpus} without WORLD_SIZE: starting {args.gpus} ranks under torch.distributed.run")
        sys.exit(relay(launch_cmd(sys.argv[1:], args.gpus, free_port())))
    # Native libraries write to fd 1 (RCCL prints a version banner at communicator
    # init): route fd 1 to stderr and keep the real stdout for the one JSON line.
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    assert world == args.gpus  # world_plan
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    lz = ge.load_package()
    h = lz.Handle(local)
    c4 = args.config == "c4"
    c4rank = args.config == "c4rank"
    if c4rank and world != 1:
        raise SystemExit("--config c4rank runs one rank's share on ONE GPU (the 8-GPU run is --config c4)")
    b = args.b
    seed = 20261015
    # the global operator and this rank's rows [r0, r1)
    if c4:  # strong scaling: a fixed n_total split over the ranks
        n_total = args.n
        bounds = [n_total * g // world for g in range(world + 1)]
    else:  # weak scaling: n rows per rank
        n_total = args.n * world
        bounds = [args.n * g for g in range(world + 1)]
    r0, r1 = bounds[rank], bounds[rank + 1]
    n = r1 - r0
    t_gen = time.time()
    if world == 1:
        A = lz.gen_banded(n, args.nnz_per_row, args.halfwidth, seed)
    else:
        A = lz.gen_banded_local(n_total, r0, r1, args.nnz_per_row, args.halfwidth, seed)
    B = lz.uniform_B(n, b, seed, r0=r0)
    log(f"[rank {rank}] generated rows [{r0}, {r1}) of n={n_total}: nnz={A.nnz} in {time.time() - t_gen:.1f}s")
    kw = dict(dtype=torch.float64, device="cuda")
    m_max = max(args.steps, args.warmup, 1)
    q = torch.zeros(m_max * b, **kw)
    alpha = torch.zeros(m_max, b, b, **kw)
    beta = torch.zeros(m_max + 1, b, b, **kw)
    Bd = torch.from_numpy(B).cuda()
    dist_path = world > 1 or args.dist
    lc, lc_rank = 84, 0

    def make_runner(exchange):
        """(run(m), description, halo rows) for this rank's path."""
        if not dist_path:
            Ad = lz.CsrDevice.from_host(A)
            Q0, Q1, W = (torch.zeros(n, b, **kw) for _ in range(3))

            def run(m):
                h.block_lanczos_blas(Ad, Bd, m, lc, q, alpha, beta, Q0, Q1, W, fused=not args.unfused)
            return run, "single", 0, Ad
        if exchange == "halo":
            # only the referenced off-rank rows move each step
            ccol, rcnt, hrows = lz.halo_plan(A.col, np.asarray(bounds, np.int64), rank)
            h.halo_init(r0, n, rcnt, hrows)
            nh = int(hrows.size)
            Ad = lz.CsrDevice.from_host(lz.CsrHost(A.n, A.row_ptr, ccol, A.val), n_cols=n + nh)
            X0, X1 = (torch.zeros(n + nh, b, **kw) for _ in range(2))
            log(f"[rank {rank}] halo rows {nh}")

            def run(m):
                h.block_lanczos_halo(Ad, Bd, m, lc, lc_rank, q, alpha, beta, X0, X1)
            return run, f"rows{world}+rccl_halo({nh} halo rows on rank {rank})", nh, Ad
        # all-gather (north star): padded slabs, columns in the padded numbering
        n_pad = max(bounds[g + 1] - bounds[g] for g in range(world))
        pcol = lz.remap_cols_padded(A.col, np.asarray(bounds, np.int64), n_pad)
        Ad = lz.CsrDevice.from_host(lz.CsrHost(A.n, A.row_ptr, pcol, A.val), n_cols=n_pad * world)
        Bp = torch.zeros(n_pad, b, **kw)
        Bp[:n] = Bd
        Q0, W = (torch.zeros(n_pad, b, **kw) for _ in range(2))
        X_full = torch.zeros(n_pad * world, b, **kw)

        def run(m):
            h.block_lanczos_dist(Ad, n_pad, n_pad * world, Bp, m, lc, lc_rank, q, alpha, beta, Q0, W, X_full)
        return run, f"rows{world}+rccl_allgather", 0, Ad

    if dist_path:
        uid = [lz.comm_unique_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(uid, src=0)
        h.comm_init(world, rank, uid[0])
    run, parallelism, halo_rows, Ad = make_runner(args.exchange)

    def timed(run_fn, K, W):
        """W warmup steps, then exactly K steps between barriers; max over ranks.
        Only the roofline kernel's class records HIP events in the timed region
        (each recorded launch adds two event records to the stream)."""
        if W > 0:
            run_fn(W)
        torch.cuda.synchronize()
        h.prof_enable(True, classes=[h.PROF_SPMM_PASS])
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run_fn(K)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        prof = {c: h.prof_read(c) for c in (h.PROF_SPMM_PASS, h.PROF_UPDATE_PASS, h.PROF_SMALL, h.PROF_GRAM)}
        h.prof_enable(False)
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el, prof

    elapsed, prof = timed(run, args.steps, args.warmup)
    # ---- the run checks itself: device error word, finite outputs
    err = h.device_error()
    if err != 0:
        raise RuntimeError(f"device error word {err}: a persistent kernel abandoned a bounded spin; "
                           "the timed results are invalid")
    if not bool(torch.isfinite(alpha[: args.steps]).all()):
        raise RuntimeError("non-finite alpha in the timed run")
    K = args.steps
    al_gpu = alpha[:K].cpu().numpy()
    be_gpu = beta[: K + 1].cpu().numpy()
    q_gpu = q[: K * b].cpu().numpy()
    spmm_ms, spmm_cnt = prof[h.PROF_SPMM_PASS]
    # per-class breakdown of the other kernels from a short untimed run with every class recorded
    K_bd = min(K, 5)
    h.prof_enable(True)
    run(K_bd)
    torch.cuda.synchronize()
    upd_ms, upd_cnt = h.prof_read(h.PROF_UPDATE_PASS)
    small_ms, _ = h.prof_read(h.PROF_SMALL)
    gram_ms, _ = h.prof_read(h.PROF_GRAM)
    h.prof_enable(False)
    if h.device_error() != 0:
        raise RuntimeError("device error word set in the breakdown run")

    # ---- N > 1: the first steps against the CPU oracle on the GLOBAL operator (rank 0
    # builds it; every rank learns the verdict).  A multi-GPU line is never printed
    # unchecked.
    ref_g = None
    parity = None
    if world > 1:
        m_chk = min(K, args.parity_steps)
        verdict = [None]
        if rank == 0:
            t_o = time.time()
            A_g = lz.gen_banded(n_total, args.nnz_per_row, args.halfwidth, seed)
            B_g = lz.uniform_B(n_total, b, seed)
            orc = ge.load_oracle()
            qo, ao, bo = orc.block_lanczos(A_g, B_g, m_chk, lc)
            ref_g = (ao, bo, qo)
            del A_g, B_g
            parity = compare_run(lz, m_chk, b, (al_gpu, be_gpu, q_gpu), ref_g, 1e-9, RITZ_TOL)
            parity.update({"device_error": err, "against": f"oracle/lz_oracle.c on the global n={n_total} operator "
                                                           f"and start block (rank 0), {world} ranks' result",
                           "oracle_s": round(time.time() - t_o, 1)})
            log(f"N>1 parity: {parity}")
            verdict = [parity["ok"]]
        dist.broadcast_object_list(verdict, src=0)
        if not verdict[0]:
            raise RuntimeError(f"multi-GPU parity check against the oracle failed: {parity}")

    # ---- N > 1: the other exchange form (halo <-> the north star's all-gather) on the same partition
    other = None
    if world > 1 and not args.no_second_exchange:
        ex2 = "allgather" if args.exchange == "halo" else "halo"
        del run, Ad
        torch.cuda.empty_cache()
        run2, par2, _, Ad = make_runner(ex2)
        el2, _ = timed(run2, K, args.warmup)
        if h.device_error() != 0:
            raise RuntimeError(f"device error word set in the {ex2} run")
        a2 = alpha[:K].cpu().numpy()
        b2_ = beta[: K + 1].cpu().numpy()
        q2_ = q[: K * b].cpu().numpy()
        other = {"exchange": ex2, "parallelism": par2, "iters_per_s": round(K / el2, 3),
                 "ms_per_step": round(el2 / K * 1e3, 4),
                 "max_dalpha_vs_headline": float(np.max(np.abs(a2 - al_gpu)))}
        verdict = [None]
        if rank == 0:
            other["parity"] = compare_run(lz, min(K, args.parity_steps), b, (a2, b2_, q2_), ref_g, 1e-9, RITZ_TOL)
            verdict = [other["parity"]["ok"]]
        dist.broadcast_object_list(verdict, src=0)
        if not verdict[0]:
            raise RuntimeError(f"{ex2} exchange: parity check against the oracle failed: {other}")
        del run2

    # ---- plain SpMM kernel (the BASELINE headline kernel) on the same operator
    plain = None
    if world == 1 and not dist_path and args.spmm_reps > 0:
        Y = torch.empty(n, b, **kw)
        h.spmm(Ad, Bd, Y)
        torch.cuda.synchronize()
        h.prof_enable(True)
        for _ in range(args.spmm_reps):
            h.spmm(Ad, Bd, Y)
        torch.cuda.synchronize()
        ms, cnt = h.prof_read(h.PROF_SPMM)
        h.prof_enable(False)
        t_avg = ms / cnt * 1e-3
        gbs = spmm_bytes(n, A.nnz, b) / t_avg / 1e9
        plain = {"kernel": spmm_kernel(A.nnz, n), "avg_ms": round(ms / cnt, 4),
                 "bytes_per_launch": spmm_bytes(n, A.nnz, b), "achieved_GBs": round(gbs, 1),
                 "frac_of_hbm_peak": round(gbs / HBM_PEAK_GBS, 4)}
        # the same figures as a roofline object, with the kernel's measured HBM traffic
        trp, srcp = pmc_traffic("k_spmm_seg", n, A.nnz, args.halfwidth, spmm_kernel(A.nnz, n))
        plain["roofline"] = {"bound": "hbm", "kernel": spmm_kernel(A.nnz, n), "achieved": round(gbs, 1),
                             "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                             "traffic": trp, "traffic_source": srcp, "avg_ms": round(ms / cnt, 4),
                             "bytes_per_launch": spmm_bytes(n, A.nnz, b),
                             # A and X read, Y written: 2 : 1
                             "stream_ceiling": stream_ceiling(gbs, "r2w1")}
        if n == 10_000_000 and args.nnz_per_row == 10.0 and args.halfwidth == 4096:
            # the tile structure's own ceiling at C3 (DESIGN.md 4 SpMM): the same kernel and instruction
            # stream with every input L2-resident (diagnostic build, LZ_SPMM_DIAG=64) -- what no HBM
            # schedule can beat without fewer gathered lines per nonzero
            plain["ceiling_frac"] = round(spmm_bytes(n, A.nnz, b) / SPMM_ALL_L2_MS * 1e-6 / HBM_PEAK_GBS, 4)
            plain["ceiling_ms"] = SPMM_ALL_L2_MS
            plain["ceiling_source"] = ("profiles/r06l_spmm_l2_ceiling.log: k_spmm_seg with every row pointer, CSR "
                                       "entry and X row L2-resident (LZ_SPMM_DIAG=64, lib/liblz_hip_diag.so), "
                                       "0.767-0.773 ms against 1.189 ms as it runs, same box")
        if not args.no_cpu_baseline:  # the CPU SpMM on the same operator and block
            orc = ge.load_oracle()
            Yc, tc = orc.csr_spmm_timed(A, B, reps=3)
            Yg = Y.cpu().numpy()
            plain["parity_max_rel"] = float(np.max(np.abs(Yg - Yc)) / max(1e-300, float(np.abs(Yc).max())))
            if not plain["parity_max_rel"] <= 1e-12:
                raise RuntimeError(f"plain SpMM differs from the oracle: {plain['parity_max_rel']}")
            plain["cpu_baseline"] = {"value": round(spmm_bytes(n, A.nnz, b) / tc / 1e9, 2), "unit": "GB/s",
                                     "ms": round(tc * 1e3, 2), "cores": orc.num_threads(), "kind": "port",
                                     "sample": "best of 3 oracle CSR SpMMs (OpenMP over rows), same A and block"}
            del Yc, Yg
        del Y

    # ---- CPU oracle on the same operator and start block, rank 0, N = 1: the CPU
    # baseline (best of the timed iterations) and the bench's own parity check
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        orc = ge.load_oracle()
        m_o = min(K, 1 + max(1, args.cpu_iters))
        t_o = time.time()
        qo, ao, bo, t_each = orc.block_lanczos_timed(A, B, m_o, lc)
        log(f"oracle: {m_o} steps in {time.time() - t_o:.1f}s")
        st_ = cpu_stats(t_each)  # the first iteration warms the caches
        cpu = {"value": st_["value"], "unit": "iters/s", "cores": orc.num_threads(), "kind": "port",
               "mean_iters_per_s": st_["mean"], "worst_iters_per_s": st_["worst"], "host_cpu": host_cpu(),
               "sample": f"best of {st_['samples']} block-Lanczos iterations (after the start-up step and one "
                         f"warm-up iteration) of the same n={n} nnz={A.nnz} b={b} fp64 operator and start "
                         f"block, oracle/lz_oracle.c OpenMP; host cores are shared on this pool, so the rate "
                         f"varies between boxes (r02: 1.85-5.31 it/s)"}
        scale = max(1.0, np.abs(ao).max(), np.abs(bo[:m_o]).max())
        r_gpu = lz.ritz_values(m_o, b, al_gpu[:m_o], be_gpu[: m_o + 1])
        r_cpu = lz.ritz_values(m_o, b, ao, bo)
        parity = {"steps_checked": m_o, "ritz_tol": RITZ_TOL,
                  "max_dalpha_rel": float(np.max(np.abs(al_gpu[:m_o] - ao)) / scale),
                  "max_dbeta_rel": float(np.max(np.abs(be_gpu[:m_o] - bo[:m_o])) / scale),
                  "max_dq": float(np.max(np.abs(q_gpu[: m_o * b] - qo))),
                  "max_dritz": float(np.max(np.abs(r_gpu - r_cpu))),
                  "device_error": err, "against": "oracle/lz_oracle.c (CPU restatement), same A and B"}
        parity["ok"] = parity["max_dritz"] <= RITZ_TOL and parity["max_dalpha_rel"] <= 1e-9
        if not parity["ok"]:
            raise RuntimeError(f"bench parity check failed: {parity}")

    # ---- BASELINE config 1 (single-vector Lanczos, n=1M, nnz=1e7): an extra line
    c2 = None
    if world == 1 and args.c2_steps > 0:
        n2 = 1_000_000
        A2 = lz.gen_banded(n2, 10.0, 4096, seed)
        A2d = lz.CsrDevice.from_host(A2)
        b2 = torch.from_numpy(lz.uniform_B(n2, 1, seed)[:, 0].copy()).cuda()
        k2 = args.c2_steps
        q2, al2, be2 = (torch.zeros(k2 + 1, **kw) for _ in range(3))
        v0, v1, v2 = (torch.zeros(n2, **kw) for _ in range(3))
        h.vector_lanczos(A2d, b2, k2, 84, q2, al2, be2, v0, v1, v2)  # warm
        torch.cuda.synchronize()
        t0c = time.perf_counter()
        h.vector_lanczos(A2d, b2, k2, 84, q2, al2, be2, v0, v1, v2)
        torch.cuda.synchronize()
        dt2 = time.perf_counter() - t0c
        c2 = {"workload": f"C2 single-vector Lanczos fp64, banded-random n={n2} nnz={A2.nnz}",
              "iters_per_s": round(k2 / dt2, 1), "us_per_iter": round(dt2 / k2 * 1e6, 2),
              "iteration_GBs": round((A2.nnz * 12 + (n2 + 1) * 8 + 7 * n2 * 8) / (dt2 / k2) / 1e9, 1),
              "note": "A + 7 n s bytes per step: SpMV pass A + 4 n s (w_j gathered, q_{j-1} read, q_j and w' "
                      "written), update pass 3 n s (w', q_j read, w' written)"}
        # the dominant kernel (the SpMV pass) against the HBM roofline: HIP events of a separate
        # solve with the two vector classes recorded
        k2p = min(k2, 50)
        h.prof_enable(True)
        h.vector_lanczos(A2d, b2, k2p, 84, q2, al2, be2, v0, v1, v2)
        torch.cuda.synchronize()
        sv_ms, sv_cnt = h.prof_read(h.PROF_SPMM_PASS)
        up_ms, up_cnt = h.prof_read(h.PROF_UPDATE_PASS)
        h.prof_enable(False)
        if sv_cnt and up_cnt:
            spmv_b = A2.nnz * 12 + (n2 + 1) * 8 + 4 * n2 * 8
            t_sv, t_up = sv_ms / sv_cnt * 1e-3, up_ms / up_cnt * 1e-3
            kn2 = "k_vl_spmv_win<double,8,512,9216>"
            tr2, src2 = pmc_traffic("k_vl_spmv_win", n2, A2.nnz, 4096, kn2)
            c2["roofline"] = {"bound": "hbm", "kernel": kn2, "bytes_per_launch": spmv_b,
                              "avg_ms": round(t_sv * 1e3, 5), "achieved": round(spmv_b / t_sv / 1e9, 1),
                              "peak": HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": round(spmv_b / t_sv / 1e9 / HBM_PEAK_GBS, 4),
                              "traffic": tr2, "traffic_source": src2,
                              "update_pass": {"kernel": "k_vl_update<double>", "bytes_per_launch": 3 * n2 * 8,
                                              "avg_ms": round(t_up * 1e3, 5),
                                              "frac": round(3 * n2 * 8 / t_up / 1e9 / HBM_PEAK_GBS, 4)},
                              "note": "HIP events around each launch of a separate solve; a launch moves "
                                      f"{spmv_b / 1e6:.0f} MB in ~{t_sv * 1e6:.0f} us, so launch ramp-up and "
                                      "tail are a visible share of it"}
        if not args.no_cpu_baseline:
            orc = ge.load_oracle()
            m2 = min(k2, 12)
            bvh = b2.cpu().numpy()
            qo2, ao2, bo2, t2 = orc.vector_lanczos_timed(A2, bvh, m2, 84)
            c2["parity"] = compare_run(lz, m2, 1, (al2.cpu().numpy()[:m2].reshape(m2, 1, 1),
                                                   np.r_[be2.cpu().numpy()[:m2], 0.0].reshape(m2 + 1, 1, 1),
                                                   q2.cpu().numpy()[:m2]),
                                       (ao2.reshape(m2, 1, 1), np.r_[bo2, 0.0].reshape(m2 + 1, 1, 1), qo2),
                                       1e-9, RITZ_TOL)
            if not c2["parity"]["ok"]:
                raise RuntimeError(f"C2 parity check failed: {c2['parity']}")
            st2 = cpu_stats(t2)
            _, ts2 = orc.csr_spmm_timed(A2, bvh[:, None], reps=5)
            c2["cpu_baseline"] = {"value": st2["value"], "unit": "iters/s", "mean": st2["mean"], "worst": st2["worst"],
                                  "cores": orc.num_threads(), "kind": "port", "host_cpu": host_cpu(),
                                  "spmv_GBs": round(spmm_bytes(n2, A2.nnz, 1) / ts2 / 1e9, 2),
                                  "sample": f"best of {st2['samples']} single-vector iterations (after one warm-up) of "
                                            f"the same operator and start vector, oracle/lz_oracle.c OpenMP "
                                            f"(deterministic chunked dots); spmv_GBs: best of 5 oracle SpMVs"}
        del A2d, v0, v1, v2

    # ---- BASELINE config 4 (block Lanczos b=32 fp32, power-law rows): an extra line
    c5 = None
    if world == 1 and args.c5_steps > 0:
        n5, k5 = 10_000_000, args.c5_steps
        A5 = lz.gen_powerlaw(n5, 10.0, 2.1, 100000, seed=seed, dtype=np.float32)
        A5d = lz.CsrDevice.from_host(A5)
        kw5 = dict(dtype=torch.float32, device="cuda")
        B5 = torch.from_numpy(lz.uniform_B(n5, 32, seed=seed + 3, dtype=np.float32)).cuda()
        q5, al5, be5 = torch.zeros(k5 * 32, **kw5), torch.zeros(k5, 32, 32, **kw5), torch.zeros(k5 + 1, 32, 32, **kw5)
        P5 = [torch.zeros(n5, 32, **kw5) for _ in range(3)]
        h.block_lanczos_blas(A5d, B5, 2, 84, q5, al5, be5, *P5)  # warm
        torch.cuda.synchronize()
        t0c = time.perf_counter()
        h.block_lanczos_blas(A5d, B5, k5, 84, q5, al5, be5, *P5)
        torch.cuda.synchronize()
        dt5 = time.perf_counter() - t0c
        c5 = {"workload": f"C5 block Lanczos b=32 fp32, power-law-degree CSR (alpha 2.1, cap 1e5) n={n5} "
                          f"nnz={A5.nnz}, max row {int(np.diff(A5.row_ptr).max())}",
              "iters_per_s": round(k5 / dt5, 2), "ms_per_iter": round(dt5 / k5 * 1e3, 3),
              "finite": bool(torch.isfinite(al5).all())}
        # rooflines: the SpMM (the dominant kernel: U = A W_j - W_{j-1} M_j, tile pass + long-tile
        # pass) and the whole iteration (beta^2 form: A + 8 n b s), HIP events of a separate solve
        k5p = min(k5, 5)
        h.prof_enable(True)
        h.block_lanczos_blas(A5d, B5, k5p, 84, q5, al5, be5, *P5)
        torch.cuda.synchronize()
        sp5_ms, sp5_cnt = h.prof_read(h.PROF_SPMM)
        el5_ms, el5_cnt = h.prof_read(h.PROF_SPMM_PASS)
        ub5_ms, ub5_cnt = h.prof_read(h.PROF_UPDATE_PASS)
        h.prof_enable(False)
        a5 = A5.nnz * 8 + (n5 + 1) * 8  # fp32 values + int32 columns + row pointers
        nbs5 = n5 * 32 * 4
        if sp5_cnt == k5p:
            # step 0 has no W_{j-1} term: A + 2 nbs, later steps A + 3 nbs
            sp5_b = k5p * (a5 + 2 * nbs5) + (k5p - 1) * nbs5
            t5 = sp5_ms * 1e-3
            kn5 = "k_spmm_seg<float,32,48,1024,false,0,false,true,false>"
            tr5, src5 = pmc_traffic("k_spmm_seg_c5", n5, A5.nnz, 0, kn5)
            c5["roofline"] = {"bound": "hbm", "kernel": kn5 + " (+ its long-tile pass, MODE 1)",
                              "bytes_per_launch": round(sp5_b / k5p), "avg_ms": round(t5 / k5p * 1e3, 4),
                              "achieved": round(sp5_b / t5 / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": round(sp5_b / t5 / 1e9 / HBM_PEAK_GBS, 4),
                              "traffic": tr5, "traffic_source": src5,
                              "bytes_note": "A (4-B values, 4-B columns) + W_j gathered once + W_{j-1} read + U "
                                            "written = A + 3 n b s (step 0: A + 2 n b s); the reference's SpMM "
                                            "model A + 2 n b s is spmm_model_bytes",
                              "spmm_model_bytes": a5 + 2 * nbs5}
            if el5_cnt and ub5_cnt:
                c5["iteration_roofline"] = {
                    "bytes_per_step": a5 + 8 * nbs5, "ms_per_step": round(dt5 / k5 * 1e3, 3),
                    "frac": round((a5 + 8 * nbs5) / (dt5 / k5) / 1e9 / HBM_PEAK_GBS, 4),
                    "kernels_ms_per_step": {"spmm": round(sp5_ms / k5p, 4), "pass_el": round(el5_ms / el5_cnt, 4),
                                            "pass_ub": round(ub5_ms / ub5_cnt, 4)},
                    "note": "beta^2 form: SpMM A + 3 nbs, pass EL 2 nbs, pass UB 3 nbs"}
        if not args.no_cpu_baseline:  # fp32: 1e-4 relative
            orc = ge.load_oracle()
            m5 = min(k5, 4)
            B5h = B5.cpu().numpy()
            qo5, ao5, bo5, t5 = orc.block_lanczos_timed(A5, B5h, m5, 84)
            scale5 = max(1.0, float(np.abs(ao5).max()), float(np.abs(bo5[:m5]).max()))
            c5["parity"] = compare_run(lz, m5, 32, (al5.cpu().numpy(), be5.cpu().numpy(), q5.cpu().numpy()),
                                       (ao5, bo5, qo5), 1e-4, 1e-4 * scale5)
            if not c5["parity"]["ok"]:
                raise RuntimeError(f"C5 parity check failed: {c5['parity']}")
            st5 = cpu_stats(t5)
            _, ts5 = orc.csr_spmm_timed(A5, B5h, reps=2)
            c5["cpu_baseline"] = {"value": st5["value"], "unit": "iters/s", "mean": st5["mean"], "worst": st5["worst"],
                                  "cores": orc.num_threads(), "kind": "port", "host_cpu": host_cpu(),
                                  "spmm_GBs": round(spmm_bytes(n5, A5.nnz, 32, 4) / ts5 / 1e9, 2),
                                  "sample": f"best of {st5['samples']} fp32 block iterations (after the start-up "
                                            f"step and one warm-up) of the same operator and start block, "
                                            f"oracle/lz_oracle.c OpenMP; spmm_GBs: best of 2 oracle SpMMs"}
        # MFMA utilisation of the C5 dense step (v_mfma_f32_32x32x2_f32), committed PMC passes
        for kern in ("k_fused_el32", "k_fused_ub32"):  # the beta^2 form's passes (the default at b = 32)
            d, src = pmc_record("mfma", kern, n5, A5.nnz, 0, kern)
            if d:
                c5.setdefault("mfma", {})[kern] = {"pmc_MfmaUtil_pct": d.get("MfmaUtil_pct"),
                                                   "mfma_flop_per_launch": d.get("mfma_flop_per_launch"),
                                                   "pmc_source": src}
        del A5d, B5, P5

    # ---- C3 stress case: uniform-random columns (half width = n), same n, nnz/row, b
    c3r = None
    if world == 1 and not dist_path and args.rand_steps > 0:
        kr = args.rand_steps
        Ar = lz.gen_banded(n, args.nnz_per_row, n, seed)
        Ard = lz.CsrDevice.from_host(Ar)
        Yr = torch.empty(n, b, **kw)
        h.spmm(Ard, Bd, Yr)
        torch.cuda.synchronize()
        h.prof_enable(True)
        for _ in range(5):
            h.spmm(Ard, Bd, Yr)
        torch.cuda.synchronize()
        ms_r, cnt_r = h.prof_read(h.PROF_SPMM)
        h.prof_enable(False)
        qr, alr, ber = torch.zeros(kr * b, **kw), torch.zeros(kr, b, b, **kw), torch.zeros(kr + 1, b, b, **kw)
        Pr = [torch.zeros(n, b, **kw) for _ in range(3)]
        h.block_lanczos_blas(Ard, Bd, 2, 84, qr, alr, ber, *Pr)  # warm
        torch.cuda.synchronize()
        t0c = time.perf_counter()
        h.block_lanczos_blas(Ard, Bd, kr, 84, qr, alr, ber, *Pr)
        torch.cuda.synchronize()
        dtr = time.perf_counter() - t0c
        t_sp = ms_r / cnt_r * 1e-3
        c3r = {"workload": f"C3 stress: uniform-random columns (half width n), b={b} fp64, n={n} nnz={Ar.nnz}",
               "iters_per_s": round(kr / dtr, 2), "ms_per_iter": round(dtr / kr * 1e3, 3),
               "spmm_ms": round(t_sp * 1e3, 4),
               "spmm_GBs": round(spmm_bytes(n, Ar.nnz, b) / t_sp / 1e9, 1),
               "spmm_frac_of_hbm_peak": round(spmm_bytes(n, Ar.nnz, b) / t_sp / 1e9 / HBM_PEAK_GBS, 4),
               "finite": bool(torch.isfinite(alr).all())}
        if not args.no_cpu_baseline:
            orc = ge.load_oracle()
            mr = min(kr, 3)
            qor, aor, bor, tr = orc.block_lanczos_timed(Ar, B, mr, 84)
            c3r["parity"] = compare_run(lz, mr, b, (alr.cpu().numpy(), ber.cpu().numpy(), qr.cpu().numpy()),
                                        (aor, bor, qor), 1e-9, RITZ_TOL)
            if not c3r["parity"]["ok"]:
                raise RuntimeError(f"C3 random-column parity check failed: {c3r['parity']}")
            str_ = cpu_stats(tr)
            c3r["cpu_baseline"] = {"value": str_["value"], "unit": "iters/s", "mean": str_["mean"],
                                   "cores": orc.num_threads(), "kind": "port", "host_cpu": host_cpu(),
                                   "sample": f"best of {str_['samples']} block iterations of the same operator, "
                                             f"oracle/lz_oracle.c OpenMP"}
        # measured HBM traffic of this SpMM (committed PMC passes of the same operator): re-fetched
        # bytes, NOT algorithmic throughput
        tr_r, src_r = pmc_traffic("k_spmm_seg_random_columns", n, Ar.nnz, n, spmm_kernel(Ar.nnz, n))
        if tr_r:
            c3r.update({"spmm_pmc_hbm_bytes": tr_r, "spmm_pmc_refetch_ratio": round(tr_r / spmm_bytes(n, Ar.nnz, b), 2),
                        "spmm_pmc_hbm_GBs_incl_refetch": round(tr_r / t_sp / 1e9, 1),
                        "pmc_source": src_r})
        else:
            c3r["spmm_pmc_note"] = src_r
        del Ard, Yr, Pr

    if rank == 0:
        value = world * K / elapsed if not c4 else K / elapsed
        fused = not args.unfused
        t_pass = spmm_ms / max(spmm_cnt, 1) * 1e-3 if spmm_cnt else None
        t_upd = upd_ms / max(upd_cnt, 1) * 1e-3 if upd_cnt else None
        roof = mfma = None
        hw = args.halfwidth
        cb = col_bytes(n, hw)
        # the wavefront step (lz_wf.hip) has no separate update pass
        wf = fused and spmm_cnt > 0 and upd_cnt == 0
        if fused and wf:
            # one solve of K steps: the first step pass 1 only, the others pass 2 + pass 1 (at N > 1 the
            # boundary tiles' pass 1 is a launch of its own: same bytes, more launches)
            tot = wf_bytes(n, A.nnz, b, K, cb=cb)
            ach = tot / (spmm_ms * 1e-3) / 1e9
            kname, kshort = wf_kernel(n, hw, A.nnz, one_gpu=not dist_path)
            d, tsrc = pmc_record("", kshort, n, A.nnz, hw, kname, nnz_tol=0.01 if world > 1 else 0.0)
            traffic = None
            if d and d.get("hbm_bytes_first_launch"):
                # the solve's bytes spread over its launches, as bytes_per_launch (at N > 1 a step is
                # several launches over the same rows: the requested tiles' pass 2, the step, the boundary)
                traffic = round((d["hbm_bytes_first_launch"] + (K - 1) * d["hbm_bytes_per_launch"]) / spmm_cnt)
            roof = {"bound": "hbm", "kernel": kname, "first_launch_kernel": wf_first_kernel(kname),
                    "achieved": round(ach, 1),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                    "traffic": traffic, "traffic_unit": "bytes/launch (mean over the profiled solve's launches)",
                    "traffic_source": tsrc, "avg_ms": round(t_pass * 1e3, 4),
                    "bytes_per_launch": round(tot / spmm_cnt),
                    # a steady launch reads A + 3nbs and writes 2nbs: ~2 : 1
                    "stream_ceiling": stream_ceiling(ach, "r2w1"),
                    "bytes_note": f"{K} steps per solve in {spmm_cnt} launches: the first step pass 1 only (A + 2nbs), "
                                  f"the others pass 2 of step j + pass 1 of step j+1 (A + 5nbs); A with {cb}-byte "
                                  f"columns"}
            # the timed solve's MFMA FLOP (its first launch pass 1 only) over its launches' kernel time
            fl = wf_mfma_flop(n, spmm_cnt) / spmm_cnt
            tf = fl / t_pass / 1e12
            ent = {"kernel": kshort, "mfma_flop_per_launch": round(fl), "avg_ms": round(t_pass * 1e3, 4),
                   "achieved": round(tf, 3), "frac": round(tf / FP64_MFMA_PEAK_TFS, 4),
                   "mfma_flop_per_steady_launch": WF_MFMA_FLOP_PER_ROW * n,
                   "flop_note": f"{spmm_cnt} launches: the first 4 v_mfma_f64_16x16x4f64 per 16-row strip (S1), "
                                f"the others 24 (V_(j+1) 12, G 4, S2 4, S1 4); 2048 FLOP each"}
            d, src = pmc_record("mfma", kshort, n, A.nnz, hw, kname)
            if d:
                ent.update({"pmc_MfmaUtil_pct": d.get("MfmaUtil_pct"),
                            "pmc_mfma_flop_per_launch": d.get("mfma_flop_per_launch"),
                            "pmc_mfma_flop_per_steady_launch": d.get("mfma_flop_per_steady_launch"),
                            "pmc_dispatch_mix": d.get("dispatch_mix"), "pmc_source": src})
                # MfmaUtil is busy / elapsed cycles at the profiled run's clock; the FLOP
                # fraction above is against the 2.4 GHz peak: the same quantity is
                # MfmaUtil x (profiled clock / 2.4 GHz)
                clk = d.get("effective_clock_GHz")
                if clk and d.get("MfmaUtil_pct") is not None:
                    ent["pmc_frac_at_peak_clock"] = round(d["MfmaUtil_pct"] / 100.0 * clk / 2.4, 4)
                    ent["pmc_note"] = (f"profiled clock {clk} GHz; MfmaUtil {d['MfmaUtil_pct']} % of the SIMD cycles "
                                       f"= {ent['pmc_frac_at_peak_clock']} of the 2.4 GHz peak, against frac {ent['frac']} "
                                       f"from the model FLOP and this run's kernel time")
            else:
                ent["pmc_note"] = src
            mfma = {"unit": "TFLOP/s", "peak": FP64_MFMA_PEAK_TFS, "dtype": "f64 (v_mfma_f64_16x16x4f64)",
                    "wavefront_step": ent}
        elif fused and t_pass:
            ach = fused_pass_bytes(n, A.nnz, b, cb=cb) / t_pass / 1e9
            kname, kshort = fused_kernel(A.nnz, n)
            traffic, tsrc = pmc_traffic(kshort, n, A.nnz, hw, kname)
            roof = {"bound": "hbm", "kernel": kname, "achieved": round(ach, 1),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                    "traffic": traffic, "traffic_unit": "bytes/launch", "traffic_source": tsrc,
                    "avg_ms": round(t_pass * 1e3, 4),
                    "bytes_per_launch": fused_pass_bytes(n, A.nnz, b, cb=cb)}
            # MFMA utilisation of the dense step (north star): algorithmic MFMA FLOP / kernel time
            # against the fp64 MFMA peak, plus the rocprofv3 MfmaUtil counter of the same kernels
            mfma = {"unit": "TFLOP/s", "peak": FP64_MFMA_PEAK_TFS, "dtype": "f64 (v_mfma_f64_16x16x4f64)",
                    "pass2_update_gram": None, "pass1_epilogue": None}
            for key, kern, kfull, fl, t in (("pass2_update_gram", "k_fused_update16", PASS2_KERNEL,
                                             PASS2_MFMA_FLOP_PER_ROW, t_upd),
                                            ("pass1_epilogue", kshort, kname, PASS1_MFMA_FLOP_PER_ROW, t_pass)):
                if not t:
                    continue
                tf = fl * n / t / 1e12
                ent = {"kernel": kern, "mfma_flop_per_launch": fl * n, "avg_ms": round(t * 1e3, 4),
                       "achieved": round(tf, 3), "frac": round(tf / FP64_MFMA_PEAK_TFS, 4)}
                d, src = pmc_record("mfma", kern, n, A.nnz, hw, kfull)
                if not d:
                    ent["pmc_note"] = src
                if d:
                    ent.update({"pmc_MfmaUtil_pct": d.get("MfmaUtil_pct"),
                                "pmc_mfma_flop_per_launch": d.get("mfma_flop_per_launch"), "pmc_source": src})
                mfma[key] = ent
        elif plain:
            roof = {"bound": "hbm", "kernel": plain["kernel"], "achieved": plain["achieved_GBs"],
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": plain["frac_of_hbm_peak"], "traffic": None}
        # iteration roofline: SURVEY.md 8(d)'s fixed convention (A + 8 n b s) and the bytes the
        # design actually moves (A + 6 n b s two-pass, A + 5 n b s wavefront); per rank
        a_bytes = A.nnz * 12 + (n + 1) * 8
        step_nbs = 5 if wf else 6
        it_s = elapsed / K
        if c4:
            workload = (f"C4 block Lanczos b=16 fp64, banded-random symmetric CSR n={n_total} total "
                        f"({world} rank(s), {n} rows on rank 0), nnz~{args.nnz_per_row:g}/row, "
                        f"halfwidth {args.halfwidth}")
        elif c4rank:
            workload = (f"C4 per-rank share on one GPU: block Lanczos b=16 fp64, banded-random symmetric CSR "
                        f"n={args.n} (one of 8 ranks of the 40M-row operator), nnz~{args.nnz_per_row:g}/row, "
                        f"halfwidth {args.halfwidth} (columns clipped to the share: no halo rows)")
        else:
            workload = ("C3 block Lanczos b=16 fp64, banded-random symmetric CSR "
                        f"n={args.n} per GPU, nnz~{args.nnz_per_row:g}/row, halfwidth {args.halfwidth}")
        out = {
            "metric": "block-Lanczos iters/sec + SpMM achieved HBM GB/s vs peak, n=10M nnz=1e8 b=16",
            "value": round(value, 3),
            "unit": "iters/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / K * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if c4 else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (splitmix64 banded-random symmetric CSR, seed 20261015)",
            "config": {"workload": workload, "config": args.config.upper(),
                       "n_total": n_total, "n_per_gpu": n, "nnz_per_gpu": A.nnz, "b": b, "m_timed": K,
                       "path": "fused" if fused else "unfused",
                       "parallelism": parallelism},
            "roofline": roof,
            "cpu_baseline": cpu,
            "parity": parity,
            "mfma": mfma,
            "extra": {
                "plain_spmm": plain,
                "other_exchange": other,
                "c2_vector_lanczos": c2,
                "c5_block32_f32_powerlaw": c5,
                "c3_random_columns_stress": c3r,
                "kernel_ms_per_step": {"fused_spmm_pass": round(spmm_ms / K, 4),
                                       "update_pass": round(upd_ms / K_bd, 4),
                                       "finish_sqrtm": round(small_ms / K_bd, 4),
                                       "gram": round(gram_ms / K_bd, 4),
                                       "note": f"fused_spmm_pass: HIP events in the timed region; the others: "
                                               f"a separate {K_bd}-step run with every class recorded"},
                # the achieved fraction of the iteration: the bytes the implemented step moves
                "iteration_frac_qfree_bytes": round((a_bytes + step_nbs * n * b * 8) / it_s / 1e9 / HBM_PEAK_GBS, 4),
                "iteration_qfree_bytes": a_bytes + step_nbs * n * b * 8,
                # NOT an achieved fraction: the SURVEY.md 8(d) model's A + 8nbs (more bytes than the
                # implemented step moves) per measured step time, kept for comparison with that convention
                "iteration_rate_vs_survey_model_A8nbs": round((a_bytes + 8 * n * b * 8) / it_s / 1e9 / HBM_PEAK_GBS, 4),
                "survey_model_bytes": a_bytes + 8 * n * b * 8,
                "iteration_bytes_note": f"qfree_bytes: A + {step_nbs}nbs, what the implemented Q-free "
                                        f"{'wavefront' if wf else 'two-pass'} step moves (A with 12-B entries; "
                                        "the roofline kernel streams 2-B columns); survey_model_bytes: SURVEY.md "
                                        "8(d)'s fixed A + 8nbs convention, not bytes this step moves; the per-solve "
                                        "final-state pass (Q0 = Q1 = Q_{m-1}, W = W_m: 6 nbs once) is inside the "
                                        "timed solve",
                "step_form": "wavefront (lz_wf.hip)" if wf else ("two-pass (lz_fused.hip)" if fused else "unfused"),
                # the gather-bound pass's natural unit: nonzeros (one 128-B X row gathered each) per second,
                # comparable across C3 (10 nnz/row) and C4 (25 nnz/row)
                "nnz_per_s_per_gpu": round(A.nnz * K / elapsed, 1),
            },
        }
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    h.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
