"""Benchmark: block-Lanczos iterations/sec + SpMM achieved HBM GB/s vs peak
(BASELINE.json metric), n = 10M, nnz = 1e8, b = 16, fp64, on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]

A "step" is one block-Lanczos iteration (fused SpMM pass + alpha finish +
update pass + beta sqrtm) over the whole synthetic operator, inputs resident in
HBM.  N = 1: config C3 on one GPU.  N > 1 (launched by torch.distributed.run):
weak scaling -- every rank owns a 10M-row slab of an N*10M-row banded operator,
row-partitioned; each iteration exchanges only the Krylov-block rows other
ranks reference (RCCL grouped send/recv, `--exchange halo`, default) or
all-gathers the block (`--exchange allgather`); `value` counts
slab-iterations/s summed over ranks.  rank 0 prints one JSON line on stdout
(native libraries' own stdout output is routed to stderr).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_PEAK_TFS = 78.6


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def spmm_bytes(n, nnz, b, sv=8):
    """Reference's A + 2B model + row_ptr: z(s_v+4) + (n+1)8 + 2 n b s_v."""
    return nnz * (sv + 4) + (n + 1) * 8 + 2 * n * b * sv


def fused_pass_bytes(n, nnz, b, sv=8):
    """Algorithmic bytes of one fused pass-1 launch (Q-free iteration): A, the
    Krylov block W_j read once, W_{j-1} read, W' written."""
    return nnz * (sv + 4) + (n + 1) * 8 + 3 * n * b * sv


def fused_kernel():
    """(full name, PMC short name) of the pass-1 kernel lz_fused.hip launches for
    b = 16 fp64 (LZ_FUSED_KERNEL selects the alternatives kept for A/B runs)."""
    v = os.environ.get("LZ_FUSED_KERNEL", "")
    if v.startswith("s"):
        return "k_fused_seg16", "k_fused_seg16"
    if v.startswith("t"):
        return "k_fused_spmm16<true>", "k_fused_spmm16"
    if v.startswith("p"):
        return f"k_fused_pf16<{8 if v[1:2] == '8' else 4}>", "k_fused_pf16"
    if not v or v.startswith("r"):
        return "k_fused_pp16<14,2376,3,2>", "k_fused_pp16"
    if v.startswith("wsq"):
        return "k_fused_ws16<15,2536,2>", "k_fused_ws16"
    if v.startswith("n"):
        return "k_fused_ws16<14,2376,3,true,2>", "k_fused_ws16"
    return "k_fused_ws16<15,2536,3,true>", "k_fused_ws16"


def spmm_kernel():
    """The plain SpMM kernel lz_csr_spmm launches for b = 16 fp64 (LZ_SPMM_KERNEL A/B)."""
    v = os.environ.get("LZ_SPMM_KERNEL", "")
    if not v or v[0] == "s":
        tr = {"3": 32, "6": 64, "9": 96}.get(v[1:2], 48)
        return f"k_spmm_seg<double,16,{tr},{tr * 16},8,nt>"
    return "k_spmm_buf<double,16,1024,2>" if v[0] == "b" else f"LZ_SPMM_KERNEL={v}"


def pmc_traffic(kernel, n, nnz, hw):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary
    (profiles/*_pmc_<kernel>.json, written by scripts/pmc_traffic.py from separate
    FETCH_SIZE / WRITE_SIZE passes of this bench command; FETCH_SIZE doubled per
    MI355X_MICROARCH.md's gfx950 note).  None unless it was taken on this workload."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_pmc_{kernel}.json")), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        w = d.get("workload", {})
        if w.get("n") == n and w.get("nnz") == nnz and w.get("halfwidth") == hw:
            return d.get("hbm_bytes_per_launch"), os.path.relpath(f, ROOT)
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=10_000_000, help="rows per GPU")
    ap.add_argument("--nnz-per-row", type=float, default=10.0)
    ap.add_argument("--halfwidth", type=int, default=4096)
    ap.add_argument("--b", type=int, default=16)
    ap.add_argument("--unfused", action="store_true")
    ap.add_argument("--cpu-iters", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--spmm-reps", type=int, default=20)
    ap.add_argument("--c2-steps", type=int, default=200, help="single-vector Lanczos steps at BASELINE config 1 (0: skip)")
    ap.add_argument("--c5-steps", type=int, default=10, help="block-32 fp32 power-law steps at BASELINE config 4 (0: skip)")
    ap.add_argument("--rand-steps", type=int, default=10,
                    help="block-Lanczos steps on the C3 uniform-random-column stress operator (0: skip)")
    ap.add_argument("--exchange", choices=["halo", "allgather"], default="halo",
                    help="multi-GPU Krylov-block exchange (N > 1, or with --dist at N = 1)")
    ap.add_argument("--dist", action="store_true",
                    help="run the distributed entry point even at N = 1 (rehearsal of the N > 1 path)")
    args = ap.parse_args()
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
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    lz = ge.load_package()
    h = lz.Handle(local)
    b, n = args.b, args.n
    seed = 20261015
    t_gen = time.time()
    dist_path = world > 1 or args.dist
    if world == 1:
        A = lz.gen_banded(n, args.nnz_per_row, args.halfwidth, seed)
    else:
        A = lz.gen_banded_local(n * world, rank * n, (rank + 1) * n, args.nnz_per_row, args.halfwidth, seed)
    B = lz.uniform_B(n, b, seed + rank)
    log(f"[rank {rank}] generated n={A.n} nnz={A.nnz} in {time.time() - t_gen:.1f}s")
    kw = dict(dtype=torch.float64, device="cuda")
    m_max = max(args.steps, args.warmup, 1)
    q = torch.zeros(m_max * b, **kw)
    alpha = torch.zeros(m_max, b, b, **kw)
    beta = torch.zeros(m_max + 1, b, b, **kw)
    Bd = torch.from_numpy(B).cuda()
    halo_rows = 0

    if not dist_path:
        Ad = lz.CsrDevice.from_host(A)
        Q0, Q1, W = (torch.zeros(n, b, **kw) for _ in range(3))

        def run(m):
            h.block_lanczos_blas(Ad, Bd, m, 84, q, alpha, beta, Q0, Q1, W, fused=not args.unfused)
    else:
        uid = [lz.comm_unique_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(uid, src=0)
        h.comm_init(world, rank, uid[0])
        if args.exchange == "halo":
            # rank g owns rows [g n, (g+1) n); only referenced off-rank rows move
            bounds = np.arange(world + 1, dtype=np.int64) * n
            ccol, rcnt, hrows = lz.halo_plan(A.col, bounds, rank)
            h.halo_init(rank * n, n, rcnt, hrows)
            halo_rows = int(hrows.size)
            Ad = lz.CsrDevice.from_host(lz.CsrHost(A.n, A.row_ptr, ccol, A.val), n_cols=n + halo_rows)
            X0, X1 = (torch.zeros(n + halo_rows, b, **kw) for _ in range(2))
            log(f"[rank {rank}] halo rows {halo_rows}")

            def run(m):
                h.block_lanczos_halo(Ad, Bd, m, 84, 0, q, alpha, beta, X0, X1)
        else:
            Ad = lz.CsrDevice.from_host(A, n_cols=n * world)
            Q0, W = (torch.zeros(n, b, **kw) for _ in range(2))
            X_full = torch.zeros(n * world, b, **kw)

            def run(m):
                h.block_lanczos_dist(Ad, n, n * world, Bd, m, 84, 0, q, alpha, beta, Q0, W, X_full)

    # ---- warmup
    if args.warmup > 0:
        run(args.warmup)
    torch.cuda.synchronize()

    # ---- timed region: exactly K steps
    h.prof_enable(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    spmm_ms, spmm_cnt = h.prof_read(h.PROF_SPMM_PASS)
    upd_ms, upd_cnt = h.prof_read(h.PROF_UPDATE_PASS)
    small_ms, small_cnt = h.prof_read(h.PROF_SMALL)
    gram_ms, gram_cnt = h.prof_read(h.PROF_GRAM)
    h.prof_enable(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    assert torch.isfinite(alpha[: args.steps]).all(), "non-finite alpha"

    # ---- plain SpMM kernel (the BASELINE headline kernel), same operator
    plain = None
    if world == 1 and args.spmm_reps > 0:
        Y = torch.empty(n, b, **kw)
        h.spmm(Ad, Q0, Y)
        torch.cuda.synchronize()
        h.prof_enable(True)
        for _ in range(args.spmm_reps):
            h.spmm(Ad, Q0, Y)
        torch.cuda.synchronize()
        ms, cnt = h.prof_read(h.PROF_SPMM)
        h.prof_enable(False)
        t_avg = ms / cnt * 1e-3
        gbs = spmm_bytes(n, A.nnz, b) / t_avg / 1e9
        plain = {"kernel": spmm_kernel(), "avg_ms": round(ms / cnt, 4),
                 "bytes_per_launch": spmm_bytes(n, A.nnz, b), "achieved_GBs": round(gbs, 1),
                 "frac_of_hbm_peak": round(gbs / HBM_PEAK_GBS, 4)}

    # ---- BASELINE config 1 (single-vector Lanczos, n=1M, nnz=1e7): an extra line
    c2 = None
    if world == 1 and args.c2_steps > 0:
        n2 = 1_000_000
        A2 = lz.gen_banded(n2, 10.0, args.halfwidth, seed)
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
              "iteration_GBs": round((A2.nnz * 12 + (n2 + 1) * 8 + 5 * n2 * 8) / (dt2 / k2) / 1e9, 1),
              "note": "A + 5 n s bytes per step (A, w read, q_{j-1} read, q_j written, w' written)"}
        del A2d, v0, v1, v2

    # ---- BASELINE config 4 (block Lanczos b=32 fp32, power-law rows): an extra line
    c5 = None
    if world == 1 and args.c5_steps > 0:
        n5, k5 = args.n, args.c5_steps
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
        h.block_lanczos_blas(Ard, Bd, 2, 84, qr, alr, ber, Q0, Q1, W)  # warm
        torch.cuda.synchronize()
        t0c = time.perf_counter()
        h.block_lanczos_blas(Ard, Bd, kr, 84, qr, alr, ber, Q0, Q1, W)
        torch.cuda.synchronize()
        dtr = time.perf_counter() - t0c
        t_sp = ms_r / cnt_r * 1e-3
        c3r = {"workload": f"C3 stress: uniform-random columns (half width n), b={b} fp64, n={n} nnz={Ar.nnz}",
               "iters_per_s": round(kr / dtr, 2), "ms_per_iter": round(dtr / kr * 1e3, 3),
               "spmm_ms": round(t_sp * 1e3, 4),
               "spmm_GBs": round(spmm_bytes(n, Ar.nnz, b) / t_sp / 1e9, 1),
               "spmm_frac_of_hbm_peak": round(spmm_bytes(n, Ar.nnz, b) / t_sp / 1e9 / HBM_PEAK_GBS, 4),
               "finite": bool(torch.isfinite(alr).all())}
        # measured HBM traffic of this SpMM (committed PMC passes of the same operator)
        tr_r, src_r = pmc_traffic("k_spmm_seg_random_columns", n, Ar.nnz, n)
        if tr_r:
            c3r.update({"spmm_pmc_hbm_bytes": tr_r, "spmm_pmc_GBs": round(tr_r / t_sp / 1e9, 1),
                        "spmm_pmc_frac_of_hbm_peak": round(tr_r / t_sp / 1e9 / HBM_PEAK_GBS, 4),
                        "pmc_source": src_r})
        del Ard, Yr

    # ---- CPU baseline: the oracle (C, OpenMP) on this operator, rank 0, N = 1
    cpu = None
    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        orc = ge.load_oracle()
        iters = max(1, args.cpu_iters)
        t_cpu = orc.time_block_iters(A, B, iters)
        cpu = {"value": round(iters / t_cpu, 4), "unit": "iters/s", "cores": orc.num_threads(),
               "kind": "port",
               "sample": f"{iters} block-Lanczos iterations (after the start-up step) of the same "
                         f"n={n} nnz={A.nnz} b={b} fp64 operator, oracle/lz_oracle.c OpenMP"}

    if rank == 0:
        K = args.steps
        value = world * K / elapsed
        fused = not args.unfused
        t_pass = spmm_ms / max(spmm_cnt, 1) * 1e-3 if spmm_cnt else None
        if fused and t_pass:
            ach = fused_pass_bytes(n, A.nnz, b) / t_pass / 1e9
            kname, kshort = fused_kernel()
            traffic, tsrc = pmc_traffic(kshort, n, A.nnz, args.halfwidth)
            roof = {"bound": "hbm", "kernel": kname, "achieved": round(ach, 1),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                    "traffic": traffic, "traffic_unit": "bytes/launch", "traffic_source": tsrc,
                    "avg_ms": round(t_pass * 1e3, 4),
                    "bytes_per_launch": fused_pass_bytes(n, A.nnz, b)}
        elif plain:
            roof = {"bound": "hbm", "kernel": plain["kernel"], "achieved": plain["achieved_GBs"],
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": plain["frac_of_hbm_peak"], "traffic": None}
        else:
            roof = None
        iter_min_bytes = A.nnz * 12 + (n + 1) * 8 + 8 * n * b * 8  # SURVEY.md 8(d) convention, fixed
        out = {
            "metric": "block-Lanczos iters/sec + SpMM achieved HBM GB/s vs peak, n=10M nnz=1e8 b=16",
            "value": round(value, 3),
            "unit": "iters/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / K * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (splitmix64 banded-random symmetric CSR, seed 20261015)",
            "config": {"workload": "C3 block Lanczos b=16 fp64, banded-random symmetric CSR "
                                   f"n={n} per GPU, nnz~{args.nnz_per_row:g}/row, halfwidth {args.halfwidth}",
                       "n_per_gpu": n, "nnz_per_gpu": A.nnz, "b": b, "m_timed": K,
                       "path": "fused" if fused else "unfused",
                       "parallelism": ("single" if not dist_path else
                                       f"rows{world}+rccl_{args.exchange}" + (f"({halo_rows} halo rows/rank)"
                                                                              if args.exchange == "halo" else ""))},
            "roofline": roof,
            "cpu_baseline": cpu,
            "extra": {
                "plain_spmm": plain,
                "c2_vector_lanczos": c2,
                "c5_block32_f32_powerlaw": c5,
                "c3_random_columns_stress": c3r,
                "kernel_ms_per_step": {"fused_spmm_pass": round(spmm_ms / K, 4),
                                       "update_pass": round(upd_ms / K, 4),
                                       "finish_sqrtm": round(small_ms / K, 4),
                                       "gram": round(gram_ms / K, 4)},
                "iteration_frac_of_roofline": round(iter_min_bytes / (elapsed / K) / 1e9 / HBM_PEAK_GBS, 4),
                "iteration_min_bytes": iter_min_bytes,
            },
        }
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    h.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
