"""The reference's own measurement harnesses (kernels/measurements/*.cu,
measure_lanczos.cu), re-run through this build's C ABI at the sizes and
precision their published numbers were taken at (from
lanczos_plots.m), plus the structured C3 companion SURVEY.md 8(f)1 names
(the Yee operator at N=120, fp64 b=16).

Bandwidth is given twice: with each harness's own byte formula (the column the
reference published) and with this build's algorithmic-bytes model.  The
reference numbers are from its (unstated, T4-class) GPU in fp32; `speedup` is
the reference's published time / ours.  HIP-event timing on the handle's
stream (the legacy default stream, which is also torch's current stream).

  python scripts/ref_harness.py > profiles/r01_ref_harness.json
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

lz = ge.load_package()
h = lz.Handle(0)
f32 = dict(dtype=torch.float32, device="cuda")
f64 = dict(dtype=torch.float64, device="cuda")
rows = []


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def emit(name, src, size, ms, ref_ms, ref_bytes, alg_bytes, note=""):
    r = {"harness": name, "reference_source": src, "size": size, "ms": round(ms, 4),
         "reference_ms": ref_ms, "speedup": round(ref_ms / ms, 2) if ref_ms else None,
         "GBs_reference_formula": round(ref_bytes / ms / 1e6, 1) if ref_bytes else None,
         "GBs_algorithmic": round(alg_bytes / ms / 1e6, 1) if alg_bytes else None}
    if note:
        r["note"] = note
    rows.append(r)
    print(json.dumps(r), file=sys.stderr, flush=True)


t0 = time.time()
# ---- Yee operator at N=160 (the published SpMM / Lanczos size), fp32
A64 = lz.matrix_a(160)
n = A64.n
A32 = lz.CsrHost(n, A64.row_ptr, A64.col, A64.val.astype(np.float32))
Ad = lz.CsrDevice.from_host(A32)
print(f"matrix_a(160): n={n} nnz={A64.nnz} ({time.time() - t0:.1f}s)", file=sys.stderr)
b = 16
X = torch.rand(n, b, **f32)
Y = torch.empty(n, b, **f32)
ms = timed(lambda: h.spmm(Ad, X, Y), 20)
# spmv_spmm.cu:384: ELL data (value + index per slot, width 4) + X + Y
emit("ELL-4 SpMM b=16 (here CSR, row-major X/Y)", "lanczos_plots.m:96-98; kernels/measurements/spmv_spmm.cu:384",
     f"Yee N=160, n={n}, nnz={A64.nnz}, fp32", ms, 16.71,
     n * 4 * 8 + 2 * n * b * 4, A64.nnz * 8 + (n + 1) * 8 + 2 * n * b * 4)
Xc = torch.rand(b, n, **f32)  # column-major X / Y (the reference's layout: ld = n)
Yc = torch.empty(b, n, **f32)
ms = timed(lambda: h.spmm(Ad, Xc, Yc, layout=lz.LZ_COL_MAJOR), 20)
emit("ELL-4 SpMM b=16 (here CSR, column-major X/Y as the reference)", "lanczos_plots.m:96-98",
     f"Yee N=160, n={n}, fp32", ms, 16.71, n * 4 * 8 + 2 * n * b * 4,
     A64.nnz * 8 + (n + 1) * 8 + 2 * n * b * 4)

# block Lanczos m=2, b=16 fp32 on the same operator (measure_lanczos.cu); unfused reference op order
m = 2
B = torch.rand(n, b, **f32) + 1.0
q, al, be = torch.zeros(m * b, **f32), torch.zeros(m, b, b, **f32), torch.zeros(m + 1, b, b, **f32)
Q0, Q1, W = (torch.zeros(n, b, **f32) for _ in range(3))
ms = timed(lambda: h.block_lanczos_blas(Ad, B, m, 5, q, al, be, Q0, Q1, W), 5)
emit("block Lanczos m=2 b=16", "lanczos_plots.m:142-144; measure_lanczos.cu:268-292",
     f"Yee N=160, n={n}, fp32 (n not recorded by the reference; inferred 24.8M)", ms, 198.0, None, None,
     "whole solve: start-up step + 1 iteration, unfused reference op order (fp32 has no fused path)")
del Ad, X, Y, Xc, Yc, B, Q0, Q1, W

# ---- dense kernels at the harness sizes, fp32 b=16
nt = 10_137_600
T = torch.rand(nt, b, **f32)
R = torch.empty(b, b, **f32)
ms = timed(lambda: h.mm_tt(T, R), 20)
emit("Gram T^T T (mm_tt)", "lanczos_plots.m:40-46; kernels/measurements/mm_tt.cu:252-253",
     f"{nt} x {b}, fp32", ms, 3.52, 2 * nt * b * 4, nt * b * 4, "the reference formula counts T twice")
T2 = torch.rand(nt, b, **f32)
ms = timed(lambda: h.mm_tt2(T, T2, R), 20)
emit("sym cross-Gram (mm_tt2)", "lanczos_plots.m:67-73; kernels/measurements/mm_tt2.cu:282-283",
     f"{nt} x {b}, fp32", ms, 6.63, 4 * nt * b * 4, 2 * nt * b * 4, "the reference formula counts both inputs twice")
del T, T2
ns = 3_072_000
Qs = torch.rand(ns, b, **f32)
S = torch.rand(b, b, **f32)
Ws = torch.empty(ns, b, **f32)
ms = timed(lambda: h.mm_ts(0.0, 1.0, Qs, S, Ws), 20)
emit("tall x small (mm_ts), W = Q S", "lanczos_plots.m:10-16; kernels/measurements/mm_ts.cu:303",
     f"{ns} x {b}, fp32", ms, 1.74, 2 * ns * b * 4, 2 * ns * b * 4)
del Qs, Ws
G = torch.rand(b, b, **f64)
G = (G @ G.T + b * torch.eye(b, **f64)).to(torch.float32)
be1, bi1 = torch.empty(b, b, **f32), torch.empty(b, b, **f32)
ms = timed(lambda: h.sqrtm(G, be1, bi1), 50)
emit("sqrtm 16x16 (+ inverse)", "lanczos_plots.m:120-121", "b=16, fp32", ms, 0.1156, None, None,
     "reference custom kernel 115.6 us, cusolver syevjBatched 76.6 us")
# both routes of the one-workgroup sqrtm at b = 16 and 32 (round 5: Newton-Schulz on the
# f64 MFMA by one wave at b = 16, four waves at b = 32; LZ_SQRTM_NS=0: the Jacobi route),
# on a well-conditioned SPD G (kappa ~ 1e3, inside the Newton-Schulz bound of 4e6)
for bs in (16, 32):
    Gd = torch.rand(bs, bs, **f64)
    Gd = Gd @ Gd.T + 0.05 * bs * torch.eye(bs, **f64)
    for dt, kw in (("fp64", f64), ("fp32", f32)):
        Gx = Gd.to(kw["dtype"])
        bo, bi = torch.empty(bs, bs, **kw), torch.empty(bs, bs, **kw)
        for route, env in (("Newton-Schulz", "1"), ("Jacobi", "0")):
            os.environ["LZ_SQRTM_NS"] = env
            ms = timed(lambda: h.sqrtm(Gx, bo, bi), 50)
            emit(f"sqrtm {bs}x{bs} (+ inverse), {route}", "lanczos_plots.m:120-121; utils/lib_utils.hpp:696-745",
                 f"b={bs}, {dt}, kappa(G)={float(torch.linalg.cond(Gd)):.1e}", ms,
                 0.1156 if bs == 16 else None, None, None,
                 "the reference publishes b = 16 only (custom kernel 115.6 us, syevjBatched 76.6 us)")
        os.environ.pop("LZ_SQRTM_NS", None)

# ---- structured C3 companion: Yee N=120, fp64, b=16, fused iteration
A = lz.matrix_a(120)
n = A.n
Ad = lz.CsrDevice.from_host(A)
X = torch.rand(n, b, **f64)
Y = torch.empty(n, b, **f64)
ms = timed(lambda: h.spmm(Ad, X, Y), 20)
emit("SpMM b=16 fp64, structured C3 companion", "SURVEY.md 8(f)1", f"Yee N=120, n={n}, nnz={A.nnz}, fp64",
     ms, None, None, A.nnz * 12 + (n + 1) * 8 + 2 * n * b * 8)
m = 20
B = torch.from_numpy(lz.uniform_B(n, b, seed=3)).cuda()
q, al, be = torch.zeros(m * b, **f64), torch.zeros(m, b, b, **f64), torch.zeros(m + 1, b, b, **f64)
Q0, Q1, W = (torch.zeros(n, b, **f64) for _ in range(3))
ms = timed(lambda: h.block_lanczos_blas(Ad, B, m, 5, q, al, be, Q0, Q1, W), 3)
emit("block Lanczos b=16 fp64 fused, structured C3 companion", "SURVEY.md 8(f)1",
     f"Yee N=120, n={n}, m={m}", ms / m, None, None, A.nnz * 12 + (n + 1) * 8 + 6 * n * b * 8,
     f"ms per iteration (whole {m}-step solve / {m}); iters/s = {1e3 * m / ms:.1f}")

print(json.dumps({"device": torch.cuda.get_device_name(0), "rows": rows}, indent=1))
