"""The rebuilt reference driver (lib/test_lanczos, csrc/test_lanczos.cpp on the
C++ drop-in layer include/lz_methods.hpp) run as its own process, the way the
reference's test_lanczos.cu:131-362 is run: its printed Ritz values and
solution lines are checked against the committed golden vectors (the CPU
restatement on the reference's own matrix_a operator and glibc-rand B)."""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RITZ_TOL = 1e-10


def run_driver(lz, *args):
    exe = os.path.join(lz.LIB_DIR, "test_lanczos")
    assert os.path.exists(exe), "lib/test_lanczos not built"
    out = subprocess.run([exe, *args], capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = out.stdout.splitlines()
    ritz = None
    sol = []
    for i, ln in enumerate(lines):
        if ln.startswith("Ritz values"):
            ritz = np.array([float(t) for t in ln.split(":", 1)[1].split()])
        if ln.startswith("Solution for block lanczos"):
            k = i + 1
            while k < len(lines) and lines[k].strip() and not lines[k].startswith(" "):
                try:
                    sol.append(float(lines[k]))
                except ValueError:
                    break
                k += 1
    assert " the size of the problem is " in out.stdout and " end Lanczos " in out.stdout
    return ritz, np.array(sol), out.stdout


def test_driver_default_command_line(lz, golden):
    """The reference's own run, no arguments (test_lanczos.cu:310-362): -N 10 -m 5,
    N_COL = 4, B column-major with rows padded to a multiple of 768 (handed to
    block_lanczos_blas in that layout), then the 10^6-step forward-Euler check."""
    ritz, sol, out = run_driver(lz)
    assert np.max(np.abs(ritz - golden["N10_b4_m5_ritz"])) <= RITZ_TOL
    assert np.allclose(sol, golden["N10_b4_m5_solution"], rtol=1e-9, atol=1e-13)
    assert " start fdtd " in out and "Solution from fdtd" in out
    rel = float(out.split("Relative error for block lanczos is")[1].split()[0])
    assert rel < 1e-7, rel  # forward Euler at dt = 1e-6 against the Krylov solution


@pytest.mark.parametrize("m,extra", [(5, []), (5, ["--unfused"]), (20, []), (5, ["--row-major-B"])])
def test_driver_block_matrix_a(lz, golden, m, extra):
    """-N 10 -m 5 / 20, N_COL = 4; B in the reference's padded column-major layout
    (default) or row-major."""
    ritz, sol, _ = run_driver(lz, "-N", "10", "-m", str(m), "--block", "4", "--fdtd-steps", "0", *extra)
    key = f"N10_b4_m{m}"
    assert ritz.size == 4 * m
    assert np.max(np.abs(ritz - golden[key + "_ritz"])) <= RITZ_TOL
    assert np.allclose(sol, golden[key + "_solution"], rtol=1e-9, atol=1e-13)


def test_driver_block16(lz, golden):
    ritz, sol, _ = run_driver(lz, "-N", "10", "-m", "5", "--block", "16", "--fdtd-steps", "0")
    assert np.max(np.abs(ritz - golden["N10_b16_m5_ritz"])) <= RITZ_TOL
    assert np.allclose(sol, golden["N10_b16_m5_solution"], rtol=1e-9, atol=1e-13)


def test_driver_vector(lz, golden):
    """--vector: single-vector Lanczos (test_VectorLanczos, test_lanczos.cu:20-127):
    the reference's output lines and its 10^5-step fdtd_vector check (:111-123)."""
    ritz, _, out = run_driver(lz, "-N", "10", "-m", "10", "--vector")
    al, be = golden["N10_vec_m10_alpha"], golden["N10_vec_m10_beta"]
    ref = lz.ritz_values(10, 1, al, np.concatenate([be, [0.0]]))
    assert np.max(np.abs(ritz - ref)) <= RITZ_TOL
    assert "The solution for vector_lanczos" in out and "Solution for block lanczos" not in out
    assert "Solution from fdtd" in out
    rel = float(out.split("Relative error for block lanczos is")[1].split()[0])
    assert rel < 1e-5, rel  # dt = 1e-5


def test_driver_fdtd(lz, golden):
    """The driver's validation run (methods/fdtd.hpp:33-56) at N = 3: Lanczos vs
    forward Euler, the reference's own convergence plateau (lanczos_plots.m:168-169)."""
    _, sol, out = run_driver(lz, "-N", "3", "-m", "8", "--block", "4", "--fdtd-steps", "200000")
    rel = float(out.split("Relative error for block lanczos is")[1].split()[0])
    assert rel < 2e-8, rel  # CPU oracle at 2e5 steps: 4.57e-9 (forward Euler O(dt))


def test_driver_vector_fp32(lz, orc, golden):
    """--vector --fp32: test_VectorLanczos<float> (test_lanczos.cu:355) on the
    driver's own operator and b, against the oracle's fp32 restatement."""
    ritz, _, _ = run_driver(lz, "-N", "10", "-m", "10", "--vector", "--fp32", "--fdtd-steps", "0")
    from conftest import golden_csr
    A = golden_csr(lz, golden, 10)
    A32 = lz.CsrHost(A.n, A.row_ptr, A.col, A.val.astype(np.float32))
    bv = lz.rand_B(A.n, 1)[:, 0].astype(np.float32)
    _, ao, bo = orc.vector_lanczos(A32, bv, 10, int(golden["lc"]))
    ref = lz.ritz_values(10, 1, ao.astype(np.float64), np.r_[bo, 0].astype(np.float64))
    assert ritz.size == 10
    assert np.max(np.abs(ritz - ref)) <= 1e-5 * np.abs(ref).max()
