"""Run-to-run determinism of single kernels / solves on the b = 32 fp32
operator of test_vranks_b32_f32 (n = 20,011, 10 nnz/row, half width 600):
  spmm      lz_csr_spmm fp32 b = 32 (plain k_spmm_seg), Y compared bitwise
  solve_e   the one-GPU solve in the pass-E form (LZ_C5_B2=0: plain SpMM + E + U)
  solve_b2  the one-GPU solve in the beta^2 form (default)
  python scripts/flake_kernels.py REPS what ..."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import __graft_entry__ as ge  # noqa: E402

lz = ge.load_package()
reps = int(sys.argv[1])
A = lz.gen_banded(20_011, 10.0, 600, seed=30, dtype=np.float32)
B = lz.uniform_B(A.n, 32, seed=31, dtype=np.float32)
h = lz.Handle(0)
Ad = lz.CsrDevice.from_host(A)
Bd = torch.from_numpy(B).cuda()
for what in sys.argv[2:]:
    first, nd = None, 0
    for it in range(reps):
        if what == "spmm":
            Y = torch.full((A.n, 32), float("nan"), dtype=torch.float32, device="cuda")
            h.spmm(Ad, Bd, Y)
            out = Y.cpu().numpy()
        else:
            if what == "solve_e":
                os.environ["LZ_C5_B2"] = "0"
            else:
                os.environ.pop("LZ_C5_B2", None)
            q, al, be = lz.run_block_lanczos(h, Ad, Bd, 2, 15_000)
            out = al.cpu().numpy()
        if first is None:
            first = out.copy()
        elif not np.array_equal(out, first):
            nd += 1
            if nd <= 3:
                diff = np.argwhere(out != first)
                print(f"{what} run {it}: {diff.shape[0]} elements differ, first {diff[:4].tolist()}", flush=True)
    print(f"{what}: {nd}/{reps - 1} runs differ from run 0", flush=True)
