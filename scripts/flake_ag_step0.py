"""Diagnose run-to-run differences of the b = 32 fp32 block Lanczos (config
C5's block, the distributed all-gather form and the one-GPU solve): solves
repeated in one process; alpha compared with the first run's, and after each
all-gather run every rank's X_full peer slot compared with the peer's B.

  python scripts/flake_ag_step0.py REPS M NRANKS   (NRANKS 0: the one-GPU solve)
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import __graft_entry__ as ge  # noqa: E402

lz = ge.load_package()
reps, m_steps, N = (int(x) for x in sys.argv[1:4])
A = lz.gen_banded(20_011, 10.0, 600, seed=30, dtype=np.float32)
B = lz.uniform_B(A.n, 32, seed=31, dtype=np.float32)
b, lc = 32, 15_000


def one_gpu():
    h = lz.Handle(0)
    Ad = lz.CsrDevice.from_host(A)
    q, al, be = lz.run_block_lanczos(h, Ad, torch.from_numpy(B).cuda(), m_steps, lc)
    assert h.device_error() == 0
    out = al.cpu().numpy(), be.cpu().numpy()
    h.close()
    return out


def dist():
    bounds = lz.partition_rows(A, N)
    n_pad = int(np.max(np.diff(bounds)))
    lc_rank = int(np.searchsorted(bounds, lc, side="right") - 1)

    def rank_fn(r, h):
        kw = dict(dtype=torch.float32, device="cuda")
        r0, r1 = int(bounds[r]), int(bounds[r + 1])
        nl = r1 - r0
        k0, k1 = int(A.row_ptr[r0]), int(A.row_ptr[r1])
        rp = (A.row_ptr[r0:r1 + 1] - A.row_ptr[r0]).astype(np.int64)
        pcol = lz.remap_cols_padded(A.col[k0:k1], bounds, n_pad)
        Ad = lz.CsrDevice.from_host(lz.CsrHost(nl, rp, pcol, A.val[k0:k1].copy()), n_cols=n_pad * N)
        Bp = torch.zeros(n_pad, b, **kw)
        Bp[:nl] = torch.from_numpy(np.ascontiguousarray(B[r0:r1])).cuda()
        W = torch.zeros(n_pad, b, **kw)
        X = torch.zeros(n_pad * N, b, **kw)
        q, al, be = (torch.zeros(m_steps * b, **kw), torch.zeros(m_steps, b, b, **kw),
                     torch.zeros(m_steps + 1, b, b, **kw))
        h.block_lanczos_dist(Ad, n_pad, n_pad * N, Bp, m_steps, lc - int(bounds[lc_rank]), lc_rank, q, al, be,
                             None, W, X)
        assert h.device_error() == 0
        return al.cpu().numpy(), be.cpu().numpy()

    res = lz.run_virtual_ranks(N, rank_fn)
    return res[0]


first, nd, nan = None, 0, 0
for it in range(reps):
    al, be = one_gpu() if N == 0 else dist()
    nan += int(not np.isfinite(al).all())
    if first is None:
        first = al.copy()
    elif not np.array_equal(al, first):
        nd += 1
        steps = [j for j in range(m_steps) if not np.array_equal(al[j], first[j])]
        print(f"run {it}: alpha differs from run 0 at steps {steps}: max rel "
              f"{np.max(np.abs(al - first)) / np.max(np.abs(first)):.2e}", flush=True)
print(f"N={N} m={m_steps} LZ_POISON={os.environ.get('LZ_POISON')}: {nd}/{reps - 1} runs differ from run 0, "
      f"{nan} with non-finite alpha", flush=True)
