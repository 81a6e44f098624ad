"""Multi-GPU decomposition on CPU: world_size 2-4 over gloo.

lz_block_lanczos_dist (csrc/lz_api.hip) runs, per rank: all-gather of the
residual slab into a padded full block, the fused pass on the rank's rows with
columns renumbered into the padded space, and two b x b all-reduces (alpha
partial, W'^T W' partial) with sqrtm redundant on every rank.  This test runs
that exact decomposition with torch.distributed (gloo) between two CPU
processes -- nnz-balanced row partition (lzh_partition_rows), the per-rank
generator (lzh_gen_banded_local), the padded column remap
(lzh_remap_cols_padded), the oracle's CSR SpMM on local rows -- and checks it
against the single-process oracle on the global operator (reference op order,
methods/block_lanczos.hpp:104-166).  The RCCL path itself runs only in the
multi-GPU bench.
"""
import os
import socket

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, b, m, hw, seed):
    import sys

    import torch
    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    import __graft_entry__ as ge

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lz, orc = ge.load_package(), ge.load_oracle()
        A = lz.gen_banded(n, 10.0, hw, seed)
        bounds = lz.partition_rows(A, world)
        r0, r1 = int(bounds[rank]), int(bounds[rank + 1])
        nl = r1 - r0
        # the per-rank generator reproduces the global operator's rows
        Al = lz.gen_banded_local(n, r0, r1, 10.0, hw, seed)
        rp = np.asarray(A.row_ptr)
        assert np.array_equal(Al.row_ptr, rp[r0:r1 + 1] - rp[r0])
        assert np.array_equal(Al.col, A.col[rp[r0]:rp[r1]])
        assert np.array_equal(Al.val, A.val[rp[r0]:rp[r1]])
        n_pad = int(np.diff(bounds).max())
        Ap = lz.CsrHost(nl, Al.row_ptr, lz.remap_cols_padded(Al.col, bounds, n_pad), Al.val)

        def allgather_rows(Wl):
            pad = np.zeros((n_pad, b))
            pad[:nl] = Wl
            parts = [torch.empty(n_pad, b, dtype=torch.float64) for _ in range(world)]
            dist.all_gather(parts, torch.from_numpy(pad))
            return torch.cat(parts).numpy()

        def allreduce(M):
            t = torch.from_numpy(np.ascontiguousarray(M))
            dist.all_reduce(t)
            return t.numpy()

        Bg = lz.uniform_B(n, b, seed=seed + 1)
        Bl = Bg[r0:r1]
        beta0, binv = orc.sqrtm_pair(allreduce(Bl.T @ Bl))
        X = allgather_rows(Bl)
        alpha = np.zeros((m, b, b))
        beta = np.zeros((m + 1, b, b))
        beta[0] = beta0
        Q = np.zeros((nl, b))
        for j in range(m):
            Wl = X[rank * n_pad: rank * n_pad + nl]
            Y = orc.csr_spmm(Ap, X)
            Qn = Wl @ binv
            Wn = Y @ binv - (Q @ beta[j] if j else 0.0)
            M = allreduce(Qn.T @ Wn)
            alpha[j] = 0.5 * (M + M.T)
            Wn = Wn - Qn @ alpha[j]
            Q = Qn
            if j + 1 < m:
                beta[j + 1], binv = orc.sqrtm_pair(allreduce(Wn.T @ Wn))
                X = allgather_rows(Wn)
        _, ao, bo = orc.block_lanczos(A, Bg, m, 0)
        scale = max(1.0, np.abs(ao).max(), np.abs(bo[:m]).max())
        assert np.max(np.abs(alpha - ao)) <= 1e-9 * scale
        assert np.max(np.abs(beta[:m] - bo[:m])) <= 1e-9 * scale
        r = lz.ritz_values(m, b, alpha, beta)
        ro = lz.ritz_values(m, b, ao, bo)
        assert np.max(np.abs(r - ro)) <= 1e-10
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,b,hw", [(2, 4, 300), (2, 16, 300), (4, 16, 900), (8, 16, 700)])
def test_row_partitioned_block_lanczos_gloo(world, b, hw):
    """All-gather form at 2 and 4 ranks (4 ranks: uneven nnz-balanced slabs,
    every slab padded, halos reaching past the neighbouring rank)."""
    import torch.multiprocessing as mp

    mp.spawn(_worker, args=(world, _free_port(), 3001, b, 6, hw, 77), nprocs=world, join=True)


def _halo_worker(rank, world, port, n, b, m, hw, seed):
    """lz_block_lanczos_halo's decomposition (csrc/lz_api.hip block_lanczos_halo16):
    halo plan (lzh_halo_plan), the count / request-list exchange of lz_halo_init,
    owner-side packing by send list, point-to-point row exchange into the halo
    runs, the fused step on compact columns -- over gloo between CPU processes."""
    import sys

    import torch
    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    import __graft_entry__ as ge

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lz, orc = ge.load_package(), ge.load_oracle()
        bounds = np.array([n * p // world for p in range(world + 1)], np.int64)
        r0, r1 = int(bounds[rank]), int(bounds[rank + 1])
        nl = r1 - r0
        Al = lz.gen_banded_local(n, r0, r1, 10.0, hw, seed)
        ccol, rcnt, hrows = lz.halo_plan(Al.col, bounds, rank)
        nh = hrows.size
        assert rcnt[rank] == 0 and rcnt.sum() == nh
        assert np.all(np.diff(hrows) > 0)
        # the compact numbering addresses the same global rows
        glob = np.concatenate([np.arange(r0, r1), hrows])
        assert np.array_equal(glob[ccol], Al.col)
        roff = np.concatenate([[0], np.cumsum(rcnt)])
        # lz_halo_init: request lists travel to their owners
        reqs = [None] * world
        dist.all_gather_object(reqs, [hrows[roff[p]:roff[p + 1]].tolist() for p in range(world)])
        send = [np.asarray(reqs[p][rank], np.int64) - r0 for p in range(world)]
        for p in range(world):
            assert send[p].size == 0 or (send[p].min() >= 0 and send[p].max() < nl)
        Ac = lz.CsrHost(nl, Al.row_ptr, ccol, Al.val)

        def exchange(Xl):
            """rows [nl, nl+nh) from their owners (ncclSend/ncclRecv group)"""
            X = np.zeros((nl + nh, b))
            X[:nl] = Xl
            ops, bufs = [], {}
            for p in range(world):
                if p == rank:
                    continue
                if send[p].size:
                    ops.append(dist.isend(torch.from_numpy(np.ascontiguousarray(Xl[send[p]])), p))
                if rcnt[p]:
                    bufs[p] = torch.empty(int(rcnt[p]), b, dtype=torch.float64)
                    ops.append(dist.irecv(bufs[p], p))
            for o in ops:
                o.wait()
            for p, t in bufs.items():
                X[nl + roff[p]: nl + roff[p + 1]] = t.numpy()
            return X

        def allreduce(M):
            t = torch.from_numpy(np.ascontiguousarray(M))
            dist.all_reduce(t)
            return t.numpy()

        Bg = lz.uniform_B(n, b, seed=seed + 1)
        Bl = Bg[r0:r1]
        beta0, binv = orc.sqrtm_pair(allreduce(Bl.T @ Bl))
        X = exchange(Bl)
        alpha = np.zeros((m, b, b))
        beta = np.zeros((m + 1, b, b))
        beta[0] = beta0
        Q = np.zeros((nl, b))
        for j in range(m):
            Y = orc.csr_spmm(Ac, X)
            Qn = X[:nl] @ binv
            Wn = Y @ binv - (Q @ beta[j] if j else 0.0)
            M = allreduce(Qn.T @ Wn)
            alpha[j] = 0.5 * (M + M.T)
            Wn = Wn - Qn @ alpha[j]
            Q = Qn
            if j + 1 < m:
                beta[j + 1], binv = orc.sqrtm_pair(allreduce(Wn.T @ Wn))
                X = exchange(Wn)
        A = lz.gen_banded(n, 10.0, hw, seed)
        _, ao, bo = orc.block_lanczos(A, Bg, m, 0)
        scale = max(1.0, np.abs(ao).max(), np.abs(bo[:m]).max())
        assert np.max(np.abs(alpha - ao)) <= 1e-9 * scale
        assert np.max(np.abs(beta[:m] - bo[:m])) <= 1e-9 * scale
        r = lz.ritz_values(m, b, alpha, beta)
        ro = lz.ritz_values(m, b, ao, bo)
        assert np.max(np.abs(r - ro)) <= 1e-10
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,hw", [(2, 300), (3, 5000), (8, 700)])
def test_halo_partitioned_block_lanczos_gloo(world, hw):
    """hw=5000 > rows per rank: every rank's halo spans both neighbours and beyond."""
    import torch.multiprocessing as mp

    mp.spawn(_halo_worker, args=(world, _free_port(), 3001, 16, 6, hw, 77), nprocs=world, join=True)


def test_halo_plan_edges():
    import sys

    sys.path.insert(0, ROOT)
    import __graft_entry__ as ge

    lz = ge.load_package()
    bounds = np.array([0, 4, 8, 12], np.int64)
    col = np.array([5, 0, 11, 9, 5, 3, 7, 11], np.int32)  # rank 1 owns rows 4..7
    cc, cnt, rows = lz.halo_plan(col, bounds, 1)
    assert rows.tolist() == [0, 3, 9, 11]
    assert cnt.tolist() == [2, 0, 2]
    assert cc.tolist() == [1, 4, 7, 6, 1, 5, 3, 7]
    cc, cnt, rows = lz.halo_plan(np.zeros(0, np.int32), bounds, 0)  # nnz = 0
    assert rows.size == 0 and cnt.tolist() == [0, 0, 0] and cc.size == 0
    with pytest.raises(lz.LanczosError):
        lz.halo_plan(np.array([12], np.int32), bounds, 0)  # column past the last row
