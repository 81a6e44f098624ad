"""The wavefront step's once-per-solve plan (lz_wf.hip wf_plan16, k_wf_deps)
against a numpy restatement of what it must hold: per pass-1 tile t of TR rows the range
[lo, hi] of tiles its own-row columns fall in (t included), the span maxima,
and pass 1's 16-bit columns (column - the start row of the entry's 16-row
strip).  Integer work: bit-exact.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def plan_ref(A, tr, xoff=0):
    n = A.n
    T = -(-n // tr)
    rp = A.row_ptr.astype(np.int64)
    col = A.col.astype(np.int64) - xoff
    row = np.repeat(np.arange(n, dtype=np.int64), np.diff(rp))
    c16 = (col - (row // 16) * 16).astype(np.int64)
    own = (col >= 0) & (col < n)
    tile = row // tr
    lo = np.arange(T, dtype=np.int64)
    hi = np.arange(T, dtype=np.int64)
    np.minimum.at(lo, tile[own], col[own] // tr)
    np.maximum.at(hi, tile[own], col[own] // tr)
    t = np.arange(T)
    spans = [int((t - lo).max()), int((hi - t).max()), int((hi - lo + 1).max())]
    bad = bool(((c16 < -32768) | (c16 > 32767)).any())
    return np.stack([lo, hi], 1), c16, spans, bad


def check(lz, handle, torch, A, xoff=0, nx=None, misalign=False):
    Ad = lz.CsrDevice.from_host(A)
    if misalign:  # a column array at an odd 4-byte offset
        buf = torch.zeros(A.nnz + 1, dtype=torch.int32, device="cuda")
        buf[1:] = Ad.col
        Ad = lz.CsrDevice(Ad.n, Ad.n_cols, Ad.row_ptr, buf[1:], Ad.val)
        assert Ad.col.data_ptr() % 16 != 0
    info, deps, c16 = handle.wf_plan(Ad, nx=nx, xoff=xoff)
    torch.cuda.synchronize()
    assert info["T"] > 0
    d_ref, c_ref, spans, bad = plan_ref(A, info["tr"], xoff)
    assert np.array_equal(deps.cpu().numpy(), d_ref)
    assert info["spans"][:3] == spans
    assert bool(info["spans"][3] & 1) == bad
    if not bad:
        assert info["col16"]
        assert np.array_equal(c16.cpu().numpy().astype(np.int64), c_ref)
    return info


@pytest.mark.parametrize("n,per_row,hw", [(200_003, 10.0, 4096), (100_000, 25.0, 20_000),
                                          (176 * 50, 10.0, 100), (40_017, 6.0, 60_000)])
def test_wf_plan_vs_numpy(lz, handle, torch_cuda, n, per_row, hw):
    A = lz.gen_banded(n, per_row, hw, seed=n + 7)
    info = check(lz, handle, torch_cuda, A)
    assert info["ok"] == (info["spans"][2] <= 1024)


def test_wf_plan_misaligned_columns(lz, handle, torch_cuda):
    A = lz.gen_banded(100_003, 10.0, 4096, seed=3)
    check(lz, handle, torch_cuda, A, misalign=True)


def test_wf_plan_rank_rows(lz, handle, torch_cuda):
    """A rank's rows [xoff, xoff + n) of a larger gather source: columns outside
    them (peers' rows) are left out of the ranges, the 16-bit columns keep
    their strip offsets."""
    n_all, r0, r1 = 300_000, 100_000, 200_000
    A = lz.gen_banded_local(n_all, r0, r1, 10.0, 3000, 5)
    check(lz, handle, torch_cuda, A, xoff=r0, nx=n_all)
