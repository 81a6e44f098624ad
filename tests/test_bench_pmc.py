"""bench.py's counter-file matching (CPU): a committed PMC summary is used only
for the launched instantiation, the current kernel source and the same
workload; a distributed rank may take the per-rank share's summary (nnz within
1 %), and says so."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

KF = "k_wf16<10,4400,2,1,2,1,false,false>"


def _write(tmp_path, nnz, sha):
    prof = tmp_path / "profiles"
    prof.mkdir(exist_ok=True)
    rec = {"kernel": "k_wf16", "kernel_full": KF, "source_sha": sha,
           "workload": {"n": 5_000_000, "nnz": nnz, "halfwidth": 65536},
           "hbm_bytes_per_launch": 17_000_000_000, "hbm_bytes_first_launch": 15_000_000_000}
    (prof / "r99_c4rank_pmc_k_wf16.json").write_text(json.dumps(rec))


def test_pmc_record_exact_and_share(tmp_path, monkeypatch):
    _write(tmp_path, 124_909_886, bench.source_sha("k_wf16"))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    d, src = bench.pmc_record("", "k_wf16", 5_000_000, 124_909_886, 65536, KF)
    assert d and "per-rank share" not in src
    d, src = bench.pmc_record("", "k_wf16", 5_000_000, 125_000_000, 65536, KF)  # single GPU: exact only
    assert d is None
    d, src = bench.pmc_record("", "k_wf16", 5_000_000, 125_000_000, 65536, KF, nnz_tol=0.01)
    assert d and "per-rank share" in src
    d, src = bench.pmc_record("", "k_wf16", 5_000_000, 130_000_000, 65536, KF, nnz_tol=0.01)
    assert d is None


def test_pmc_record_refuses_stale_or_other_kernel(tmp_path, monkeypatch):
    _write(tmp_path, 124_909_886, "0" * 16)
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    d, src = bench.pmc_record("", "k_wf16", 5_000_000, 124_909_886, 65536, KF)
    assert d is None and "stale" in src
    _write(tmp_path, 124_909_886, bench.source_sha("k_wf16"))
    d, src = bench.pmc_record("", "k_wf16", 5_000_000, 124_909_886, 65536, "k_wf16<11,1936,3,1,4,1,true,false>")
    assert d is None and "is not the launched" in src
