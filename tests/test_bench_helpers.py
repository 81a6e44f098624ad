"""bench.py's self-checks on CPU: the parity comparison that gates every bench
line (compare_run: alpha / beta / Ritz of the first steps against the oracle,
the reference's methods/block_lanczos.hpp:104-166 restated), the counter-file
guard (a rocprofv3 summary is used only for the launched instantiation on the
kernel's current source), and the stream-ceiling figure in the roofline
objects.  Nothing here touches a GPU."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _tridiag_run(rng, m, b):
    al = rng.standard_normal((m, b, b))
    al = 0.5 * (al + np.transpose(al, (0, 2, 1)))
    be = rng.standard_normal((m + 1, b, b))
    be = np.einsum("kij,klj->kil", be, be) + b * np.eye(b)  # symmetric positive definite
    q = rng.standard_normal(m * b)
    return al, be, q


def test_compare_run_accepts_equal_and_rejects_perturbed(lz):
    rng = np.random.default_rng(7)
    m, b = 4, 3
    al, be, q = _tridiag_run(rng, m, b)
    ok = bench.compare_run(lz, m, b, (al, be, q), (al, be, q), 1e-9, bench.RITZ_TOL)
    assert ok["ok"] and ok["max_dalpha_rel"] == 0.0 and ok["max_dritz"] == 0.0 and ok["max_dq"] == 0.0
    al2 = al.copy()
    al2[2, 1, 1] += 1e-6  # one alpha entry off by 1e-6: past the 1e-9 relative bar
    bad = bench.compare_run(lz, m, b, (al2, be, q), (al, be, q), 1e-9, bench.RITZ_TOL)
    assert not bad["ok"] and bad["max_dalpha_rel"] > 1e-9
    be2 = be.copy()
    be2[1] *= 1.0 + 1e-7
    assert not bench.compare_run(lz, m, b, (al, be2, q), (al, be, q), 1e-9, bench.RITZ_TOL)["ok"]
    # only the first m steps count: a later alpha (beyond the checked steps) may differ
    al3 = np.concatenate([al, rng.standard_normal((1, b, b))])
    assert bench.compare_run(lz, m, b, (al3, be, q), (al, be, q), 1e-9, bench.RITZ_TOL)["ok"]


def test_pmc_record_guards(tmp_path, monkeypatch):
    csrc = tmp_path / "csrc"
    (tmp_path / "profiles").mkdir()
    csrc.mkdir()
    (csrc / "lz_spmm.hip").write_text("// kernel source v1\n")
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "CSRC", str(csrc))
    kfull = "k_spmm_seg<double,16,48,768,false,0,false,false,false>"
    rec = {"kernel": "k_spmm_seg", "kernel_full": kfull, "source_sha": bench.source_sha("k_spmm_seg"),
           "workload": {"n": 1000, "nnz": 10000, "halfwidth": 64}, "hbm_bytes_per_launch": 12345}
    (tmp_path / "profiles" / "r09_pmc_k_spmm_seg.json").write_text(json.dumps(rec))
    d, src = bench.pmc_record("", "k_spmm_seg", 1000, 10000, 64, kfull)
    assert d and d["hbm_bytes_per_launch"] == 12345 and src.endswith("r09_pmc_k_spmm_seg.json")
    assert bench.pmc_traffic("k_spmm_seg", 1000, 10000, 64, kfull)[0] == 12345
    # another workload, another instantiation: refused
    assert bench.pmc_record("", "k_spmm_seg", 2000, 10000, 64, kfull)[0] is None
    d, why = bench.pmc_record("", "k_spmm_seg", 1000, 10000, 64, kfull.replace("768", "1024"))
    assert d is None and "is not the launched" in why
    # the kernel's source changed since the counters were taken: refused as stale
    (csrc / "lz_spmm.hip").write_text("// kernel source v2\n")
    d, why = bench.pmc_record("", "k_spmm_seg", 1000, 10000, 64, kfull)
    assert d is None and "stale" in why


def test_stream_ceiling():
    s = bench.stream_ceiling(4090.8, "r2w1")
    assert s["mix"] == "r2w1" and s["GBs"] == bench.STREAM_GBS["r2w1"]
    assert abs(s["frac"] - 4090.8 / bench.STREAM_GBS["r2w1"]) < 1e-4
    assert s["source"].startswith("profiles/") and os.path.exists(os.path.join(ROOT, s["source"].split()[0]))
    # every mix at or below the nominal peak the roofline fractions are quoted against
    assert all(0 < v < bench.HBM_PEAK_GBS for v in bench.STREAM_GBS.values())
