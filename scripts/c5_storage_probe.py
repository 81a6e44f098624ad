"""Experiment: does the STORAGE order of the gathered block matter at C5?

The rows of A (and so the tile order and load balance) stay as generated; only
the columns are relabelled, with X stored in the matching order:
  natural        A, X
  degree_sorted  col' = inv[col], X' = X[perm], perm = rows by descending degree
                 (the hot X rows packed into the first pages)
  random         the same with a random perm (control)
Each row's entries keep their CSR order, so Y is the same sums in the same
order: checked bitwise against the natural run.  (scripts/c5_reorder_probe.py
measured the full symmetric P A P^T, which also moves the hub ROWS together.)
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

lz = ge.load_package()
h = lz.Handle(0)
n, b = 10_000_000, 32
A = lz.gen_powerlaw(n, 10.0, 2.1, 100000, seed=20261015, dtype=np.float32)
deg = np.diff(A.row_ptr)
B = lz.uniform_B(n, b, seed=3, dtype=np.float32)
rng = np.random.default_rng(7)
perms = {"natural": None, "degree_sorted": np.argsort(-deg, kind="stable"), "random": rng.permutation(n)}
res, yref = {}, None
for rnd in range(3):
    for name, perm in perms.items():
        if perm is None:
            AA, XX = A, B
        else:
            inv = np.empty(n, np.int64)
            inv[perm] = np.arange(n)
            AA = lz.CsrHost(n, A.row_ptr, inv[A.col].astype(np.int32), A.val)
            XX = B[perm]
        Ad = lz.CsrDevice.from_host(AA)
        Xd = torch.from_numpy(np.ascontiguousarray(XX)).cuda()
        Y = torch.empty(n, b, dtype=torch.float32, device="cuda")
        h.spmm(Ad, Xd, Y)
        torch.cuda.synchronize()
        h.prof_enable(True)
        for _ in range(10):
            h.spmm(Ad, Xd, Y)
        torch.cuda.synchronize()
        ms, c = h.prof_read(h.PROF_SPMM)
        h.prof_enable(False)
        if yref is None:
            yref = Y.clone()
        same = bool(torch.equal(Y, yref))
        res.setdefault(name, []).append(round(ms / c, 4))
        print(f"round {rnd} {name}: spmm {ms / c:.4f} ms, Y bitwise equal to natural: {same}", flush=True)
        if not same:
            raise RuntimeError(f"{name}: Y differs")
        del Ad, Xd, Y
        torch.cuda.empty_cache()
print(json.dumps({k: {"spmm_ms": v, "median": float(np.median(v))} for k, v in res.items()}))
