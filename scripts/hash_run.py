"""Bitwise A/B of two library builds: a short fused C3-shaped run (n = 2M,
m = 8) and a hash of its alpha, beta and q.  Run once per build, e.g.
  LZ_HIP_LIB=.../lib/head/liblz_hip.so python scripts/hash_run.py; python scripts/hash_run.py"""
import hashlib, os, sys
import torch
sys.path.insert(0, os.getcwd())
import __graft_entry__ as ge
lz = ge.load_package(); h = lz.Handle(0)
n, b, m = 2_000_000, 16, 8
A = lz.gen_banded(n, 10.0, 4096, 20261015); Ad = lz.CsrDevice.from_host(A)
Bd = torch.from_numpy(lz.uniform_B(n, b, 20261015)).cuda()
kw = dict(dtype=torch.float64, device="cuda")
q = torch.zeros(m * b, **kw); al = torch.zeros(m, b, b, **kw); be = torch.zeros(m + 1, b, b, **kw)
Q0, Q1, W = (torch.zeros(n, b, **kw) for _ in range(3))
h.block_lanczos_blas(Ad, Bd, m, 84, q, al, be, Q0, Q1, W); torch.cuda.synchronize()
print("hash", hashlib.sha256(al.cpu().numpy().tobytes() + be.cpu().numpy().tobytes() + q.cpu().numpy().tobytes()).hexdigest()[:16])
