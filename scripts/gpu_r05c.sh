#!/bin/bash
# Round 5: isolate the b = 32 fp32 distributed failure (Newton-Schulz sqrtm on / off).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -v -k "newton_schulz" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/ns.log 2>&1; echo "ns tests rc=$?"; grep -E "PASS|FAIL" $O/ns.log | tail -30
for ns in 0 1; do
LZ_SQRTM_NS=$ns timeout -k 10 300 python -u -m pytest tests/test_gpu_vranks.py tests/test_gpu_lanczos.py -m gpu -v -k "b32 or f32" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/b32_ns$ns.log 2>&1; echo "b32 ns=$ns rc=$?"; grep -E "PASS|FAIL" $O/b32_ns$ns.log | tail -30
done
python - <<'PY'
import os, sys, time, numpy as np, torch
sys.path.insert(0, os.getcwd())
import __graft_entry__ as ge
lz = ge.load_package(); orc = ge.load_oracle()
h = lz.Handle(0)
rng = np.random.default_rng(1)
for cond in (1e1, 1e3, 1e5):
    Q, _ = np.linalg.qr(rng.standard_normal((32, 32)))
    ev = np.power(cond, -np.arange(32) / 31)
    G = (Q * ev) @ Q.T; G = 0.5 * (G + G.T)
    s, si = orc.sqrtm_pair(G)
    for ns in ("1", "0"):
        os.environ["LZ_SQRTM_NS"] = ns
        b = torch.empty(32, 32, dtype=torch.float64, device="cuda"); bi = torch.empty_like(b)
        Gd = torch.from_numpy(G).cuda()
        h.sqrtm(Gd, b, bi); torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(20): h.sqrtm(Gd, b, bi)
        torch.cuda.synchronize(); us = (time.perf_counter() - t) / 20 * 1e6
        print(f"cond {cond:.0e} ns={ns} {us:.1f} us  dbeta {np.abs(b.cpu().numpy()-s).max()/np.abs(s).max():.2e}  dbinv {np.abs(bi.cpu().numpy()-si).max()/np.abs(si).max():.2e}")
PY
