"""Time the one-workgroup b x b kernels (sqrtm, gram finish) in isolation."""
import json, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge
lz = ge.load_package()
h = lz.Handle(0)
out = {}
for b in (4, 16, 32):
    for cond in (1e2, 1e12):
        torch.manual_seed(0)
        Qm, _ = torch.linalg.qr(torch.randn(b, b, dtype=torch.float64))
        ev = torch.logspace(0, -torch.log10(torch.tensor(cond)).item(), b, dtype=torch.float64)
        G = (Qm * ev) @ Qm.T
        G = 0.5 * (G + G.T)
        Gd = G.cuda()
        be = torch.empty_like(Gd); bi = torch.empty_like(Gd); eg = torch.empty(b, dtype=torch.float64, device="cuda")
        h.sqrtm(Gd, be, bi, eg); torch.cuda.synchronize()
        h.prof_enable(True)
        for _ in range(50):
            h.sqrtm(Gd, be, bi, eg)
        torch.cuda.synchronize()
        ms, cnt = h.prof_read(h.PROF_SMALL)
        h.prof_enable(False)
        err = (be.cpu() @ be.cpu() - G).abs().max().item() / G.abs().max().item()
        eerr = (eg.cpu() - torch.sort(ev).values).abs().max().item()
        out[f"sqrtm_b{b}_cond{cond:g}"] = dict(us=round(ms / cnt * 1e3, 2), rel_err=err, eig_err=eerr)
print(json.dumps(out, indent=1))
