"""Achievable HBM streaming rate on this box (calibration for the roofline):
torch copy (1R+1W) and a 2R+1W add over 1.28 GB blocks (the C3 block size)."""
import json, torch
n = 10_000_000 * 16
x = torch.rand(n, dtype=torch.float64, device="cuda")
y = torch.rand(n, dtype=torch.float64, device="cuda")
z = torch.empty_like(x)
def t(f, reps=20):
    f(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps): f()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps
ms_copy = t(lambda: z.copy_(x))
ms_add = t(lambda: torch.add(x, y, out=z))
ms_sum = t(lambda: x.sum())
print(json.dumps({"copy_TBs": 2 * n * 8 / ms_copy / 1e9, "add_TBs": 3 * n * 8 / ms_add / 1e9,
                  "read_TBs": n * 8 / ms_sum / 1e9}))
