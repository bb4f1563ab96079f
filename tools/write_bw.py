"""Write-only, read-only and copy bandwidth of the GPU's HBM at C5's column sizes (8 x 8 GiB of
int64 columns = the gather's 64 B per match over 2^30 matches): is the C5 gather's 68.7 GB of
column stores bound by the write rate?  torch kernels only (fill_, sum, copy_), timed with events."""
import torch

def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = []
    for _ in range(reps):
        a.record(); fn(); b.record(); b.synchronize()
        out.append(a.elapsed_time(b))
    return min(out)

n = 1 << 30  # int64 per column: 8 GiB
cols = [torch.empty(n, dtype=torch.int64, device="cuda") for _ in range(8)]
ms = timed(lambda: [c.fill_(7) for c in cols])
print(f"fill 8 x 8 GiB: {ms:.2f} ms, {8 * n * 8 / ms / 1e6:.0f} GB/s")
big = torch.empty(8 * n, dtype=torch.int64, device="cuda")
ms = timed(lambda: big.fill_(3))
print(f"fill 64 GiB one buffer: {ms:.2f} ms, {8 * n * 8 / ms / 1e6:.0f} GB/s")
del big
ms = timed(lambda: [c.sum() for c in cols])
print(f"read (sum) 8 x 8 GiB: {ms:.2f} ms, {8 * n * 8 / ms / 1e6:.0f} GB/s")
half = cols[:4]
dst = cols[4:]
ms = timed(lambda: [d.copy_(s) for d, s in zip(dst, half)])
print(f"copy 4 x 8 GiB: {ms:.2f} ms, {2 * 4 * n * 8 / ms / 1e6:.0f} GB/s (read + write)")
