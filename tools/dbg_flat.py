import os, sys
sys.path[:0] = ["/root/repo", "/root/repo/chunk-compaction-in-vectorized-execution-simd_amd"]
import torch, ccj
ccj.device_init(0)
n = 1 << 30
t = ccj.Table.reference(ccj.LP, 1 << 26, 1, ccj.LAYOUT_DEVICE)
keys = ccj.gen_uniform_keys(n, 42, 1 << 26)
out = t.probe_partitioned(keys, 2048)
torch.cuda.synchronize()
for _ in range(2):
    t.probe_partitioned(keys, 2048, out=out)
torch.cuda.synchronize()
