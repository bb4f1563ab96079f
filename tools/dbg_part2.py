import sys
sys.path[:0] = ["/root/repo", "/root/repo/chunk-compaction-in-vectorized-execution-simd_amd"]
import torch, ccj
ccj.device_init(0)
n = 1 << int(sys.argv[1])
t = ccj.Table.reference(ccj.LP, 1 << 26, 1, ccj.LAYOUT_DEVICE)
keys = ccj.gen_uniform_keys(n, 42, 1 << 26)
out = t.probe_partitioned(keys, 2048)
for _ in range(3):
    t.probe_partitioned(keys, 2048, out=out)
for _ in range(3):
    t.probe(keys, 2048, out=out)
torch.cuda.synchronize()
