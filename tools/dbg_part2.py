import sys
sys.path[:0] = ["/root/repo", "/root/repo/chunk-compaction-in-vectorized-execution-simd_amd"]
import torch, ccj
from oracle import oracle as O
ccj.device_init(0)
n = 1 << int(sys.argv[1])
t = ccj.Table.reference(ccj.LP, 1 << 26, 1, ccj.LAYOUT_DEVICE)
keys = ccj.gen_uniform_keys(n, 42, 1 << 26)
out = t.probe_partitioned(keys, 2048)
for _ in range(3):
    t.probe_partitioned(keys, 2048, out=out)
torch.cuda.synchronize()
m, l2 = ccj.result_checksum(out, 2048, row_map=out["row_map"][:n].to(torch.int64))
print("partitioned", m, l2 == O.count_uniform(42, 0, n, 1 << 26, 1 << 26, 1, threads=16)[1], flush=True)
out2 = t.probe(keys, 2048)
for _ in range(3):
    t.probe(keys, 2048, out=out2)
torch.cuda.synchronize()
