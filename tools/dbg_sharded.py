"""Bisect the sharded-probe verification at growing sizes (world 1 process group)."""
import os
import sys
sys.path[:0] = ["/root/repo", "/root/repo/chunk-compaction-in-vectorized-execution-simd_amd"]
import torch
import torch.distributed as dist
import ccj
import ccj_dist
from oracle import oracle as O

ccj.device_init(0)
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29555")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
for lg in (22, 26, 28):
    n = 1 << lg
    keys = ccj.gen_uniform_keys(n, 42, 1 << 26)
    fp = ccj.FixedOwnerPartitioner(n, 1, n + 4096)
    ok = torch.zeros(n + 4096, dtype=torch.int64, device="cuda")
    orow = torch.zeros(n + 4096, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    fp(keys, 5, ok, orow, cnt, st)
    torch.cuda.synchronize()
    print("partition", lg, int(cnt.item()), int(st.item()), bool((ok[:n] == keys).all()),
          bool((orow[:n].to(torch.int64) == torch.arange(n, device="cuda") + 5).all()), flush=True)
for lg, b in ((22, 1), (26, 1), (26, 4), (28, 1), (28, 4), (30, 4)):
    n = 1 << lg
    sp = ccj_dist.ShardedProbe(1 << 26, 1, n, 2048, 1, 0, batches=b)
    keys = ccj.gen_uniform_keys(n, 42, 1 << 26)
    got = sp.step(keys, 0, verify=True)
    want = O.count_uniform(42, 0, n, 1 << 26, 1 << 26, 1)
    out = sp.table.probe(keys, 2048, rounds=False)
    c2 = ccj.result_checksum(out, 2048)
    print("sharded", lg, b, got == want, got, want, c2, flush=True)
    del sp, keys, out
    torch.cuda.empty_cache()
dist.destroy_process_group()
