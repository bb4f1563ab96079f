import sys, time
sys.path[:0] = ["/root/repo", "/root/repo/chunk-compaction-in-vectorized-execution-simd_amd"]
import torch, ccj
from oracle import oracle as O
ccj.device_init(0)
for lg in [24, 27, 28, 29, 30]:
    n = 1 << lg
    t = ccj.Table.reference(ccj.LP, 1 << 26, 1, ccj.LAYOUT_DEVICE)
    keys = ccj.gen_uniform_keys(n, 42, 1 << 26)
    out = t.probe_partitioned(keys, 2048)
    torch.cuda.synchronize()
    cnt = int(out["count"].to(torch.int64).sum().item())
    rm = out["row_map"][:n]
    print(lg, "status", int(out["status"].item()), "matches", cnt, "rowmap min/max", int(rm.min()), int(rm.max()), flush=True)
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record(); t.probe_partitioned(keys, 2048, out=out); e.record(); torch.cuda.synchronize()
    print("  ms", s.elapsed_time(e), flush=True)
    del out, keys, t
    torch.cuda.empty_cache()
