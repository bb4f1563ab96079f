"""Host-side issue timeline of the one-rank sharded rehearsal (ON THE GPU BOX):
python3 tools/reh_host_trace.py  -> for one timed run of 2 steps, the host time at which each
partition / exchange / probe call returned (ms from the run's start).  A gap means the host was
blocked inside a call, i.e. the issuing thread, not the GPU, serialised the pipeline."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "chunk-compaction-in-vectorized-execution-simd_amd")]
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import ccj  # noqa: E402
import ccj_dist  # noqa: E402


def main():
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    n_probe = 1 << 30
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        sp = ccj_dist.ShardedProbe(1 << 27, 1, n_probe, 2048, 1, 0, stream=stream, batches=4)
        keys = ccj.gen_uniform_keys(n_probe, 42, 1 << 27, first_row=0, stream=stream)
    torch.cuda.synchronize()
    sp.run(keys, 0, steps=2)
    torch.cuda.synchronize()
    log = []
    t0 = time.perf_counter()
    for name in ("_partition", "_exchange", "_probe"):
        f = getattr(sp, name)

        def wrap(*a, _f=f, _n=name, **k):
            s = time.perf_counter()
            r = _f(*a, **k)
            log.append((_n, a[0] if _n == "_exchange" else a[1],
                        (s - t0) * 1e3, (time.perf_counter() - t0) * 1e3))
            return r
        setattr(sp, name, wrap)
    t0 = time.perf_counter()
    sp.run(keys, 0, steps=2)
    t_issue = (time.perf_counter() - t0) * 1e3
    torch.cuda.synchronize()
    t_all = (time.perf_counter() - t0) * 1e3
    for n, i, s, e in log:
        print(f"{n:11s} {i:3d} call {s:8.2f} -> {e:8.2f} ms ({e - s:6.2f})")
    print(f"issue {t_issue:.1f} ms, run {t_all:.1f} ms")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
