"""CPU stand-in for bench.py's N > 1 step (bench.py --ops-module tests/bench_host_ops.py): the
oracle-backed ops object of tests/test_dist_cpu.py plus the two calls bench_multi makes on its own
(the probe key stream and the work accounting).  Test infrastructure only: it lets
tests/test_bench_launch_cpu.py run bench.py's self-launcher and its N > 1 line with gloo, no GPU.
Set BENCH_OPS_FAIL_RANK=r to make rank r fail (exit-status propagation)."""
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE)]

from test_dist_cpu import HostOps  # noqa: E402


class BenchHostOps(HostOps):
    def probe_keys(self, seed, first_row, n, rng):
        from oracle import oracle as O
        return torch.from_numpy(O.uniform_keys(seed, first_row, first_row + n, rng))

    def probe_cost(self, keys, stream):
        return int(keys.numel()), 0  # (slots examined, matches): a stand-in, S-bar = 1


def make_ops(rank):
    if os.environ.get("BENCH_OPS_FAIL_RANK") == str(rank):
        raise RuntimeError(f"rank {rank}: failing on purpose (BENCH_OPS_FAIL_RANK)")
    return BenchHostOps(subs=8)
