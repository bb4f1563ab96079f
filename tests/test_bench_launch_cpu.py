"""bench.py --gpus N without an outside launcher starts its own N ranks (torch.distributed.run as a
child process) and prints rank 0's line; here on CPU with gloo and an oracle-backed ops object
(tests/bench_host_ops.py) instead of the HIP kernels: exactly one JSON line on stdout, the N > 1
line's diagnostic fields, exact L1/L2, and a failing rank's exit status propagated."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--ops-module", os.path.join(ROOT, "tests", "bench_host_ops.py"), "--n-build-per-gpu", "4096",
        "--n-probe", "12288", "--chunk", "256", "--steps", "2", "--warmup", "1", "--batches", "3", "--group", "2",
        "--no-cpu", "--no-verify"]


def run_bench(world, extra_env=None, extra_args=()):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(extra_env or {})
    env["OMP_NUM_THREADS"] = "1"
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world)] + ARGS +
                          list(extra_args), capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)


@pytest.mark.parametrize("world,scaling", [(2, "weak"), (2, "strong"), (4, "strong")])
def test_self_launch_one_json_line(world, scaling):
    """weak: 12288 probe keys per rank; strong: 12288 in total (12288 / N per rank)."""
    from oracle import oracle as O
    p = run_bench(world, extra_args=["--scaling", scaling])
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["steps"] == 2 and d["scaling"] == scaling
    for k in ("partition_ms", "exchange_ms", "local_probe_ms", "xgmi_bytes_per_step", "xgmi_useful_bytes_per_step"):
        assert k in d, k
    assert d["parity"]["exact_size_fallback_steps"] == 0
    n_build, n_probe = 4096 * world, 12288 if scaling == "weak" else 12288 // world
    assert d["config"]["n_probe_per_gpu"] == n_probe
    want = O.count_uniform(42, 0, world * n_probe, n_build, n_build, 1)
    assert (d["parity"]["matches"], int(d["parity"]["l2"], 16)) == want
    assert d["config"]["batches"] == 3 and d["config"]["group"] == 2


def test_self_launch_failing_rank_propagates():
    p = run_bench(2, {"BENCH_OPS_FAIL_RANK": "1"})
    assert p.returncode != 0
    assert not [ln for ln in p.stdout.splitlines() if ln.strip().startswith("{")]
