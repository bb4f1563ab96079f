"""bench.py end to end at small sizes, one process per workload: the JSON line of the driver's
contract for every workload and path (C2 partitioned with the reference-order paths beside it, and
the tuning build's rank-walk A/B, C2 ordered, C3 with compaction, C5 with payload columns, the main.cpp pipeline),
with the bench's own full-size-style parity checks green.  Catches a broken bench path before the
driver's round-end run does."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--steps", "2", "--warmup", "1", "--no-cpu", "--n-build", str(1 << 21), "--n-probe", str(1 << 24)]


def run_bench(*extra):
    p = subprocess.run([sys.executable, "bench.py", *SMALL, *extra], cwd=ROOT, capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["value"] > 0 and line["n_gpus"] == 1 and line["higher_is_better"]
    assert "roofline" in line and line["roofline"]["frac"] > 0
    return line


def test_bench_c2_with_other_paths():
    line = run_bench("--n-build-per-gpu", str(1 << 21))
    par = line["parity"]
    assert par["status_flags"] == 0 and par["l1_ok"] and par["l2_ok"]
    paths = {o["path"]: o for o in line["other_paths"]}
    assert set(paths) == {"ordered", "chunk"}
    for o in paths.values():
        assert o["check"]["status_flags"] == 0 and o["check"]["l1_ok"] and o["check"]["l2_ok"]
    assert paths["ordered"]["check"]["equals_chunk_path_l3"]
    # BASELINE configs[2] and [4] in the same line (the driver's default run measures them too)
    ow = {o["workload"][:2]: o for o in line["other_workloads"]}
    assert set(ow) == {"C3", "C5"}, line["other_workloads"]
    for o in ow.values():
        assert o["value"] > 0 and o["roofline"]["frac"] > 0
        assert o["parity"]["status_flags"] == 0 and o["parity"]["l1_ok"] and o["parity"]["l2_ok"]
    assert ow["C3"]["parity"]["compaction_keeps_all"] and ow["C3"]["compaction_ms"] > 0
    assert ow["C5"]["parity"]["payload_cols_ok"]
    # C3's frac on SURVEY §8(d)'s bytes over probe + compaction; round 5's figure kept beside it
    r3 = ow["C3"]["roofline"]
    assert r3["frac_csr"] > 0 and r3["kernel_ms"] == pytest.approx(r3["probe_kernel_ms"] + r3["compaction_kernel_ms"])
    assert r3["alg_probe_bytes_per_tuple"] == pytest.approx(8 + 4 + 8 * r3["chain_keys_per_tuple"] + 12 * r3["m_bar"])
    # the gather kernel that actually ran, and no traffic pasted from a profile of another shape / build
    assert ow["C5"]["roofline"]["gather_kernel_run"].startswith("gather_payload_cols_sub<8>")  # slab order
    for r in (line["roofline"], r3, ow["C5"]["roofline"]):
        assert r["traffic"] is None or r["traffic_stale"] is False
    # the multi-GPU protocol at N = 1 on the C4 per-GPU shape: the N = 1 point of the curve
    sr = line["scaling_reference"]
    assert sr["ms_per_step"] > 0 and sr["l1_ok"] and sr["l2_ok"], sr
    assert sr["config"]["n_build_total"] == 1 << 21 and sr["config"]["n_probe_per_gpu"] == 1 << 24


def test_bench_c2_tuning_build_with_rank_ab():
    """--lib tuning: the same line, with the rank walk (tuning build only) timed beside the headline."""
    line = run_bench("--lib", "tuning", "--no-other-workloads", "--no-scaling-reference")
    par = line["parity"]
    assert par["status_flags"] == 0 and par["l1_ok"] and par["l2_ok"]
    paths = {o["path"]: o for o in line["other_paths"]}
    assert set(paths) == {"ordered", "chunk", "rank"}
    for o in paths.values():
        assert o["check"]["status_flags"] == 0 and o["check"]["l1_ok"] and o["check"]["l2_ok"]
    assert paths["ordered"]["check"]["equals_chunk_path_l3"]


def test_bench_c2_ordered_headline():
    line = run_bench("--path", "ordered", "--no-other", "--no-other-workloads", "--no-scaling-reference")
    assert line["path"] == "ordered" and line["parity"]["l1_ok"] and line["parity"]["l2_ok"]


@pytest.mark.parametrize("path", ["partitioned", "ordered", "chunk"])
def test_bench_c3(path):
    """C3 on every path; the ordered and chunk paths compact the reference's real Next results."""
    line = run_bench("--workload", "c3", "--path", path)
    par = line["parity"]
    assert par["status_flags"] == 0 and par["l1_ok"] and par["l2_ok"] and par["compaction_keeps_all"]
    assert line["path"] == path


def test_bench_c3_reference_cpu_baseline():
    """C3's cpu_baseline: the reference's own chaining loop (oracle/_ref/ref_driver, compiled from its
    sources) on a sample of the same stream, its match count checked against the oracle's."""
    if not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "ref_driver")):
        pytest.skip("oracle/_ref/ref_driver not built")
    p = subprocess.run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--n-build", str(1 << 21),
                        "--n-probe", str(1 << 24), "--workload", "c3", "--cpu-sample", str(1 << 22)], cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    cpu = json.loads(p.stdout.strip().splitlines()[-1])["cpu_baseline"]
    assert cpu is not None and cpu["kind"] == "reference" and cpu["matches_ok"] and cpu["value"] > 0, cpu


def test_bench_c5():
    line = run_bench("--workload", "c5")
    par = line["parity"]
    assert par["status_flags"] == 0 and par["l1_ok"] and par["l2_ok"] and par["payload_cols_ok"]


def test_bench_pipeline():
    p = subprocess.run([sys.executable, "bench.py", "--workload", "pipeline", "--steps", "2", "--warmup", "1",
                        "--no-cpu", "--pipe-lhs", "2000000", "--pipe-rhs", "200000"], cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["value"] > 0
