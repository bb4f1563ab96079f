"""Checks that run against the tuning build (libccj_tuning.so, `make tuning`) in child pytests.

  - The rank walk (csrc/ccj_rank.hip) is built into libccj_tuning.so only: the product
    library refuses its index and its flag, and the rank walk's own checks (tests/rank_walk_checks.py:
    the slot-array walk's matches, row order, misses, rows / position mode, segmented counts, runs
    crossing windows) run against the tuning build.
  - The LDS-DMA walks' DPP address moves are checked there against ds_bpermute (dpp_check: a mismatch
    raises CCJ_FLAG_INTERNAL in the probe's status): the partitioned / ordered walk tests of
    tests/test_probe_gpu.py, which require status 0, run on the tuning build too."""
import os
import subprocess
import sys

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import ccj  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TUNING = os.path.join(ROOT, "chunk-compaction-in-vectorized-execution-simd_amd", "libccj_tuning.so")


@pytest.fixture(scope="module", autouse=True)
def _device():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ccj.device_init(0)


def test_product_library_refuses_the_rank_walk():
    table = ccj.Table.reference(ccj.LP, 1 << 20, 1, ccj.LAYOUT_DEVICE)
    with pytest.raises(ccj.CCJError, match="libccj_tuning.so only"):
        table.build_rank_index()
    keys = ccj.gen_uniform_keys(1 << 20, 5, 1 << 20)
    with pytest.raises(ccj.CCJError, match="libccj_tuning.so only"):
        table.probe_partitioned(keys, 2048, rows=True, rank=True, part=table.alloc_partitioned(1 << 20, 2048))
    table.free()


def test_rank_walk_checks_on_the_tuning_build():
    assert os.path.exists(TUNING), "libccj_tuning.so missing: make -C chunk-compaction-in-vectorized-execution-simd_amd"
    env = dict(os.environ, CCJ_LIB_PATH=TUNING)
    p = subprocess.run([sys.executable, "-m", "pytest", os.path.join(ROOT, "tests", "rank_walk_checks.py"), "-q", "-x",
                        "-p", "no:cacheprovider"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-2000:]
    assert " passed" in p.stdout and "failed" not in p.stdout


def test_walk_dpp_address_checks_on_the_tuning_build():
    """probe_walk1 / probe_walk2 with the tuning build's DPP check on (every DMA address each lane
    received equals its partner lane's computed one): the walk tests of test_probe_gpu.py — long runs
    across windows and the table's end, every chunk width, rows / positions / plain modes, the ordered
    path's round-word walk — pass with status 0, i.e. no CCJ_FLAG_INTERNAL."""
    assert os.path.exists(TUNING), "libccj_tuning.so missing: make -C chunk-compaction-in-vectorized-execution-simd_amd"
    env = dict(os.environ, CCJ_LIB_PATH=TUNING)
    sel = ("partitioned_walk_long_runs or partitioned_distinct_keys_every_chunk_width or partitioned_probe_rows_mode "
           "or partitioned_probe_walks or ordered_probe_equals_chunk_probe")
    p = subprocess.run([sys.executable, "-m", "pytest", os.path.join(ROOT, "tests", "test_probe_gpu.py"), "-q", "-x",
                        "-k", sel, "-p", "no:cacheprovider"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=900)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-2000:]
    assert " passed" in p.stdout and "failed" not in p.stdout


def test_every_timing_ablation_runs_clean_on_the_tuning_build():
    """tests/ablation_checks.py: each timing-only ablation bit of the tuning build (CCJ_ABLATE,
    CCJ_OWNER_ABLATE, CCJ_GATHER_ABLATE) once on every path that reads it, small sizes, one child
    process: no fault, only defined status flags, and clean runs afterwards."""
    assert os.path.exists(TUNING), "libccj_tuning.so missing: make -C chunk-compaction-in-vectorized-execution-simd_amd"
    env = dict(os.environ, CCJ_LIB_PATH=TUNING)
    p = subprocess.run([sys.executable, "-m", "pytest", os.path.join(ROOT, "tests", "ablation_checks.py"), "-q", "-x",
                        "-p", "no:cacheprovider"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-2000:]
    assert " passed" in p.stdout and "failed" not in p.stdout
