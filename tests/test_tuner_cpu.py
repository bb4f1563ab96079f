"""The compaction-threshold tuner (host/ccj_tuner.h: the UCB-tuned bandit of
negative_feedback.hpp:20-260) on synthetic rewards, compiled with the host compiler: it settles on
the best threshold, and restarts its exploration when the rewards shift (the :66-82 detector)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "chunk-compaction-in-vectorized-execution-simd_amd", "host")


@pytest.fixture(scope="module")
def selftest(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("tuner") / "tuner_selftest")
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-I", HOST, "-o", exe,
                    os.path.join(HOST, "tuner_selftest.cpp")], check=True)
    out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout
    return {t[0]: ([int(x) for x in t[1:-2]], int(t[-1])) for t in (l.split() for l in out.splitlines())}


def test_tuner_settles_on_best_threshold(selftest):
    sel, restarts = selftest["stationary"]
    assert len(sel) == 5  # thresholds {1, 32, 64, 128, 256} at chunk 256 (arms >= 256 collapse)
    assert sel.index(max(sel)) == 2 and sel[2] > 0.8 * sum(sel)
    assert restarts == 0


def test_tuner_restarts_after_shift(selftest):
    sel, restarts = selftest["shift"]
    assert restarts >= 1
    assert sel.index(max(sel)) == 4 and sel[4] > 0.6 * sum(sel)
