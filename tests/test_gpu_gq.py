"""The device GQ (engine_dev.h d_gq: glibc-derived thresholds counted around a bare v_log_f32 guess) equals the
reference's int(-10 log10(1 - pb) + 0.5) / 100 cut-off (NucFamGenotypeLikelihood.cpp OutputVCF :1818-1820) for every
pb tested: +-64 ulps around each threshold, the 0.9999999999 cut-off, tiny and 2^20 random values
(tests/native/gq_check.hip, built by __graft_entry__.build())."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "native", "build", "gq_check")


@pytest.mark.gpu
def test_device_gq_matches_glibc():
    assert os.path.exists(EXE), "build gq_check first (__graft_entry__.build())"
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert " 0 mismatches" in r.stdout
