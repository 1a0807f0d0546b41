"""The device libm (sp_libm.h) reproduces the host glibc float libm bit for bit.

Runs tools/libm_exhaustive.cpp (same header, compiled for the host without FP contraction) on a
strided sample of all 2^32 inputs per function (the full sweep's log is tests/golden/
libm_exhaustive_full.txt).  The device build compiles the identical source with explicit fma()
and -ffp-contract=off, so host equality carries over; the GPU parity tests check it end to end."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("libm") / "libm_ex")
    subprocess.run(["g++", "-O2", "-std=c++17", "-mavx2", "-mfma", "-ffp-contract=off", "-fno-builtin", "-pthread",
                    os.path.join(ROOT, "tools", "libm_exhaustive.cpp"), "-o", exe, "-lm"], check=True, timeout=300)
    return exe


@pytest.mark.parametrize("fn", ["expf", "logf", "sinf", "cosf", "sincosf", "erff", "acosf", "atanf", "fmod1", "roundf", "powf", "atan2f"])
def test_libm_matches_glibc(checker, fn):
    out = subprocess.run([checker, fn, "4099", "4"], capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stdout
    assert "mismatches=0" in out.stdout


def test_full_sweep_log():
    log = os.path.join(ROOT, "tests", "golden", "libm_exhaustive_full.txt")
    if not os.path.exists(log):
        pytest.skip("full 2^32 sweep log not recorded yet")
    text = open(log).read()
    for fn in ["expf", "logf", "sinf", "cosf", "sincosf", "erff", "acosf", "atanf", "fmod1", "roundf"]:
        assert f"{fn} checked=4294967296 mismatches=0" in text
