"""rt_libm.h / rt_srgb_lut.h (the device's glibc-exact logf, pow(x, 5) and sRGB decode) pinned
exhaustively against this host's glibc: every float in (0, 1] for logf (the polar normal
sampler's domain) and every float in [-1, 1] for pow5 (Schlick Fresnel), see
tools/libm_check.cpp."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tools", "libm_check.cpp")


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("libm") / "libm_check")
    subprocess.run(["g++", "-O2", "-mfma", "-ffp-contract=off", "-fopenmp", "-std=c++17", SRC, "-o", exe], check=True)
    return exe


@pytest.mark.slow
def test_logf_and_pow5_exhaustive(checker):
    r = subprocess.run([checker, "check"], capture_output=True, text=True, timeout=600)
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["logf_checked"] == 0x3F800000
    assert res["pow5_checked"] == 2 * (0x3F800000 + 1)
    assert res["logf_mismatch"] == 0 and res["pow5_mismatch"] == 0
    assert r.returncode == 0


def test_srgb_lut_is_glibc_powf(checker):
    r = subprocess.run([checker, "lut"], capture_output=True, text=True, check=True)
    committed = open(os.path.join(ROOT, "raytracing-hw_amd", "csrc", "rt_srgb_lut.h")).read()
    assert r.stdout == committed


@pytest.mark.slow
def test_gamma_quantizer_thresholds(checker):
    """rt_quant_lut.h: the 8-bit gamma step's thresholds from glibc powf (the generator
    also checks the quantizer is monotonic over every float in [0, 1])."""
    r = subprocess.run([checker, "quant"], capture_output=True, text=True, check=True, timeout=600)
    committed = open(os.path.join(ROOT, "raytracing-hw_amd", "csrc", "rt_quant_lut.h")).read()
    assert r.stdout == committed
