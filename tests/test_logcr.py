"""The staged Viterbi log (pytorch_hmm_amd/csrc/logcr.h) on every positive normal fp32 input.

The chains take the reference's emission log(obs + 1e-8) (hmm.py:152) with the sum in fp32 and
the log correctly rounded.  tools/logcr_check.cpp compiles the device header for the host (same
fp64 operations, explicit fma) and compares it, input by input, with the correctly rounded
log and with the previous fp64-libm path.
"""
import os
import re
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

# inputs within 2^-60 of a rounding midpoint: one ulp off, as (float)log((double)s) is there too
KNOWN_OFF = {0x3C413D3A, 0x4C5D65A5, 0x65D890D3, 0x6F31A8EC}


def _build(tmp_path):
    exe = str(tmp_path / "logcr_check")
    subprocess.run(["g++", "-O2", "-fopenmp", "-ffp-contract=off", "-o", exe,
                    os.path.join(ROOT, "tools", "logcr_check.cpp"), "-lm"], check=True)
    return exe


def _run(exe, lo, hi):
    out = subprocess.run([exe, hex(lo), hex(hi)], check=True, capture_output=True, text=True).stdout
    bad = {int(m, 16) for m in re.findall(r"^bad (0x[0-9a-f]+)", out, re.M)}
    n_bad, n_old, n_chk = map(int, re.search(r"mismatches (\d+) olddiff (\d+) checked (\d+)", out).groups())
    return bad, n_bad, n_old, n_chk


def test_logcr_every_positive_normal_float(tmp_path):
    exe = _build(tmp_path)
    bad, n_bad, n_old, n_chk = _run(exe, 0x00800000, 0x7F800000)
    assert n_chk == 0x7F000000
    assert n_bad == len(bad) and bad == KNOWN_OFF, sorted(hex(b) for b in bad)
    assert n_old == 1  # s = 0x1.2f1fd6p+3: the double-rounded libm path is the one off


def test_logcr_specials_and_subnormals(tmp_path):
    # +0 and positive subnormals (scaled by 2^24 in the kernel), +inf and the nans, -0 and
    # negative subnormals, -inf and negative nans; the negative normals all give nan as well
    # (the full 2^32 sweep is the same program with no arguments, ~1 min on 8 cores)
    exe = _build(tmp_path)
    for lo, hi in ((0x00000000, 0x00800000), (0x7F800000, 0x80800000), (0xBF800000, 0xBF900000),
                   (0xFF800000, 0x100000000)):
        bad, n_bad, n_old, n_chk = _run(exe, lo, hi)
        assert n_chk == hi - lo and n_bad == 0 and n_old == 0, (hex(lo), sorted(hex(b) for b in bad))


def test_logcr_probability_range_matches_previous_path(tmp_path):
    # the whole OBS_PROB domain of softmax emissions: s = p + 1e-8 in [1e-8, 1 + 1e-8]
    exe = _build(tmp_path)
    bad, n_bad, n_old, _ = _run(exe, 0x322BCC77, 0x3F800001)
    assert bad == {0x3C413D3A}
    assert n_old == 0
