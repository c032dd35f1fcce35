"""normalize_unit (csrc/pt_device.h) replaces glm's normalize, v * (1 / sqrt(dot(v, v))), by an
integer formula when dot(v, v) is within NU_ULPS floats of 1.  Check that formula against IEEE
float32 sqrt and division (numpy rounds both correctly) for EVERY such d, and that the window
the device uses lies inside the range where the formula holds."""
import re

import numpy as np

from conftest import PKG

ONE = 0x3F800000


def _formula(k):
    m = -2 * (k >> 1) if k >= 0 else ((((1 - k) >> 1) + 1) >> 1)
    return np.array([ONE + m], np.uint32).view(np.float32)[0]


def _ieee(k):
    d = np.array([ONE + k], np.uint32).view(np.float32)[0]
    with np.errstate(all="ignore"):
        return np.float32(1.0) / np.sqrt(d)


def _device_window():
    src = open(f"{PKG}/csrc/pt_device.h").read()
    return int(re.search(r"constexpr int NU_ULPS = (\d+);", src).group(1))


def test_formula_matches_ieee_over_a_wide_window():
    # it holds for -4096 <= k <= 2897 (beyond, the dropped second-order terms of the expansions
    # reach a rounding boundary); the device uses a far smaller window
    for k in range(-4096, 2898):
        assert _formula(k).view(np.uint32) == _ieee(k).view(np.uint32), k


def test_device_window_is_covered():
    nu = _device_window()
    assert 16 <= nu <= 2048
    for k in range(-nu, nu + 1):
        assert _formula(k) == _ieee(k)
