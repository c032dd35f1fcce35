"""The shared float helpers behind the bit-exact parity (CPU, no GPU):

* include/pt/pt_libm.h's float sincos for |x| < 8 (round 3): accuracy against sin / cos in double
  on a stride of every float of (-8, 8) (the exhaustive pass, max 1.49 / 1.55 ulp, is in the
  header's comment; this keeps a 1/61 sample of it);
* pt_device.h's div_by_pi: identical bits to IEEE x / PI for 0 and every float of [2^-30, 1]
  (tools/check_div_by_pi.c, exhaustive over that range).
"""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SINCOS_CHECK = r'''
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include "pt/pt_libm.h"
int main(void) {
    double maxs = 0, maxc = 0;
    for (uint32_t b = 0; b < 0x41000000u; b += 61) {
        for (int sg = 0; sg < 2; ++sg) {
            uint32_t bb = b | (sg ? 0x80000000u : 0u);
            float x; memcpy(&x, &bb, 4);
            float s, c; pt_sincosf(x, &s, &c);
            double rs = sin((double)x), rc = cos((double)x);
            float fs = fabsf((float)rs), fc = fabsf((float)rc);
            double us = nextafterf(fs, INFINITY) - fs, uc = nextafterf(fc, INFINITY) - fc;
            double es = fabs(s - rs) / us, ec = fabs(c - rc) / uc;
            if (es > maxs) maxs = es;
            if (ec > maxc) maxc = ec;
        }
    }
    printf("%.4f %.4f\n", maxs, maxc);
    return 0;
}
'''


def _cc(tmp_path, name, src=None, path=None):
    exe = str(tmp_path / name)
    if src is not None:
        path = str(tmp_path / (name + ".c"))
        with open(path, "w") as f:
            f.write(src)
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fno-fast-math", "-I" + os.path.join(REPO, "include"),
                    "-o", exe, path, "-lm"], check=True)
    return exe


def test_float_sincos_accuracy(tmp_path):
    out = subprocess.run([_cc(tmp_path, "sincos", src=SINCOS_CHECK)], check=True, capture_output=True, text=True)
    es, ec = (float(v) for v in out.stdout.split())
    assert es <= 1.5 and ec <= 1.6, (es, ec)


def test_div_by_pi_exact(tmp_path):
    exe = _cc(tmp_path, "divpi", path=os.path.join(REPO, "tools", "check_div_by_pi.c"))
    out = subprocess.run([exe], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
