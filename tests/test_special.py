"""The committed special-function coefficients (csrc/cse_special.hpp, written by
tools/gen_special.py) hold the error bounds the kernels are documented with,
evaluated in fp32 in the kernels' own order (Horner, one rounding per FMA):

  - MMSE bracket h(v) = e^{-v/2}[(1+v) I0(v/2) + v I1(v/2)] (mmse.py:88-96):
    relative error < 5e-7 on [1e-12, 80];
  - OMLSA's LSA exponent 0.5 log2(e) E1(v) (advanced_mmse.py:100-104) as the
    kernel forms it, Pn(v')/Dn(v') - 0.5 log2(v') + 0.5 log2(log2 e) with
    v' = min(v log2 e, CSE_LSA_VMAX2): absolute error < 2e-6 on [1e-12, 80];
    Dn stays in (0.02, 1] (the kernel's overflow argument).

CPU only: reads the header as text, scipy.special for the reference values.
"""

import os
import re

import numpy as np
from scipy.special import exp1, i0e, i1e

HDR = os.path.join(os.path.dirname(__file__), "..", "classical_speech_enhancement_amd", "csrc",
                   "cse_special.hpp")


def _consts():
    text = open(HDR).read()
    arrays = {m.group(1): np.array([np.float32(float(x.rstrip("f")))
                                    for x in m.group(2).split(",")])
              for m in re.finditer(r"float (CSE_\w+)\[\d+\] = \{([^}]*)\}", text)}
    scalars = {m.group(1): float(m.group(2)) for m in
               re.finditer(r"float (CSE_\w+) = ([-0-9.e]+)f", text)}
    for m in re.finditer(r"float (CSE_HB_U0) = ([0-9.e-]+)f, (CSE_HB_U1) = ([0-9.e-]+)f", text):
        scalars[m.group(1)], scalars[m.group(3)] = float(m.group(2)), float(m.group(4))
    return arrays, scalars


def _horner32(c, t):
    t = np.asarray(t, dtype=np.float32)
    acc = np.full_like(t, c[-1])
    for ck in c[-2::-1]:
        acc = (acc.astype(np.float64) * t + np.float64(ck)).astype(np.float32)  # fma: one rounding
    return acc


def test_lsa_rational_abs_error():
    a, s = _consts()
    l2e = np.float32(1.4426950408889634)
    v = np.concatenate([np.logspace(-12, 0, 20001), np.linspace(1, 80, 40001)])
    v2 = np.minimum((v.astype(np.float32) * l2e).astype(np.float32), np.float32(s["CSE_LSA_VMAX2"]))
    pn = _horner32(a["CSE_LSAP"], v2).astype(np.float64)
    dn = _horner32(a["CSE_LSAD"], v2).astype(np.float64)
    assert dn.min() > 0.02 and dn.max() <= 1.0 + 1e-6
    lg = pn / dn - 0.5 * np.log2(v2.astype(np.float64)) + 0.5 * np.log2(1.4426950408889634)
    err = np.max(np.abs(lg - 0.5 * 1.4426950408889634 * exp1(v)))
    assert err < 2e-6, err


def test_mmse_bracket_rel_error():
    a, s = _consts()
    split, u0, u1 = s["CSE_HA_SPLIT"], s["CSE_HB_U0"], s["CSE_HB_U1"]
    v = np.concatenate([np.logspace(-12, np.log10(split), 20001), np.linspace(split, 80, 40001)])
    v32 = v.astype(np.float32)
    ta = ((v32 - np.float32(2.0)) * np.float32(0.5)).astype(np.float32)
    u = (1.0 / v32.astype(np.float64)).astype(np.float32)
    tb = (u.astype(np.float64) * 2.0 - (u0 + u1)) * (1.0 / (u1 - u0))
    pa = _horner32(a["CSE_HA"], ta).astype(np.float64)
    pb = _horner32(a["CSE_HB"], tb.astype(np.float32)).astype(np.float64)
    approx = np.where(v32 <= split, pa, np.sqrt(v32.astype(np.float64)) * pb)
    ref = (1 + v) * i0e(v / 2) + v * i1e(v / 2)
    err = np.max(np.abs(approx / ref - 1))
    assert err < 5e-7, err
