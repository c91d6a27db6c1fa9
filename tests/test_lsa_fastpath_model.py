"""Host model of the certified LSA fast path (csrc/lsa_wave.h lsa_fast_reg64, modelled in
tools/lsa_fastpath_sim.py): column reduction + shortest augmenting paths from it, used only
under the uniqueness certificate.  On CPU, against scipy itself:
  * whenever the certificate holds, the assignment is scipy's;
  * matrices with several optimal assignments (exact ties) are never certified;
  * the fast path needs fewer augmenting-path steps than scipy's own algorithm on
    SAP-like matrices (shared task profile + small per-agent terms).
The kernel's parity against scipy on the GPU: tests/test_gpu_sap.py."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tools"))
scipy_opt = pytest.importorskip("scipy.optimize")

from lsa_fastpath_sim import fast_path, scipy_steps  # noqa: E402


def _sap_like(rng, n):
    return (rng.normal(size=(1, n)) + 0.05 * rng.normal(size=(n, n))).astype(np.float32)


@pytest.mark.parametrize("kind", ["sap", "uniform", "ints"])
def test_certified_means_scipy(kind):
    rng = np.random.RandomState({"sap": 1, "uniform": 2, "ints": 3}[kind])
    certified = 0
    for k in range(6):
        n = (64, 48, 17)[k % 3]
        if kind == "sap":
            Q = _sap_like(rng, n)
        elif kind == "uniform":
            Q = rng.rand(n, n).astype(np.float32)
        else:
            Q = rng.randint(0, 3, size=(n, n)).astype(np.float32)
        C = -Q.astype(np.float64)
        ref = scipy_opt.linear_sum_assignment(Q, maximize=True)[1]
        x, _, ok = fast_path(C)
        # the fast path always finds AN optimal assignment
        assert np.isclose(C[np.arange(n), x].sum(), C[np.arange(n), ref].sum(), rtol=0, atol=1e-9)
        if ok:
            assert np.array_equal(x, ref)
        certified += ok
    if kind == "ints":
        assert certified == 0  # small-integer matrices have many optima
    else:
        assert certified == 6


def test_fast_path_takes_fewer_steps_on_sap_like():
    rng = np.random.RandomState(5)
    ts = tf = 0
    for _ in range(3):
        C = -_sap_like(rng, 64).astype(np.float64)
        a, s = scipy_steps(C)
        b, f, ok = fast_path(C)
        assert ok and np.array_equal(a, b)
        ts, tf = ts + s, tf + f
    assert tf < 0.8 * ts, (tf, ts)
