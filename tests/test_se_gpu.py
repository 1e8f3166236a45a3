"""GPU state evolution (se.hip, ldpc_sparc_amd.sparc_se) against the
reference's outputs (tests/golden/se_golden.npz, the reference run with seeded
numpy samples).  Bar: psi and tau within 1e-10 relative (the device sums the
Monte-Carlo mean in a different order), identical stopping iteration."""
import os
import sys

import numpy as np
import pytest

from ldpc_sparc_amd import sparc_se

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
from make_golden_se import CASES  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", list(CASES))
def test_state_evolution_matches_reference(se_golden, name):
    cp, var, t_max, mc, seed = CASES[name]
    np.random.seed(seed)
    code_params = dict(cp)
    psi, tau = sparc_se.sparc_se(var, code_params, t_max, mc)
    np.testing.assert_allclose(psi, se_golden[name + "_psi"], rtol=1e-10, atol=1e-14)
    np.testing.assert_allclose(tau, se_golden[name + "_tau"], rtol=1e-10)
    assert 'complex' in code_params and 'modulated' in code_params  # check_code_params rewrote it


def test_expectation_vector_and_scalar():
    rng = np.random.default_rng(0)
    u = rng.standard_normal((300, 64))
    from oracle import se_ref
    taus = np.array([0.05, 0.1, 0.3])
    E = sparc_se.sparc_se_E(taus, 1, u)
    for t, e in zip(taus, E):
        assert abs(e - se_ref.se_E(t, 1, u)) <= 1e-12 * abs(e)
    assert abs(sparc_se.sparc_se_E(0.2, 2, u) - se_ref.se_E(0.2, 2, u)) <= 1e-12
