import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running statistical test")


@pytest.fixture(scope="session")
def ldpc_golden():
    import numpy as np
    return np.load(os.path.join(REPO, "tests", "golden", "ldpc_golden.npz"))


@pytest.fixture(scope="session")
def oracle_built():
    """Build oracle/_build (and oracle/_ref when the reference is present)."""
    import subprocess
    lib = os.path.join(REPO, "oracle", "_build", "libbp_oracle.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle")], check=True,
                       capture_output=True)
    return lib


@pytest.fixture(scope="session")
def sparc_golden():
    import numpy as np
    return np.load(os.path.join(REPO, "tests", "golden", "sparc_golden.npz"))


@pytest.fixture(scope="session")
def sophie_golden():
    import numpy as np
    return np.load(os.path.join(REPO, "tests", "golden", "sophie_golden.npz"))


@pytest.fixture(scope="session")
def integrated_golden():
    import numpy as np
    return np.load(os.path.join(REPO, "tests", "golden", "integrated_golden.npz"))


@pytest.fixture(scope="session")
def se_golden():
    import numpy as np
    return np.load(os.path.join(REPO, "tests", "golden", "se_golden.npz"))
