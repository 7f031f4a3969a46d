import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd")
for p in (PKG_ROOT, os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def goldens():
    import numpy as np
    d = np.load(os.path.join(ROOT, "tests", "golden", "pmpc_goldens.npz"))
    return {k: d[k] for k in d.files}


@pytest.fixture(scope="session")
def rmpc_goldens():
    import numpy as np
    d = np.load(os.path.join(ROOT, "tests", "golden", "rmpc_goldens.npz"))
    return {k: d[k] for k in d.files}


@pytest.fixture(scope="session")
def lmpc_goldens():
    import numpy as np
    d = np.load(os.path.join(ROOT, "tests", "golden", "lmpc_goldens.npz"))
    return {k: d[k] for k in d.files}
