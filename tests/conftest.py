import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    if os.environ.get("DMX_LIBV"):   # a diagnostic library variant (tools/build_var.sh), e.g. the claim guard
        import deflate_compression_amd as D
        D.LIB_PATH = os.path.abspath(os.environ["DMX_LIBV"])
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def golden_cases():
    import golden_inputs
    return golden_inputs.cases()


@pytest.fixture(scope="session")
def golden_tokens():
    import numpy as np
    z = np.load(os.path.join(REPO, "tests", "golden", "ref_tokens.npz"), allow_pickle=False)
    return {k: z[k] for k in z.files}
