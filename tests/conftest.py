import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "hybrid-als-twotower-recommender_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG_DIR, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C-ABI)")


@pytest.fixture(scope="session")
def device():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test ran without a visible HIP device")
    return torch.device("cuda", 0)


def load_golden(name):
    import json

    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def dec_score(d):
    """Inverse of make_golden.enc_score: exact numpy scalar."""
    import numpy as np

    t = d["t"]
    if t == "int":
        return int(d["v"])
    if t == "float32":
        return np.float32(d["v"])
    if t == "float64":
        return np.float64(d["v"])
    return float(d["v"])


def dec_pairs(pairs):
    return [(int(i), dec_score(s)) for i, s in pairs]
