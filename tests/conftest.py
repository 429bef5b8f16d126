import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

GOLDEN = os.path.join(HERE, "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) — run with -m gpu")
    config.addinivalue_line("markers", "slow: full-size (BASELINE config) parity runs")


@pytest.fixture(scope="session")
def oracle():
    import oracle_bind
    oracle_bind.load()
    return oracle_bind


def golden_cases():
    import json
    with open(os.path.join(GOLDEN, "MANIFEST.json")) as f:
        return json.load(f)["cases"]


def load_golden(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    if "inputs" in z.files:
        return z["inputs"], z["expected"]
    if name == "cfg1_f32_p2_1MiB":
        ins = np.stack([(0.5 + np.random.default_rng(1000 + r).random(262144)).astype(np.float32) for r in range(2)])
        return ins, z["expected"]
    raise KeyError(name)


@pytest.fixture(scope="session")
def gpu():
    """The tips_amd library on a real device. Fails (never skips) without one:
    gpu-marked tests only run with -m gpu, on the MI355X box."""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("no HIP device visible for a gpu-marked test")
    import tips_amd
    from tips_amd import _lib
    _lib.lib()  # loud failure if the .so is missing
    tips_amd.init()
    return tips_amd
