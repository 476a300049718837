import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long CPU test")
    # make sure the checker and the product library exist (cheap no-ops when built)
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True)
    if not os.path.exists(os.path.join(ROOT, "smallz4_amd", "lib", "libsmallz4_amd.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "smallz4_amd", "csrc")], check=False)


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        return json.load(f)["cases"]


@pytest.fixture(scope="session")
def compressor():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import smallz4_amd
    return smallz4_amd.Compressor(device=0)
