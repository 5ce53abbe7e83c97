import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ringo-snark_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP library)")


@pytest.fixture(scope="session")
def fields():
    import json
    F = json.load(open(os.path.join(ROOT, "tests", "golden", "fields.json")))
    return {k: int(v["q_hex"], 16) for k, v in F.items()}
