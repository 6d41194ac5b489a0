import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "diffusion-models-moe_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

import pytest  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")


# ---- near-tie / flip accounting: GPU parity tests record how many rows they compared, how many sat within fp16
# near-tie distance of the top-k boundary and how many of those flipped. Written at session end to the JSON file
# named by SDMOE_PARITY_REPORT (the GPU runs set it under gpurun_out/; copies are kept under profiles/).
_PARITY = []


@pytest.fixture(scope="session")
def parity_report():
    def add(test, **counts):
        _PARITY.append(dict(test=test, **{k: (int(v) if not isinstance(v, float) else v) for k, v in counts.items()}))
    return add


def pytest_sessionfinish(session, exitstatus):
    path = os.environ.get("SDMOE_PARITY_REPORT")
    if path and _PARITY:
        import json
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump(_PARITY, f, indent=1)
