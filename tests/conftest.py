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


class heartbeat:
    """Context manager printing a progress line every `every` seconds from a daemon thread (long CPU-oracle phases of
    a GPU test: the GPU box kills a command that writes nothing for minutes). Use with pytest -s."""

    def __init__(self, what, every=30.0):
        self.what, self.every = what, every

    def __enter__(self):
        import threading
        import time
        self._stop = threading.Event()
        t0 = time.time()

        # also appended under gpurun_out/ (the GPU box watches that directory too; pytest captures stdout without -s)
        log = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "heartbeat.log")

        def run():
            while not self._stop.wait(self.every):
                line = f"[{self.what}] {time.time() - t0:.0f} s"
                print(line, flush=True)
                try:
                    os.makedirs(os.path.dirname(log), exist_ok=True)
                    with open(log, "a") as f:
                        f.write(line + "\n")
                except OSError:
                    pass
        self._t = threading.Thread(target=run, daemon=True)
        self._t.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        self._t.join()
        return False
