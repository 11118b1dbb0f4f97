import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (REPO, HERE, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def ctx():
    import depthmapx_amd as dmx
    c = dmx.Context(0)
    yield c
    c.close()


def pytest_runtest_logreport(report):
    """DMX_TEST_DURATIONS=<file>: append each test phase's duration as it ends (a run cut off by a time limit
    still leaves the record of what took the time)."""
    path = os.environ.get("DMX_TEST_DURATIONS")
    if path and report.when in ("setup", "call"):
        with open(path, "a") as f:
            f.write("%.2f %s %s %s\n" % (report.duration, report.when, report.outcome, report.nodeid))
