import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def oracle():
    from oracle_lib import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


# Lines the parity tests want in the log even when they pass (per-utterance error
# distributions, decision-flip counts): printed in the terminal summary.
REPORT: list = []


@pytest.fixture(scope="session")
def parity_report():
    return REPORT


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    if REPORT:
        terminalreporter.section("parity report")
        for line in REPORT:
            terminalreporter.write_line(line)


def pytest_collection_finish(session):
    """GPU runs: initialise torch's HIP runtime before libafs touches the device (torch
    refuses to initialise after another runtime copy in the process has), so tests may mix
    torch device tensors with the C ABI."""
    if any(item.get_closest_marker("gpu") for item in session.items):
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.init()
        except Exception:
            pass
