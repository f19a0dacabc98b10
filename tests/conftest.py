"""pytest configuration: `-m gpu` tests need an MI355X (run them through gpurun);
everything else runs on CPU.  Paths: the host package lives in python-mpc_amd/
(a directory name that is not an identifier) and the oracle in oracle/."""
import os
import sys

import numpy as np
import pytest
import scipy.sparse as sparse

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "python-mpc_amd"), os.path.join(ROOT, "oracle"), ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run via gpurun")


def pytest_terminal_summary(terminalreporter):
    """The agreement fractions every device-vs-oracle batch check observed (tests/parity.py)."""
    import parity
    if not parity.RECORDS:
        return
    terminalreporter.section("parity agreement (device vs oracle)")
    for label, n, fs, fi, nd, du, note in parity.RECORDS:
        terminalreporter.write_line(f"{label}: {n} instances, status {fs:.4f}, iterations {fi:.4f}, "
                                    f"{nd} disagreeing (each held to the termination test), "
                                    f"max |du| where equal {du:.2e}{note}")


def load_golden(name):
    """Return dict of arrays + scipy CSC P/A from a tests/golden fixture."""
    d = dict(np.load(os.path.join(GOLDEN, name), allow_pickle=False))
    for k in ("P", "A"):
        if k + "_data" in d:
            shape = tuple(int(v) for v in d.pop(k + "_shape"))
            d[k] = sparse.csc_matrix((d.pop(k + "_data"), d.pop(k + "_indices"), d.pop(k + "_indptr")), shape=shape)
    return d


@pytest.fixture(scope="session")
def golden():
    return load_golden
