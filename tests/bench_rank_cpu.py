"""One rank of bench.py on CPU with the oracle stand-in (tests/_fake_batch.py) --
started by tests/test_multiproc.py through bench.launch; TEST INFRASTRUCTURE ONLY."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, ROOT, os.path.join(ROOT, "python-mpc_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import bench  # noqa: E402
from _fake_batch import FakeBatch  # noqa: E402

if __name__ == "__main__":
    bench.main(sys.argv[1:], solver_cls=FakeBatch, device="cpu")
