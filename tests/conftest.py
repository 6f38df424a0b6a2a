import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a MI355X (runs the HIP library)")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected without a GPU")
    from geomesa_amd import _lib
    _lib.load()
    return _lib.context()


class JavaRandom:
    """java.util.Random (48-bit LCG), as used by the reference tests' `new Random(-574)`."""

    def __init__(self, seed):
        self.seed = (seed ^ 0x5DEECE66D) & ((1 << 48) - 1)

    def next(self, bits):
        self.seed = (self.seed * 0x5DEECE66D + 0xB) & ((1 << 48) - 1)
        r = self.seed >> (48 - bits)
        if r >= 1 << (bits - 1):
            r -= 1 << bits
        return r

    def nextInt(self, bound):
        if bound & (-bound) == bound:
            return (bound * (self.next(31) & 0x7FFFFFFF)) >> 31
        while True:
            bits = self.next(31) & 0x7FFFFFFF
            val = bits % bound
            if bits - val + (bound - 1) < (1 << 31):
                return val

    def nextDouble(self):
        return (((self.next(26) & ((1 << 26) - 1)) << 27) + (self.next(27) & ((1 << 27) - 1))) * (1.0 / (1 << 53))


@pytest.fixture
def jrandom():
    return JavaRandom


def load_geoms():
    import re
    r = re.compile(r"\((\d+\.\d*),(\d+\.\d*),(\d+\.\d*),(\d+\.\d*)\)")
    out = []
    with open(os.path.join(GOLDEN, "geoms.list")) as f:
        for line in f:
            m = r.search(line)
            if m:
                out.append(tuple(float(m.group(i)) for i in range(1, 5)))
    return out
