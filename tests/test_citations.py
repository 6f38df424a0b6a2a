"""Every Scala/Java file:line citation in the repo points inside the cited reference file.

Runs only where the reference checkout exists (this container); the GPU box has none."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not os.path.isdir("/root/reference"), reason="reference checkout absent")
def test_citations_in_range():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import check_citations
    bad = check_citations.check(ROOT)
    assert not bad, "\n".join("%s:%d: %s (%s)" % b for b in bad)
