"""GPU: the driver's round-end smoke() (one fp32 and one f16 generator step against the oracle) as a test, so a
change that breaks it fails the -m gpu suite first."""
import pytest

pytestmark = pytest.mark.gpu


def test_graft_entry_smoke():
    import __graft_entry__
    __graft_entry__.smoke()
