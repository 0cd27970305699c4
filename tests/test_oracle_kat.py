"""The CPU restatement against the reference's own known-answer tables (pins the oracle)."""
import glob
import os

import pytest

from kat import check
from oracle_sm import OracleStateMachine

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KATS = sorted(glob.glob(os.path.join(GOLDEN, "kat_*.tbl")))

# TestContext: message_body_size_max = 64 * 128 -> batch_max = 64 (state_machine.zig:2202-2208).
KAT_BATCH_MAX = 64


def test_kat_inventory():
    assert len(KATS) == 25


@pytest.mark.parametrize("path", KATS, ids=[os.path.basename(p)[4:-4] for p in KATS])
def test_oracle_kat(path):
    sm = OracleStateMachine(batch_max=KAT_BATCH_MAX)
    check(sm, open(path).read())
