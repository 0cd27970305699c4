"""The reference's known-answer tables on the MI355X engine, through the C ABI."""
import glob
import os

import pytest

from kat import check

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KATS = sorted(glob.glob(os.path.join(GOLDEN, "kat_*.tbl")))


@pytest.mark.gpu
@pytest.mark.parametrize("path", KATS, ids=[os.path.basename(p)[4:-4] for p in KATS])
def test_gpu_kat(path):
    from tigerbeetle_amd import StateMachine

    sm = StateMachine(batch_max=64, accounts_max=1024, transfers_max=4096)
    try:
        check(sm, open(path).read())
    finally:
        sm.close()
