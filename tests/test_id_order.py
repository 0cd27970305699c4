"""Id orders of `tigerbeetle benchmark --id-order` (cli.zig:97, 263-265): IdPermutation
(testing/id.zig:8-48) restated in tigerbeetle_amd/workload.py (numpy) and csrc/workload.hip
(device). CPU: the reference's own round-trip test ("IdPermutation", id.zig:76-98: decode(encode(v))
== v for its DefaultPrng(123) values), and the numpy Xoshiro256++ against the scalar restatement of
Zig std's generator (tests/test_checksum.py, pinned there by the reference's checksum stability
vectors). GPU: the device rewrite equals the numpy one."""
import numpy as np
import pytest

from test_checksum import Xoshiro256
from tigerbeetle_amd import workload
from tigerbeetle_amd.types import ACCOUNT_DTYPE, TRANSFER_DTYPE

M64, M128 = (1 << 64) - 1, (1 << 128) - 1


def _decode(lo, hi, order):
    v = int(lo) | (int(hi) << 64)
    if order == 0:
        return v
    if order == 2:
        return M128 - v
    return (v >> 32) & M64  # @truncate(id >> 32) into usize


def test_reference_round_trip():
    """id.zig:76-98 with the same PRNG draws (DefaultPrng.init(123)): identity, inversion and random
    (its seed is the stream's first u64), values random.int(usize), i and maxInt(usize) - i."""
    x = Xoshiro256(123)
    perms = [(0, 0), (2, 0), (1, None)]
    for order, seed in perms:
        if seed is None:
            seed = x.next()
        vals = []
        for i in range(20):
            vals += [x.next(), i, M64 - i]
        vals = [v for v in vals if v != 0]  # the engine's ids are index + 1 > 0
        lo, hi = workload.encode_ids(np.array(vals, np.uint64), order, seed)
        assert [_decode(a, b, order) for a, b in zip(lo, hi)] == vals


def test_random_matches_scalar_xoshiro():
    seed = workload.benchmark_permutation_seed(42)
    assert seed == Xoshiro256(42).next()  # benchmark_load.zig:120-125
    data = np.array([1, 2, 3, 10_000, 1 << 40, M64], np.uint64)
    lo, hi = workload.encode_ids(data, 1, seed)
    mask = M128 & ~(M64 << 32)
    for d, a, b in zip(data.tolist(), lo, hi):
        g = Xoshiro256((seed + d) & M64)
        r = g.next() | (g.next() << 64)
        assert int(a) | (int(b) << 64) == (((d << 32) | (r & mask)) & M128)


def test_permute_records_cpu():
    a = workload.accounts(0, 100, seed=3)
    t = workload.transfers_uniform(0, 100, seed=3, n_accounts=100)
    seed = workload.benchmark_permutation_seed(3)
    for order in (1, 2, 3):
        a2 = workload.permute_ids(a.copy(), order, seed)
        t2 = workload.permute_ids(t.copy(), order, seed)
        ids = {(int(x), int(y)) for x, y in zip(a2["id_lo"], a2["id_hi"])}
        assert len(ids) == 100
        assert {(int(x), int(y)) for x, y in zip(t2["debit_account_id_lo"], t2["debit_account_id_hi"])} <= ids
        assert {(int(x), int(y)) for x, y in zip(t2["credit_account_id_lo"], t2["credit_account_id_hi"])} <= ids
        assert (t2["id_hi"] != 0).all()


def test_time_ids_strictly_increasing():
    """The time-based order (docs/develop/data-modeling.md:186-203): 48-bit milliseconds above 80
    random bits, incremented within a millisecond; strictly increasing u128 ids, high word nonzero,
    a new millisecond every 2^18 ids."""
    n = (1 << 18) * 3 + 1000
    lo, hi = workload.encode_ids(np.arange(1, n + 1, dtype=np.uint64), 3, 77)
    v = [int(a) | (int(b) << 64) for a, b in zip(lo, hi)]
    assert all(x < y for x, y in zip(v, v[1:]))
    assert (hi != 0).all()
    ms = [x >> 80 for x in v]
    assert ms[0] == workload.TIME_BASE_MS and ms[-1] == workload.TIME_BASE_MS + 3
    assert ms[(1 << 18) - 1] == ms[0] and ms[1 << 18] == ms[0] + 1


@pytest.mark.gpu
@pytest.mark.parametrize("order", [1, 2, 3])
def test_permute_ids_device(order):
    import torch

    from tigerbeetle_amd import _lib

    L = _lib.lib()
    n, seed = 5000, workload.benchmark_permutation_seed(44)
    for dt, gen, kind in ((ACCOUNT_DTYPE, workload.accounts(0, n, seed=4), 0),
                          (TRANSFER_DTYPE, workload.transfers_uniform(0, n, seed=4, n_accounts=n), 1)):
        d = torch.from_numpy(np.frombuffer(gen.tobytes(), np.uint8).copy()).cuda()
        torch.cuda.synchronize()
        _lib.check(L.tbg_gen_permute_ids(d.data_ptr(), n, kind, order, seed, None), "permute")
        torch.cuda.synchronize()
        got = np.frombuffer(d.cpu().numpy().tobytes(), dt)
        assert got.tobytes() == workload.permute_ids(gen.copy(), order, seed).tobytes()
