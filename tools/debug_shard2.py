"""Diagnostic: the uniform-stream test flow, per-window integrity checks on every shard."""
import sys

import numpy as np

sys.path.insert(0, "tests")
from oracle_sm import OracleStateMachine  # noqa: E402
from test_gpu_shard import LocalShards  # noqa: E402
from test_gpu_window import oracle_batches  # noqa: E402

from tigerbeetle_amd import workload  # noqa: E402
from tigerbeetle_amd.sharding import shard_of  # noqa: E402
from tigerbeetle_amd.types import Operation  # noqa: E402

BM = 8190


def run(G, check_every):
    n_acc, n_xfer, win = 30_000, 250_000, 8
    sh = LocalShards(G, BM, n_acc // G + 4096, n_xfer // G + 16384, win * BM)
    ref = OracleStateMachine(batch_max=BM)
    acc = workload.accounts(0, n_acc, seed=9)
    accb = [acc[i:i + BM] for i in range(0, n_acc, BM)]
    for w0 in range(0, len(accb), win):
        assert sh.commit_window(Operation.create_accounts, accb[w0:w0 + win]) == oracle_batches(
            ref, Operation.create_accounts, accb[w0:w0 + win])
    xf = workload.transfers_uniform(0, n_xfer, seed=9, n_accounts=n_acc)
    xfb = [xf[i:i + BM] for i in range(0, n_xfer, BM)]
    for k, w0 in enumerate(range(0, len(xfb), win)):
        g = sh.commit_window(Operation.create_transfers, xfb[w0:w0 + win])
        r = oracle_batches(ref, Operation.create_transfers, xfb[w0:w0 + win])
        if g != r:
            print(f"G={G} window {k}: reply mismatch")
            return False
        if check_every or w0 + win >= len(xfb):
            ga, ra = sh.dump_accounts(), ref.dump_accounts()
            gt, rt = sh.dump_transfers(), ref.dump_transfers()
            bad = []
            if ga.tobytes() != ra.tobytes():
                diff = np.nonzero(ga.view(np.uint8).reshape(-1, 128).any(1) != 0)[0]
                rows = np.nonzero((ga.view(np.uint8).reshape(-1, 128) != ra.view(np.uint8).reshape(-1, 128)).any(1))[0]
                bad.append(f"accounts differ in {len(rows)} rows, first {rows[:5].tolist()}; "
                           f"zero ids {int((ga['id_lo'] == 0).sum())}")
                j = rows[0]
                bad.append(f"  gpu {ga[j]}\n  ref {ra[j]}")
            if gt.tobytes() != rt.tobytes():
                rows = np.nonzero((gt.view(np.uint8).reshape(-1, 128) != rt.view(np.uint8).reshape(-1, 128)).any(1))[0] \
                    if len(gt) == len(rt) else []
                bad.append(f"transfers differ: len {len(gt)} vs {len(rt)}, rows {len(rows)}")
            if bad:
                print(f"G={G} window {k}: " + "\n".join(bad))
                for r_, s in enumerate(sh.shards):
                    st = s.stats()
                    a = s.sm.dump_accounts()
                    print(f"   shard {r_}: accounts {st['accounts']} transfers {st['transfers']} "
                          f"zero-id accounts {int((a['id_lo'] == 0).sum())} "
                          f"owned-ok {bool((shard_of(a['id_lo'], a['id_hi'], G) == r_).all())}")
                return False
    print(f"G={G}: ok")
    sh.close()
    ref.close()
    return True


for G in [int(x) for x in sys.argv[1].split(",")]:
    run(G, check_every=len(sys.argv) > 2)
