"""Debug: sharded general path pulse_next vs the restatement, per batch (GPU box)."""
import sys

import numpy as np

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from chaos import Chaos, run_protocol  # noqa: E402
from oracle_sm import OracleStateMachine  # noqa: E402
from test_gpu_shard import LocalShards  # noqa: E402
from tigerbeetle_amd.types import NS_PER_S, Operation  # noqa: E402


def live(xs, st):
    m = ((xs["flags"] & 2) != 0) & (xs["timeout"] > 0) & (st == 1)
    e = xs["timestamp"][m] + xs["timeout"][m].astype(np.uint64) * np.uint64(NS_PER_S)
    return sorted(zip(e.tolist(), xs["timestamp"][m].tolist()))


G, bm = 3, 8
sh = LocalShards(G, bm, 1024, 1 << 14, bm)
ref = OracleStateMachine(batch_max=bm)
ch = Chaos(7100, n_accounts=10, pending=0.9, postvoid=0.05, limits=0.0, balancing=0.0, linked=0.05, invalid=0.0)
for b in range(40):
    if b < 2:
        ev, op = ch.accounts_batch(bm), Operation.create_accounts
    else:
        ev, op = ch.transfers_batch(bm), Operation.create_transfers
    tick = 5 * NS_PER_S if b % 8 == 7 else 0
    pn0 = (sh.shards[0].pulse_next(), ref.pulse_next_timestamp())
    g, fast = sh.commit_any(op, [ev], tick)
    r = run_protocol(ref, op, ev, tick)
    pn = (sh.shards[0].pulse_next(), ref.pulse_next_timestamp())
    print(b, "fast" if fast else "gen", "T", sh.prepare_timestamp, "pn before", pn0, "after", pn, "reply", g == [r])
    if pn[0] != pn[1] or g != [r]:
        rx, rs = ref.dump_transfers(), ref.dump_transfer_status()
        print(" ref live", live(rx, rs)[:12])
        for k, s in enumerate(sh.shards):
            print(" shard", k, "live", live(s.sm.dump_transfers(), s.sm.dump_transfer_status())[:12])
        print(" ref statuses", np.bincount(rs, minlength=5))
        print(" shard statuses", sum(np.bincount(s.sm.dump_transfer_status(), minlength=5) for s in sh.shards))
        break
