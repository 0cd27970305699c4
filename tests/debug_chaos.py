"""Debug helper: replay a chaos seed on GPU and oracle, stop at the first diverging batch and
print the diverging events with their engine class bits."""
import sys

import numpy as np

_here = __import__("os").path.dirname(__import__("os").path.abspath(__file__))
sys.path.insert(0, _here)
sys.path.insert(0, __import__("os").path.dirname(_here))
from chaos import Chaos, run_protocol  # noqa: E402
from oracle_sm import OracleStateMachine  # noqa: E402

from tigerbeetle_amd import StateMachine, _lib  # noqa: E402
from tigerbeetle_amd.types import NS_PER_S, Operation, get_u128  # noqa: E402

CLS = ["STATIC", "REACH", "U", "W", "LINKED", "TSNZ", "INSERT", "PENDING", "POSTVOID", "POST", "READS_DR",
       "READS_CR", "PV_PRE", "COMMIT", "INSERTED"]


def main(seed, batches, batch_max, **kw):
    gpu = StateMachine(batch_max=batch_max, accounts_max=1 << 12, transfers_max=1 << 16)
    ref = OracleStateMachine(batch_max=batch_max)
    ch = Chaos(seed, **kw)
    for b in range(batches):
        if b < 3:
            ev, op = ch.accounts_batch(ch.rng.randint(1, batch_max)), Operation.create_accounts
        else:
            n = ch.rng.choice([1, 2, 5, batch_max // 2, batch_max])
            ev, op = ch.transfers_batch(n), Operation.create_transfers
        tick = NS_PER_S if (b % 3 == 0) else 0
        r1 = run_protocol(gpu, op, ev, tick)
        r2 = run_protocol(ref, op, ev, tick)
        if r1 != r2:
            n = len(ev)
            cls = np.zeros(n, np.uint32)
            code = np.zeros(n, np.uint32)
            _lib.lib().tbg_debug_last_batch(gpu.h, cls.ctypes.data, code.ctypes.data, n)
            g = dict(np.frombuffer(r1, "<u4").reshape(-1, 2).tolist())
            r = dict(np.frombuffer(r2, "<u4").reshape(-1, 2).tolist())
            print(f"batch {b} n={n} op={op.name} T={gpu.prepare_timestamp}")
            for i in range(n):
                if g.get(i, 0) != r.get(i, 0):
                    e = ev[i]
                    bits = [nm for k, nm in enumerate(CLS) if cls[i] >> k & 1]
                    print(f"  i={i} gpu={g.get(i, 0)} ref={r.get(i, 0)} cls={bits} id={get_u128(e, 'id')} "
                          f"dr={get_u128(e, 'debit_account_id')} cr={get_u128(e, 'credit_account_id')} "
                          f"amt={get_u128(e, 'amount')} pid={get_u128(e, 'pending_id')} flags={e['flags']:#x} "
                          f"timeout={e['timeout']} ledger={e['ledger']}")
            # context: other events touching the same ids / accounts
            return
    print("no divergence")


if __name__ == "__main__":
    main(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), n_accounts=300, id_space=4000)
