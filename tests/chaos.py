"""Randomized request streams that hit every path of the commit logic: linked chains (incl. open
chains and rollbacks), duplicate ids inside and across batches, two-phase pending/post/void with
timeouts and expiry, balancing, account limits, overflow-sized amounts, non-zero timestamps and
invalid fields. Seeded and deterministic; used for GPU-vs-oracle differential tests."""
import random

import numpy as np

from tigerbeetle_amd.types import ACCOUNT_DTYPE, TRANSFER_DTYPE, U128_MAX, set_u128


def _pick(rng, choices):
    r = rng.random()
    acc = 0.0
    for p, v in choices:
        acc += p
        if r < acc:
            return v
    return choices[-1][1]


class Chaos:
    def __init__(self, seed, n_accounts=40, id_space=400, huge=False, limits=0.3, linked=0.15, pending=0.3,
                 postvoid=0.25, balancing=0.08, invalid=0.05, history=0.0):
        self.rng = random.Random(seed)
        self.n_accounts = n_accounts
        self.id_space = id_space
        self.huge = huge
        self.p = dict(limits=limits, linked=linked, pending=pending, postvoid=postvoid, balancing=balancing,
                      invalid=invalid, history=history)
        self.pending_ids = []
        self.history = []  # recent transfer events, for idempotent retries

    def accounts_batch(self, n):
        rng = self.rng
        a = np.zeros(n, ACCOUNT_DTYPE)
        for i in range(n):
            ident = rng.randint(1, self.n_accounts + 3)
            set_u128(a[i], "id", ident)
            a[i]["ledger"] = 1 if rng.random() < 0.9 else 2
            a[i]["code"] = rng.randint(1, 3)
            f = 0
            if rng.random() < self.p["limits"]:
                f |= 2 if rng.random() < 0.5 else 4
            if rng.random() < self.p["linked"]:
                f |= 1
            if rng.random() < 0.02:
                f |= 6  # mutually exclusive
            if self.p["history"] and rng.random() < self.p["history"]:
                f |= 8  # flags.history: historical_balance rows (get_account_balances)
            a[i]["flags"] = f
            a[i]["user_data_64"] = rng.randint(0, 2)
            if rng.random() < self.p["invalid"]:
                k = rng.randint(0, 4)
                if k == 0:
                    a[i]["reserved"] = 1
                elif k == 1:
                    a[i]["timestamp"] = 7
                elif k == 2:
                    set_u128(a[i], "debits_posted", 5)
                elif k == 3:
                    a[i]["ledger"] = 0
                else:
                    set_u128(a[i], "id", 0)
        return a

    def _amount(self):
        rng = self.rng
        if self.huge and rng.random() < 0.1:
            return U128_MAX - rng.randint(0, 1000)
        if rng.random() < 0.05:
            return 0
        return rng.randint(1, 200)

    def transfers_batch(self, n):
        rng = self.rng
        t = np.zeros(n, TRANSFER_DTYPE)
        for i in range(n):
            if self.history and rng.random() < 0.12:
                # retry of an earlier event, sometimes with one field changed (exists* paths)
                t[i] = self.history[rng.randrange(len(self.history))]
                t[i]["timestamp"] = 0
                k = rng.randint(0, 9)
                if k == 1:
                    t[i]["user_data_128_lo"] += 1
                elif k == 2:
                    t[i]["user_data_64"] += 1
                elif k == 3:
                    t[i]["user_data_32"] += 1
                elif k == 4:
                    t[i]["timeout"] = (int(t[i]["timeout"]) + 1) & 0xFFFFFFFF
                elif k == 5:
                    t[i]["code"] = t[i]["code"] % 3 + 1
                elif k == 6:
                    t[i]["amount_lo"] += 1
                elif k == 7:
                    t[i]["flags"] ^= 1
                continue
            ident = rng.randint(1, self.id_space)
            set_u128(t[i], "id", ident)
            kind = rng.random()
            if kind < self.p["postvoid"] and self.pending_ids:
                pid = rng.choice(self.pending_ids) if rng.random() < 0.85 else rng.randint(1, self.id_space)
                set_u128(t[i], "pending_id", pid)
                t[i]["flags"] = 4 if rng.random() < 0.6 else 8
                amt = rng.choice([0, 0, rng.randint(1, 150)])
                set_u128(t[i], "amount", amt)
                if rng.random() < 0.2:
                    set_u128(t[i], "debit_account_id", rng.randint(1, self.n_accounts))
                if rng.random() < 0.1:
                    t[i]["ledger"] = 1
                if rng.random() < 0.3:
                    t[i]["user_data_32"] = rng.randint(0, 2)
            else:
                dr = rng.randint(1, self.n_accounts + 2)
                cr = rng.randint(1, self.n_accounts + 2)
                set_u128(t[i], "debit_account_id", dr)
                set_u128(t[i], "credit_account_id", cr)
                set_u128(t[i], "amount", self._amount())
                t[i]["ledger"] = 1 if rng.random() < 0.95 else 2
                t[i]["code"] = rng.randint(1, 3)
                f = 0
                if rng.random() < self.p["pending"]:
                    f |= 2
                    t[i]["timeout"] = rng.choice([0, 1, 2, 3, 5])
                    self.pending_ids.append(ident)
                    if len(self.pending_ids) > 200:
                        self.pending_ids.pop(0)
                if rng.random() < self.p["balancing"]:
                    f |= rng.choice([16, 32, 48])
                t[i]["flags"] = f
                t[i]["user_data_64"] = rng.randint(0, 2)
            if rng.random() < self.p["linked"]:
                t[i]["flags"] |= 1
            if rng.random() < self.p["invalid"]:
                k = rng.randint(0, 13)
                if k == 0:
                    t[i]["timestamp"] = 5
                elif k == 1:
                    t[i]["flags"] |= 1 << 9
                elif k == 2:
                    t[i]["code"] = 0
                elif k == 3:
                    set_u128(t[i], "id", 0)
                elif k == 4:
                    t[i]["timeout"] = 9
                elif k == 5:
                    t[i]["flags"] |= 12
                elif k == 6:
                    set_u128(t[i], "id", U128_MAX)
                elif k == 7:
                    set_u128(t[i], "debit_account_id", rng.choice([0, U128_MAX]))
                elif k == 8:
                    set_u128(t[i], "credit_account_id", rng.choice([0, U128_MAX]))
                elif k == 9:
                    set_u128(t[i], "pending_id", rng.choice([0, U128_MAX, 3]))
                elif k == 10:
                    t[i]["ledger"] = 0
                elif k == 11:
                    t[i]["ledger"] = 3
                elif k == 12:
                    t[i]["timeout"] = 0xFFFFFFFF
                    t[i]["flags"] |= 2
                else:
                    t[i]["code"] = 9
            self.history.append(t[i].copy())
            if len(self.history) > 300:
                self.history.pop(0)
        return t


def run_protocol(sm, operation, events, tick_ns=0):
    """One commit under the harness protocol (state_machine.zig:2719-2739); returns reply bytes."""
    from tigerbeetle_amd.types import Operation

    data = events.tobytes()
    sm.prepare_timestamp += tick_ns
    sm.prepare_timestamp += 1
    sm.prepare(operation, data)
    T = sm.prepare_timestamp
    if sm.pulse():
        sm.prefetch_timestamp = T
        sm.prefetch(1, Operation.pulse, b"")
        sm.commit(0, 1, T, Operation.pulse, b"")
    sm.prefetch_timestamp = T
    sm.prefetch(2, operation, data)
    return sm.commit(0, 2, T, operation, data)
