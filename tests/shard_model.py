"""CPU model of the hash-sharded commit (tigerbeetle_amd/csrc/shard.h). TEST INFRASTRUCTURE.

Restates the per-shard protocol in numpy/Python so that the decomposition itself can be checked on
CPU with real torch.distributed (gloo) collectives, world size > 1, without a GPU:

  prep     each shard writes, per event, only the facts it owns (debit / credit account ledger and
           limit bit, transfer-id exists code) into a (1 + E) x 4 int32 word array; word 0 = trailer
  exchange element-wise sum across shards (dist.all_reduce)
  decide   each shard decides its home batches (a contiguous range of the window's batches) from
           the summed words (+ linked chains) and sets one commit flag per home event
  exchange element-wise sum of the commit flags across shards
  apply    owned effects of committed events only (id owner stores the record, account owners add
           the amount)

Validation order follows state_machine.zig:1421-1489 (create_account / create_transfer heads), the
exists comparisons :1450-1460 and :1587-1606, chains :1240-1300. Only the sharded class is modelled
(no limits, balancing, two-phase or in-window duplicates); the test streams stay inside it.
"""
import numpy as np

from tigerbeetle_amd.sharding import shard_of
from tigerbeetle_amd.types import U128_MAX, get_u128

CONT = -1
TRANSFER_FIELDS_EXISTS = [  # create_transfer_exists order (:1587-1606), codes 36..45, then 46
    ("flags", 36), ("debit_account_id", 37), ("credit_account_id", 38), ("amount", 39),
    ("user_data_128", 41), ("user_data_64", 42), ("user_data_32", 43), ("timeout", 44), ("code", 45)]
ACCOUNT_FIELDS_EXISTS = [  # create_account_exists order (:1450-1460), codes 15..20, then 21
    ("flags", 15), ("user_data_128", 16), ("user_data_64", 17), ("user_data_32", 18), ("ledger", 19),
    ("code", 20)]
U128_FIELDS = {"id", "debit_account_id", "credit_account_id", "amount", "pending_id", "user_data_128",
               "debits_pending", "debits_posted", "credits_pending", "credits_posted"}


def field(rec, name):
    return get_u128(rec, name) if name in U128_FIELDS else int(rec[name])


def ca_static(a):
    """create_account validation (:1424-1439); CONT if it passes."""
    if int(a["timestamp"]) != 0:
        return 3
    if int(a["reserved"]) != 0:
        return 4
    f = int(a["flags"])
    if f & 0xFFF0:
        return 5
    ident = field(a, "id")
    if ident == 0:
        return 6
    if ident == U128_MAX:
        return 7
    if (f & 2) and (f & 4):
        return 8
    for name, code in (("debits_pending", 9), ("debits_posted", 10), ("credits_pending", 11),
                       ("credits_posted", 12)):
        if field(a, name) != 0:
            return code
    if int(a["ledger"]) == 0:
        return 13
    if int(a["code"]) == 0:
        return 14
    return CONT


def ct_static(t):
    """create_transfer head and single-phase validation (:1465-1489); CONT if it passes."""
    if int(t["timestamp"]) != 0:
        return 3
    f = int(t["flags"])
    if f & 0xFFC0:
        return 4
    ident = field(t, "id")
    if ident == 0:
        return 5
    if ident == U128_MAX:
        return 6
    assert not f & 0x3E, "outside the modelled class"
    dr, cr = field(t, "debit_account_id"), field(t, "credit_account_id")
    if dr == 0:
        return 8
    if dr == U128_MAX:
        return 9
    if cr == 0:
        return 10
    if cr == U128_MAX:
        return 11
    if cr == dr:
        return 12
    if field(t, "pending_id") != 0:
        return 13
    if int(t["timeout"]) != 0:
        return 17
    if field(t, "amount") == 0:
        return 18
    if int(t["ledger"]) == 0:
        return 19
    if int(t["code"]) == 0:
        return 20
    return CONT


def exists_code(ev, stored, fields, exists):
    for name, code in fields:
        if field(ev, name) != field(stored, name):
            return code
    return exists


class ShardModel:
    def __init__(self, G, me):
        self.G, self.me = G, me
        self.accounts = {}   # id -> stored record (owned)
        self.transfers = {}  # id -> stored record (owned)

    def owns(self, rec, name):
        return int(shard_of(rec[name + "_lo"], rec[name + "_hi"], self.G)) == self.me

    def prep(self, op, events):
        words = np.zeros((1 + len(events), 4), np.int64)
        static = []
        for i, ev in enumerate(events):
            code = ca_static(ev) if op == "a" else ct_static(ev)
            static.append(code)
            if code != CONT:
                continue
            v = words[1 + i]
            if op == "a":
                if self.owns(ev, "id"):
                    st = self.accounts.get(field(ev, "id"))
                    v[2] = 1 + (0 if st is None else exists_code(ev, st, ACCOUNT_FIELDS_EXISTS, 21))
                continue
            for side, col in (("debit_account_id", 0), ("credit_account_id", 1)):
                if self.owns(ev, side):
                    acc = self.accounts.get(field(ev, side))
                    if acc is not None:
                        v[col] = int(acc["ledger"])
            if self.owns(ev, "id"):
                st = self.transfers.get(field(ev, "id"))
                v[2] = 1 + (0 if st is None else exists_code(ev, st, TRANSFER_FIELDS_EXISTS, 46))
        return words, static

    @staticmethod
    def decide(op, events, words, static):
        codes = []
        for i, ev in enumerate(events):
            code = static[i]
            if code == CONT:
                x, y, z = (int(c) for c in words[1 + i][:3])
                if op == "a":
                    code = z - 1
                elif x == 0:
                    code = 21
                elif y == 0:
                    code = 22
                elif x != y:
                    code = 23
                elif int(ev["ledger"]) != x:
                    code = 24
                else:
                    code = z - 1
            codes.append(code)
        # linked chains (:1240-1300): first failure back-fills the chain, open chain at batch end
        n = len(events)
        i = 0
        while i < n:
            if not int(events[i]["flags"]) & 1:
                i += 1
                continue
            j = i
            while j < n - 1 and int(events[j]["flags"]) & 1:
                j += 1
            end = j  # last member (unlinked, or the batch's last event)
            if int(events[end]["flags"]) & 1:
                codes[end] = 2  # linked_event_chain_open
            f = next((k for k in range(i, end + 1) if codes[k] != 0), None)
            if f is not None:
                for k in range(i, end + 1):
                    if k != f and not (k == end and codes[end] == 2):
                        codes[k] = 1
            i = end + 1
        return codes

    def apply(self, op, events, commit, timestamps):
        for i, ev in enumerate(events):
            if not commit[i]:
                continue
            rec = ev.copy()
            rec["timestamp"] = timestamps[i]
            if op == "a":
                if self.owns(ev, "id"):
                    self.accounts[field(ev, "id")] = rec
                continue
            amount = field(ev, "amount")
            for side, bal in (("debit_account_id", "debits_posted"), ("credit_account_id", "credits_posted")):
                if self.owns(ev, side):
                    acc = self.accounts[field(ev, side)]
                    v = field(acc, bal) + amount
                    acc[bal + "_lo"] = v & (2**64 - 1)
                    acc[bal + "_hi"] = v >> 64
            if self.owns(ev, "id"):
                self.transfers[field(ev, "id")] = rec
