"""CPU model of the routed hash-sharded commit (tigerbeetle_amd/csrc/route.h). TEST INFRASTRUCTURE.

Restates the per-shard protocol in numpy/Python, with the device's exact block layouts, so that the
decomposition can be checked on CPU with real torch.distributed (gloo) all-to-alls at world size > 1,
and its message blocks compared byte for byte with the engine's (tests/test_gpu_route.py):

  route    the home validates its events (state_machine.zig:1424-1439, 1465-1489), stamps them
           (:1253) and writes one block per destination: the record to the id owner, {account id,
           amount, side} to each account owner, in event order                        -> exchange A
  own      each owner answers what it owns: the id's claim (in-window duplicates) and exists code
           (:1450-1460, 1587-1606); the account's state, ledger and limit/history flag -> exchange B
  decide   each home decides its events from the replies (:1496-1507) and chains (:1240-1300) and
           writes a commit byte per message plus committed records per 1024-chunk   -> exchange C
  apply    every shard ORs the verdicts; the owners apply the committed messages in (home, message)
           order: balances, records appended in timestamp order.

Only the class is modelled (no limits, balancing, two-phase); a window outside it is rejected by the
verdict like on the device.
"""
import struct

import numpy as np

from tigerbeetle_amd.sharding import shard_of
from tigerbeetle_amd.types import ACCOUNT_DTYPE, TRANSFER_DTYPE, U128_MAX, get_u128

CONT = -1
TRANSFER_FIELDS_EXISTS = [  # create_transfer_exists order (:1587-1606), codes 36..45, then 46
    ("flags", 36), ("debit_account_id", 37), ("credit_account_id", 38), ("amount", 39),
    ("user_data_128", 41), ("user_data_64", 42), ("user_data_32", 43), ("timeout", 44), ("code", 45)]
ACCOUNT_FIELDS_EXISTS = [  # create_account_exists order (:1450-1460), codes 15..20, then 21
    ("flags", 15), ("user_data_128", 16), ("user_data_64", 17), ("user_data_32", 18), ("ledger", 19),
    ("code", 20)]
U128_FIELDS = {"id", "debit_account_id", "credit_account_id", "amount", "pending_id", "user_data_128",
               "debits_pending", "debits_posted", "credits_pending", "credits_posted"}
HDR_A, HDR_B, HDR_C, CHUNK = 256, 64, 64, 1024
RV_DUP, RV_CAP, RV_OVF, RV_UNSUP, RV_HUGE = 1, 2, 4, 8, 16
RI_DUP = 0x40


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
    """create_transfer head and single-phase validation (:1465-1489); CONT if it passes. Returns
    (code, outside the class)."""
    if int(t["timestamp"]) != 0:
        return 3, False
    f = int(t["flags"])
    if f & 0xFFC0:
        return 4, False
    ident = field(t, "id")
    if ident == 0:
        return 5, False
    if ident == U128_MAX:
        return 6, False
    assert not f & 0x0C, "post/void: outside the modelled class"
    dr, cr = field(t, "debit_account_id"), field(t, "credit_account_id")
    if dr == 0:
        return 8, False
    if dr == U128_MAX:
        return 9, False
    if cr == 0:
        return 10, False
    if cr == U128_MAX:
        return 11, False
    if cr == dr:
        return 12, False
    if field(t, "pending_id") != 0:
        return 13, False
    if not f & 2 and int(t["timeout"]) != 0:
        return 17, False
    if not f & 0x30 and field(t, "amount") == 0:
        return 18, False
    if int(t["ledger"]) == 0:
        return 19, False
    if int(t["code"]) == 0:
        return 20, False
    return CONT, bool(f & 0x32)  # pending / balancing: valid, outside the class


def exists_code(ev, stored, fields, exists):
    for name, code in fields:
        if field(ev, name) != field(stored, name):
            return code
    return exists


def al16(x):
    return (x + 15) & ~15


def cap1(n, G):
    return 0 if n == 0 else al16(min(n // G + n // (8 * G) + 256, n))


def cap2(n, G, xfer):
    return 0 if (n == 0 or not xfer) else al16(min(2 * n // G + 2 * n // (8 * G) + 256, 2 * n))


class Layout:
    """csrc/route.h RtLayout and its block sizes."""

    def __init__(self, G, n_home, xfer):
        self.G, self.n, self.xfer = G, list(n_home), xfer
        self.c1 = [cap1(n, G) for n in n_home]
        self.c2 = [cap2(n, G, xfer) for n in n_home]

    def blk_a(self, s):
        return HDR_A + self.c1[s] * 128 + self.c2[s] * 32

    def b_side(self, s):
        return HDR_B + al16(self.c1[s])

    def blk_b(self, s):
        return self.b_side(s) + self.c2[s] * 8

    def nch(self, s):
        return (self.c1[s] + CHUNK - 1) // CHUNK

    def c_hdr(self, s):
        return HDR_C + al16(4 * self.nch(s))

    def c_side(self, s):
        return self.c_hdr(s) + al16(self.c1[s])

    def blk_c(self, s):
        return self.c_side(s) + al16(self.c2[s])


class ShardModel:
    def __init__(self, G, me):
        self.G, self.me = G, me
        self.accounts = {}   # id -> stored record (owned), in insertion (= timestamp) order
        self.transfers = {}  # id -> stored record (owned)
        self.x_id_max = 0

    def owner(self, rec, name):
        return int(shard_of(rec[name + "_lo"], rec[name + "_hi"], self.G))

    # ---- route (home) ---------------------------------------------------------------------------
    def route(self, op, batches, timestamps, bounds):
        """batches: the whole window (the model only reads its home batches); timestamps: per batch.
        Returns the A send blocks (one bytes object per destination)."""
        G, me = self.G, self.me
        n_home = [sum(len(batches[b]) for b in range(bounds[s], bounds[s + 1])) for s in range(G)]
        L = Layout(G, n_home, op == "t")
        self.L, self.op = L, op
        home = [(b, j) for b in range(bounds[me], bounds[me + 1]) for j in range(len(batches[b]))]
        self.home = home
        self.batches, self.bounds = batches, bounds
        ids, sides = [[] for _ in range(G)], [[] for _ in range(G)]
        self.static, self.pos, self.ledger, verdict, nonmono = [], [], [], 0, False
        prev = None
        for (b, j) in home:
            ev = batches[b][j]
            T = timestamps[b]
            rec = ev.copy()
            rec["timestamp"] = T - len(batches[b]) + j + 1
            if op == "a":
                code, unsup = ca_static(ev), False
            else:
                code, unsup = ct_static(ev)
                if prev is not None and not field(ev, "id") > prev:
                    nonmono = True
                prev = field(ev, "id")
            if unsup:
                verdict |= RV_UNSUP
            self.static.append(code)
            self.ledger.append(int(ev["ledger"]))
            if code != CONT:
                self.pos.append(None)
                continue
            if op == "t" and field(ev, "amount") >> 64:
                verdict |= RV_HUGE
            o_id = self.owner(ev, "id")
            k_id = len(ids[o_id])
            ids[o_id].append(rec.tobytes())
            if op == "a":
                self.pos.append((o_id, k_id))
                continue
            amount = field(ev, "amount") & (2**64 - 1)
            o_dr, o_cr = self.owner(ev, "debit_account_id"), self.owner(ev, "credit_account_id")
            k_dr = len(sides[o_dr])
            sides[o_dr].append(struct.pack("<QQQII", int(ev["debit_account_id_lo"]), int(ev["debit_account_id_hi"]),
                                           amount, 0, 0))
            k_cr = len(sides[o_cr])
            sides[o_cr].append(struct.pack("<QQQII", int(ev["credit_account_id_lo"]), int(ev["credit_account_id_hi"]),
                                           amount, 1, 0))
            self.pos.append((o_id, k_id, o_dr, k_dr, o_cr, k_cr))
        E = len(home)
        first = batches[home[0][0]][home[0][1]] if E else None
        last = batches[home[-1][0]][home[-1][1]] if E else None
        out = []
        for d in range(G):
            if len(ids[d]) > L.c1[me] or len(sides[d]) > L.c2[me]:
                verdict |= RV_CAP
            blk = bytearray(L.blk_a(me))
            flags = (1 if nonmono else 0) | (2 if E else 0)
            fl = (int(first["id_lo"]), int(first["id_hi"])) if E else (0, 0)
            ll = (int(last["id_lo"]), int(last["id_hi"])) if E else (0, 0)
            struct.pack_into("<IIII4Q", blk, 0, min(len(ids[d]), L.c1[me]), min(len(sides[d]), L.c2[me]), E, flags,
                             *fl, *ll)
            for k, r in enumerate(ids[d][: L.c1[me]]):
                blk[HDR_A + k * 128: HDR_A + (k + 1) * 128] = r
            s0 = HDR_A + L.c1[me] * 128
            for k, m in enumerate(sides[d][: L.c2[me]]):
                blk[s0 + k * 32: s0 + (k + 1) * 32] = m
            out.append(bytes(blk))
        self.home_verdict = verdict
        return out

    # ---- own (owner) ----------------------------------------------------------------------------
    def own(self, recv_a):
        """recv_a: one A block per source shard. Returns the B send blocks (one per home)."""
        G, L, xfer = self.G, self.L, self.op == "t"
        hdr = [struct.unpack_from("<IIII4Q", recv_a[s], 0) for s in range(G)]
        mono, last, first, any_ = True, None, None, False
        for h in hdr:
            if not h[3] & 2:
                continue
            if h[3] & 1:
                mono = False
            f, l = h[4] | (h[5] << 64), h[6] | (h[7] << 64)
            if any_ and not f > last:
                mono = False
            if not any_:
                first = f
            any_, last = True, l
        claim = (not xfer) or not mono
        self.recv_a, self.hdr = recv_a, hdr
        nid, nside = sum(h[0] for h in hdr), sum(h[1] for h in hdr)
        verdict = 0
        stored = self.transfers if xfer else self.accounts
        if nid > 10**12:  # (the model's stores are unbounded: no capacity verdict)
            verdict |= RV_CAP
        seen = set()
        out = []
        self.slots = {}
        for s in range(G):
            blk = bytearray(L.blk_b(s))
            struct.pack_into("<I", blk, 0, verdict)
            for k in range(hdr[s][0]):
                raw = recv_a[s][HDR_A + k * 128: HDR_A + (k + 1) * 128]
                ev = np.frombuffer(raw, TRANSFER_DTYPE if xfer else ACCOUNT_DTYPE)[0]
                ident = field(ev, "id")
                dup = False
                if claim:
                    dup = ident in seen
                    seen.add(ident)
                st = stored.get(ident)
                if st is None:
                    code = 0
                elif xfer:
                    code = exists_code(ev, st, TRANSFER_FIELDS_EXISTS, 46)
                else:
                    code = exists_code(ev, st, ACCOUNT_FIELDS_EXISTS, 21)
                blk[HDR_B + k] = (1 + code) | (RI_DUP if dup else 0)
            for k in range(hdr[s][1]):
                o = HDR_A + L.c1[s] * 128 + k * 32
                lo, hi, amount, side, _ = struct.unpack_from("<QQQII", recv_a[s], o)
                acc = self.accounts.get(lo | (hi << 64))
                st, ledger = 0, 0
                if acc is not None:
                    st, ledger = 1, int(acc["ledger"])
                    lim = 4 if side else 2
                    if int(acc["flags"]) & (lim | 8):
                        st |= 2
                struct.pack_into("<II", blk, L.b_side(s) + k * 8, ledger, st)
            out.append(bytes(blk))
        self.prefix = mono and nid and first is not None and first > self.x_id_max
        return out

    # ---- decide (home) --------------------------------------------------------------------------
    def decide(self, recv_b):
        """recv_b: one B block per owner. Returns (per home batch the reply bytes, the C send blocks)."""
        G, L, me, xfer = self.G, self.L, self.me, self.op == "t"
        verdict = self.home_verdict
        for o in range(G):
            verdict |= struct.unpack_from("<I", recv_b[o], 0)[0]
        codes, lim = [], []
        for i, code in enumerate(self.static):
            li = False
            if code == CONT:
                p = self.pos[i]
                idr = recv_b[p[0]][HDR_B + p[1]]
                if idr & RI_DUP:
                    verdict |= RV_DUP
                idcode = (idr & 0x3F) - 1
                if not xfer:
                    code = idcode
                else:
                    dl, ds = struct.unpack_from("<II", recv_b[p[2]], L.b_side(me) + p[3] * 8)
                    cl, cs = struct.unpack_from("<II", recv_b[p[4]], L.b_side(me) + p[5] * 8)
                    if not ds & 1:
                        code = 21
                    elif not cs & 1:
                        code = 22
                    elif dl != cl:
                        code = 23
                    elif self.ledger[i] != dl:
                        code = 24
                    else:
                        code = idcode
                        li = bool((ds | cs) & 2)
            codes.append(code)
            lim.append(li)
        # linked chains (:1240-1300) per home batch: first failure back-fills, open chain at batch end
        commit = [False] * len(codes)
        replies = []
        i = 0
        for b in range(self.bounds[me], self.bounds[me + 1]):
            ev = self.batches[b]
            n = len(ev)
            c = codes[i: i + n]
            j = 0
            while j < n:
                if not int(ev[j]["flags"]) & 1:
                    j += 1
                    continue
                e = j
                while e < n - 1 and int(ev[e]["flags"]) & 1:
                    e += 1
                if int(ev[e]["flags"]) & 1:
                    c[e] = 2  # linked_event_chain_open
                f = next((k for k in range(j, e + 1) if c[k] != 0), None)
                if f is not None:
                    for k in range(j, e + 1):
                        if k != f and not (k == e and c[e] == 2):
                            c[k] = 1
                j = e + 1
            for j in range(n):
                commit[i + j] = c[j] == 0
                if c[j] == 0 and xfer and lim[i + j]:
                    verdict |= RV_UNSUP
            replies.append(np.array([(j, c[j]) for j in range(n) if c[j] != 0], np.uint32).reshape(-1, 2).tobytes())
            i += n
        out = [bytearray(L.blk_c(me)) for _ in range(G)]
        for d in range(G):
            struct.pack_into("<I", out[d], 0, verdict)
        for i, p in enumerate(self.pos):
            if p is None:
                continue
            cb = 1 if commit[i] else 0
            out[p[0]][L.c_hdr(me) + p[1]] = cb
            if cb:
                o = HDR_C + 4 * (p[1] // CHUNK)
                struct.pack_into("<I", out[p[0]], o, struct.unpack_from("<I", out[p[0]], o)[0] + 1)
            if xfer:
                out[p[2]][L.c_side(me) + p[3]] = cb
                out[p[4]][L.c_side(me) + p[5]] = cb
        return replies, [bytes(x) for x in out]

    # ---- apply (owners) -------------------------------------------------------------------------
    def apply(self, recv_c):
        """recv_c: one C block per home. Returns the global verdict (nothing applied when set)."""
        G, L, xfer = self.G, self.L, self.op == "t"
        verdict = 0
        for s in range(G):
            verdict |= struct.unpack_from("<I", recv_c[s], 0)[0]
        if verdict:
            return verdict
        for s in range(G):
            for k in range(self.hdr[s][1]):
                if not recv_c[s][L.c_side(s) + k]:
                    continue
                o = HDR_A + L.c1[s] * 128 + k * 32
                lo, hi, amount, side, _ = struct.unpack_from("<QQQII", self.recv_a[s], o)
                acc = self.accounts[lo | (hi << 64)]
                bal = "credits_posted" if side else "debits_posted"
                v = field(acc, bal) + amount
                acc[bal + "_lo"] = v & (2**64 - 1)
                acc[bal + "_hi"] = v >> 64
        for s in range(G):
            for k in range(self.hdr[s][0]):
                if not recv_c[s][L.c_hdr(s) + k]:
                    continue
                raw = self.recv_a[s][HDR_A + k * 128: HDR_A + (k + 1) * 128]
                rec = np.frombuffer(raw, TRANSFER_DTYPE if xfer else ACCOUNT_DTYPE)[0].copy()
                ident = field(rec, "id")
                if xfer:
                    self.transfers[ident] = rec
                    self.x_id_max = max(self.x_id_max, ident)
                else:
                    self.accounts[ident] = rec
        return 0
