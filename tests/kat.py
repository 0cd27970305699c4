"""Table-driven known-answer tests: parser + harness.

`parse()` mirrors the reference table parser (src/testing/table.zig:8-93): whitespace-separated
columns, `_` = field default, a leading letter on an integer is a comment (`A1` -> 1), a leading
`-n` on an unsigned integer means `maxInt - n`, and a trailing `// ...` is a comment.

`check()` mirrors the harness `check()` (src/state_machine.zig:2507-2765): rows accumulate a
request and the expected reply; `commit <operation>` bumps `prepare_timestamp` by one, calls
`prepare()`, runs a pulse first when `pulse()` says so (same timestamp), executes the operation at
`prepare_timestamp` and compares the reply bytes exactly.

The state machine under test is any object exposing the StateMachine boundary:
`prepare_timestamp`, `prepare(operation, input)`, `pulse()`, `prefetch(op, operation, input)`,
`commit(client, op, timestamp, operation, input) -> bytes`, plus the test hook
`setup_balances(id, dp, dpo, cp, cpo)` (the harness `setup` action, :2545-2561).
"""
import numpy as np

from tigerbeetle_amd.types import (
    ACCOUNT_DTYPE,
    BALANCE_DTYPE,
    FILTER_CREDITS,
    FILTER_DEBITS,
    FILTER_DTYPE,
    FILTER_REVERSED,
    RESULT_DTYPE,
    TRANSFER_DTYPE,
    U64_MAX,
    U128_MAX,
    CreateAccountResult,
    CreateTransferResult,
    Operation,
    set_u128,
)

# Column schemas: (name, kind, default). kind: int bit width, or ("opt", token), or "result".
ACCOUNT_COLUMNS = [
    ("id", 128, None), ("debits_pending", 128, 0), ("debits_posted", 128, 0),
    ("credits_pending", 128, 0), ("credits_posted", 128, 0), ("user_data_128", 128, 0),
    ("user_data_64", 64, 0), ("user_data_32", 32, 0), ("reserved", 1, 0), ("ledger", 32, None),
    ("code", 16, None), ("flags_linked", ("opt", "LNK"), None),
    ("flags_debits_must_not_exceed_credits", ("opt", "D<C"), None),
    ("flags_credits_must_not_exceed_debits", ("opt", "C<D"), None),
    ("flags_history", ("opt", "HIST"), None), ("flags_padding", 12, 0), ("timestamp", 64, 0),
    ("result", ("enum", CreateAccountResult), None),
]  # TestCreateAccount, state_machine.zig:2349-2392

TRANSFER_COLUMNS = [
    ("id", 128, None), ("debit_account_id", 128, None), ("credit_account_id", 128, None),
    ("amount", 128, 0), ("pending_id", 128, 0), ("user_data_128", 128, 0), ("user_data_64", 64, 0),
    ("user_data_32", 32, 0), ("timeout", 32, 0), ("ledger", 32, None), ("code", 16, None),
    ("flags_linked", ("opt", "LNK"), None), ("flags_pending", ("opt", "PEN"), None),
    ("flags_post_pending_transfer", ("opt", "POS"), None),
    ("flags_void_pending_transfer", ("opt", "VOI"), None),
    ("flags_balancing_debit", ("opt", "BDR"), None), ("flags_balancing_credit", ("opt", "BCR"), None),
    ("flags_padding", 7, 0), ("timestamp", 64, 0),
    ("result", ("enum", CreateTransferResult), None),
]  # TestCreateTransfer, state_machine.zig:2394-2441

RESULT_TRANSFER_COLUMNS = TRANSFER_COLUMNS[:-1]  # TestGetAccountTransfersResult, state_machine.zig:2459-2500

FILTER_COLUMNS = [
    ("account_id", 128, None), ("timestamp_min_transfer_id", ("nint", 128), None),
    ("timestamp_max_transfer_id", ("nint", 128), None), ("limit", 32, None),
    ("flags_debits", ("opt", "DR"), None), ("flags_credits", ("opt", "CR"), None),
    ("flags_reversed", ("opt", "REV"), None),
]  # TestAccountFilter, state_machine.zig:2443-2457

REQUIRED = object()


def _int(token, bits):
    off = 1 if token[0].isalpha() else 0
    mx = (1 << bits) - 1
    if token[off] == "-":
        return mx - int(token[off + 1:])
    return int(token[off:])


def _parse_struct(columns, tokens):
    row = {}
    for name, kind, default in columns:
        has_default = not (default is None and not (isinstance(kind, tuple) and kind[0] in ("opt", "nint")))
        if has_default and tokens and tokens[0] == "_":
            tokens.pop(0)
            row[name] = default
            continue
        tok = tokens.pop(0)
        if isinstance(kind, int):
            row[name] = _int(tok, kind)
        elif kind[0] == "opt":
            assert tok == kind[1], (name, tok)
            row[name] = True
        elif kind[0] == "nint":  # an optional integer: `_` = null
            row[name] = _int(tok, kind[1])
        elif kind[0] == "enum":
            row[name] = kind[1][tok]
    return row


def parse(table):
    """Returns a list of (action, payload) tuples."""
    actions = []
    for raw in table.split("\n"):
        line = raw.strip()
        if not line or line.startswith("#"):
            continue
        tokens = line.split()
        if "//" in tokens:
            tokens = tokens[: tokens.index("//")]
        kind = tokens.pop(0)
        if kind == "account":
            actions.append(("account", _parse_struct(ACCOUNT_COLUMNS, tokens)))
        elif kind == "transfer":
            actions.append(("transfer", _parse_struct(TRANSFER_COLUMNS, tokens)))
        elif kind == "setup":
            vals = [_int(t, 128) for t in tokens[:5]]
            tokens = tokens[5:]
            actions.append(("setup", vals))
        elif kind == "tick":
            value = int(tokens.pop(0))
            unit = tokens.pop(0)
            assert unit == "seconds"
            actions.append(("tick", value))
        elif kind == "commit":
            actions.append(("commit", Operation[tokens.pop(0)]))
        elif kind == "lookup_account":
            ident = _int(tokens.pop(0), 128)
            if tokens[0] == "_":
                tokens.pop(0)
                bal = None
            else:
                bal = [_int(tokens.pop(0), 128) for _ in range(4)]
            actions.append(("lookup_account", (ident, bal)))
        elif kind == "lookup_transfer":
            ident = _int(tokens.pop(0), 128)
            variant = tokens.pop(0)
            tok = tokens.pop(0)
            if variant == "exists":
                val = tok in ("1", "true", "T")
                assert val or tok in ("0", "false", "F")
            else:
                assert variant == "amount"
                val = _int(tok, 128)
            actions.append(("lookup_transfer", (ident, variant, val)))
        elif kind in ("get_account_transfers", "get_account_balances"):
            actions.append((kind, _parse_struct(FILTER_COLUMNS, tokens)))
        elif kind == "get_account_transfers_result":
            actions.append((kind, _parse_struct(RESULT_TRANSFER_COLUMNS, tokens)))
        elif kind == "get_account_balances_result":
            actions.append((kind, [_int(tokens.pop(0), 128) for _ in range(5)]))
        else:
            raise ValueError("unsupported row: " + line)
        assert not tokens, ("trailing tokens", line, tokens)
    return actions


def account_record(a, timestamp=None):
    """TestCreateAccount.event (state_machine.zig:2369-2391)."""
    r = np.zeros(1, ACCOUNT_DTYPE)
    for f in ("id", "debits_pending", "debits_posted", "credits_pending", "credits_posted", "user_data_128"):
        set_u128(r[0], f, a[f])
    r[0]["user_data_64"] = a["user_data_64"]
    r[0]["user_data_32"] = a["user_data_32"]
    r[0]["reserved"] = a["reserved"]
    r[0]["ledger"] = a["ledger"]
    r[0]["code"] = a["code"]
    flags = (
        (1 if a["flags_linked"] else 0)
        | (2 if a["flags_debits_must_not_exceed_credits"] else 0)
        | (4 if a["flags_credits_must_not_exceed_debits"] else 0)
        | (8 if a["flags_history"] else 0)
        | (a["flags_padding"] << 4)
    )
    r[0]["flags"] = flags
    r[0]["timestamp"] = a["timestamp"] if timestamp is None else timestamp
    return r


def transfer_record(t, timestamp=None):
    """TestCreateTransfer.event (state_machine.zig:2416-2440)."""
    r = np.zeros(1, TRANSFER_DTYPE)
    for f in ("id", "debit_account_id", "credit_account_id", "amount", "pending_id", "user_data_128"):
        set_u128(r[0], f, t[f])
    for f in ("user_data_64", "user_data_32", "timeout", "ledger", "code"):
        r[0][f] = t[f]
    flags = (
        (1 if t["flags_linked"] else 0)
        | (2 if t["flags_pending"] else 0)
        | (4 if t["flags_post_pending_transfer"] else 0)
        | (8 if t["flags_void_pending_transfer"] else 0)
        | (16 if t["flags_balancing_debit"] else 0)
        | (32 if t["flags_balancing_credit"] else 0)
        | (t["flags_padding"] << 6)
    )
    r[0]["flags"] = flags
    r[0]["timestamp"] = t["timestamp"] if timestamp is None else timestamp
    return r


def _execute(sm, op, operation, request):
    """TestContext.execute (state_machine.zig:2270-2297)."""
    timestamp = sm.prepare_timestamp
    sm.prefetch_timestamp = timestamp
    sm.prefetch(op, operation, request)
    return sm.commit(0, 1, timestamp, operation, request)


def check(sm, table):
    """Run one KAT table against state machine `sm`; raises AssertionError on any mismatch."""
    accounts, transfers = {}, {}
    request, reply = [], []
    op = 1
    operation = None
    n_events = 0
    for action, p in parse(table):
        if action == "setup":
            assert operation is None
            sm.setup_balances(*p)
        elif action == "tick":
            interval = abs(p) * 1_000_000_000
            sm.prepare_timestamp = (sm.prepare_timestamp + (interval if p > 0 else U64_MAX - interval)) & U64_MAX
        elif action == "account":
            assert operation in (None, Operation.create_accounts)
            operation = Operation.create_accounts
            request.append(account_record(p).tobytes())
            n_events += 1
            if p["result"] == CreateAccountResult.ok:
                ts = sm.prepare_timestamp + 1 + n_events
                accounts[p["id"]] = account_record(p, ts if p["timestamp"] == 0 else None)
            else:
                reply.append(np.array([(n_events - 1, int(p["result"]))], RESULT_DTYPE).tobytes())
        elif action == "transfer":
            assert operation in (None, Operation.create_transfers)
            operation = Operation.create_transfers
            request.append(transfer_record(p).tobytes())
            n_events += 1
            if p["result"] == CreateTransferResult.ok:
                ts = sm.prepare_timestamp + 1 + n_events
                transfers[p["id"]] = transfer_record(p, ts if p["timestamp"] == 0 else None)
            else:
                reply.append(np.array([(n_events - 1, int(p["result"]))], RESULT_DTYPE).tobytes())
        elif action == "lookup_account":
            assert operation in (None, Operation.lookup_accounts)
            operation = Operation.lookup_accounts
            ident, bal = p
            request.append(ident.to_bytes(16, "little"))
            if bal is not None:
                rec = accounts[ident].copy()
                for f, v in zip(("debits_pending", "debits_posted", "credits_pending", "credits_posted"), bal):
                    set_u128(rec[0], f, v)
                reply.append(rec.tobytes())
        elif action == "lookup_transfer":
            assert operation in (None, Operation.lookup_transfers)
            operation = Operation.lookup_transfers
            ident, variant, val = p
            request.append(ident.to_bytes(16, "little"))
            if variant == "exists":
                if val:
                    reply.append(transfers[ident].tobytes())
            else:
                rec = transfers[ident].copy()
                set_u128(rec[0], "amount", val)
                reply.append(rec.tobytes())
        elif action in ("get_account_transfers", "get_account_balances"):
            # state_machine.zig:2648-2700: timestamp bounds name a transfer whose timestamp they take
            op_q = Operation[action]
            assert operation in (None, op_q)
            operation = op_q
            f = np.zeros(1, FILTER_DTYPE)
            set_u128(f[0], "account_id", p["account_id"])
            for key, col in (("timestamp_min_transfer_id", "timestamp_min"),
                             ("timestamp_max_transfer_id", "timestamp_max")):
                f[0][col] = 0 if p[key] is None else int(transfers[p[key]][0]["timestamp"])
            f[0]["limit"] = p["limit"]
            f[0]["flags"] = ((FILTER_DEBITS if p["flags_debits"] else 0) | (FILTER_CREDITS if p["flags_credits"] else 0)
                             | (FILTER_REVERSED if p["flags_reversed"] else 0))
            request.append(f.tobytes())
        elif action == "get_account_transfers_result":
            assert operation == Operation.get_account_transfers
            reply.append(transfer_record(p, int(transfers[p["id"]][0]["timestamp"])).tobytes())
        elif action == "get_account_balances_result":
            assert operation == Operation.get_account_balances
            b = np.zeros(1, BALANCE_DTYPE)
            for f_, v in zip(("debits_pending", "debits_posted", "credits_pending", "credits_posted"), p[1:]):
                set_u128(b[0], f_, v)
            b[0]["timestamp"] = transfers[p[0]][0]["timestamp"]
            reply.append(b.tobytes())
        elif action == "commit":
            assert operation in (None, p)
            req = b"".join(request)
            sm.prepare_timestamp += 1
            sm.prepare(p, req)
            if sm.pulse():
                size = len(_execute(sm, op, Operation.pulse, b""))
                assert size == 0
                op += 1
            actual = _execute(sm, op, p, req)
            expected = b"".join(reply)
            if actual != expected:
                raise AssertionError(_diff(p, expected, actual))
            request, reply = [], []
            operation = None
            n_events = 0
            op += 1
    assert operation is None and not request and not reply


def _diff(operation, expected, actual):
    if operation in (Operation.create_accounts, Operation.create_transfers):
        e = np.frombuffer(expected, RESULT_DTYPE).tolist()
        a = np.frombuffer(actual, RESULT_DTYPE).tolist()
        return f"{operation.name}: expected {e}\n actual {a}"
    dt = {Operation.lookup_accounts: ACCOUNT_DTYPE, Operation.get_account_balances: BALANCE_DTYPE}.get(
        operation, TRANSFER_DTYPE)
    e = np.frombuffer(expected, dt)
    a = np.frombuffer(actual, dt)
    return f"{operation.name}: expected {len(e)} records\n{e}\n actual {len(a)} records\n{a}"
