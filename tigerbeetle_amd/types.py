"""Wire records and result codes (mirrors include/tb_types.h).

Layouts follow the reference extern structs byte for byte: Account (src/tigerbeetle.zig:7-40),
Transfer (:80-111), Create*sResult (:267-285). u128 fields are two little-endian u64 words
(`<name>_lo`, `<name>_hi`) so numpy can hold them; helpers convert to/from Python ints.
"""
import enum

import numpy as np

U128_MAX = (1 << 128) - 1
U64_MAX = (1 << 64) - 1
BATCH_MAX = 8190  # state_machine.zig:58-81 with message_body_size_max = 1 MiB - 256 B
NS_PER_S = 1_000_000_000
TIMESTAMP_MIN = 1
TIMESTAMP_MAX = U64_MAX - 1


def _u128(name):
    return [(name + "_lo", "<u8"), (name + "_hi", "<u8")]


ACCOUNT_DTYPE = np.dtype(
    _u128("id") + _u128("debits_pending") + _u128("debits_posted") + _u128("credits_pending")
    + _u128("credits_posted") + _u128("user_data_128")
    + [("user_data_64", "<u8"), ("user_data_32", "<u4"), ("reserved", "<u4"), ("ledger", "<u4"),
       ("code", "<u2"), ("flags", "<u2"), ("timestamp", "<u8")]
)
TRANSFER_DTYPE = np.dtype(
    _u128("id") + _u128("debit_account_id") + _u128("credit_account_id") + _u128("amount")
    + _u128("pending_id") + _u128("user_data_128")
    + [("user_data_64", "<u8"), ("user_data_32", "<u4"), ("timeout", "<u4"), ("ledger", "<u4"),
       ("code", "<u2"), ("flags", "<u2"), ("timestamp", "<u8")]
)
RESULT_DTYPE = np.dtype([("index", "<u4"), ("result", "<u4")])
# AccountFilter (tigerbeetle.zig:288-322) and AccountBalance (:65-78)
FILTER_DTYPE = np.dtype(_u128("account_id") + [("timestamp_min", "<u8"), ("timestamp_max", "<u8"),
                                               ("limit", "<u4"), ("flags", "<u4"), ("reserved", "u1", (24,))])
BALANCE_DTYPE = np.dtype(_u128("debits_pending") + _u128("debits_posted") + _u128("credits_pending")
                         + _u128("credits_posted") + [("timestamp", "<u8"), ("reserved", "u1", (56,))])
FILTER_DEBITS, FILTER_CREDITS, FILTER_REVERSED = 1, 2, 4
assert ACCOUNT_DTYPE.itemsize == 128 and TRANSFER_DTYPE.itemsize == 128 and RESULT_DTYPE.itemsize == 8
assert FILTER_DTYPE.itemsize == 64 and BALANCE_DTYPE.itemsize == 128


def set_u128(rec, name, value):
    rec[name + "_lo"] = value & U64_MAX
    rec[name + "_hi"] = (value >> 64) & U64_MAX


def get_u128(rec, name):
    return int(rec[name + "_lo"]) | (int(rec[name + "_hi"]) << 64)


class Operation(enum.IntEnum):
    """state_machine.zig:341-350 (vsr_operations_reserved = 128)."""
    pulse = 128
    create_accounts = 129
    create_transfers = 130
    lookup_accounts = 131
    lookup_transfers = 132
    get_account_transfers = 133
    get_account_balances = 134


class AccountFlags(enum.IntFlag):
    """tigerbeetle.zig:42-63."""
    linked = 1 << 0
    debits_must_not_exceed_credits = 1 << 1
    credits_must_not_exceed_debits = 1 << 2
    history = 1 << 3


class TransferFlags(enum.IntFlag):
    """tigerbeetle.zig:127-140."""
    linked = 1 << 0
    pending = 1 << 1
    post_pending_transfer = 1 << 2
    void_pending_transfer = 1 << 3
    balancing_debit = 1 << 4
    balancing_credit = 1 << 5


class TransferPendingStatus(enum.IntEnum):
    """tigerbeetle.zig:113-125."""
    none = 0
    pending = 1
    posted = 2
    voided = 3
    expired = 4


class CreateAccountResult(enum.IntEnum):
    """tigerbeetle.zig:145-180."""
    ok = 0
    linked_event_failed = 1
    linked_event_chain_open = 2
    timestamp_must_be_zero = 3
    reserved_field = 4
    reserved_flag = 5
    id_must_not_be_zero = 6
    id_must_not_be_int_max = 7
    flags_are_mutually_exclusive = 8
    debits_pending_must_be_zero = 9
    debits_posted_must_be_zero = 10
    credits_pending_must_be_zero = 11
    credits_posted_must_be_zero = 12
    ledger_must_not_be_zero = 13
    code_must_not_be_zero = 14
    exists_with_different_flags = 15
    exists_with_different_user_data_128 = 16
    exists_with_different_user_data_64 = 17
    exists_with_different_user_data_32 = 18
    exists_with_different_ledger = 19
    exists_with_different_code = 20
    exists = 21


class CreateTransferResult(enum.IntEnum):
    """tigerbeetle.zig:185-265."""
    ok = 0
    linked_event_failed = 1
    linked_event_chain_open = 2
    timestamp_must_be_zero = 3
    reserved_flag = 4
    id_must_not_be_zero = 5
    id_must_not_be_int_max = 6
    flags_are_mutually_exclusive = 7
    debit_account_id_must_not_be_zero = 8
    debit_account_id_must_not_be_int_max = 9
    credit_account_id_must_not_be_zero = 10
    credit_account_id_must_not_be_int_max = 11
    accounts_must_be_different = 12
    pending_id_must_be_zero = 13
    pending_id_must_not_be_zero = 14
    pending_id_must_not_be_int_max = 15
    pending_id_must_be_different = 16
    timeout_reserved_for_pending_transfer = 17
    amount_must_not_be_zero = 18
    ledger_must_not_be_zero = 19
    code_must_not_be_zero = 20
    debit_account_not_found = 21
    credit_account_not_found = 22
    accounts_must_have_the_same_ledger = 23
    transfer_must_have_the_same_ledger_as_accounts = 24
    pending_transfer_not_found = 25
    pending_transfer_not_pending = 26
    pending_transfer_has_different_debit_account_id = 27
    pending_transfer_has_different_credit_account_id = 28
    pending_transfer_has_different_ledger = 29
    pending_transfer_has_different_code = 30
    exceeds_pending_transfer_amount = 31
    pending_transfer_has_different_amount = 32
    pending_transfer_already_posted = 33
    pending_transfer_already_voided = 34
    pending_transfer_expired = 35
    exists_with_different_flags = 36
    exists_with_different_debit_account_id = 37
    exists_with_different_credit_account_id = 38
    exists_with_different_amount = 39
    exists_with_different_pending_id = 40
    exists_with_different_user_data_128 = 41
    exists_with_different_user_data_64 = 42
    exists_with_different_user_data_32 = 43
    exists_with_different_timeout = 44
    exists_with_different_code = 45
    exists = 46
    overflows_debits_pending = 47
    overflows_credits_pending = 48
    overflows_debits_posted = 49
    overflows_credits_posted = 50
    overflows_debits = 51
    overflows_credits = 52
    overflows_timeout = 53
    exceeds_credits = 54
    exceeds_debits = 55
