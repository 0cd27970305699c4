/*
 * tb_types.h — TigerBeetle wire records and result codes, as plain C.
 *
 * Byte-for-byte the layout of the reference's extern structs (little-endian, 16-B aligned):
 *   Account                 reference src/tigerbeetle.zig:7-40      (128 B)
 *   AccountFlags            reference src/tigerbeetle.zig:42-63     (u16 bitfield)
 *   Transfer                reference src/tigerbeetle.zig:80-111    (128 B)
 *   TransferFlags           reference src/tigerbeetle.zig:127-140   (u16 bitfield)
 *   TransferPendingStatus   reference src/tigerbeetle.zig:113-125
 *   CreateAccountResult     reference src/tigerbeetle.zig:145-180
 *   CreateTransferResult    reference src/tigerbeetle.zig:185-265
 *   Create*sResult          reference src/tigerbeetle.zig:267-285   (8 B {index, result})
 *   Operation codes         reference src/state_machine.zig:341-350 (vsr_operations_reserved = 128)
 *
 * u128 fields are stored as {lo, hi} u64 pairs so the header is usable from C, C++ and HIP
 * without relying on __int128 in the ABI.
 */
#ifndef TB_TYPES_H
#define TB_TYPES_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tb_uint128 {
    uint64_t lo;
    uint64_t hi;
} tb_uint128_t;

typedef struct __attribute__((aligned(16))) tb_account {
    tb_uint128_t id;              /*   0 */
    tb_uint128_t debits_pending;  /*  16 */
    tb_uint128_t debits_posted;   /*  32 */
    tb_uint128_t credits_pending; /*  48 */
    tb_uint128_t credits_posted;  /*  64 */
    tb_uint128_t user_data_128;   /*  80 */
    uint64_t user_data_64;        /*  96 */
    uint32_t user_data_32;        /* 104 */
    uint32_t reserved;            /* 108 */
    uint32_t ledger;              /* 112 */
    uint16_t code;                /* 116 */
    uint16_t flags;               /* 118 */
    uint64_t timestamp;           /* 120 */
} tb_account_t;

typedef struct __attribute__((aligned(16))) tb_transfer {
    tb_uint128_t id;                /*   0 */
    tb_uint128_t debit_account_id;  /*  16 */
    tb_uint128_t credit_account_id; /*  32 */
    tb_uint128_t amount;            /*  48 */
    tb_uint128_t pending_id;        /*  64 */
    tb_uint128_t user_data_128;     /*  80 */
    uint64_t user_data_64;          /*  96 */
    uint32_t user_data_32;          /* 104 */
    uint32_t timeout;               /* 108 */
    uint32_t ledger;                /* 112 */
    uint16_t code;                  /* 116 */
    uint16_t flags;                 /* 118 */
    uint64_t timestamp;             /* 120 */
} tb_transfer_t;

typedef struct tb_create_result {
    uint32_t index;
    uint32_t result;
} tb_create_result_t;

/* AccountFlags (tigerbeetle.zig:42-63). */
enum {
    TB_ACCOUNT_LINKED = 1u << 0,
    TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS = 1u << 1,
    TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS = 1u << 2,
    TB_ACCOUNT_HISTORY = 1u << 3,
    TB_ACCOUNT_PADDING_MASK = 0xFFF0u
};

/* TransferFlags (tigerbeetle.zig:127-140). */
enum {
    TB_TRANSFER_LINKED = 1u << 0,
    TB_TRANSFER_PENDING = 1u << 1,
    TB_TRANSFER_POST_PENDING = 1u << 2,
    TB_TRANSFER_VOID_PENDING = 1u << 3,
    TB_TRANSFER_BALANCING_DEBIT = 1u << 4,
    TB_TRANSFER_BALANCING_CREDIT = 1u << 5,
    TB_TRANSFER_PADDING_MASK = 0xFFC0u
};

/* TransferPendingStatus (tigerbeetle.zig:113-125). */
enum {
    TB_PENDING_NONE = 0,
    TB_PENDING_PENDING = 1,
    TB_PENDING_POSTED = 2,
    TB_PENDING_VOIDED = 3,
    TB_PENDING_EXPIRED = 4
};

/* TransferPending groove object (state_machine.zig:259-269): keyed by the pending transfer's
 * timestamp. 16 B. */
typedef struct tb_transfer_pending_t {
    uint64_t timestamp;
    uint8_t status;  /* TB_PENDING_* */
    uint8_t padding[7];
} tb_transfer_pending_t;

/* AccountFilter (tigerbeetle.zig:288-322): the input of get_account_transfers and
 * get_account_balances. 64 B. timestamp_min / timestamp_max 0 = unbounded (inclusive bounds). */
typedef struct __attribute__((aligned(16))) tb_account_filter {
    tb_uint128_t account_id; /*  0 */
    uint64_t timestamp_min;  /* 16 */
    uint64_t timestamp_max;  /* 24 */
    uint32_t limit;          /* 32 */
    uint32_t flags;          /* 36: TB_FILTER_* */
    uint8_t reserved[24];    /* 40 */
} tb_account_filter_t;

/* AccountFilterFlags (tigerbeetle.zig:309-322). */
enum {
    TB_FILTER_DEBITS = 1u << 0,
    TB_FILTER_CREDITS = 1u << 1,
    TB_FILTER_REVERSED = 1u << 2
};

/* AccountBalance (tigerbeetle.zig:65-78): one row of get_account_balances. 128 B. */
typedef struct __attribute__((aligned(16))) tb_account_balance {
    tb_uint128_t debits_pending;  /*  0 */
    tb_uint128_t debits_posted;   /* 16 */
    tb_uint128_t credits_pending; /* 32 */
    tb_uint128_t credits_posted;  /* 48 */
    uint64_t timestamp;           /* 64 */
    uint8_t reserved[56];         /* 72 */
} tb_account_balance_t;

/* AccountBalancesGrooveValue (state_machine.zig:296-315): the account_balances groove row that
 * historical_balance (:1806-1841) inserts, keyed by the transfer's timestamp; a side's account id is
 * 0 when that account has no flags.history. 256 B. */
typedef struct __attribute__((aligned(16))) tb_account_balances_value {
    tb_uint128_t dr_account_id;      /*   0 */
    tb_uint128_t dr_debits_pending;  /*  16 */
    tb_uint128_t dr_debits_posted;   /*  32 */
    tb_uint128_t dr_credits_pending; /*  48 */
    tb_uint128_t dr_credits_posted;  /*  64 */
    tb_uint128_t cr_account_id;      /*  80 */
    tb_uint128_t cr_debits_pending;  /*  96 */
    tb_uint128_t cr_debits_posted;   /* 112 */
    tb_uint128_t cr_credits_pending; /* 128 */
    tb_uint128_t cr_credits_posted;  /* 144 */
    uint64_t timestamp;              /* 160 */
    uint8_t reserved[88];            /* 168 */
} tb_account_balances_value_t;

/* Operation (state_machine.zig:341-350). */
enum {
    TB_OP_PULSE = 128,
    TB_OP_CREATE_ACCOUNTS = 129,
    TB_OP_CREATE_TRANSFERS = 130,
    TB_OP_LOOKUP_ACCOUNTS = 131,
    TB_OP_LOOKUP_TRANSFERS = 132,
    TB_OP_GET_ACCOUNT_TRANSFERS = 133,
    TB_OP_GET_ACCOUNT_BALANCES = 134
};

/* CreateAccountResult (tigerbeetle.zig:145-180). */
enum {
    TB_CA_OK = 0,
    TB_CA_LINKED_EVENT_FAILED = 1,
    TB_CA_LINKED_EVENT_CHAIN_OPEN = 2,
    TB_CA_TIMESTAMP_MUST_BE_ZERO = 3,
    TB_CA_RESERVED_FIELD = 4,
    TB_CA_RESERVED_FLAG = 5,
    TB_CA_ID_MUST_NOT_BE_ZERO = 6,
    TB_CA_ID_MUST_NOT_BE_INT_MAX = 7,
    TB_CA_FLAGS_ARE_MUTUALLY_EXCLUSIVE = 8,
    TB_CA_DEBITS_PENDING_MUST_BE_ZERO = 9,
    TB_CA_DEBITS_POSTED_MUST_BE_ZERO = 10,
    TB_CA_CREDITS_PENDING_MUST_BE_ZERO = 11,
    TB_CA_CREDITS_POSTED_MUST_BE_ZERO = 12,
    TB_CA_LEDGER_MUST_NOT_BE_ZERO = 13,
    TB_CA_CODE_MUST_NOT_BE_ZERO = 14,
    TB_CA_EXISTS_WITH_DIFFERENT_FLAGS = 15,
    TB_CA_EXISTS_WITH_DIFFERENT_USER_DATA_128 = 16,
    TB_CA_EXISTS_WITH_DIFFERENT_USER_DATA_64 = 17,
    TB_CA_EXISTS_WITH_DIFFERENT_USER_DATA_32 = 18,
    TB_CA_EXISTS_WITH_DIFFERENT_LEDGER = 19,
    TB_CA_EXISTS_WITH_DIFFERENT_CODE = 20,
    TB_CA_EXISTS = 21
};

/* CreateTransferResult (tigerbeetle.zig:185-265). */
enum {
    TB_CT_OK = 0,
    TB_CT_LINKED_EVENT_FAILED = 1,
    TB_CT_LINKED_EVENT_CHAIN_OPEN = 2,
    TB_CT_TIMESTAMP_MUST_BE_ZERO = 3,
    TB_CT_RESERVED_FLAG = 4,
    TB_CT_ID_MUST_NOT_BE_ZERO = 5,
    TB_CT_ID_MUST_NOT_BE_INT_MAX = 6,
    TB_CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE = 7,
    TB_CT_DEBIT_ACCOUNT_ID_MUST_NOT_BE_ZERO = 8,
    TB_CT_DEBIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX = 9,
    TB_CT_CREDIT_ACCOUNT_ID_MUST_NOT_BE_ZERO = 10,
    TB_CT_CREDIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX = 11,
    TB_CT_ACCOUNTS_MUST_BE_DIFFERENT = 12,
    TB_CT_PENDING_ID_MUST_BE_ZERO = 13,
    TB_CT_PENDING_ID_MUST_NOT_BE_ZERO = 14,
    TB_CT_PENDING_ID_MUST_NOT_BE_INT_MAX = 15,
    TB_CT_PENDING_ID_MUST_BE_DIFFERENT = 16,
    TB_CT_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER = 17,
    TB_CT_AMOUNT_MUST_NOT_BE_ZERO = 18,
    TB_CT_LEDGER_MUST_NOT_BE_ZERO = 19,
    TB_CT_CODE_MUST_NOT_BE_ZERO = 20,
    TB_CT_DEBIT_ACCOUNT_NOT_FOUND = 21,
    TB_CT_CREDIT_ACCOUNT_NOT_FOUND = 22,
    TB_CT_ACCOUNTS_MUST_HAVE_THE_SAME_LEDGER = 23,
    TB_CT_TRANSFER_MUST_HAVE_THE_SAME_LEDGER_AS_ACCOUNTS = 24,
    TB_CT_PENDING_TRANSFER_NOT_FOUND = 25,
    TB_CT_PENDING_TRANSFER_NOT_PENDING = 26,
    TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_DEBIT_ACCOUNT_ID = 27,
    TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_CREDIT_ACCOUNT_ID = 28,
    TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_LEDGER = 29,
    TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_CODE = 30,
    TB_CT_EXCEEDS_PENDING_TRANSFER_AMOUNT = 31,
    TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_AMOUNT = 32,
    TB_CT_PENDING_TRANSFER_ALREADY_POSTED = 33,
    TB_CT_PENDING_TRANSFER_ALREADY_VOIDED = 34,
    TB_CT_PENDING_TRANSFER_EXPIRED = 35,
    TB_CT_EXISTS_WITH_DIFFERENT_FLAGS = 36,
    TB_CT_EXISTS_WITH_DIFFERENT_DEBIT_ACCOUNT_ID = 37,
    TB_CT_EXISTS_WITH_DIFFERENT_CREDIT_ACCOUNT_ID = 38,
    TB_CT_EXISTS_WITH_DIFFERENT_AMOUNT = 39,
    TB_CT_EXISTS_WITH_DIFFERENT_PENDING_ID = 40,
    TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_128 = 41,
    TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_64 = 42,
    TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_32 = 43,
    TB_CT_EXISTS_WITH_DIFFERENT_TIMEOUT = 44,
    TB_CT_EXISTS_WITH_DIFFERENT_CODE = 45,
    TB_CT_EXISTS = 46,
    TB_CT_OVERFLOWS_DEBITS_PENDING = 47,
    TB_CT_OVERFLOWS_CREDITS_PENDING = 48,
    TB_CT_OVERFLOWS_DEBITS_POSTED = 49,
    TB_CT_OVERFLOWS_CREDITS_POSTED = 50,
    TB_CT_OVERFLOWS_DEBITS = 51,
    TB_CT_OVERFLOWS_CREDITS = 52,
    TB_CT_OVERFLOWS_TIMEOUT = 53,
    TB_CT_EXCEEDS_CREDITS = 54,
    TB_CT_EXCEEDS_DEBITS = 55
};

/* message_body_size_max = message_size_max (1 MiB, config.zig:153) - header (256 B,
 * vsr/message_header.zig:72); batch_max = body / max(sizeof Event, sizeof Result)
 * (state_machine.zig:58-81) = 8190 for create_accounts / create_transfers. */
#define TB_MESSAGE_BODY_SIZE_MAX (1048576u - 256u)
#define TB_BATCH_MAX 8190u

#define TB_NS_PER_S 1000000000ull
/* TimestampRange (lsm/timestamp_range.zig:4-5). */
#define TB_TIMESTAMP_MIN 1ull
#define TB_TIMESTAMP_MAX 0xFFFFFFFFFFFFFFFEull

#ifdef __cplusplus
} /* extern "C" */

static_assert(sizeof(tb_account_t) == 128, "Account is 128 B");
static_assert(sizeof(tb_transfer_t) == 128, "Transfer is 128 B");
static_assert(sizeof(tb_create_result_t) == 8, "Create*sResult is 8 B");
static_assert(sizeof(tb_account_filter_t) == 64, "AccountFilter is 64 B");
static_assert(sizeof(tb_account_balance_t) == 128, "AccountBalance is 128 B");
static_assert(sizeof(tb_account_balances_value_t) == 256, "AccountBalancesGrooveValue is 256 B");
#else
_Static_assert(sizeof(tb_account_t) == 128, "Account is 128 B");
_Static_assert(sizeof(tb_transfer_t) == 128, "Transfer is 128 B");
_Static_assert(sizeof(tb_create_result_t) == 8, "Create*sResult is 8 B");
_Static_assert(sizeof(tb_account_filter_t) == 64, "AccountFilter is 64 B");
_Static_assert(sizeof(tb_account_balance_t) == 128, "AccountBalance is 128 B");
_Static_assert(sizeof(tb_account_balances_value_t) == 256, "AccountBalancesGrooveValue is 256 B");
#endif

#endif /* TB_TYPES_H */
