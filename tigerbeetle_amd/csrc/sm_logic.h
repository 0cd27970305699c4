// sm_logic.h — the reference's per-event decision logic, as stateless device functions.
//
// Each function restates one block of src/state_machine.zig in the reference's evaluation order
// (precedence is reproduced by evaluation order, never by min(enum)).
// They return a CreateTransferResult / CreateAccountResult code, or CONT to continue.
#pragma once
#include "dev_common.h"

// create_transfer head (state_machine.zig:1465-1468).
__device__ __attribute__((always_inline)) inline uint32_t ct_head(const tb_transfer_t& t) {
  if (t.flags & TB_TRANSFER_PADDING_MASK) return TB_CT_RESERVED_FLAG;
  const u128 id = U(t.id);
  if (id == 0) return TB_CT_ID_MUST_NOT_BE_ZERO;
  if (id == MAX128) return TB_CT_ID_MUST_NOT_BE_INT_MAX;
  return CONT;
}

// create_transfer field validation, single-phase/pending branch (:1474-1489).
__device__ __attribute__((always_inline)) inline uint32_t ct_validate(const tb_transfer_t& t) {
  const u128 dr = U(t.debit_account_id), cr = U(t.credit_account_id);
  if (dr == 0) return TB_CT_DEBIT_ACCOUNT_ID_MUST_NOT_BE_ZERO;
  if (dr == MAX128) return TB_CT_DEBIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX;
  if (cr == 0) return TB_CT_CREDIT_ACCOUNT_ID_MUST_NOT_BE_ZERO;
  if (cr == MAX128) return TB_CT_CREDIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX;
  if (cr == dr) return TB_CT_ACCOUNTS_MUST_BE_DIFFERENT;
  if (U(t.pending_id) != 0) return TB_CT_PENDING_ID_MUST_BE_ZERO;
  if (!(t.flags & TB_TRANSFER_PENDING) && t.timeout != 0) return TB_CT_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER;
  if (!(t.flags & (TB_TRANSFER_BALANCING_DEBIT | TB_TRANSFER_BALANCING_CREDIT)) && U(t.amount) == 0)
    return TB_CT_AMOUNT_MUST_NOT_BE_ZERO;
  if (t.ledger == 0) return TB_CT_LEDGER_MUST_NOT_BE_ZERO;
  if (t.code == 0) return TB_CT_CODE_MUST_NOT_BE_ZERO;
  return CONT;
}

// Ledger checks once both accounts are found (:1503-1504).
__device__ __attribute__((always_inline)) inline uint32_t ct_ledgers(const tb_transfer_t& t, uint32_t dr_ledger, uint32_t cr_ledger) {
  if (dr_ledger != cr_ledger) return TB_CT_ACCOUNTS_MUST_HAVE_THE_SAME_LEDGER;
  if (t.ledger != dr_ledger) return TB_CT_TRANSFER_MUST_HAVE_THE_SAME_LEDGER_AS_ACCOUNTS;
  return CONT;
}

// create_transfer_exists (:1587-1606).
__device__ __attribute__((always_inline)) inline uint32_t ct_exists(const tb_transfer_t& t, const tb_transfer_t& e) {
  if (t.flags != e.flags) return TB_CT_EXISTS_WITH_DIFFERENT_FLAGS;
  if (U(t.debit_account_id) != U(e.debit_account_id)) return TB_CT_EXISTS_WITH_DIFFERENT_DEBIT_ACCOUNT_ID;
  if (U(t.credit_account_id) != U(e.credit_account_id)) return TB_CT_EXISTS_WITH_DIFFERENT_CREDIT_ACCOUNT_ID;
  if (U(t.amount) != U(e.amount)) return TB_CT_EXISTS_WITH_DIFFERENT_AMOUNT;
  if (U(t.user_data_128) != U(e.user_data_128)) return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_128;
  if (t.user_data_64 != e.user_data_64) return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_64;
  if (t.user_data_32 != e.user_data_32) return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_32;
  if (t.timeout != e.timeout) return TB_CT_EXISTS_WITH_DIFFERENT_TIMEOUT;
  if (t.code != e.code) return TB_CT_EXISTS_WITH_DIFFERENT_CODE;
  return TB_CT_EXISTS;
}

// post_or_void_pending_transfer steps before the pending lookup (:1614-1624).
__device__ __attribute__((always_inline)) inline uint32_t pv_validate(const tb_transfer_t& t) {
  const uint16_t f = t.flags;
  if ((f & TB_TRANSFER_POST_PENDING) && (f & TB_TRANSFER_VOID_PENDING)) return TB_CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
  if (f & TB_TRANSFER_PENDING) return TB_CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
  if (f & TB_TRANSFER_BALANCING_DEBIT) return TB_CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
  if (f & TB_TRANSFER_BALANCING_CREDIT) return TB_CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
  const u128 pid = U(t.pending_id);
  if (pid == 0) return TB_CT_PENDING_ID_MUST_NOT_BE_ZERO;
  if (pid == MAX128) return TB_CT_PENDING_ID_MUST_NOT_BE_INT_MAX;
  if (pid == U(t.id)) return TB_CT_PENDING_ID_MUST_BE_DIFFERENT;
  if (t.timeout != 0) return TB_CT_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER;
  return CONT;
}

// Checks against the found pending transfer p, up to (excluding) the exists check (:1629-1654).
// Outputs the posted/voided amount.
__device__ __attribute__((always_inline)) inline uint32_t pv_against(const tb_transfer_t& t, const tb_transfer_t& p, u128* amount_out) {
  if (!(p.flags & TB_TRANSFER_PENDING)) return TB_CT_PENDING_TRANSFER_NOT_PENDING;
  const u128 tdr = U(t.debit_account_id), tcr = U(t.credit_account_id);
  if (tdr > 0 && tdr != U(p.debit_account_id)) return TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_DEBIT_ACCOUNT_ID;
  if (tcr > 0 && tcr != U(p.credit_account_id)) return TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_CREDIT_ACCOUNT_ID;
  if (t.ledger > 0 && t.ledger != p.ledger) return TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_LEDGER;
  if (t.code > 0 && t.code != p.code) return TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_CODE;
  const u128 pa = U(p.amount);
  const u128 amount = U(t.amount) > 0 ? U(t.amount) : pa;
  if (amount > pa) return TB_CT_EXCEEDS_PENDING_TRANSFER_AMOUNT;
  if ((t.flags & TB_TRANSFER_VOID_PENDING) && amount < pa) return TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_AMOUNT;
  *amount_out = amount;
  return CONT;
}

// post_or_void_pending_transfer_exists (:1743-1804).
__device__ __attribute__((always_inline)) inline uint32_t pv_exists(const tb_transfer_t& t, const tb_transfer_t& e, const tb_transfer_t& p) {
  if (t.flags != e.flags) return TB_CT_EXISTS_WITH_DIFFERENT_FLAGS;
  if (U(t.amount) == 0) {
    if (U(e.amount) != U(p.amount)) return TB_CT_EXISTS_WITH_DIFFERENT_AMOUNT;
  } else {
    if (U(t.amount) != U(e.amount)) return TB_CT_EXISTS_WITH_DIFFERENT_AMOUNT;
  }
  if (U(t.pending_id) != U(e.pending_id)) return TB_CT_EXISTS_WITH_DIFFERENT_PENDING_ID;
  if (U(t.user_data_128) == 0) {
    if (U(e.user_data_128) != U(p.user_data_128)) return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_128;
  } else if (U(t.user_data_128) != U(e.user_data_128)) {
    return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_128;
  }
  if (t.user_data_64 == 0) {
    if (e.user_data_64 != p.user_data_64) return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_64;
  } else if (t.user_data_64 != e.user_data_64) {
    return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_64;
  }
  if (t.user_data_32 == 0) {
    if (e.user_data_32 != p.user_data_32) return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_32;
  } else if (t.user_data_32 != e.user_data_32) {
    return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_32;
  }
  return TB_CT_EXISTS;
}

// Pending status switch (:1658-1670).
__device__ __attribute__((always_inline)) inline uint32_t pv_status(uint8_t status) {
  switch (status) {
    case TB_PENDING_POSTED: return TB_CT_PENDING_TRANSFER_ALREADY_POSTED;
    case TB_PENDING_VOIDED: return TB_CT_PENDING_TRANSFER_ALREADY_VOIDED;
    case TB_PENDING_EXPIRED: return TB_CT_PENDING_TRANSFER_EXPIRED;
    default: return CONT;
  }
}

// The posting/voiding transfer record that post_or_void inserts (:1672-1686).
__device__ __attribute__((always_inline)) inline tb_transfer_t pv_record(const tb_transfer_t& t, const tb_transfer_t& p, u128 amount) {
  tb_transfer_t t2;
  t2.id = t.id;
  t2.debit_account_id = p.debit_account_id;
  t2.credit_account_id = p.credit_account_id;
  // (selects on the 64-bit words: a select between the two struct members would be one between
  // their addresses, which keeps both records in scratch memory instead of registers)
  const bool own128 = (t.user_data_128.lo | t.user_data_128.hi) != 0;
  t2.user_data_128.lo = own128 ? t.user_data_128.lo : p.user_data_128.lo;
  t2.user_data_128.hi = own128 ? t.user_data_128.hi : p.user_data_128.hi;
  t2.user_data_64 = t.user_data_64 > 0 ? t.user_data_64 : p.user_data_64;
  t2.user_data_32 = t.user_data_32 > 0 ? t.user_data_32 : p.user_data_32;
  t2.ledger = p.ledger;
  t2.code = p.code;
  t2.pending_id = t.pending_id;
  t2.timeout = 0;
  t2.timestamp = t.timestamp;
  t2.flags = t.flags;
  t2.amount = W(amount);
  return t2;
}

__device__ __attribute__((always_inline)) inline uint64_t expires_at_of(const tb_transfer_t& p) {
  return p.timestamp + (uint64_t)p.timeout * TB_NS_PER_S;
}

struct Bal {
  u128 dp, dpo, cp, cpo;
};
__device__ __attribute__((always_inline)) inline Bal load_bal(const tb_account_t* a) {
  Bal b;
  b.dp = U(a->debits_pending);
  b.dpo = U(a->debits_posted);
  b.cp = U(a->credits_pending);
  b.cpo = U(a->credits_posted);
  return b;
}
__device__ __attribute__((always_inline)) inline void store_bal(tb_account_t* a, const Bal& b) {
  a->debits_pending = W(b.dp);
  a->debits_posted = W(b.dpo);
  a->credits_pending = W(b.cp);
  a->credits_posted = W(b.cpo);
}

// Balance-dependent tail of create_transfer (:1509-1547): balancing clamp, overflow checks,
// timeout overflow, limits. Returns OK with the (clamped) amount, or the failing code.
__device__ __attribute__((always_inline)) inline uint32_t ct_balances(const tb_transfer_t& t, const Bal& dr, uint16_t dr_flags, const Bal& cr,
                                       uint16_t cr_flags, u128* amount_out) {
  const uint16_t f = t.flags;
  const bool bdr = f & TB_TRANSFER_BALANCING_DEBIT, bcr = f & TB_TRANSFER_BALANCING_CREDIT;
  u128 amount = U(t.amount);
  if ((bdr || bcr) && amount == 0) amount = (u128)0xFFFFFFFFFFFFFFFFull;  // u64 max (:1512)
  if (bdr) {
    const u128 bal = dr.dpo + dr.dp;
    const u128 avail = dr.cpo > bal ? dr.cpo - bal : 0;
    if (avail < amount) amount = avail;
    if (amount == 0) return TB_CT_EXCEEDS_CREDITS;
  }
  if (bcr) {
    const u128 bal = cr.cpo + cr.cp;
    const u128 avail = cr.dpo > bal ? cr.dpo - bal : 0;
    if (avail < amount) amount = avail;
    if (amount == 0) return TB_CT_EXCEEDS_DEBITS;
  }
  if (f & TB_TRANSFER_PENDING) {
    if (ovf128(amount, dr.dp)) return TB_CT_OVERFLOWS_DEBITS_PENDING;
    if (ovf128(amount, cr.cp)) return TB_CT_OVERFLOWS_CREDITS_PENDING;
  }
  if (ovf128(amount, dr.dpo)) return TB_CT_OVERFLOWS_DEBITS_POSTED;
  if (ovf128(amount, cr.cpo)) return TB_CT_OVERFLOWS_CREDITS_POSTED;
  if (ovf128(amount, dr.dp + dr.dpo)) return TB_CT_OVERFLOWS_DEBITS;
  if (ovf128(amount, cr.cp + cr.cpo)) return TB_CT_OVERFLOWS_CREDITS;
  if (ovf64(t.timestamp, (uint64_t)t.timeout * TB_NS_PER_S)) return TB_CT_OVERFLOWS_TIMEOUT;
  if ((dr_flags & TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS) && dr.dp + dr.dpo + amount > dr.cpo)
    return TB_CT_EXCEEDS_CREDITS;
  if ((cr_flags & TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS) && cr.cp + cr.cpo + amount > cr.dpo)
    return TB_CT_EXCEEDS_DEBITS;
  *amount_out = amount;
  return TB_CT_OK;
}

// create_account validation (state_machine.zig:1424-1439).
__device__ __attribute__((always_inline)) inline uint32_t ca_validate(const tb_account_t& a) {
  if (a.reserved != 0) return TB_CA_RESERVED_FIELD;
  if (a.flags & TB_ACCOUNT_PADDING_MASK) return TB_CA_RESERVED_FLAG;
  const u128 id = U(a.id);
  if (id == 0) return TB_CA_ID_MUST_NOT_BE_ZERO;
  if (id == MAX128) return TB_CA_ID_MUST_NOT_BE_INT_MAX;
  if ((a.flags & TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS) && (a.flags & TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS))
    return TB_CA_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
  if (U(a.debits_pending) != 0) return TB_CA_DEBITS_PENDING_MUST_BE_ZERO;
  if (U(a.debits_posted) != 0) return TB_CA_DEBITS_POSTED_MUST_BE_ZERO;
  if (U(a.credits_pending) != 0) return TB_CA_CREDITS_PENDING_MUST_BE_ZERO;
  if (U(a.credits_posted) != 0) return TB_CA_CREDITS_POSTED_MUST_BE_ZERO;
  if (a.ledger == 0) return TB_CA_LEDGER_MUST_NOT_BE_ZERO;
  if (a.code == 0) return TB_CA_CODE_MUST_NOT_BE_ZERO;
  return CONT;
}

// create_account_exists (:1450-1460). Compares the whole u16 flags, linked included.
__device__ __attribute__((always_inline)) inline uint32_t ca_exists(const tb_account_t& a, const tb_account_t& e) {
  if (a.flags != e.flags) return TB_CA_EXISTS_WITH_DIFFERENT_FLAGS;
  if (U(a.user_data_128) != U(e.user_data_128)) return TB_CA_EXISTS_WITH_DIFFERENT_USER_DATA_128;
  if (a.user_data_64 != e.user_data_64) return TB_CA_EXISTS_WITH_DIFFERENT_USER_DATA_64;
  if (a.user_data_32 != e.user_data_32) return TB_CA_EXISTS_WITH_DIFFERENT_USER_DATA_32;
  if (a.ledger != e.ledger) return TB_CA_EXISTS_WITH_DIFFERENT_LEDGER;
  if (a.code != e.code) return TB_CA_EXISTS_WITH_DIFFERENT_CODE;
  return TB_CA_EXISTS;
}
