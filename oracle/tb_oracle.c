/*
 * tb_oracle.c — CPU restatement of the reference StateMachine commit path.
 *
 * TEST INFRASTRUCTURE ONLY. This file is the parity oracle and the single-threaded CPU baseline
 * (bench.py cpu_baseline kind "port"). Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it; the product (libtbgpu.so, tigerbeetle_amd/) never does.
 *
 * The reference (kdrag0n/tigerbeetle, Zig 0.11) cannot be built here (no zig toolchain), so this
 * restatement is pinned by the reference's own table-driven known-answer tests
 * (src/state_machine.zig:2767-3360, transcribed under tests/golden/kat_*.tbl), which the CPU test
 * suite runs against it byte-for-byte.
 *
 * Each function cites the reference file:line it follows (paths relative to the reference root).
 * Storage is in-memory: open-addressing hash maps stand in for the LSM grooves' get/insert/update
 * (src/lsm/groove.zig:617-1000), an undo log stands in for scope_open/scope_close
 * (src/lsm/cache_map.zig:254-301), and a lazily-validated binary heap stands in for the
 * `expires_at` index tree scanned by ExpirePendingTransfers (src/state_machine.zig:2018-2173).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/tb_types.h"

typedef unsigned __int128 u128;

static inline u128 U(tb_uint128_t v) { return ((u128)v.hi << 64) | v.lo; }
static inline tb_uint128_t W(u128 v) {
    tb_uint128_t r = {(uint64_t)v, (uint64_t)(v >> 64)};
    return r;
}
static const u128 MAX128 = ~(u128)0;

/* sum_overflows (state_machine.zig:2002-2007). */
static inline int ovf128(u128 a, u128 b) { return a + b < a; }
static inline int ovf64(uint64_t a, uint64_t b) { return a + b < a; }

/* ----------------------------------------------------------------------------------------------
 * Open-addressing map: u128 key -> u32 value (linear probing, backward-shift delete).
 * -------------------------------------------------------------------------------------------- */
typedef struct {
    tb_uint128_t *keys;
    uint32_t *vals; /* UINT32_MAX = empty */
    uint64_t cap;   /* power of two */
    uint64_t count;
} omap;

static inline uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}
static inline uint64_t hkey(tb_uint128_t k) { return mix64(k.lo ^ mix64(k.hi + 0x9e3779b97f4a7c15ull)); }
static inline int keq(tb_uint128_t a, tb_uint128_t b) { return a.lo == b.lo && a.hi == b.hi; }

static void omap_init(omap *m, uint64_t cap) {
    m->cap = cap;
    m->count = 0;
    m->keys = (tb_uint128_t *)calloc(cap, sizeof(tb_uint128_t));
    m->vals = (uint32_t *)malloc(cap * sizeof(uint32_t));
    memset(m->vals, 0xff, cap * sizeof(uint32_t));
}
static void omap_free(omap *m) {
    free(m->keys);
    free(m->vals);
}
static uint32_t omap_get(const omap *m, tb_uint128_t k) {
    uint64_t mask = m->cap - 1, i = hkey(k) & mask;
    for (;;) {
        uint32_t v = m->vals[i];
        if (v == UINT32_MAX) return UINT32_MAX;
        if (keq(m->keys[i], k)) return v;
        i = (i + 1) & mask;
    }
}
static void omap_put_raw(omap *m, tb_uint128_t k, uint32_t v) {
    uint64_t mask = m->cap - 1, i = hkey(k) & mask;
    for (;;) {
        if (m->vals[i] == UINT32_MAX) {
            m->keys[i] = k;
            m->vals[i] = v;
            m->count++;
            return;
        }
        if (keq(m->keys[i], k)) {
            m->vals[i] = v;
            return;
        }
        i = (i + 1) & mask;
    }
}
static void omap_put(omap *m, tb_uint128_t k, uint32_t v) {
    if ((m->count + 1) * 2 > m->cap) {
        omap old = *m;
        omap_init(m, old.cap * 2);
        for (uint64_t i = 0; i < old.cap; i++)
            if (old.vals[i] != UINT32_MAX) omap_put_raw(m, old.keys[i], old.vals[i]);
        omap_free(&old);
    }
    omap_put_raw(m, k, v);
}
static void omap_del(omap *m, tb_uint128_t k) {
    uint64_t mask = m->cap - 1, i = hkey(k) & mask;
    for (;;) {
        if (m->vals[i] == UINT32_MAX) return;
        if (keq(m->keys[i], k)) break;
        i = (i + 1) & mask;
    }
    /* backward-shift deletion */
    uint64_t j = i;
    for (;;) {
        j = (j + 1) & mask;
        if (m->vals[j] == UINT32_MAX) break;
        uint64_t home = hkey(m->keys[j]) & mask;
        /* can the entry at j move to i?  yes iff home is not cyclically in (i, j] */
        int in_range = (i <= j) ? (home > i && home <= j) : (home > i || home <= j);
        if (!in_range) {
            m->keys[i] = m->keys[j];
            m->vals[i] = m->vals[j];
            i = j;
        }
    }
    m->vals[i] = UINT32_MAX;
    m->count--;
}

/* ----------------------------------------------------------------------------------------------
 * Expiry index: min-heap of (expires_at, timestamp) pushed at pending creation, lazily validated
 * against the pending-status map (an index entry is live iff its TransferPending status is
 * `pending`: both removal sites — post/void at state_machine.zig:1699 and expiry at :1921 — also
 * move the status away from `pending`, and chain rollback restores both together).
 * -------------------------------------------------------------------------------------------- */
typedef struct {
    uint64_t expires_at, timestamp;
} xentry;

typedef struct {
    xentry *a;
    uint64_t n, cap;
} xheap;

static inline int xless(xentry x, xentry y) {
    return x.expires_at < y.expires_at || (x.expires_at == y.expires_at && x.timestamp < y.timestamp);
}
static void xheap_push(xheap *h, xentry e) {
    if (h->n == h->cap) {
        h->cap = h->cap ? h->cap * 2 : 1024;
        h->a = (xentry *)realloc(h->a, h->cap * sizeof(xentry));
    }
    uint64_t i = h->n++;
    while (i > 0) {
        uint64_t p = (i - 1) / 2;
        if (!xless(e, h->a[p])) break;
        h->a[i] = h->a[p];
        i = p;
    }
    h->a[i] = e;
}
static void xheap_pop(xheap *h) {
    xentry e = h->a[--h->n];
    uint64_t i = 0;
    for (;;) {
        uint64_t c = 2 * i + 1;
        if (c >= h->n) break;
        if (c + 1 < h->n && xless(h->a[c + 1], h->a[c])) c++;
        if (!xless(h->a[c], e)) break;
        h->a[i] = h->a[c];
        i = c;
    }
    if (h->n) h->a[i] = e;
}

/* ----------------------------------------------------------------------------------------------
 * Undo log (scope_open/scope_close, state_machine.zig:1190-1218; cache_map.zig:254-301).
 * -------------------------------------------------------------------------------------------- */
enum { U_ACC_UPDATE, U_ACC_INSERT, U_XFER_INSERT, U_PEND_INSERT, U_PEND_UPDATE };
typedef struct {
    uint32_t kind;
    uint32_t idx;       /* account index / pending status slot */
    tb_uint128_t key;   /* id or timestamp */
    tb_uint128_t bal[4];/* old balances for U_ACC_UPDATE */
    uint8_t status;     /* old status for U_PEND_UPDATE */
} undo_rec;

typedef struct tbo_state {
    /* accounts groove */
    omap acc_map;
    tb_account_t *acc;
    uint64_t acc_n, acc_cap;
    /* transfers groove */
    omap xfer_map;
    tb_transfer_t *xfer;
    uint64_t xfer_n, xfer_cap;
    /* transfers_pending groove: timestamp -> status slot */
    omap pend_map;
    uint8_t *pend_status;
    uint32_t *pend_xfer; /* pending slot -> index of the pending transfer record */
    uint64_t pend_n, pend_cap;
    /* expires_at index */
    xheap xh;
    uint64_t pulse_next_timestamp; /* ExpirePendingTransfers.pulse_next_timestamp (:2063) */
    uint32_t batch_max;            /* constants.batch_max.create_transfers (pulse cap, :1016-1022) */
    uint64_t commit_timestamp;
    /* account_balances groove (state_machine.zig:296-315): one row per transfer record (same
     * index, so the transfer insert's undo also drops it); hist_side bit 0 = dr side, bit 1 = cr */
    tb_uint128_t (*hist)[8];
    uint8_t *hist_side;
    uint64_t hist_cap;
    /* scope */
    int scope_active;
    undo_rec *undo;
    uint64_t undo_n, undo_cap;
} tbo_state;

static void undo_push(tbo_state *s, undo_rec r) {
    if (!s->scope_active) return;
    if (s->undo_n == s->undo_cap) {
        s->undo_cap = s->undo_cap ? s->undo_cap * 2 : 256;
        s->undo = (undo_rec *)realloc(s->undo, s->undo_cap * sizeof(undo_rec));
    }
    s->undo[s->undo_n++] = r;
}

static void scope_open(tbo_state *s) {
    s->scope_active = 1;
    s->undo_n = 0;
}

/* scope_close(.persist | .discard): discard replays the log in reverse (LIFO). */
static void scope_close(tbo_state *s, int discard) {
    if (discard) {
        while (s->undo_n) {
            undo_rec *r = &s->undo[--s->undo_n];
            switch (r->kind) {
            case U_ACC_UPDATE: {
                tb_account_t *a = &s->acc[r->idx];
                a->debits_pending = r->bal[0];
                a->debits_posted = r->bal[1];
                a->credits_pending = r->bal[2];
                a->credits_posted = r->bal[3];
            } break;
            case U_ACC_INSERT:
                omap_del(&s->acc_map, r->key);
                s->acc_n--;
                break;
            case U_XFER_INSERT:
                omap_del(&s->xfer_map, r->key);
                s->xfer_n--;
                break;
            case U_PEND_INSERT:
                omap_del(&s->pend_map, r->key);
                s->pend_n--;
                break;
            case U_PEND_UPDATE:
                s->pend_status[r->idx] = r->status;
                break;
            }
        }
    }
    s->undo_n = 0;
    s->scope_active = 0;
}

/* ----------------------------------------------------------------------------------------------
 * Groove operations.
 * -------------------------------------------------------------------------------------------- */
static tb_account_t *get_account(tbo_state *s, tb_uint128_t id) {
    uint32_t i = omap_get(&s->acc_map, id);
    return i == UINT32_MAX ? NULL : &s->acc[i];
}
static tb_transfer_t *get_transfer(tbo_state *s, tb_uint128_t id) {
    uint32_t i = omap_get(&s->xfer_map, id);
    return i == UINT32_MAX ? NULL : &s->xfer[i];
}
static int get_pending_slot(tbo_state *s, uint64_t ts) {
    tb_uint128_t k = {ts, 0};
    uint32_t i = omap_get(&s->pend_map, k);
    return i == UINT32_MAX ? -1 : (int)i;
}

static void insert_account(tbo_state *s, const tb_account_t *a) {
    if (s->acc_n == s->acc_cap) {
        s->acc_cap = s->acc_cap ? s->acc_cap * 2 : 1024;
        s->acc = (tb_account_t *)realloc(s->acc, s->acc_cap * sizeof(tb_account_t));
    }
    s->acc[s->acc_n] = *a;
    omap_put(&s->acc_map, a->id, (uint32_t)s->acc_n);
    s->acc_n++;
    undo_rec r = {0};
    r.kind = U_ACC_INSERT;
    r.key = a->id;
    undo_push(s, r);
}

static void update_account(tbo_state *s, tb_account_t *a, u128 dp, u128 dpo, u128 cp, u128 cpo) {
    undo_rec r = {0};
    r.kind = U_ACC_UPDATE;
    r.idx = (uint32_t)(a - s->acc);
    r.bal[0] = a->debits_pending;
    r.bal[1] = a->debits_posted;
    r.bal[2] = a->credits_pending;
    r.bal[3] = a->credits_posted;
    undo_push(s, r);
    a->debits_pending = W(dp);
    a->debits_posted = W(dpo);
    a->credits_pending = W(cp);
    a->credits_posted = W(cpo);
}

static void insert_transfer(tbo_state *s, const tb_transfer_t *t) {
    if (s->xfer_n == s->xfer_cap) {
        s->xfer_cap = s->xfer_cap ? s->xfer_cap * 2 : 1024;
        s->xfer = (tb_transfer_t *)realloc(s->xfer, s->xfer_cap * sizeof(tb_transfer_t));
    }
    s->xfer[s->xfer_n] = *t;
    if (s->xfer_n >= s->hist_cap) {
        s->hist_cap = s->xfer_cap;
        s->hist = (tb_uint128_t(*)[8])realloc(s->hist, s->hist_cap * sizeof(*s->hist));
        s->hist_side = (uint8_t *)realloc(s->hist_side, s->hist_cap);
    }
    s->hist_side[s->xfer_n] = 0;
    omap_put(&s->xfer_map, t->id, (uint32_t)s->xfer_n);
    s->xfer_n++;
    undo_rec r = {0};
    r.kind = U_XFER_INSERT;
    r.key = t->id;
    undo_push(s, r);
    /* derived `expires_at` index (state_machine.zig:229-238): pending with timeout > 0 */
    if ((t->flags & TB_TRANSFER_PENDING) && t->timeout > 0) {
        xentry e = {t->timestamp + (uint64_t)t->timeout * TB_NS_PER_S, t->timestamp};
        xheap_push(&s->xh, e);
    }
}

/* historical_balance (state_machine.zig:1806-1841): the row of the transfer just inserted (the
 * last record), with each history account's balances after the transfer. */
static void historical_balance(tbo_state *s, const tb_account_t *dr, const tb_account_t *cr) {
    if (!((dr->flags | cr->flags) & TB_ACCOUNT_HISTORY)) return;
    const uint64_t i = s->xfer_n - 1;
    uint8_t side = 0;
    if (dr->flags & TB_ACCOUNT_HISTORY) {
        side |= 1;
        s->hist[i][0] = dr->debits_pending;
        s->hist[i][1] = dr->debits_posted;
        s->hist[i][2] = dr->credits_pending;
        s->hist[i][3] = dr->credits_posted;
    }
    if (cr->flags & TB_ACCOUNT_HISTORY) {
        side |= 2;
        s->hist[i][4] = cr->debits_pending;
        s->hist[i][5] = cr->debits_posted;
        s->hist[i][6] = cr->credits_pending;
        s->hist[i][7] = cr->credits_posted;
    }
    s->hist_side[i] = side;
}

static void insert_pending(tbo_state *s, uint64_t ts, uint8_t status) {
    if (s->pend_n == s->pend_cap) {
        s->pend_cap = s->pend_cap ? s->pend_cap * 2 : 1024;
        s->pend_status = (uint8_t *)realloc(s->pend_status, s->pend_cap);
        s->pend_xfer = (uint32_t *)realloc(s->pend_xfer, s->pend_cap * sizeof(uint32_t));
    }
    s->pend_status[s->pend_n] = status;
    s->pend_xfer[s->pend_n] = (uint32_t)(s->xfer_n - 1); /* inserted right after its transfer */
    tb_uint128_t k = {ts, 0};
    omap_put(&s->pend_map, k, (uint32_t)s->pend_n);
    s->pend_n++;
    undo_rec r = {0};
    r.kind = U_PEND_INSERT;
    r.key = k;
    undo_push(s, r);
}

static void update_pending(tbo_state *s, int slot, uint8_t status) {
    undo_rec r = {0};
    r.kind = U_PEND_UPDATE;
    r.idx = (uint32_t)slot;
    r.status = s->pend_status[slot];
    undo_push(s, r);
    s->pend_status[slot] = status;
}

/* ----------------------------------------------------------------------------------------------
 * create_account (state_machine.zig:1421-1460)
 * -------------------------------------------------------------------------------------------- */
static uint32_t create_account_exists(const tb_account_t *a, const tb_account_t *e) {
    if (a->flags != e->flags) return TB_CA_EXISTS_WITH_DIFFERENT_FLAGS;
    if (U(a->user_data_128) != U(e->user_data_128)) return TB_CA_EXISTS_WITH_DIFFERENT_USER_DATA_128;
    if (a->user_data_64 != e->user_data_64) return TB_CA_EXISTS_WITH_DIFFERENT_USER_DATA_64;
    if (a->user_data_32 != e->user_data_32) return TB_CA_EXISTS_WITH_DIFFERENT_USER_DATA_32;
    if (a->ledger != e->ledger) return TB_CA_EXISTS_WITH_DIFFERENT_LEDGER;
    if (a->code != e->code) return TB_CA_EXISTS_WITH_DIFFERENT_CODE;
    return TB_CA_EXISTS;
}

static uint32_t create_account(tbo_state *s, const tb_account_t *a) {
    if (a->reserved != 0) return TB_CA_RESERVED_FIELD;
    if (a->flags & TB_ACCOUNT_PADDING_MASK) return TB_CA_RESERVED_FLAG;
    if (U(a->id) == 0) return TB_CA_ID_MUST_NOT_BE_ZERO;
    if (U(a->id) == MAX128) return TB_CA_ID_MUST_NOT_BE_INT_MAX;
    if ((a->flags & TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS) &&
        (a->flags & TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS))
        return TB_CA_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    if (U(a->debits_pending) != 0) return TB_CA_DEBITS_PENDING_MUST_BE_ZERO;
    if (U(a->debits_posted) != 0) return TB_CA_DEBITS_POSTED_MUST_BE_ZERO;
    if (U(a->credits_pending) != 0) return TB_CA_CREDITS_PENDING_MUST_BE_ZERO;
    if (U(a->credits_posted) != 0) return TB_CA_CREDITS_POSTED_MUST_BE_ZERO;
    if (a->ledger == 0) return TB_CA_LEDGER_MUST_NOT_BE_ZERO;
    if (a->code == 0) return TB_CA_CODE_MUST_NOT_BE_ZERO;
    const tb_account_t *e = get_account(s, a->id);
    if (e) return create_account_exists(a, e);
    insert_account(s, a);
    s->commit_timestamp = a->timestamp;
    return TB_CA_OK;
}

/* ----------------------------------------------------------------------------------------------
 * create_transfer (state_machine.zig:1462-1606)
 * -------------------------------------------------------------------------------------------- */
static uint32_t create_transfer_exists(const tb_transfer_t *t, const tb_transfer_t *e) {
    if (t->flags != e->flags) return TB_CT_EXISTS_WITH_DIFFERENT_FLAGS;
    if (U(t->debit_account_id) != U(e->debit_account_id)) return TB_CT_EXISTS_WITH_DIFFERENT_DEBIT_ACCOUNT_ID;
    if (U(t->credit_account_id) != U(e->credit_account_id)) return TB_CT_EXISTS_WITH_DIFFERENT_CREDIT_ACCOUNT_ID;
    if (U(t->amount) != U(e->amount)) return TB_CT_EXISTS_WITH_DIFFERENT_AMOUNT;
    if (U(t->user_data_128) != U(e->user_data_128)) return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_128;
    if (t->user_data_64 != e->user_data_64) return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_64;
    if (t->user_data_32 != e->user_data_32) return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_32;
    if (t->timeout != e->timeout) return TB_CT_EXISTS_WITH_DIFFERENT_TIMEOUT;
    if (t->code != e->code) return TB_CT_EXISTS_WITH_DIFFERENT_CODE;
    return TB_CT_EXISTS;
}

/* post_or_void_pending_transfer_exists (state_machine.zig:1743-1804) */
static uint32_t post_or_void_exists(const tb_transfer_t *t, const tb_transfer_t *e, const tb_transfer_t *p) {
    if (t->flags != e->flags) return TB_CT_EXISTS_WITH_DIFFERENT_FLAGS;
    if (U(t->amount) == 0) {
        if (U(e->amount) != U(p->amount)) return TB_CT_EXISTS_WITH_DIFFERENT_AMOUNT;
    } else {
        if (U(t->amount) != U(e->amount)) return TB_CT_EXISTS_WITH_DIFFERENT_AMOUNT;
    }
    if (U(t->pending_id) != U(e->pending_id)) return TB_CT_EXISTS_WITH_DIFFERENT_PENDING_ID;
    if (U(t->user_data_128) == 0) {
        if (U(e->user_data_128) != U(p->user_data_128)) return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_128;
    } else {
        if (U(t->user_data_128) != U(e->user_data_128)) return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_128;
    }
    if (t->user_data_64 == 0) {
        if (e->user_data_64 != p->user_data_64) return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_64;
    } else {
        if (t->user_data_64 != e->user_data_64) return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_64;
    }
    if (t->user_data_32 == 0) {
        if (e->user_data_32 != p->user_data_32) return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_32;
    } else {
        if (t->user_data_32 != e->user_data_32) return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_32;
    }
    return TB_CT_EXISTS;
}

/* post_or_void_pending_transfer (state_machine.zig:1608-1741) */
static uint32_t post_or_void_pending_transfer(tbo_state *s, const tb_transfer_t *t) {
    const uint16_t f = t->flags;
    if ((f & TB_TRANSFER_POST_PENDING) && (f & TB_TRANSFER_VOID_PENDING)) return TB_CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    if (f & TB_TRANSFER_PENDING) return TB_CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    if (f & TB_TRANSFER_BALANCING_DEBIT) return TB_CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    if (f & TB_TRANSFER_BALANCING_CREDIT) return TB_CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE;

    const u128 pending_id = U(t->pending_id);
    if (pending_id == 0) return TB_CT_PENDING_ID_MUST_NOT_BE_ZERO;
    if (pending_id == MAX128) return TB_CT_PENDING_ID_MUST_NOT_BE_INT_MAX;
    if (pending_id == U(t->id)) return TB_CT_PENDING_ID_MUST_BE_DIFFERENT;
    if (t->timeout != 0) return TB_CT_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER;

    const tb_transfer_t *p = get_transfer(s, t->pending_id);
    if (!p) return TB_CT_PENDING_TRANSFER_NOT_FOUND;
    if (!(p->flags & TB_TRANSFER_PENDING)) return TB_CT_PENDING_TRANSFER_NOT_PENDING;

    tb_account_t *dr = get_account(s, p->debit_account_id);
    tb_account_t *cr = get_account(s, p->credit_account_id);

    if (U(t->debit_account_id) > 0 && U(t->debit_account_id) != U(p->debit_account_id))
        return TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_DEBIT_ACCOUNT_ID;
    if (U(t->credit_account_id) > 0 && U(t->credit_account_id) != U(p->credit_account_id))
        return TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_CREDIT_ACCOUNT_ID;
    if (t->ledger > 0 && t->ledger != p->ledger) return TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_LEDGER;
    if (t->code > 0 && t->code != p->code) return TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_CODE;

    const u128 p_amount = U(p->amount);
    const u128 amount = U(t->amount) > 0 ? U(t->amount) : p_amount;
    if (amount > p_amount) return TB_CT_EXCEEDS_PENDING_TRANSFER_AMOUNT;
    if ((f & TB_TRANSFER_VOID_PENDING) && amount < p_amount) return TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_AMOUNT;

    const tb_transfer_t *e = get_transfer(s, t->id);
    if (e) return post_or_void_exists(t, e, p);

    const int pslot = get_pending_slot(s, p->timestamp);
    switch (s->pend_status[pslot]) {
    case TB_PENDING_PENDING: break;
    case TB_PENDING_POSTED: return TB_CT_PENDING_TRANSFER_ALREADY_POSTED;
    case TB_PENDING_VOIDED: return TB_CT_PENDING_TRANSFER_ALREADY_VOIDED;
    case TB_PENDING_EXPIRED: return TB_CT_PENDING_TRANSFER_EXPIRED;
    default: abort();
    }

    /* Copy what we still need from p before the insert may reallocate the transfer array. */
    const tb_transfer_t pc = *p;
    tb_transfer_t t2;
    memset(&t2, 0, sizeof t2);
    t2.id = t->id;
    t2.debit_account_id = pc.debit_account_id;
    t2.credit_account_id = pc.credit_account_id;
    t2.user_data_128 = U(t->user_data_128) > 0 ? t->user_data_128 : pc.user_data_128;
    t2.user_data_64 = t->user_data_64 > 0 ? t->user_data_64 : pc.user_data_64;
    t2.user_data_32 = t->user_data_32 > 0 ? t->user_data_32 : pc.user_data_32;
    t2.ledger = pc.ledger;
    t2.code = pc.code;
    t2.pending_id = t->pending_id;
    t2.timeout = 0;
    t2.timestamp = t->timestamp;
    t2.flags = t->flags;
    t2.amount = W(amount);
    insert_transfer(s, &t2);

    if (pc.timeout > 0) {
        const uint64_t expires_at = pc.timestamp + (uint64_t)pc.timeout * TB_NS_PER_S;
        /* quirk: the posting transfer stays inserted (state_machine.zig:1689-1696) */
        if (expires_at <= t->timestamp) return TB_CT_PENDING_TRANSFER_EXPIRED;
        /* index removal (:1699) is implied by the status update below (see xheap comment) */
        if (s->pulse_next_timestamp == expires_at) s->pulse_next_timestamp = TB_TIMESTAMP_MIN;
    }

    update_pending(s, pslot, (f & TB_TRANSFER_POST_PENDING) ? TB_PENDING_POSTED : TB_PENDING_VOIDED);

    u128 dp = U(dr->debits_pending) - p_amount, dpo = U(dr->debits_posted);
    u128 ccp = U(cr->credits_pending) - p_amount, cpo = U(cr->credits_posted);
    if (f & TB_TRANSFER_POST_PENDING) {
        dpo += amount;
        cpo += amount;
    }
    update_account(s, dr, dp, dpo, U(dr->credits_pending), U(dr->credits_posted));
    update_account(s, cr, U(cr->debits_pending), U(cr->debits_posted), ccp, cpo);
    historical_balance(s, dr, cr); /* :1732-1736 */
    s->commit_timestamp = t->timestamp;
    return TB_CT_OK;
}

static uint32_t create_transfer(tbo_state *s, const tb_transfer_t *t) {
    const uint16_t f = t->flags;
    if (f & TB_TRANSFER_PADDING_MASK) return TB_CT_RESERVED_FLAG;
    if (U(t->id) == 0) return TB_CT_ID_MUST_NOT_BE_ZERO;
    if (U(t->id) == MAX128) return TB_CT_ID_MUST_NOT_BE_INT_MAX;
    if (f & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING)) return post_or_void_pending_transfer(s, t);

    const u128 dr_id = U(t->debit_account_id), cr_id = U(t->credit_account_id);
    if (dr_id == 0) return TB_CT_DEBIT_ACCOUNT_ID_MUST_NOT_BE_ZERO;
    if (dr_id == MAX128) return TB_CT_DEBIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX;
    if (cr_id == 0) return TB_CT_CREDIT_ACCOUNT_ID_MUST_NOT_BE_ZERO;
    if (cr_id == MAX128) return TB_CT_CREDIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX;
    if (cr_id == dr_id) return TB_CT_ACCOUNTS_MUST_BE_DIFFERENT;

    if (U(t->pending_id) != 0) return TB_CT_PENDING_ID_MUST_BE_ZERO;
    if (!(f & TB_TRANSFER_PENDING) && t->timeout != 0) return TB_CT_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER;
    const int bdr = (f & TB_TRANSFER_BALANCING_DEBIT) != 0, bcr = (f & TB_TRANSFER_BALANCING_CREDIT) != 0;
    if (!bdr && !bcr && U(t->amount) == 0) return TB_CT_AMOUNT_MUST_NOT_BE_ZERO;
    if (t->ledger == 0) return TB_CT_LEDGER_MUST_NOT_BE_ZERO;
    if (t->code == 0) return TB_CT_CODE_MUST_NOT_BE_ZERO;

    tb_account_t *dr = get_account(s, t->debit_account_id);
    if (!dr) return TB_CT_DEBIT_ACCOUNT_NOT_FOUND;
    tb_account_t *cr = get_account(s, t->credit_account_id);
    if (!cr) return TB_CT_CREDIT_ACCOUNT_NOT_FOUND;
    if (dr->ledger != cr->ledger) return TB_CT_ACCOUNTS_MUST_HAVE_THE_SAME_LEDGER;
    if (t->ledger != dr->ledger) return TB_CT_TRANSFER_MUST_HAVE_THE_SAME_LEDGER_AS_ACCOUNTS;

    const tb_transfer_t *e = get_transfer(s, t->id);
    if (e) return create_transfer_exists(t, e);

    const u128 dr_dp = U(dr->debits_pending), dr_dpo = U(dr->debits_posted);
    const u128 dr_cp = U(dr->credits_pending), dr_cpo = U(dr->credits_posted);
    const u128 cr_dp = U(cr->debits_pending), cr_dpo = U(cr->debits_posted);
    const u128 cr_cp = U(cr->credits_pending), cr_cpo = U(cr->credits_posted);

    u128 amount = U(t->amount);
    if (bdr || bcr) {
        if (amount == 0) amount = (u128)UINT64_MAX; /* u64 max, not u128 (:1512) */
    }
    if (bdr) {
        const u128 dr_balance = dr_dpo + dr_dp;
        const u128 avail = dr_cpo > dr_balance ? dr_cpo - dr_balance : 0; /* -| */
        if (avail < amount) amount = avail;
        if (amount == 0) return TB_CT_EXCEEDS_CREDITS;
    }
    if (bcr) {
        const u128 cr_balance = cr_cpo + cr_cp;
        const u128 avail = cr_dpo > cr_balance ? cr_dpo - cr_balance : 0;
        if (avail < amount) amount = avail;
        if (amount == 0) return TB_CT_EXCEEDS_DEBITS;
    }

    const int pending = (f & TB_TRANSFER_PENDING) != 0;
    if (pending) {
        if (ovf128(amount, dr_dp)) return TB_CT_OVERFLOWS_DEBITS_PENDING;
        if (ovf128(amount, cr_cp)) return TB_CT_OVERFLOWS_CREDITS_PENDING;
    }
    if (ovf128(amount, dr_dpo)) return TB_CT_OVERFLOWS_DEBITS_POSTED;
    if (ovf128(amount, cr_cpo)) return TB_CT_OVERFLOWS_CREDITS_POSTED;
    if (ovf128(amount, dr_dp + dr_dpo)) return TB_CT_OVERFLOWS_DEBITS;
    if (ovf128(amount, cr_cp + cr_cpo)) return TB_CT_OVERFLOWS_CREDITS;
    if (ovf64(t->timestamp, (uint64_t)t->timeout * TB_NS_PER_S)) return TB_CT_OVERFLOWS_TIMEOUT;
    /* Account.debits_exceed_credits / credits_exceed_debits (tigerbeetle.zig:31-39) */
    if ((dr->flags & TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS) && dr_dp + dr_dpo + amount > dr_cpo)
        return TB_CT_EXCEEDS_CREDITS;
    if ((cr->flags & TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS) && cr_cp + cr_cpo + amount > cr_dpo)
        return TB_CT_EXCEEDS_DEBITS;

    tb_transfer_t t2 = *t;
    t2.amount = W(amount);
    insert_transfer(s, &t2);
    if (pending) {
        update_account(s, dr, dr_dp + amount, dr_dpo, dr_cp, dr_cpo);
        update_account(s, cr, cr_dp, cr_dpo, cr_cp + amount, cr_cpo);
        insert_pending(s, t2.timestamp, TB_PENDING_PENDING);
    } else {
        update_account(s, dr, dr_dp, dr_dpo + amount, dr_cp, dr_cpo);
        update_account(s, cr, cr_dp, cr_dpo, cr_cp, cr_cpo + amount);
    }
    historical_balance(s, dr, cr); /* :1570-1574 */
    if (t->timeout > 0) {
        const uint64_t expires_at = t->timestamp + (uint64_t)t->timeout * TB_NS_PER_S;
        if (expires_at < s->pulse_next_timestamp) s->pulse_next_timestamp = expires_at;
    }
    s->commit_timestamp = t->timestamp;
    return TB_CT_OK;
}

/* ----------------------------------------------------------------------------------------------
 * execute (state_machine.zig:1220-1306): chains, timestamps, back-filled linked_event_failed.
 * -------------------------------------------------------------------------------------------- */
typedef uint32_t (*event_fn)(tbo_state *, const void *);
static uint32_t ca_thunk(tbo_state *s, const void *e) { return create_account(s, (const tb_account_t *)e); }
static uint32_t ct_thunk(tbo_state *s, const void *e) { return create_transfer(s, (const tb_transfer_t *)e); }

static uint32_t execute(tbo_state *s, uint64_t timestamp, const uint8_t *events, uint32_t n, tb_create_result_t *out,
                        event_fn fn) {
    uint32_t count = 0;
    int64_t chain = -1;
    int chain_broken = 0;
    for (uint32_t i = 0; i < n; i++) {
        uint8_t ev[128] __attribute__((aligned(16)));
        memcpy(ev, events + (size_t)i * 128, 128);
        const uint16_t flags = *(const uint16_t *)(ev + 118);
        const uint64_t ev_ts = *(const uint64_t *)(ev + 120);
        const int linked = (flags & 1u) != 0; /* linked is bit 0 in both Account and Transfer flags */
        uint32_t result;
        if (linked && chain < 0) {
            chain = i;
            scope_open(s);
        }
        if (linked && i == n - 1) {
            result = TB_CT_LINKED_EVENT_CHAIN_OPEN;
        } else if (chain_broken) {
            result = TB_CT_LINKED_EVENT_FAILED;
        } else if (ev_ts != 0) {
            result = TB_CT_TIMESTAMP_MUST_BE_ZERO;
        } else {
            *(uint64_t *)(ev + 120) = timestamp - n + i + 1;
            result = fn(s, ev);
        }
        if (result != 0) {
            if (chain >= 0) {
                if (!chain_broken) {
                    chain_broken = 1;
                    scope_close(s, 1);
                    for (uint32_t j = (uint32_t)chain; j < i; j++) {
                        out[count].index = j;
                        out[count].result = TB_CT_LINKED_EVENT_FAILED;
                        count++;
                    }
                }
            }
            out[count].index = i;
            out[count].result = result;
            count++;
        }
        if (chain >= 0 && (!linked || result == TB_CT_LINKED_EVENT_CHAIN_OPEN)) {
            if (!chain_broken) scope_close(s, 0);
            chain = -1;
            chain_broken = 0;
        }
    }
    return count;
}

/* ----------------------------------------------------------------------------------------------
 * Pulse: prefetch_expire_pending_transfers + ExpirePendingTransfers.finish + execute_expire
 * (state_machine.zig:1010-1105, 1874-1929, 2112-2166). The scan covers keys
 * [(timestamp_min, timestamp_min), (timestamp_max, timestamp_max)] ascending and skips values whose
 * timestamp has the composite-key tombstone bit (bit 63) set (lsm/composite_key.zig:25-57,
 * lsm/scan_range.zig:78-80); the buffer-full check precedes each `next()`
 * (lsm/scan_lookup.zig:151-156).
 * -------------------------------------------------------------------------------------------- */
static int xentry_in_scan_range(xentry e) {
    if (e.timestamp & (1ull << 63)) return 0;  /* composite-key tombstone bit */
    if (e.expires_at > TB_TIMESTAMP_MAX) return 0;
    return 1;
}

/* Returns the pending slot of a live, scan-visible entry, or -1 for an entry the scan never
 * yields (dead, or outside the scan's key range). */
static int xentry_slot(tbo_state *s, xentry e) {
    if (!xentry_in_scan_range(e)) return -1;
    int slot = get_pending_slot(s, e.timestamp);
    if (slot < 0 || s->pend_status[slot] != TB_PENDING_PENDING) return -1;
    return slot;
}

uint32_t tbo_pulse(tbo_state *s, uint64_t timestamp) {
    uint32_t produced = 0;
    int seen = 0, buffer_finished = 0;
    uint64_t value_next_expired_at = 0;
    for (;;) {
        if (produced == s->batch_max) { /* scan_lookup.zig:151-156 */
            buffer_finished = 1;
            break;
        }
        int slot = -1;
        while (s->xh.n && (slot = xentry_slot(s, s->xh.a[0])) < 0) xheap_pop(&s->xh);
        if (!s->xh.n) break; /* scan_finished */
        const xentry top = s->xh.a[0];
        seen = 1;
        value_next_expired_at = top.expires_at; /* value_next (:2147-2166) */
        if (top.expires_at > timestamp) break;  /* exclude_and_stop */
        xheap_pop(&s->xh);
        produced++;
        /* execute_expire_pending_transfers (:1889-1925) */
        const tb_transfer_t *x = &s->xfer[s->pend_xfer[slot]];
        tb_account_t *dr = get_account(s, x->debit_account_id);
        tb_account_t *cr = get_account(s, x->credit_account_id);
        const u128 amt = U(x->amount);
        update_account(s, dr, U(dr->debits_pending) - amt, U(dr->debits_posted), U(dr->credits_pending),
                       U(dr->credits_posted));
        update_account(s, cr, U(cr->debits_pending), U(cr->debits_posted), U(cr->credits_pending) - amt,
                       U(cr->credits_posted));
        update_pending(s, slot, TB_PENDING_EXPIRED);
    }
    /* ExpirePendingTransfers.finish (:2112-2145) */
    if (buffer_finished) {
        s->pulse_next_timestamp = value_next_expired_at;
    } else if (!seen || value_next_expired_at <= timestamp) {
        s->pulse_next_timestamp = TB_TIMESTAMP_MAX;
    } else {
        s->pulse_next_timestamp = value_next_expired_at;
    }
    return produced;
}

/* ----------------------------------------------------------------------------------------------
 * Public oracle API (ctypes). Mirrors the StateMachine boundary (state_machine.zig:543-596,
 * 1107-1146) plus the test harness hooks `setup` (:2545-2561) and lookups (:1309-1344).
 * -------------------------------------------------------------------------------------------- */
tbo_state *tbo_create(uint32_t batch_max) {
    tbo_state *s = (tbo_state *)calloc(1, sizeof(tbo_state));
    omap_init(&s->acc_map, 1024);
    omap_init(&s->xfer_map, 1024);
    omap_init(&s->pend_map, 1024);
    s->pulse_next_timestamp = TB_TIMESTAMP_MIN;
    s->batch_max = batch_max ? batch_max : TB_BATCH_MAX;
    return s;
}

void tbo_destroy(tbo_state *s) {
    if (!s) return;
    omap_free(&s->acc_map);
    omap_free(&s->xfer_map);
    omap_free(&s->pend_map);
    free(s->acc);
    free(s->xfer);
    free(s->pend_status);
    free(s->pend_xfer);
    free(s->xh.a);
    free(s->undo);
    free(s->hist);
    free(s->hist_side);
    free(s);
}

/* input_valid (state_machine.zig:543-572) */
int tbo_input_valid(uint32_t operation, uint64_t len, uint32_t batch_max) {
    switch (operation) {
    case TB_OP_PULSE: return len == 0;
    case TB_OP_CREATE_ACCOUNTS:
    case TB_OP_CREATE_TRANSFERS: return len % 128 == 0 && len <= (uint64_t)batch_max * 128;
    case TB_OP_LOOKUP_ACCOUNTS:
    case TB_OP_LOOKUP_TRANSFERS: return len % 16 == 0 && len <= (uint64_t)batch_max * 16;
    case TB_OP_GET_ACCOUNT_TRANSFERS:
    case TB_OP_GET_ACCOUNT_BALANCES: return len == 64;
    default: return 0;
    }
}

/* pulse() (state_machine.zig:589-596) */
int tbo_pulse_needed(const tbo_state *s, uint64_t prepare_timestamp) {
    return s->pulse_next_timestamp <= prepare_timestamp;
}
uint64_t tbo_pulse_next_timestamp(const tbo_state *s) { return s->pulse_next_timestamp; }

uint32_t tbo_create_accounts(tbo_state *s, uint64_t timestamp, const tb_account_t *events, uint32_t n,
                             tb_create_result_t *out) {
    return execute(s, timestamp, (const uint8_t *)events, n, out, ca_thunk);
}

uint32_t tbo_create_transfers(tbo_state *s, uint64_t timestamp, const tb_transfer_t *events, uint32_t n,
                              tb_create_result_t *out) {
    return execute(s, timestamp, (const uint8_t *)events, n, out, ct_thunk);
}

/* execute_lookup_accounts / execute_lookup_transfers (state_machine.zig:1309-1344) */
uint32_t tbo_lookup_accounts(tbo_state *s, const tb_uint128_t *ids, uint32_t n, tb_account_t *out) {
    uint32_t c = 0;
    for (uint32_t i = 0; i < n; i++) {
        const tb_account_t *a = get_account(s, ids[i]);
        if (a) out[c++] = *a;
    }
    return c;
}
uint32_t tbo_lookup_transfers(tbo_state *s, const tb_uint128_t *ids, uint32_t n, tb_transfer_t *out) {
    uint32_t c = 0;
    for (uint32_t i = 0; i < n; i++) {
        const tb_transfer_t *t = get_transfer(s, ids[i]);
        if (t) out[c++] = *t;
    }
    return c;
}

/* test `setup` action (state_machine.zig:2545-2561): poke balances directly */
int tbo_setup_balances(tbo_state *s, tb_uint128_t id, tb_uint128_t dp, tb_uint128_t dpo, tb_uint128_t cp,
                       tb_uint128_t cpo) {
    tb_account_t *a = get_account(s, id);
    if (!a) return -1;
    a->debits_pending = dp;
    a->debits_posted = dpo;
    a->credits_pending = cp;
    a->credits_posted = cpo;
    return 0;
}

uint64_t tbo_account_count(const tbo_state *s) { return s->acc_n; }
uint64_t tbo_transfer_count(const tbo_state *s) { return s->xfer_n; }

/* Dense dumps, in insertion (= timestamp) order, for whole-state parity checks. */
uint64_t tbo_dump_accounts(const tbo_state *s, tb_account_t *out, uint64_t cap) {
    uint64_t n = s->acc_n < cap ? s->acc_n : cap;
    memcpy(out, s->acc, n * sizeof(tb_account_t));
    return n;
}
uint64_t tbo_dump_transfers(const tbo_state *s, tb_transfer_t *out, uint64_t cap) {
    uint64_t n = s->xfer_n < cap ? s->xfer_n : cap;
    memcpy(out, s->xfer, n * sizeof(tb_transfer_t));
    return n;
}
/* Pending status of a transfer (by its timestamp); 0 = none. */
uint32_t tbo_pending_status(tbo_state *s, uint64_t timestamp) {
    int slot = get_pending_slot(s, timestamp);
    return slot < 0 ? 0 : s->pend_status[slot];
}
/* Pending status of every stored transfer, in store (= timestamp) order; 0 = none. */
uint64_t tbo_dump_transfer_status(tbo_state *s, uint8_t *out, uint64_t cap) {
    uint64_t n = s->xfer_n < cap ? s->xfer_n : cap;
    for (uint64_t i = 0; i < n; i++) {
        int slot = get_pending_slot(s, s->xfer[i].timestamp);
        out[i] = slot < 0 ? 0 : s->pend_status[slot];
    }
    return n;
}

/* ----------------------------------------------------------------------------------------------
 * get_account_transfers / get_account_balances (state_machine.zig:786-996, 1346-1419). The
 * reference scans the transfers groove's debit_account_id / credit_account_id indexes (a union of
 * the two when both flags are set) over the timestamp range, ascending or descending, into a buffer
 * of min(limit, batch_max) results; an invalid filter (get_scan_from_filter, :931-944) or, for
 * balances, a missing account or one without flags.history gives an empty reply. Records are kept
 * in timestamp order, so the scan is a filtered walk over them.
 * -------------------------------------------------------------------------------------------- */
static int filter_valid(const tb_account_filter_t *f) {
    const u128 id = U(f->account_id);
    if (id == 0 || id == MAX128) return 0;
    if (f->timestamp_min == UINT64_MAX || f->timestamp_max == UINT64_MAX) return 0;
    if (f->timestamp_max != 0 && f->timestamp_min > f->timestamp_max) return 0;
    if (f->limit == 0) return 0;
    if (!(f->flags & (TB_FILTER_DEBITS | TB_FILTER_CREDITS))) return 0;
    if (f->flags & ~(uint32_t)(TB_FILTER_DEBITS | TB_FILTER_CREDITS | TB_FILTER_REVERSED)) return 0;
    for (int k = 0; k < 24; k++)
        if (f->reserved[k]) return 0;
    return 1;
}

/* Indexes of the matching transfer records, in scan order, at most `cap`. */
static uint32_t account_scan(const tbo_state *s, const tb_account_filter_t *f, uint32_t cap, uint32_t *idx) {
    const uint64_t tmin = f->timestamp_min ? f->timestamp_min : TB_TIMESTAMP_MIN;
    const uint64_t tmax = f->timestamp_max ? f->timestamp_max : TB_TIMESTAMP_MAX;
    const int rev = (f->flags & TB_FILTER_REVERSED) != 0;
    uint32_t n = 0;
    for (uint64_t k = 0; k < s->xfer_n && n < cap; k++) {
        const uint64_t i = rev ? s->xfer_n - 1 - k : k;
        const tb_transfer_t *t = &s->xfer[i];
        if (t->timestamp < tmin || t->timestamp > tmax) continue;
        const int dr = (f->flags & TB_FILTER_DEBITS) && U(t->debit_account_id) == U(f->account_id);
        const int cr = (f->flags & TB_FILTER_CREDITS) && U(t->credit_account_id) == U(f->account_id);
        if (dr || cr) idx[n++] = (uint32_t)i;
    }
    return n;
}

uint32_t tbo_get_account_transfers(tbo_state *s, const tb_account_filter_t *f, tb_transfer_t *out) {
    if (!filter_valid(f)) return 0;
    const uint32_t cap = f->limit < s->batch_max ? f->limit : s->batch_max;
    uint32_t *idx = (uint32_t *)malloc((size_t)cap * sizeof(uint32_t));
    const uint32_t n = account_scan(s, f, cap, idx);
    for (uint32_t k = 0; k < n; k++) out[k] = s->xfer[idx[k]];
    free(idx);
    return n;
}

uint32_t tbo_get_account_balances(tbo_state *s, const tb_account_filter_t *f, tb_account_balance_t *out) {
    const tb_account_t *a = get_account(s, f->account_id);
    if (!a || !(a->flags & TB_ACCOUNT_HISTORY) || !filter_valid(f)) return 0;
    const uint32_t cap = f->limit < s->batch_max ? f->limit : s->batch_max;
    uint32_t *idx = (uint32_t *)malloc((size_t)cap * sizeof(uint32_t));
    const uint32_t n = account_scan(s, f, cap, idx);
    uint32_t c = 0;
    for (uint32_t k = 0; k < n; k++) {
        const uint32_t i = idx[k];
        const tb_transfer_t *t = &s->xfer[i];
        /* the side of the queried account (execute_get_account_balances, :1392-1410); a record
         * without its row (the expired post/void quirk) is skipped: the reference would reach
         * `unreachable` in its scan lookup (lsm/scan_lookup.zig) */
        int side = U(t->debit_account_id) == U(f->account_id) ? 0 : 1;
        if (!(s->hist_side[i] & (1u << side))) continue;
        tb_account_balance_t b;
        memset(&b, 0, sizeof b);
        b.debits_pending = s->hist[i][4 * side + 0];
        b.debits_posted = s->hist[i][4 * side + 1];
        b.credits_pending = s->hist[i][4 * side + 2];
        b.credits_posted = s->hist[i][4 * side + 3];
        b.timestamp = t->timestamp;
        out[c++] = b;
    }
    free(idx);
    return c;
}

/* The account_balances groove's rows (state_machine.zig:296-315) in timestamp order: what a forest
 * hands to StateMachine.open. Returns the row count (rows written up to cap). */
uint64_t tbo_dump_account_balances(const tbo_state *s, tb_account_balances_value_t *out, uint64_t cap) {
    uint64_t n = 0;
    for (uint64_t i = 0; i < s->xfer_n; i++) {
        const uint8_t side = s->hist_side[i];
        if (!side) continue;
        if (n < cap) {
            tb_account_balances_value_t r;
            memset(&r, 0, sizeof r);
            const tb_transfer_t *t = &s->xfer[i];
            if (side & 1) {
                r.dr_account_id = t->debit_account_id;
                r.dr_debits_pending = s->hist[i][0];
                r.dr_debits_posted = s->hist[i][1];
                r.dr_credits_pending = s->hist[i][2];
                r.dr_credits_posted = s->hist[i][3];
            }
            if (side & 2) {
                r.cr_account_id = t->credit_account_id;
                r.cr_debits_pending = s->hist[i][4];
                r.cr_debits_posted = s->hist[i][5];
                r.cr_credits_pending = s->hist[i][6];
                r.cr_credits_posted = s->hist[i][7];
            }
            r.timestamp = t->timestamp;
            out[n] = r;
        }
        n++;
    }
    return n;
}
