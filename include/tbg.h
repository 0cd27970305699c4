/*
 * tbg.h — C ABI of the MI355X batch-apply engine (libtbgpu.so).
 *
 * The engine replaces the body of the reference StateMachine's commit path for create_accounts,
 * create_transfers and pulse (src/state_machine.zig:543-1306, 1421-1929). Each entry point names
 * the reference interface it stands in for. Plain pointers and sizes only; all functions return
 * 0 on success and a negative status on failure. A failure is fatal for the caller (the reference
 * `commit` is infallible, state_machine.zig:1107-1115; device errors must panic the replica), and
 * the engine never partially applies a batch it rejected up front (bad input, capacity).
 *
 * Threading: an engine is driven by one host thread at a time (the replica event loop,
 * state_machine.zig:606-607: one prefetch or commit in flight).
 */
#ifndef TBG_H
#define TBG_H

#include <stddef.h>
#include <stdint.h>

#include "tb_types.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tbg_engine tbg_engine;

typedef struct tbg_config {
    int32_t device;          /* HIP device ordinal */
    uint32_t batch_max;      /* constants.batch_max (state_machine.zig:58-81); 0 = 8190 */
    uint64_t accounts_max;   /* capacity of the account store */
    uint64_t transfers_max;  /* capacity of the transfer store */
    uint32_t window_events_max; /* events per commit window (tbg_commit_window); 0 = batch_max */
    uint32_t flags;          /* TBG_FLAG_* */
    uint32_t shard_count;    /* 0: unsharded engine; G >= 1: this engine is one of G hash shards */
    uint32_t shard_index;    /* this engine's shard, < shard_count */
} tbg_config;

/* Keep a change log of each committed create_* window (tbg_window_changes): the write-back stream
   to the LSM forest. Costs three small kernels per window; off by default. */
#define TBG_FLAG_CHANGE_LOG 8u
/* Decide balance-limit windows on the sequential walker only (no account-parallel resolver). */
#define TBG_FLAG_NO_RESOLVER 1u
/* Walk W events on the single sequential walker only (no component-parallel walkers). */
#define TBG_FLAG_NO_COMPONENTS 2u
/* Resolve balance-limit windows with the wait-based account walkers (resolver.h) instead of the
   default windowed relaxation (relax.h). Same results; kept for comparison. */
#define TBG_FLAG_RES_WAIT 4u
/* Reject (TBG_E_WINDOW) every multi-batch window in which a pulse falls due, instead of modelling
   the pulses inside windows that span a second or more (tigerbeetle_amd/csrc/xwin.h). */
#define TBG_FLAG_NO_XWIN 16u
/* Resolve balance-limit windows with the grid-wide windowed relaxation (relax.h) even when their
   hot accounts fit the single-workgroup chunked resolver (chunks.h, the default). Same results. */
#define TBG_FLAG_NO_CHUNKS 32u
/* Commit every transfer window through the general path (no one-pass fused commit of order-free
   windows, tigerbeetle_amd/csrc/fused.h). Same results; for A/B timing and tests. */
#define TBG_FLAG_NO_FUSED 64u

#define TBG_OK 0
#define TBG_E_INVALID (-1)   /* input_valid() would reject the request */
#define TBG_E_CAPACITY (-2)  /* store capacity exceeded (no state changed) */
#define TBG_E_DEVICE (-3)    /* HIP runtime / device failure: fatal */
#define TBG_E_STATE (-4)     /* API misuse (e.g. commit timestamp not increasing) */
#define TBG_E_UNSUPPORTED (-5) /* sharded engine: a window outside the sharded class (nothing applied) */
#define TBG_E_WINDOW (-6)    /* a commit window spanned a due pulse it could not model: it and every window
                                queued after it were skipped (see tbg_commit_window); resubmit them in
                                smaller windows */

/* StateMachine.init (state_machine.zig:455-477) / deinit (:479-484). */
int tbg_create(const tbg_config *config, tbg_engine **out);
int tbg_destroy(tbg_engine *engine);

/* StateMachine.input_valid (state_machine.zig:543-572), a static function in the reference
 * (replica.zig:4855 calls StateMachine.input_valid(operation, body)): `engine` may be NULL, which
 * means batch_max = 8190. Returns 1 valid, 0 invalid. */
int tbg_input_valid(const tbg_engine *engine, uint32_t operation, uint64_t input_len);

/* StateMachine.pulse (state_machine.zig:589-596): *needed = pulse_next_timestamp <= prepare_ts, with
 * the reference's exact pulse_next_timestamp (lowered by every timeout creation that ran ok, also in
 * a chain rolled back later; reset to timestamp_min by a post/void of the transfer whose expiry it
 * holds; set by each pulse's finish). A host compare after a synchronous commit (which reads the value
 * back with its reply); synchronizes only when windows were queued since. */
int tbg_pulse_needed(tbg_engine *engine, uint64_t prepare_timestamp, int *needed);

/* StateMachine.prefetch (state_machine.zig:598-648): stages the request on the device and resolves
 * account/transfer slots asynchronously. Optional: commit() prefetches itself if this was not
 * called for the same input. */
int tbg_prefetch(tbg_engine *engine, uint64_t op, uint32_t operation, const void *input, uint64_t input_len,
                 uint64_t prefetch_timestamp);

/* StateMachine.commit (state_machine.zig:1107-1146) for every operation: pulse, create_accounts,
 * create_transfers, lookup_accounts, lookup_transfers, get_account_transfers and
 * get_account_balances (input: one tb_account_filter_t; reply: Transfer / AccountBalance records,
 * :1346-1419). Writes exactly the reply bytes the reference writes into `output` (for create_*:
 * packed {u32 index, u32 result} for non-ok events, ascending index) and the byte count into
 * *output_len. Synchronous. On a shard: pulses go through the general path (pulse_general in
 * tigerbeetle_amd/sharding.py), lookups and queries through tbg_shard_lookup / tbg_shard_query
 * (TBG_E_STATE here). */
int tbg_commit(tbg_engine *engine, uint64_t op, uint64_t timestamp, uint32_t operation, const void *input,
               uint64_t input_len, void *output, uint64_t output_cap, uint64_t *output_len);

/* Device-resident streaming form of commit for create_transfers / create_accounts: events already
 * in HBM, results left in HBM (d_results: n x 8 B; d_result_count: u32), fully asynchronous on the
 * engine's stream. If `auto_pulse` is set, the pulse decision pulse_next <= prepare_timestamp and
 * the pulse itself (at `timestamp`) run on the device before the batch, as the replica would. */
int tbg_commit_device(tbg_engine *engine, uint32_t operation, uint64_t timestamp, const void *d_events, uint32_t n,
                      void *d_results, uint32_t *d_result_count, int auto_pulse, uint64_t prepare_timestamp);

/* Super-batching: commits n_batches consecutive prepared batches (events contiguous in HBM at
 * d_events, batch b has batch_events[b] events and commit timestamp batch_timestamps[b]) in one
 * pass, with results identical to committing them one by one under the harness protocol (a pulse
 * check before every batch, state_machine.zig:2719-2739). Replies land in d_results, concatenated
 * per batch: batch b's replies are entries [d_batch_base[b], d_batch_base[b+1]), each with a
 * batch-relative index. With `auto_pulse`, the pulse decision for the first batch
 * (pulse_next <= prepare_timestamp) and the pulse run first, on the device. A pulse that expires
 * nothing inside the window (after a post/void reset pulse_next) is modelled exactly. A window whose
 * batches span a second or more models the pulses with expiries inside it too (csrc/xwin.h) when no
 * decision of it reads a balance, it writes no history row and no inner pulse can reach the scan
 * cap; otherwise it is rejected after its first pulse (that pulse applied, nothing else). Any other
 * window in which a pulse with expiries would fall due is rejected whole (its pulse included). A
 * rejected window skips every window queued after it too: tbg_sync() returns TBG_E_WINDOW and
 * tbg_windows_committed() tells how many windows were applied; resubmitting the same batches is
 * exact. Asynchronous on the engine stream. n_batches <= 128, total events <= window_events_max.
 * An order-free transfer window (plain creates between unlimited accounts, ids strictly increasing)
 * is committed by the one-pass fused kernels (csrc/fused.h); while a stream stays order-free its
 * windows launch nothing else, and a window that turns out not to be is re-run through the general
 * path at the next tbg_sync (or any call that reads state). So d_events, d_results and d_batch_base
 * must stay valid until tbg_sync returns. */
int tbg_commit_window(tbg_engine *engine, uint32_t operation, const void *d_events, uint32_t n_batches,
                      const uint32_t *batch_events, const uint64_t *batch_timestamps, void *d_results,
                      uint32_t *d_batch_base, int auto_pulse, uint64_t prepare_timestamp);

/* Host-fed form of tbg_commit_window: the replica's prepare bodies in host memory
 * (replica.zig:4151-4158 hands commit the message body). The window is staged into one of two
 * device slots on a copy stream, so the H2D of the next window overlaps this one's kernels; the
 * replies come back into h_results / h_batch_base (layout as tbg_commit_window; h_results must hold
 * one entry per event). Asynchronous: *ticket names the window for tbg_host_window_done. Host
 * buffers must be pinned (tbg_host_alloc) for the copies to overlap. */
int tbg_commit_window_host(tbg_engine *engine, uint32_t operation, const void *h_events, uint32_t n_batches,
                           const uint32_t *batch_events, const uint64_t *batch_timestamps, void *h_results,
                           uint32_t *h_batch_base, int auto_pulse, uint64_t prepare_timestamp, uint64_t *ticket);
/* *done = 1 once window `ticket` finished (h_events reusable, replies written). */
int tbg_host_window_done(tbg_engine *engine, uint64_t ticket, int *done);
/* Pinned, device-mapped host memory (hipHostMalloc, mapped) for message buffers the engine reads
 * from / writes to. */
int tbg_host_alloc(size_t bytes, void **out);
int tbg_host_free(void *p);
/* Page-locks and maps a caller-owned host range in place (hipHostRegister, mapped), e.g. a replica's
 * message pool (vsr/message_pool.zig allocates every message buffer once at startup): a 16 B-aligned
 * tbg_prefetch / tbg_commit request inside a registered or tbg_host_alloc range is read by the kernels
 * in place over PCIe (create_transfers: the fused pass itself, which copies it through to HBM; the
 * other operations: one copy kernel), without the copy into the engine's staging buffer or a
 * copy-engine transfer. The request must stay unchanged until its commit returns. */
int tbg_host_register(void *p, size_t bytes);
int tbg_host_unregister(void *p);

/* Waits for all work queued on the engine's stream. TBG_E_WINDOW (reported once) if a window was
 * rejected (see tbg_commit_window). */
int tbg_sync(tbg_engine *engine);
/* Create_* windows (and single-batch commits) applied by the device, and submitted by the host,
 * since tbg_create: after TBG_E_WINDOW, windows [applied, submitted) changed nothing. Synchronizes. */
int tbg_windows_committed(tbg_engine *engine, uint64_t *applied, uint64_t *submitted);
/* The engine's HIP stream (hipStream_t), for callers that time or order around it. */
void *tbg_stream(tbg_engine *engine);
/* Copies n bytes of device memory to `host` after the work queued on the engine stream, and waits:
 * a kernel on the stream writes them through the engine's mapped pinned block, so no copy-engine
 * handoff (~10 us each side) is paid on a small read (replies, counts). Any n, any alignment. */
int tbg_read_device(tbg_engine *engine, void *host, const void *d_src, uint64_t n);

/* Hash-sharded commit over G GPUs of one node (tigerbeetle_amd/csrc/shard.h). The replacement for
 * the same commit (state_machine.zig:1220-1306) when accounts are partitioned across engines:
 * account a lives on shard tbg_shard_of(a.id), transfer t on shard tbg_shard_of(t.id). Every shard
 * receives the same window (same arguments as tbg_commit_window) and is the home of a contiguous
 * range of its batches (it writes their replies):
 *   1. tbg_shard_prepare_window: one pass over the window; the owners validate and resolve what they
 *      own (accounts, transfer ids) and write tbg_shard_exchange_bytes(operation, E, G) bytes of owner
 *      facts at d_exchange: a 16 B trailer (two alternating verdict words), fixed-size counters (per
 *      shard its store room, 64 owned-id slots, 4096 ledger-mismatch slots of 8 B), then 2 B per
 *      create_transfers event / 1 B per create_accounts event (csrc/shard.h xch_view). d_exchange
 *      must be ONE buffer per shard, zeroed once at allocation and reused for every window: each
 *      window zeroes the counters and the other verdict word for the next one (tbg_reset / tbg_open
 *      restart the alternation on every shard alike);
 *   2. the caller sums those bytes element-wise across all G shards in place, ordered on the engine
 *      stream (ncclAllReduce(uint8, ncclSum) over xGMI, e.g. torch.distributed.all_reduce); every bit
 *      has exactly one writer, so the byte-wise sum is exact;
 *   3. tbg_shard_commit_window: every shard decides every event from the summed facts (the same
 *      outcome everywhere, so no second exchange), writes the replies of its home batches
 *      [home_first, home_first + home_count) (d_results / d_batch_base as tbg_commit_window, for the
 *      home batches only, d_batch_base[0..home_count]) and applies the owned effects of the committed
 *      events.
 * Sharded class: create_accounts and create_transfers without limits, balancing, two-phase or
 * in-window duplicate ids, overflow-free. Any other window is rejected whole on every shard:
 * tbg_sync returns TBG_E_UNSUPPORTED and no shard has applied it. Asynchronous on the engine stream. */
uint32_t tbg_shard_of(uint64_t id_lo, uint64_t id_hi, uint32_t shard_count);
uint64_t tbg_shard_exchange_bytes(uint32_t operation, uint32_t n_events, uint32_t shard_count);
int tbg_shard_prepare_window(tbg_engine *engine, uint32_t operation, const void *d_events, uint32_t n_batches,
                             const uint32_t *batch_events, const uint64_t *batch_timestamps, void *d_exchange);
int tbg_shard_commit_window(tbg_engine *engine, const void *d_exchange, uint32_t home_first, uint32_t home_count,
                            void *d_results, uint32_t *d_batch_base);

/* Routed sharded commit: partitioned ingestion (tigerbeetle_amd/csrc/route.h). Shard r receives only
 * the events of its HOME batches [home_bounds[r], home_bounds[r+1]) of the window (home_bounds has
 * shard_count + 1 entries, home_bounds[0] = 0, home_bounds[G] = n_batches, the same array on every
 * shard; rank order = batch order), plus the whole window's batch sizes and timestamps. Per window:
 *   tbg_route_prepare   stamps and validates the home events (state_machine.zig:1253, 1424-1439,
 *                       1465-1489) and writes one message block per destination shard: the stamped
 *                       record to the id owner, a 32 B {account id, amount, side} to each account owner;
 *   exchange A          all-to-all of those blocks (ncclSend/ncclRecv grouped; torch all_to_all_single);
 *   tbg_route_own       the owners check what they own: id claims (in-window duplicates) and `exists`
 *                       (:1506-1507, 1450-1460), the accounts (found, ledger, limit / history flags);
 *   exchange B          all-to-all of the replies back to the homes;
 *   tbg_route_decide    each home decides its events (:1496-1507, chains :1240-1300): commit bytes;
 *   exchange C          all-to-all of the commit bytes to the owners;
 *   tbg_route_apply     home replies (d_results / d_batch_base as tbg_commit_window, for the home batches
 *                       only) and the owners' effects: balance adds, records appended in timestamp order.
 * tbg_route_buffers(phase 0 / 1 / 2 = A / B / C) gives the exchange's device buffers: send_bytes[s] bytes
 * at d_send for shard s, blocks concatenated in shard order, likewise recv_bytes[s] at d_recv from shard s
 * (the splits of an uneven all-to-all). Each step is asynchronous on the engine stream; the exchanges
 * must be ordered on it. Class and rejection as tbg_shard_prepare_window's (TBG_E_UNSUPPORTED at
 * tbg_sync, nothing applied on any shard): the caller then gathers the whole window and commits it
 * through the general path. Sharded engines of at most 16 shards. A routed window holds up to G x 128
 * batches, each home's part at most 128 batches and window_events_max events. */
int tbg_route_prepare(tbg_engine *engine, uint32_t operation, const void *d_home_events, uint32_t n_batches,
                      const uint32_t *batch_events, const uint64_t *batch_timestamps, const uint32_t *home_bounds);
int tbg_route_buffers(tbg_engine *engine, uint32_t phase, void **d_send, uint64_t *send_bytes, void **d_recv,
                      uint64_t *recv_bytes);
/* The six exchange buffers (A send, A recv, B send, B recv, C send, C recv) are allocated by the engine
 * at its first routed window, or are the caller's: tbg_route_buffer_bytes gives their sizes for any
 * window of at most window_events_max events, tbg_route_attach binds them (16 B-aligned device memory,
 * e.g. tensors a collective library registers), before the first routed window. */
int tbg_route_buffer_bytes(tbg_engine *engine, uint64_t *bytes);
int tbg_route_attach(tbg_engine *engine, void *const *buffers);
int tbg_route_own(tbg_engine *engine);
int tbg_route_decide(tbg_engine *engine);
int tbg_route_apply(tbg_engine *engine, void *d_results, uint32_t *d_batch_base);

/* A hash-sharded group: G engines (one per GPU, or several on one GPU for tests) behind the
 * StateMachine interface, driven by one host thread (tigerbeetle_amd/csrc/group.inc). The replacement
 * for the reference's single StateMachine when accounts are partitioned across the GPUs of a node: a
 * replica calls tbg_group_pulse_needed / tbg_group_prefetch / tbg_group_commit exactly where it calls
 * pulse() / prefetch() / commit() (vsr/replica.zig:3764-3772, 4149-4159, 9459-9487), with the same
 * reply bytes as one engine. create_* batches go through the routed order-free path (tbg_route_*) and,
 * outside its class, through the general path (gathers, a scratch engine per shard, tbg_shard_apply);
 * pulses and lookups / queries gather from the owners. The exchanges are the group's own: device copies
 * (TBG_EXCHANGE_COPY) or one RCCL communicator per GPU (TBG_EXCHANGE_RCCL: ncclCommInitAll over the G
 * devices, librccl opened at creation; grouped ncclAllReduce / ncclSend / ncclRecv on the engine
 * streams). accounts_max / transfers_max are per shard. tbg_group_commit_window commits host-resident
 * batches under the harness protocol (a pulse check before every batch, state_machine.zig:2719-2739),
 * replies as tbg_commit_window's into host buffers. tbg_group_engine names shard r's engine (dumps,
 * stats, digests of its part of the state). */
typedef struct tbg_group tbg_group;
#define TBG_EXCHANGE_COPY 0u
#define TBG_EXCHANGE_RCCL 1u
typedef struct tbg_group_config {
    uint32_t shard_count;      /* G, 1..16 */
    uint32_t exchange;         /* TBG_EXCHANGE_* */
    const int32_t *devices;    /* G HIP device ordinals (RCCL: distinct) */
    uint32_t batch_max;        /* 0 = 8190 */
    uint32_t window_events_max;
    uint64_t accounts_max;     /* per shard */
    uint64_t transfers_max;    /* per shard */
    uint32_t flags;            /* TBG_FLAG_* of the shard engines */
    uint32_t reserved;
} tbg_group_config;
int tbg_group_create(const tbg_group_config *config, tbg_group **out);
int tbg_group_destroy(tbg_group *group);
int tbg_group_pulse_needed(tbg_group *group, uint64_t prepare_timestamp, int *needed);
int tbg_group_prefetch(tbg_group *group, uint64_t op, uint32_t operation, const void *input, uint64_t input_len,
                       uint64_t prefetch_timestamp);
int tbg_group_commit(tbg_group *group, uint64_t op, uint64_t timestamp, uint32_t operation, const void *input,
                     uint64_t input_len, void *output, uint64_t output_cap, uint64_t *output_len);
int tbg_group_commit_window(tbg_group *group, uint32_t operation, const void *h_events, uint32_t n_batches,
                            const uint32_t *batch_events, const uint64_t *batch_timestamps, void *h_results,
                            uint32_t *h_batch_base);
int tbg_group_engine(tbg_group *group, uint32_t shard, tbg_engine **engine);

/* StateMachine.open (state_machine.zig:527-541), after a restart or a state sync: an empty engine
 * takes the LSM forest's objects: every Account and every Transfer in timestamp order (the grooves'
 * object trees are keyed by timestamp) and, per transfer, its TransferPending status (0 none,
 * 1 pending, 2 posted, 3 voided, 4 expired; NULL = all 0), and the account_balances groove's rows
 * (historical_balance, :1806-1841; sorted by timestamp). pulse_next_timestamp starts at
 * timestamp_min, as in a freshly initialised StateMachine (:2063). TBG_E_STATE if not empty. A shard
 * is handed the same whole set and keeps what it owns (accounts and transfers by tbg_shard_of(id); a
 * status and a history row go with their transfer). */
int tbg_open(tbg_engine *engine, const tb_account_t *accounts, uint64_t n_accounts, const tb_transfer_t *transfers,
             uint64_t n_transfers, const uint8_t *pending_status,
             const tb_account_balances_value_t *account_balances, uint64_t n_account_balances);
/* StateMachine.reset (state_machine.zig:486-501): back to an empty state machine. */
int tbg_reset(tbg_engine *engine);
/* Prefetch completion (state_machine.zig:598-648 completes through a callback, possibly on the next
 * tick, groove.zig:753-757): *done = 1 once the device work of the last tbg_prefetch finished. */
int tbg_prefetch_poll(tbg_engine *engine, int *done);
/* StateMachine.compact (:1148-1173) / checkpoint (:1175-1188). The forest's beat belongs to the
 * replica; the engine's part is a barrier: every window committed so far is applied (and its
 * write-back stream can be drained) once these return TBG_OK. */
int tbg_compact(tbg_engine *engine, uint64_t op);
int tbg_checkpoint(tbg_engine *engine);
/* Whole-state digest for cross-replica determinism checks: out[0] accounts, out[1] transfers,
 * out[2] pending statuses (position-sensitive 64-bit sums, tigerbeetle_amd/digest.py restates
 * them), out[3] pulse_next_timestamp. Synchronizes. */
int tbg_digest(tbg_engine *engine, uint64_t out[4]);

/* TigerBeetle's checksum (vsr/checksum.zig:50-59: AEGIS-128L MAC, zero key) of n messages in HBM:
 * message k is the d_sizes[k] bytes at d_base + d_offsets[k]; its u128 checksum (little-endian, as
 * the Header fields store it) lands at d_out + 16 k. The replacement for checksum() on the prepare
 * bodies and headers a replica verifies (Header.valid_checksum / valid_checksum_body,
 * vsr/message_header.zig:105-137) and the replies it signs (replica.zig:4199-4202), for whole commit
 * windows or AOF files at once (tigerbeetle_amd/csrc/checksum.hip). Any alignment; 16-byte-aligned
 * messages load fastest. Asynchronous on `stream` (a hipStream_t; NULL = the default stream). */
int tbg_checksum(const void *d_base, const uint64_t *d_offsets, const uint32_t *d_sizes, uint32_t n, void *d_out,
                 void *stream);

/* tbg_commit_window's `auto_pulse` = TBG_WINDOW_LOG: the batches come from a replica's log (an AOF,
 * the journal), where every pulse is a prepare of its own (vsr.Operation.pulse, replica.zig:
 * 9459-9487) committed with tbg_commit(TB_OP_PULSE): no pulse is run or modelled between or before
 * the window's batches. */
#define TBG_WINDOW_LOG 2

/* Client-side reply demultiplexing (DemuxerType, state_machine.zig:133-176): a client that packed
 * several requests' events into one create_* batch splits the reply per request. init takes the
 * reply body (its results are rewritten in place); each decode(event_offset, event_count) returns
 * the results of the next request, indexes rebased to it, with monotonically increasing disjoint
 * ranges. Lookups and queries are not batched: event_offset must be 0 and the whole reply is
 * returned. TBG_E_INVALID for other operations or misaligned replies. Host-only. */
typedef struct tbg_demuxer {
    void *results;
    uint32_t count;
    uint32_t operation;
} tbg_demuxer;
int tbg_demux_init(tbg_demuxer *demuxer, uint32_t operation, void *reply, uint32_t reply_size);
int tbg_demux_decode(tbg_demuxer *demuxer, uint32_t event_offset, uint32_t event_count, void **results,
                     uint32_t *results_size);

/* Replay of an append-only file of prepares (aof.zig:23-55: entries of magic u128, 4080 B of
 * metadata, then the prepare message, each padded to 4096 B) into the engine, as a replica applies
 * its log: entries are checked in file order like AOF.Iterator.next (aof.zig:176-228: short read,
 * magic, header checksum, body checksum, hash chain parent == previous checksum) — every checksum of
 * the file verified on the GPU in bulk (tbg_checksum) — and the valid prefix is applied: runs of
 * create_accounts / create_transfers prepares as commit windows (TBG_WINDOW_LOG, batch timestamps
 * = header.timestamp), vsr pulse prepares as pulses; control-plane prepares, lookups and queries are
 * skipped (they change no state). Returns TBG_OK for a clean file, TBG_E_INVALID with
 * stats.error / stats.error_entry at the first bad entry (everything before it applied). `h_aof` is
 * host memory (e.g. an mmap of the file). */
#define TBG_AOF_OK 0
#define TBG_AOF_SHORT_READ 1      /* error.AOFShortRead */
#define TBG_AOF_MAGIC 2           /* error.AOFMagicNumberMismatch */
#define TBG_AOF_CHECKSUM 3        /* error.AOFChecksumMismatch */
#define TBG_AOF_BODY_CHECKSUM 4   /* error.AOFBodyChecksumMismatch */
#define TBG_AOF_CHAIN 5           /* error.AOFChecksumChainMismatch */
#define TBG_AOF_INPUT 6           /* a create_* prepare body that input_valid() rejects */
#define TBG_AOF_NO_CHAIN 1u       /* flags: skip the hash-chain check (Iterator.validate_chain = false) */
typedef struct tbg_aof_stats {
    uint64_t entries;        /* entries applied (prepares, pulses and skipped ones) */
    uint64_t prepares;       /* create_* prepares committed */
    uint64_t pulses;         /* pulse prepares committed */
    uint64_t skipped;        /* other prepares */
    uint64_t windows;        /* commit windows launched */
    uint64_t events;         /* create_* events committed */
    uint64_t failed_events;  /* of which failed with a result code */
    int64_t error_entry;     /* index of the first bad entry, -1 if none */
    int32_t error;           /* TBG_AOF_* */
    int32_t reserved;
} tbg_aof_stats;
int tbg_aof_replay(tbg_engine *engine, const void *h_aof, uint64_t size, uint32_t flags, tbg_aof_stats *stats);

/* Sharded engines, general class (tigerbeetle_amd/csrc/shard_gx.inc): a batch outside the
 * order-free class (balance limits, balancing, two-phase, in-window duplicate ids) or with a pulse
 * due before it is decided on every shard identically from its gathered read set:
 *   tbg_shard_gather(phase 1), sum across the shards, tbg_shard_gather(phase 2) into the buffer's
 *   second region, sum that region, then every shard opens its scratch unsharded engine from the
 *   gathered objects (tbg_reset + tbg_open_device, the shards' common pulse_next_timestamp),
 *   commits the batch there with its pulse (tbg_commit_window, auto_pulse), and applies the
 *   post-batch objects it owns (tbg_device_state of the scratch engine -> tbg_shard_apply).
 * The buffer (tbg_shard_gather_bytes, 256-byte aligned) holds one writer per slot, so its byte-wise
 * sum is the union. The C-ABI steps are device work on the engine stream; the Python driver
 * (tigerbeetle_amd/sharding.py) dedupes and orders the gathered objects. */
uint64_t tbg_shard_gather_bytes(uint32_t n_events, uint32_t shard_count, uint32_t batch_max, uint64_t *phase2_offset);
int tbg_shard_gather(tbg_engine *engine, uint32_t operation, const void *d_events, uint32_t n_events,
                     uint64_t timestamp, uint32_t phase, void *d_buffer);
/* The general class a whole window at a time (tigerbeetle_amd/csrc/shard_gw.inc; replaces one gather
 * round per batch). Every shard lists the objects it owns of the window's read set, each once (phase 1:
 * the accounts and stored transfers the events name, every live entry due at or before t_last — the
 * window's last batch timestamp — and the smallest live entry beyond it; phase 2: the accounts of the
 * phase-1 transfers), and the lists are concatenated across the shards by sums:
 *   tbg_gw_collect(phase): this shard's counts into its words of d_counts (16 x G bytes, the rest
 *     zeroed); sum d_counts across the shards;
 *   tbg_gw_write(phase): (synchronous: reads the summed counts) zero-fills the regions and writes this
 *     shard's records at its offset: phase 1 accounts [0, a1) of d_accounts and transfers [0, x1) of
 *     d_transfers / d_status (*n_accounts = a1, *n_transfers = x1), phase 2 accounts [a1, a1 + a2)
 *     (*n_accounts = a2); sum those regions. *overflow = 1 (phase 1) when a shard had more than due_cap
 *     entries due: nothing written, commit the window batch by batch (tbg_shard_gather);
 *   tbg_gw_commit: the scratch engine `scratch` (an unsharded engine of this process whose
 *     accounts_max records fit d_accounts: its account store is bound to it) keeps the acc_base
 *     accounts it held after the previous general window (0: it starts over; then tbg_gw_collect must
 *     have been called with restart = 1, and the accounts are gathered at d_accounts + acc_base),
 *     takes the gathered records (transfers sorted by timestamp) with no host round trip, commits the
 *     window (tbg_commit_window semantics, replies into d_results / d_batch_base), and this shard
 *     applies its part (every scratch account it owns that changed, its gathered transfers' statuses,
 *     the new records it owns, its pulse_next_timestamp). Asynchronous. The scratch may be kept only
 *     while nothing but general windows commits on the shards: restart after any other commit, pulse or
 *     open;
 *   tbg_gw_result: waits; *rejected = 1 when the scratch engine rejected the window (a pulse inside it
 *     reaching the expiry cap, or one falling due in a window that reads balances): nothing was applied
 *     on the shard, commit it batch by batch (and restart the scratch). *scratch_accounts: the
 *     next window's acc_base. TBG_E_CAPACITY when this shard's stores could not take its new records
 *     (nothing applied on it). */
int tbg_gw_collect(tbg_engine *engine, uint32_t operation, const void *d_events, uint32_t n_events, uint64_t t_last,
                   uint32_t phase, uint32_t due_cap, const void *d_gathered_transfers, uint32_t n_gathered_transfers,
                   void *d_counts, int restart);
int tbg_gw_write(tbg_engine *engine, uint32_t phase, const void *d_counts, void *d_accounts, uint64_t accounts_cap,
                 void *d_transfers, uint8_t *d_status, uint64_t transfers_cap, uint32_t *n_accounts,
                 uint32_t *n_transfers, int *overflow);
int tbg_gw_commit(tbg_engine *engine, tbg_engine *scratch, uint32_t operation, const void *d_events,
                  uint32_t n_batches, const uint32_t *batch_events, const uint64_t *batch_timestamps, void *d_accounts,
                  uint64_t acc_base, const void *d_transfers, const uint8_t *d_status, void *d_results,
                  uint32_t *d_batch_base, int auto_pulse, uint64_t prepare_timestamp);
int tbg_gw_result(tbg_engine *engine, tbg_engine *scratch, int *rejected, uint64_t *scratch_accounts);
/* d_history / d_history_side (tbg_device_history of the scratch engine, may be NULL): the history
 * row beside each of d_transfers, kept with the transfers this shard inserts. With
 * TBG_FLAG_CHANGE_LOG the shard's write-back stream (tbg_window_changes) then lists what changed on
 * this shard: updated accounts, inserted records, TransferPending rows. */
int tbg_shard_apply(tbg_engine *engine, const tb_account_t *d_accounts, uint64_t n_accounts,
                    const tb_transfer_t *d_transfers, const uint8_t *d_status, uint64_t n_transfers,
                    const void *d_history, const uint8_t *d_history_side, uint64_t pulse_next_timestamp);

/* Reads on a sharded engine (tigerbeetle_amd/csrc/shard_read.inc): every shard gets the same request
 * body and writes what it owns into its part of a device buffer; the caller sums the buffer
 * byte-wise across the shards in place (the same uint8 all-reduce as the commit path; one writer per
 * byte); then any shard builds the reply, byte-identical to an unsharded engine's tbg_commit reply.
 *   lookup_accounts / lookup_transfers (state_machine.zig:1309-1344): tbg_shard_lookup_bytes(n ids),
 *     tbg_shard_lookup (asynchronous), sum, tbg_shard_lookup_reply (synchronous);
 *   get_account_transfers / get_account_balances (:786-996, 1346-1419):
 *     tbg_shard_query_bytes(shard_count, batch_max), tbg_shard_query (synchronous: each shard's
 *     first min(limit, batch_max) matches in scan order, with their history rows), sum,
 *     tbg_shard_query_merge (the regions merged by timestamp in scan order, cut at the limit). */
uint64_t tbg_shard_lookup_bytes(uint32_t n_ids);
int tbg_shard_lookup(tbg_engine *engine, uint32_t operation, const void *input, uint64_t input_len, void *d_buffer);
int tbg_shard_lookup_reply(tbg_engine *engine, const void *d_buffer, uint64_t input_len, void *output,
                           uint64_t output_cap, uint64_t *output_len);
uint64_t tbg_shard_query_bytes(uint32_t shard_count, uint32_t batch_max);
int tbg_shard_query(tbg_engine *engine, uint32_t operation, const void *filter, uint64_t filter_len, void *d_buffer);
int tbg_shard_query_merge(tbg_engine *engine, uint32_t operation, const void *filter, const void *d_buffer,
                          void *output, uint64_t output_cap, uint64_t *output_len);
/* Unsharded engines: open (as tbg_open) from device-resident objects in timestamp order with the
 * given pulse_next_timestamp; and the device view of the whole state (valid until the next call
 * that changes it). */
int tbg_open_device(tbg_engine *engine, const tb_account_t *d_accounts, uint64_t n_accounts,
                    const tb_transfer_t *d_transfers, const uint8_t *d_status, uint64_t n_transfers,
                    uint64_t pulse_next_timestamp);
int tbg_device_state(tbg_engine *engine, const tb_account_t **accounts, uint64_t *n_accounts,
                     const tb_transfer_t **transfers, const uint8_t **status, uint64_t *n_transfers,
                     uint64_t *pulse_next_timestamp);
/* The history rows beside those transfer records (128 B per slot: the debit then the credit
 * account's four balances after the transfer) and per slot the sides present (bit 0 debit, bit 1
 * credit). */
int tbg_device_history(tbg_engine *engine, const void **rows, const uint8_t **sides);

/* Test hook mirroring the harness `setup` action (state_machine.zig:2545-2561). */
int tbg_setup_balances(tbg_engine *engine, const tb_uint128_t *id, const tb_uint128_t *debits_pending,
                       const tb_uint128_t *debits_posted, const tb_uint128_t *credits_pending,
                       const tb_uint128_t *credits_posted);

typedef struct tbg_stats {
    uint64_t accounts;        /* accounts stored */
    uint64_t transfers;       /* transfers stored */
    uint64_t expiry_entries;  /* entries in the live expires_at list */
    uint64_t pulse_next_timestamp;
    uint64_t events_total;    /* create_* events committed through the engine */
    uint64_t walker_events;   /* of which ran on the sequential walker */
    uint64_t resolver_events; /* of which the account-parallel resolver decided */
    uint64_t component_events; /* of which component-parallel walkers decided */
    uint64_t sorted_transfers; /* leading transfer records in the sorted id prefix (not hashed) */
    uint64_t chunked_windows;  /* balance-limit windows the chunked resolver decided */
    uint64_t fused_windows;    /* order-free transfer windows committed in one pass (fused.h) */
    uint64_t ovf_rescans;     /* times the overflow bound was re-tightened (restore.h k_ovf_rescan) */
} tbg_stats;
int tbg_get_stats(tbg_engine *engine, tbg_stats *out);

/* Debug: cumulative resolver counters (see host.inc); up to 8 values. */
/* Debug: entries in use of the account and transfer hash tables (every window in flight settled).
 * Bounded by the stored accounts / hashed transfers: an aborted fused window leaves no entry behind. */
int tbg_debug_table_used(tbg_engine *engine, uint64_t *accounts_used, uint64_t *transfers_used);
int tbg_debug_counters(tbg_engine *engine, uint64_t *out, uint32_t n);

/* Write-back stream of the last commit call (TBG_FLAG_CHANGE_LOG; state_machine.zig groove side
 * effects: groove.insert/update, lsm/groove.zig:905-1000), covering its pulse and its create_*
 * window: every account record whose balances they changed (current values, ascending creation
 * order) followed by the accounts the window created, every transfer record it inserted (commit
 * order), and the TransferPending rows inserted or updated (new pending transfers, earlier ones
 * posted, voided or expired; ascending timestamp). On a shard: what changed among the objects it owns
 * (an order-free window, or the general path's tbg_shard_apply). Synchronous.
 * TBG_E_CAPACITY if a buffer is too small (the counts are still written); TBG_E_STATE without the
 * flag. */
int tbg_window_changes(tbg_engine *engine, tb_account_t *accounts, uint64_t accounts_cap, uint64_t *accounts_count,
                       tb_transfer_t *transfers, uint64_t transfers_cap, uint64_t *transfers_count,
                       tb_transfer_pending_t *pending, uint64_t pending_cap, uint64_t *pending_count);

/* Whole-state dumps in creation (= timestamp) order, for parity checks. */
int tbg_dump_accounts(tbg_engine *engine, tb_account_t *out, uint64_t cap, uint64_t *count);
int tbg_dump_transfers(tbg_engine *engine, tb_transfer_t *out, uint64_t cap, uint64_t *count);
/* Pending status per stored transfer (0 none, 1 pending, 2 posted, 3 voided, 4 expired). */
int tbg_dump_transfer_status(tbg_engine *engine, uint8_t *out, uint64_t cap, uint64_t *count);
/* Device pointers to the dense stores (for on-device digests); valid until the next commit. */
int tbg_device_stores(tbg_engine *engine, const tb_account_t **accounts, const tb_transfer_t **transfers);

/* Synthetic request streams generated directly in HBM (tigerbeetle_amd/csrc/workload.hip),
 * shaped like the reference benchmark (src/tigerbeetle/benchmark_load.zig:206-327). `stream` is a
 * hipStream_t (e.g. tbg_stream(engine)). Bit-identical to tigerbeetle_amd/workload.py. */
/* Id orders of `tigerbeetle benchmark --id-order` (cli.zig:97, 263-265; testing/id.zig:8-48): rewrite,
 * in place, the sequential ids (data = index + 1) of `count` generated records in HBM as
 * IdPermutation.encode(data): order 0 sequential, 1 random (pseudo-UUID from Xoshiro256(seed +% data),
 * the reference's own ids for permutation seed `seed`), 2 reversed (maxInt(u128) - data). Accounts: the
 * id; transfers (`transfers` = 1): the id, both account ids and pending_id (0 and ids >= 2^64 stay). */
int tbg_gen_permute_ids(void *d_records, uint64_t count, uint32_t transfers, uint32_t order, uint64_t seed,
                        void *stream);
int tbg_gen_accounts(void *d_out, uint64_t first, uint64_t count, uint64_t seed, uint32_t ledger, uint16_t code,
                     uint16_t flags, void *stream);
int tbg_gen_transfers_uniform(void *d_out, uint64_t first, uint64_t count, uint64_t seed, uint64_t n_accounts,
                              uint64_t id_offset, void *stream);
/* Mixed streams: transfer `first + k` of `count` generated records with (first + k) % every == every - 1
 * becomes a pending create (flags.pending, `timeout` seconds); every == 0 leaves them all. */
int tbg_gen_mark_pending(void *d_records, uint64_t first, uint64_t count, uint64_t every, uint32_t timeout,
                         void *stream);

/* Per-phase kernel timing with HIP events on the engine stream. Phases: 0 prep, 1 resolve
 * (account-parallel resolver), 2 classify, 3 wcount, 4 wlist, 5 walk, 6 final, 7 pulse (all five
 * pulse kernels), 8 cpw (component walkers). enable: < 0 every phase, 0 off, > 0 a bitmask of
 * phases (each timed phase costs the stream two event records). collect() synchronizes, returns
 * the summed milliseconds and launch counts per phase since the last collect, and resets. */
int tbg_timing_enable(tbg_engine *engine, int enable);
int tbg_timing_collect(tbg_engine *engine, double *ms, uint64_t *launches, uint32_t n_phases);

/* Introspection of the last create_* batch: per-event class bits and final codes (debugging). */
int tbg_debug_last_batch(tbg_engine *engine, uint32_t *cls, uint32_t *code, uint32_t n);

/* cfg3: accounts with debits_must_not_exceed_credits on rank < limited_top and on ~half the rest
 * (ranks >= n_accounts are unlimited treasury accounts); funding transfers credit account k from
 * treasury account k % treasury; Zipf-distributed transfers over a u64 CDF table in HBM
 * (tigerbeetle_amd.workload.zipf_cdf). */
int tbg_gen_accounts_cfg3(void *d_out, uint64_t first, uint64_t count, uint64_t seed, uint64_t n_accounts,
                          uint64_t limited_top, void *stream);
int tbg_gen_funding_cfg3(void *d_out, uint64_t first, uint64_t count, uint64_t seed, uint64_t n_accounts,
                         uint64_t treasury, uint64_t amount, uint64_t id_offset, void *stream);
int tbg_gen_transfers_zipf(void *d_out, uint64_t first, uint64_t count, uint64_t seed, uint64_t n_accounts,
                           const void *d_cdf, uint64_t id_offset, void *stream);
/* cfg4: two-phase (30 % pending with 1-60 s timeouts, ~20 % post / ~10 % void of earlier pending
 * transfers) with ~10 % of events in linked chains of 2-8, a quarter of them with an injected
 * failure. */
int tbg_gen_transfers_cfg4(void *d_out, uint64_t first, uint64_t count, uint64_t seed, uint64_t n_accounts,
                           uint64_t batch, uint64_t id_offset, void *stream);

/* Library build identification ("gfx950 ..."). */
const char *tbg_version(void);

#ifdef __cplusplus
}
#endif

#endif /* TBG_H */
