// shard_gw.h — host/device state of the sharded general window (shard_gw.inc), declared before the
// engine struct (host.inc) that holds it.
#pragma once
#include "restore.h"

struct GwLists {
  uint32_t* acc_mark;  // per owned account slot: the gather epoch that listed it
  uint32_t* x_mark;    // per owned transfer slot
  uint32_t* acc_list;  // listed account slots: phase 1, then phase 2
  uint32_t* x_list;    // listed transfer slots (phase 1)
  uint32_t* cnt;       // [0] accounts phase 1, [1] transfers, [2] accounts phase 2, [3] due entries,
                       // [4] nd_slot, [6..7] nd_min (u64)
  uint32_t acc_cap, x_cap;
};

// This shard's rows of the exchange order.
struct GwOwn {
  uint32_t a1_off, a1_cnt, a1_tot, a2_off, a2_cnt, a2_tot, x1_off, x1_cnt, x1_tot;
};

struct GwState {
  GwLists L;
  uint32_t gep;               // gather epoch (bumped per window)
  uint32_t cap_events, cap_due;
  GwOwn own;
  uint32_t due_overflow;      // a shard had more than due_cap entries due in the window's span
  uint32_t* perm;             // per scratch transfer slot: its row of the exchange order
  unsigned long long *tkey_in, *tkey_out;
  uint32_t* tval_in;
  void* sort_tmp;
  size_t sort_tmp_bytes;
  uint32_t x_sort_cap;
  uint32_t* flags;            // new-record ownership flags, then ranks (apply)
  uint32_t* ranks;
  uint32_t flags_cap;
  LoadBound* lb;
  // The scratch engine's accounts persist across consecutive general windows (nothing else changes
  // them meanwhile; the caller restarts the scratch after any other commit): per owned account the
  // scratch generation that holds it, per scratch account slot this shard's slot of it (NONE32: another
  // shard's), the generation, and the scratch's account count before this window's gathered ones.
  uint32_t* acc_sc;
  uint32_t* sc2my;
  uint64_t sc2my_cap;
  uint32_t sc_gen;
  uint32_t acc_base;
};

