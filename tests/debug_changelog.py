import sys, os
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
os.chdir("/root/repo")
import numpy as np
from chaos import Chaos
from oracle_sm import OracleStateMachine
from test_gpu_window import commit_window, oracle_batches
from tigerbeetle_amd.types import NS_PER_S, Operation
from tigerbeetle_amd import StateMachine
seed, win, bm = 0, 4, 64
gpu = StateMachine(batch_max=bm, accounts_max=1 << 12, transfers_max=1 << 17, window_events_max=win * bm, change_log=True)
ref = OracleStateMachine(batch_max=bm)
ch = Chaos(500 + seed, n_accounts=60, id_space=3000)
for w in range(10):
    x0 = ref.dump_transfers()
    tick = NS_PER_S if w >= 3 else 0
    if w < 2 or w == 6:
        op = Operation.create_accounts
        batches = [ch.accounts_batch(ch.rng.randint(1, bm)) for _ in range(win)]
    else:
        op = Operation.create_transfers
        batches = [ch.transfers_batch(ch.rng.randint(1, bm)) for _ in range(win)]
    g = commit_window(gpu, op, batches, tick); r = oracle_batches(ref, op, batches, tick)
    print("window", w, "replies equal", g == r)
    x1 = ref.dump_transfers(); gx = gpu.dump_transfers()
    print(" store equal", gx.tobytes() == x1.tobytes(), len(gx), len(x1))
    la, lx, rows = gpu.window_changes()
    new = x1[len(x0):]
    if lx.tobytes() != new.tobytes():
        print(" changelog differs", len(lx), len(new))
        for k in range(min(len(lx), len(new))):
            if lx[k].tobytes() != new[k].tobytes():
                print("  rec", k, "gpu", lx[k], "\n  ref", new[k]); break
        st = gpu.stats(); print(st)
        break
