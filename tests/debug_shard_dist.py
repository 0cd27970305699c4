"""Debug: two-rank gloo general path, status mismatches vs the restatement (GPU box)."""
import os
import sys
import tempfile

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import numpy as np  # noqa: E402

import test_gpu_shard_general as t  # noqa: E402
from chaos import run_protocol  # noqa: E402
from oracle_sm import OracleStateMachine  # noqa: E402

if __name__ == "__main__":
    import torch.multiprocessing as mp

    d = tempfile.mkdtemp()
    mp.spawn(t._rank_main, args=(2, t._free_port(), 7200, 16, d), nprocs=2, join=True)
    ref = OracleStateMachine(batch_max=16)
    for op, ev, tick in t._dist_stream(7200, 16):
        run_protocol(ref, op, ev, tick)
    xs = [np.load(os.path.join(d, f"xfer{r}.npy")) for r in range(2)]
    sts = [np.load(os.path.join(d, f"st{r}.npy")) for r in range(2)]
    rx, rs = ref.dump_transfers(), ref.dump_transfer_status()
    pos = {int(ts): k for k, ts in enumerate(rx["timestamp"])}
    bad = 0
    for r in range(2):
        for k in range(len(xs[r])):
            j = pos[int(xs[r]["timestamp"][k])]
            if sts[r][k] != rs[j]:
                bad += 1
                if bad < 10:
                    print("rank", r, "slot", k, "ts", int(xs[r]["timestamp"][k]), "flags", int(xs[r]["flags"][k]),
                          "timeout", int(xs[r]["timeout"][k]), "shard st", int(sts[r][k]), "ref st", int(rs[j]))
    print("mismatches", bad, "of", len(rx))

    # the same stream in-process (LocalShards, general path for every batch)
    import torch

    from test_gpu_shard import LocalShards
    from tigerbeetle_amd.sharding import commit_general_batch

    sh = LocalShards(2, 16, 1024, 1 << 14, 16)
    ref2 = OracleStateMachine(batch_max=16)
    ts = 0
    for b, (op, ev, tick) in enumerate(t._dist_stream(7200, 16)):
        ts += tick + 1 + len(ev)
        d_ev = torch.from_numpy(np.frombuffer(ev.tobytes(), np.uint8).copy()).cuda()
        torch.cuda.synchronize()
        g = commit_general_batch(sh.shards, sh.summed, op, d_ev.data_ptr(), len(ev), ts)
        r = run_protocol(ref2, op, ev, tick)
        st_sh = t._statuses(sh)
        st_ref = ref2.dump_transfer_status()
        if g != r or st_sh.tobytes() != st_ref.tobytes():
            print("in-process: batch", b, "reply", g == r, "statuses", st_sh.tolist(), st_ref.tolist())
            break
    else:
        print("in-process: all equal")
