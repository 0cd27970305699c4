"""One rank of torch.distributed "nccl" (RCCL on ROCm) driving the sharded engine: the RCCL calls the
multi-GPU bench makes (all_to_all_single with uneven splits for routed windows, all_reduce for the
general path's gathers and pulses), on the engine stream, with a world of one (this pool hands out
one GPU per call, and RCCL refuses two ranks on one device). Replies are compared with the
unsharded engine on the same batches. Run by tests/test_gpu_rccl.py in its own process:

    python tests/rccl_one_rank.py PORT
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)


def main():
    import torch
    import torch.distributed as dist

    from test_gpu_window import commit_window
    from tigerbeetle_amd import StateMachine, workload
    from tigerbeetle_amd.sharding import ShardedStateMachine, alltoall_nccl, exchange_nccl
    from tigerbeetle_amd.state_machine import to_host
    from tigerbeetle_amd.types import NS_PER_S, Operation

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%s" % sys.argv[1], rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    BM, n_acc, win = 1024, 5000, 4
    sh = ShardedStateMachine(1, 0, exchange_nccl, device=0, batch_max=BM, accounts_max=n_acc + 1024,
                             transfers_max=1 << 16, window_events_max=win * BM)
    sh.alltoall = alltoall_nccl
    ref = StateMachine(batch_max=BM, accounts_max=n_acc + 1024, transfers_max=1 << 16, window_events_max=win * BM)
    ts = 0

    def routed(op, batches):
        nonlocal ts
        ns, tss = [], []
        for b in batches:
            ts += 1 + len(b)
            ns.append(len(b))
            tss.append(ts)
        data = np.concatenate([np.frombuffer(b.tobytes(), np.uint8) for b in batches])
        d_ev = torch.from_numpy(data.copy()).cuda()
        d_res = torch.zeros(len(data) // 128 * 8, dtype=torch.uint8, device="cuda")
        d_base = torch.zeros(len(ns) + 1, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        if sh.pulse(tss[0]):
            sh.commit_pulse(tss[0])
        first, count = sh.commit_window_routed(op, d_ev.data_ptr(), ns, tss, d_res.data_ptr(), d_base.data_ptr())
        sh.sync()
        torch.cuda.synchronize()
        rb, base = to_host(d_res).tobytes(), to_host(d_base)
        return [rb[base[k] * 8: base[k + 1] * 8] for k in range(count)]

    def general(op, batches):
        nonlocal ts
        ns, tss = [], []
        for b in batches:
            ts += 1 + len(b)
            ns.append(len(b))
            tss.append(ts)
        data = np.concatenate([np.frombuffer(b.tobytes(), np.uint8) for b in batches])
        d_ev = torch.from_numpy(data.copy()).cuda()
        torch.cuda.synchronize()
        out = sh.commit_general_window(op, d_ev.data_ptr(), ns, tss)
        sh.sync()
        return out

    acc = [workload.accounts(f, min(BM, n_acc - f), seed=3) for f in range(0, n_acc, BM)]
    for w0 in range(0, len(acc), win):
        assert routed(Operation.create_accounts, acc[w0:w0 + win]) == commit_window(ref, Operation.create_accounts,
                                                                                   acc[w0:w0 + win])
    n_routed = 0
    for w in range(4):  # uniform: the routed class (three RCCL all-to-alls per window)
        xb = [workload.transfers_uniform((w * win + k) * BM, BM, seed=3, n_accounts=n_acc) for k in range(win)]
        assert routed(Operation.create_transfers, xb) == commit_window(ref, Operation.create_transfers, xb), w
        n_routed += 1
    # two-phase (cfg4's generator): the general path, its gathers summed by RCCL all-reduces
    for w in range(2):
        xb = [workload.transfers_cfg4((64 + w * win + k) * BM, BM, 3, n_acc, BM) for k in range(win)]
        g = general(Operation.create_transfers, xb)
        r = commit_window(ref, Operation.create_transfers, xb)
        assert g == r, w
    assert sh.pulse_next() == ref.pulse_next_timestamp()
    print("rccl one-rank ok: %d routed windows, 2 general windows (backend %s)" % (n_routed, dist.get_backend()))
    sh.close()
    ref.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
