"""Probe: does torch.cuda.synchronize() wait for work on the engine's non-blocking stream?"""
import torch

from tigerbeetle_amd import StateMachine, _lib

sm = StateMachine(batch_max=8190, accounts_max=1024, transfers_max=1024)
ext = torch.cuda.ExternalStream(sm.stream)
buf = torch.empty(60_000_000 * 128, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
L = _lib.lib()
for trial in range(3):
    _lib.check(L.tbg_gen_transfers_uniform(buf.data_ptr(), 0, 60_000_000, 1, 1000, 0, sm.stream), "gen")
    before = ext.query()
    torch.cuda.synchronize()
    after = ext.query()
    print(f"trial {trial}: engine stream idle before sync={before}, after torch.cuda.synchronize()={after}",
          flush=True)
sm.close()
