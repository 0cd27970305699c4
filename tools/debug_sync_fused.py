"""GPU box: per-batch fused-window count of the synchronous prefetch/commit path after one batch
outside the fused class (pending transfers with timeouts), then clean batches."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from chaos import run_protocol  # noqa: E402
from test_gpu_fused import BM, _accounts, _engines  # noqa: E402
from tigerbeetle_amd import workload  # noqa: E402
from tigerbeetle_amd.types import Operation  # noqa: E402

n_acc = 2000
gpu, ref = _engines(n_acc + 2, 1 << 19)
_accounts(gpu, ref, n_acc + 2, flags={n_acc: 2})
first = 0
for b in range(14):
    ev = workload.transfers_uniform(first, BM, seed=41, n_accounts=n_acc)
    first += BM
    if b == 2:
        ev["flags"][::37] = 2
        ev["timeout"][::37] = 1
    tick = 2 * 10**9 if b == 3 else 0
    same = run_protocol(gpu, Operation.create_transfers, ev, tick) == run_protocol(ref, Operation.create_transfers, ev, tick)
    st = gpu.stats()
    print(b, "same" if same else "DIFF", "fused", st["fused_windows"], "pulse_next", st["pulse_next_timestamp"],
          "expiry", st["expiry_entries"], flush=True)
gpu.close()
