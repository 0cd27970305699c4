"""Host restatement of the engine's whole-state digest (tbg_digest, csrc/restore.h): position-
sensitive 64-bit sums over the dense account and transfer stores and the pending statuses. Lets a
caller compare a GPU engine's state with records it holds on the host (another replica, the CPU
restatement's dumps) without copying the engine's stores back."""
import numpy as np

M64 = (1 << 64) - 1
C1, C2 = np.uint64(0xFF51AFD7ED558CCD), np.uint64(0xC4CEB9FE1A85EC53)


def mix64(x):
    x = x ^ (x >> np.uint64(33))
    x = x * C1
    x = x ^ (x >> np.uint64(33))
    x = x * C2
    return x ^ (x >> np.uint64(33))


def _records(records):
    """Sum over records (n x 128 B) of digest_record(words, slot)."""
    n = len(records)
    if n == 0:
        return 0
    w = np.frombuffer(np.ascontiguousarray(records).tobytes(), np.uint64).reshape(n, 16)
    slot = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        h = np.uint64(0x243F6A8885A308D3) ^ slot
        for k in range(16):
            h = mix64(h ^ w[:, k] ^ np.uint64(k << 56))
        h = mix64(h + slot * np.uint64(0x9E3779B97F4A7C15))
    return int(h.sum(dtype=np.uint64))


def _statuses(status):
    n = len(status)
    if n == 0:
        return 0
    with np.errstate(over="ignore"):
        k = np.arange(n, dtype=np.uint64)
        return int(mix64((k << np.uint64(8)) | status.astype(np.uint64)).sum(dtype=np.uint64))


def digest(accounts, transfers, status, pulse_next):
    """[accounts, transfers, statuses, pulse_next_timestamp], as tbg_digest returns them."""
    return [_records(accounts), _records(transfers), _statuses(np.asarray(status, np.uint8)), int(pulse_next)]
