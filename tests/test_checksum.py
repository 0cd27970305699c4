"""TigerBeetle's checksum (vsr/checksum.zig): AEGIS-128L MAC with a zero key.

The CPU restatement (oracle/aegis.c) is pinned by the reference's own known answers: the two test
vectors (vsr/checksum.zig:54, 100-111) and the "checksum stability" hash over 896 cases
(:146-195: zeros of 0..127 bytes, 64-byte one-hot messages, Xoshiro256(92)-filled messages of
13..268 bytes). The GPU kernel (csrc/checksum.hip, tbg_checksum) is checked against the same known
answers and against the restatement on random messages of every length class, at unaligned
offsets, and on whole-window bodies (1 MiB prepares)."""
import ctypes
import os
import random

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
M64 = (1 << 64) - 1
VECTORS = [
    (bytes(16), int.from_bytes((0xf72ad48dd05dd1656133101cd4be3a26).to_bytes(16, "big"), "little")),
    (b"", 0x49F174618255402DE6E7E3C40D60CC83),
]
STABILITY = 0x82dcaacf4875b279446825b6830d1263


def _oracle():
    L = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
    L.tbo_checksum.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
    return L


def oracle_checksum(data):
    out = ctypes.create_string_buffer(16)
    _oracle().tbo_checksum(bytes(data), len(data), out)
    return int.from_bytes(out.raw, "little")


class Xoshiro256:
    """Zig std.rand.Xoshiro256 (xoshiro256++, SplitMix64 seeding) and its fill(): the generator the
    stability test draws its messages from."""

    def __init__(self, seed):
        s = seed & M64
        self.s = []
        for _ in range(4):
            s = (s + 0x9e3779b97f4a7c15) & M64
            z = s
            z = ((z ^ (z >> 30)) * 0xbf58476d1ce4e5b9) & M64
            z = ((z ^ (z >> 27)) * 0x94d049bb133111eb) & M64
            self.s.append(z ^ (z >> 31))

    @staticmethod
    def _rotl(x, k):
        return ((x << k) | (x >> (64 - k))) & M64

    def next(self):
        s0, s1, s2, s3 = self.s
        r = (self._rotl((s0 + s3) & M64, 23) + s0) & M64
        t = (s1 << 17) & M64
        s2 ^= s0
        s3 ^= s1
        s1 ^= s2
        s0 ^= s3
        s2 ^= t
        s3 = self._rotl(s3, 45)
        self.s = [s0, s1, s2, s3]
        return r

    def fill(self, n):
        out = bytearray()
        while len(out) + 8 <= n:
            out += self.next().to_bytes(8, "little")
        if len(out) != n:
            out += self.next().to_bytes(8, "little")[: n - len(out)]
        return bytes(out)


def stability_messages():
    msgs = [bytes(k) for k in range(128)]
    for k in range(64 * 8):
        m = bytearray(64)
        m[k // 8] = 1 << (k % 8)
        msgs.append(bytes(m))
    prng = Xoshiro256(92)
    msgs += [prng.fill(k + 13) for k in range(256)]
    return msgs


def test_oracle_vectors():
    for src, want in VECTORS:
        assert oracle_checksum(src) == want


def test_oracle_stability():
    cases = [oracle_checksum(m) for m in stability_messages()]
    assert len(set(cases)) == 896 and 0 not in cases
    blob = b"".join(c.to_bytes(16, "little") for c in cases)
    assert oracle_checksum(blob) == STABILITY


def _gpu(messages, align=16, gap=0, seed=0):
    """Packs messages into one device buffer (offsets aligned to `align` plus a random `gap`) and
    checksums them in one launch."""
    import torch

    from tigerbeetle_amd.checksum import as_u128, checksum_device

    rng = random.Random(seed)
    offsets, pos = [], 0
    for m in messages:
        pos = (pos + align - 1) // align * align + (rng.randint(0, gap) if gap else 0)
        offsets.append(pos)
        pos += len(m)
    buf = np.zeros(max(pos, 1), np.uint8)
    for o, m in zip(offsets, messages):
        buf[o:o + len(m)] = np.frombuffer(m, np.uint8)
    d = torch.from_numpy(buf).cuda()
    tags = checksum_device(d, offsets, [len(m) for m in messages])
    torch.cuda.synchronize()
    return as_u128(tags)


@pytest.mark.gpu
def test_gpu_vectors_and_stability():
    assert _gpu([v[0] for v in VECTORS]) == [v[1] for v in VECTORS]
    cases = _gpu(stability_messages())
    blob = b"".join(c.to_bytes(16, "little") for c in cases)
    assert _gpu([blob]) == [STABILITY]


@pytest.mark.gpu
@pytest.mark.parametrize("align,gap", [(16, 0), (1, 0), (1, 13), (4, 5)])
def test_gpu_random_lengths(align, gap):
    """Lengths 0..3000 (every tail size mod 32, several chunk boundaries of the staging) at aligned and
    unaligned offsets, message counts not a multiple of the 8 per wave."""
    rng = random.Random(align * 100 + gap)
    lens = list(range(0, 70)) + [rng.randint(0, 3000) for _ in range(150)] + [1023, 1024, 1025, 2048, 2049]
    msgs = [bytes(rng.getrandbits(8) for _ in range(n)) for n in lens]
    assert _gpu(msgs, align, gap, seed=gap) == [oracle_checksum(m) for m in msgs]


@pytest.mark.gpu
def test_gpu_prepare_bodies():
    """Prepare-sized bodies (up to 8190 x 128 B) of a commit window: mixed sizes in one launch."""
    from tigerbeetle_amd import workload

    sizes = [8190, 1, 4000, 8190, 7, 8190, 0, 333, 8190, 12]
    msgs = [workload.transfers_uniform(k * 8190, n, seed=3, n_accounts=1000).tobytes() for k, n in enumerate(sizes)]
    assert _gpu(msgs) == [oracle_checksum(m) for m in msgs]
