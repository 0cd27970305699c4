"""Test infrastructure: writes append-only files of prepares in the reference's on-disk format
(aof.zig:23-55 AOFEntry = magic u128, AOFEntryMetadata {primary u64, replica u64, reserved[4064]},
the prepare message padded with zeros to a 4096-byte sector multiple; vsr/message_header.zig:552-605
Header.Prepare), with checksums from the CPU restatement (oracle/aegis.c), and a log recorder that
runs the restatement under the replica's protocol (lockstep.replica_commit) so pulses land in the
log as prepares of their own (vsr.Operation.pulse = 4)."""
import struct

from test_checksum import oracle_checksum
from tigerbeetle_amd.types import Operation

MAGIC = 312960301372567410560647846651901451202
SECTOR = 4096
VSR_PULSE = 4
COMMAND_PREPARE = 6


def prepare_header(operation, body, op, timestamp, parent, cluster=7, client=0x1234, request=0, view=0):
    """Header.Prepare bytes (256) with checksum_body and checksum set."""
    h = bytearray(256)
    struct.pack_into("<16s", h, 80, cluster.to_bytes(16, "little"))
    struct.pack_into("<I", h, 96, 256 + len(body))           # size
    struct.pack_into("<I", h, 104, view)                     # view
    struct.pack_into("<H", h, 112, 0)                        # protocol
    h[114] = COMMAND_PREPARE
    struct.pack_into("<16s", h, 128, parent.to_bytes(16, "little"))
    struct.pack_into("<16s", h, 208, client.to_bytes(16, "little"))
    struct.pack_into("<QQQ", h, 224, op, op, timestamp)      # op, commit, timestamp
    struct.pack_into("<I", h, 248, request)
    h[252] = operation
    struct.pack_into("<16s", h, 32, oracle_checksum(body).to_bytes(16, "little"))
    struct.pack_into("<16s", h, 0, oracle_checksum(bytes(h[16:])).to_bytes(16, "little"))
    return bytes(h)


def entry(header, body, replica=0, primary=0):
    e = bytearray(MAGIC.to_bytes(16, "little"))
    e += struct.pack("<QQ", primary, replica) + bytes(4064)
    e += header + body
    e += bytes((-len(e)) % SECTOR)
    return bytes(e)


class AofLog:
    """Accumulates prepares into an AOF image with a consistent hash chain."""

    def __init__(self):
        self.entries = []  # (offset, header bytes)
        self.data = bytearray()
        self.parent = 0
        self.op = 1

    def append(self, operation, body, timestamp):
        h = prepare_header(operation, body, self.op, timestamp, self.parent)
        self.entries.append((len(self.data), h))
        self.data += entry(h, body)
        self.parent = int.from_bytes(h[:16], "little")
        self.op += 1

    def append_raw(self, header, body):
        self.entries.append((len(self.data), header))
        self.data += entry(header, body)


def record(ref, requests, realtime_fn):
    """Runs `requests` [(operation, events)] through the restatement under the replica protocol
    (a pulse is a prepare of its own when pulse() says so, replica.zig:9459-9487, 5763-5771) and
    logs every prepare. Returns (AofLog, replies)."""
    log = AofLog()
    replies = []
    for k, (operation, events) in enumerate(requests):
        realtime = realtime_fn(k, ref.prepare_timestamp)
        if ref.pulse():
            ref.prepare_timestamp = max(max(ref.prepare_timestamp, ref.commit_timestamp) + 1, realtime)
            T = ref.prepare_timestamp
            ref.prefetch_timestamp = T
            ref.prefetch(0, Operation.pulse, b"")
            ref.commit(0, 0, T, Operation.pulse, b"")
            log.append(VSR_PULSE, b"", T)
        data = events.tobytes()
        ref.prepare_timestamp = max(max(ref.prepare_timestamp, ref.commit_timestamp) + 1, realtime)
        ref.prepare(operation, data)
        T = ref.prepare_timestamp
        ref.prefetch_timestamp = T
        ref.prefetch(0, operation, data)
        replies.append(ref.commit(0, 0, T, operation, data))
        log.append(int(operation), data, T)
    return log, replies
