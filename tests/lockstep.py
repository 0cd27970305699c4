"""Test harness pieces for the pulse decision (state_machine.zig:589-596).

`Lockstep` drives the GPU engine and the CPU restatement with the same StateMachine calls and
asserts, call by call, that every `pulse()` decision, every reply and the pulse_next_timestamp after
every commit are identical. `replica_commit` is the commit protocol of a solo primary
(vsr/replica.zig), in which a pulse is a prepare of its own and takes a timestamp, so a wrong
decision shifts every later stored timestamp.
"""
from tigerbeetle_amd.types import Operation


class Lockstep:
    def __init__(self, gpu, ref):
        self.gpu, self.ref = gpu, ref
        self.batch_max = gpu.batch_max
        self.decisions = 0
        self.pulses = 0
        self.resets = 0  # commits after which pulse_next_timestamp == timestamp_min (a post/void reset)

    def _both(self, name, value):
        setattr(self.gpu, name, value)
        setattr(self.ref, name, value)

    prepare_timestamp = property(lambda s: s.gpu.prepare_timestamp, lambda s, v: s._both("prepare_timestamp", v))
    prefetch_timestamp = property(lambda s: s.gpu.prefetch_timestamp, lambda s, v: s._both("prefetch_timestamp", v))
    commit_timestamp = property(lambda s: s.gpu.commit_timestamp, lambda s, v: s._both("commit_timestamp", v))

    def input_valid(self, operation, data):
        a, b = self.gpu.input_valid(operation, data), self.ref.input_valid(operation, data)
        assert a == b
        return a

    def prepare(self, operation, data):
        self.gpu.prepare(operation, data)
        self.ref.prepare(operation, data)
        assert self.gpu.prepare_timestamp == self.ref.prepare_timestamp

    def pulse(self):
        a, b = self.gpu.pulse(), self.ref.pulse()
        assert a == b, (f"pulse() at prepare_timestamp {self.ref.prepare_timestamp}: gpu {a} ref {b} "
                        f"(pulse_next gpu {self.gpu.pulse_next_timestamp()} ref {self.ref.pulse_next_timestamp()})")
        self.decisions += 1
        self.pulses += int(a)
        return a

    def prefetch(self, op, operation, data):
        self.gpu.prefetch(op, operation, data)
        self.ref.prefetch(op, operation, data)

    def commit(self, client, op, timestamp, operation, data):
        a = self.gpu.commit(client, op, timestamp, operation, data)
        b = self.ref.commit(client, op, timestamp, operation, data)
        assert a == b, f"{Operation(operation).name} at {timestamp}: replies differ"
        pa, pb = self.gpu.pulse_next_timestamp(), self.ref.pulse_next_timestamp()
        assert pa == pb, f"pulse_next_timestamp after {Operation(operation).name} at {timestamp}: gpu {pa} ref {pb}"
        self.resets += int(pb == 1 and operation == Operation.create_transfers)
        return a

    def setup_balances(self, *args):
        self.gpu.setup_balances(*args)
        self.ref.setup_balances(*args)


def replica_commit(sm, op, operation, events, realtime):
    """One client request on a solo primary. pulse_needed() (vsr/replica.zig:9459-9478) asks the
    state machine's pulse() against the last prepare's timestamp before the request is prepared; a
    pulse is then a prepare of its own, stamped prepare_timestamp = max(max(prepare_timestamp,
    commit_timestamp) + 1, realtime) (:5763-5771; prepare() adds 0 for a pulse,
    state_machine.zig:575-587), and committed before the request. Returns (reply, op, pulsed)."""
    pulsed = False
    if sm.pulse():
        sm.prepare_timestamp = max(max(sm.prepare_timestamp, sm.commit_timestamp) + 1, realtime)
        T = sm.prepare_timestamp
        sm.prefetch_timestamp = T
        sm.prefetch(op, Operation.pulse, b"")
        sm.commit(0, op, T, Operation.pulse, b"")
        op += 1
        pulsed = True
    data = events.tobytes()
    sm.prepare_timestamp = max(max(sm.prepare_timestamp, sm.commit_timestamp) + 1, realtime)
    sm.prepare(operation, data)
    T = sm.prepare_timestamp
    sm.prefetch_timestamp = T
    sm.prefetch(op, operation, data)
    return sm.commit(0, op, T, operation, data), op + 1, pulsed
