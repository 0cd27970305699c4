"""The client's reply Demuxer (state_machine.zig:133-176) over the C ABI (tbg_demux_*, host-only)."""
import ctypes

from . import _lib


class Demuxer:
    """Splits one reply body per packed request: decode(event_offset, event_count) returns the next
    request's results (bytes), indexes rebased to it. The reply buffer is rewritten in place, as the
    reference does."""

    def __init__(self, operation, reply):
        self._buf = ctypes.create_string_buffer(bytes(reply), max(len(reply), 1))
        self._dm = _lib.Demuxer()
        _lib.check(_lib.lib().tbg_demux_init(ctypes.byref(self._dm), int(operation), self._buf, len(reply)),
                   "demux_init")

    def decode(self, event_offset, event_count):
        ptr, size = ctypes.c_void_p(), ctypes.c_uint32()
        _lib.check(_lib.lib().tbg_demux_decode(ctypes.byref(self._dm), event_offset, event_count, ctypes.byref(ptr),
                                               ctypes.byref(size)), "demux_decode")
        return ctypes.string_at(ptr.value, size.value) if size.value else b""
