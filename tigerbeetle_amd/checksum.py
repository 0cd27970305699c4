"""TigerBeetle's checksum (vsr/checksum.zig:50-59, AEGIS-128L MAC with a zero key) on the GPU for many
messages at once (csrc/checksum.hip, C-ABI tbg_checksum). Device tensors in, device tensor out."""
import numpy as np

from . import _lib


def checksum_device(data, offsets, sizes, stream=None):
    """data: uint8 CUDA tensor; offsets (int64) / sizes (int32): the messages inside it, as CUDA
    tensors or sequences. Returns a (n, 16) uint8 CUDA tensor: each message's u128 checksum in
    little-endian bytes. Asynchronous on `stream` (a torch.cuda.Stream, default: the current one)."""
    import torch

    dev = data.device
    offsets = torch.as_tensor(offsets, dtype=torch.int64, device=dev)
    sizes = torch.as_tensor(sizes, dtype=torch.int32, device=dev)
    n = int(offsets.numel())
    assert int(sizes.numel()) == n
    out = torch.empty((max(n, 1), 16), dtype=torch.uint8, device=dev)
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    _lib.check(_lib.lib().tbg_checksum(data.data_ptr(), offsets.data_ptr(), sizes.data_ptr(), n, out.data_ptr(),
                                       s.cuda_stream), "checksum")
    return out[:n]


def as_u128(tags):
    """(n, 16) little-endian tag bytes (host array or CUDA tensor) -> list of Python ints."""
    a = tags.cpu().numpy() if hasattr(tags, "cpu") else np.asarray(tags)
    return [int.from_bytes(bytes(r), "little") for r in a.reshape(-1, 16)]
