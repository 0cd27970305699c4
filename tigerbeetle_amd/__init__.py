"""tigerbeetle_amd — MI355X-native batch-apply engine for TigerBeetle's StateMachine commit path.

The product is the C-ABI library libtbgpu.so (include/tbg.h, HIP kernels in csrc/); this package
is its host-side mirror of the reference StateMachine interface.
"""
from .state_machine import StateMachine  # noqa: F401
from .types import (  # noqa: F401
    ACCOUNT_DTYPE,
    BATCH_MAX,
    RESULT_DTYPE,
    TRANSFER_DTYPE,
    CreateAccountResult,
    CreateTransferResult,
    Operation,
)
