"""hbbft_amd — MI355X-native batched threshold-crypto verifier for hbbft's per-epoch hot path.

The compute path is the HIP library ``hbbft_amd/libhbtc.so`` (gfx950 kernels behind the C ABI
of ``include/hbtc.h``); ``hbbft_amd._native`` binds it with ctypes; ``protocol`` (Coin,
ThresholdDecryption), ``skg`` (SyncKeyGen) and ``broadcast`` (Reliable Broadcast coding) mirror
the hbbft call sites as batch queues; ``shard`` plans multi-GPU splits; ``wire`` restates the
bincode framing.  Nothing here falls back to the CPU: if the library is missing, calls raise
``NativeUnavailable``.
"""
from ._native import (ACCEPT, DECODE_ERR, DUPLICATE_ENTRY, INSTANCE_ERR,  # noqa: F401
                      NOT_ENOUGH_SHARES, REJECT, UNKNOWN_SENDER, Context, HbtcError,
                      NativeUnavailable)

__all__ = ["Context", "HbtcError", "NativeUnavailable", "ACCEPT", "REJECT", "DECODE_ERR",
           "UNKNOWN_SENDER", "INSTANCE_ERR", "NOT_ENOUGH_SHARES", "DUPLICATE_ENTRY"]
