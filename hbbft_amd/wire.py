"""bincode 1.0 framing of the threshold_crypto values hbbft puts on the wire or under encryption
(Cargo.toml pins bincode 1.0.0).

  point      a compressed G1 / G2 point inside a SignatureShare / DecryptionShare: serde
             `serialize_bytes` -> u64 little-endian length + the 48 / 96 bytes
  FieldWrap  an Fr scalar (SyncKeyGen Ack values, src/sync_key_gen.rs:374-376,485): u64 LE length
             32 + the 32-byte big-endian representation; deserialization fails for a wrong
             length or a value >= r (Fault::ValueDeserialization, :485-492)
  Poly       a row polynomial (SyncKeyGen Part rows, :319-320,359): u64 LE coefficient count +
             every coefficient as a FieldWrap; a failure is InvalidPartMessage (:359-365)

The point framing follows SURVEY.md §8a A14; the Fr layout restates threshold_crypto's serde_impl
and is parity-unpinned (no fixture in the reference holds these bytes).  Device-side unframing of
share batches: hbtc_unframe_points (include/hbtc.h).
"""
import struct

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


class WireError(ValueError):
    """bincode / serde refused the bytes."""


def frame_point(c):
    c = bytes(c)
    if len(c) not in (48, 96):
        raise ValueError("compressed G1 (48 B) or G2 (96 B) expected")
    return struct.pack("<Q", len(c)) + c


def unframe_point(b, size):
    b = bytes(b)
    if len(b) != 8 + size or struct.unpack_from("<Q", b)[0] != size:
        raise WireError("bad point frame")
    return b[8:]


def fr_to_wire(v):
    v = int(v)
    if not 0 <= v < R:
        raise ValueError("scalar out of range")
    return struct.pack("<Q", 32) + v.to_bytes(32, "big")


def fr_from_wire(b, pos=0):
    """(value, next position); WireError on a bad length, short input or a value >= r."""
    b = bytes(b)
    if len(b) < pos + 8:
        raise WireError("short FieldWrap")
    n = struct.unpack_from("<Q", b, pos)[0]
    if n != 32 or len(b) < pos + 8 + 32:
        raise WireError("bad FieldWrap length")
    v = int.from_bytes(b[pos + 8:pos + 40], "big")
    if v >= R:
        raise WireError("FieldWrap value >= r")
    return v, pos + 40


def fr_value_from_wire(b):
    """A message holding one FieldWrap<Fr> (an Ack value).  bincode 1.0's `deserialize` stops
    after the last field and ignores what follows (no trailing-bytes check before bincode 1.3's
    Options), so bytes appended after the value are ignored here too."""
    return fr_from_wire(b)[0]


def poly_to_wire(coeffs):
    return struct.pack("<Q", len(coeffs)) + b"".join(fr_to_wire(c) for c in coeffs)


def poly_from_wire(b):
    b = bytes(b)
    if len(b) < 8:
        raise WireError("short Poly")
    n = struct.unpack_from("<Q", b)[0]
    if 8 + 40 * n > len(b):  # short; bytes after the last coefficient are ignored (bincode 1.0)
        raise WireError("bad Poly length")
    out, pos = [], 8
    for _ in range(n):
        v, pos = fr_from_wire(b, pos)
        out.append(v)
    return out
