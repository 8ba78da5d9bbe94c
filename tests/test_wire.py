"""bincode framing (hbbft_amd/wire.py): round trips and the refusals that map to hbbft faults
(ValueDeserialization, InvalidPartMessage; src/sync_key_gen.rs:359-365,485-492)."""
import pytest

from hbbft_amd import wire


def test_fieldwrap_roundtrip_and_refusals():
    for v in (0, 1, wire.R - 1, 12345678901234567890):
        b = wire.fr_to_wire(v)
        assert len(b) == 40 and wire.fr_value_from_wire(b) == v
    with pytest.raises(wire.WireError):
        wire.fr_value_from_wire(b"\x21" + bytes(39))           # length 33
    with pytest.raises(wire.WireError):
        wire.fr_value_from_wire(wire.fr_to_wire(5)[:8] + wire.R.to_bytes(32, "big"))  # == r
    # bincode 1.0 (Cargo.toml:21) ignores bytes after the last field: a value with bytes
    # appended decodes to the same value (reference nodes accept it)
    assert wire.fr_value_from_wire(wire.fr_to_wire(5) + b"\0") == 5
    assert wire.fr_value_from_wire(wire.fr_to_wire(wire.R - 1) + bytes(range(17))) == wire.R - 1
    with pytest.raises(wire.WireError):
        wire.fr_value_from_wire(wire.fr_to_wire(5)[:30])       # short


def test_poly_roundtrip_and_refusals():
    coeffs = [3, wire.R - 2, 0, 77]
    b = wire.poly_to_wire(coeffs)
    assert wire.poly_from_wire(b) == coeffs
    assert wire.poly_from_wire(wire.poly_to_wire([])) == []
    with pytest.raises(wire.WireError):
        wire.poly_from_wire(b[:-1])
    with pytest.raises(wire.WireError):
        wire.poly_from_wire((5).to_bytes(8, "little") + b[8:])
    # bytes appended after the last coefficient are ignored, as bincode 1.0 does
    assert wire.poly_from_wire(b + b"\x01\x02\x03") == coeffs
    assert wire.poly_from_wire((3).to_bytes(8, "little") + b[8:]) == coeffs[:3]


def test_appended_bytes_agree_with_rules_oracle():
    from oracle import hbbft_rules as rules
    coeffs = [9, 8, 7]
    for extra in (b"", b"\0", bytes(41)):
        assert rules._poly_from_wire(wire.poly_to_wire(coeffs) + extra) == coeffs
        assert wire.poly_from_wire(wire.poly_to_wire(coeffs) + extra) == coeffs
        assert rules._fr_from_wire(wire.fr_to_wire(11) + extra)[0] == 11
        assert wire.fr_value_from_wire(wire.fr_to_wire(11) + extra) == 11


def test_point_frames():
    g1, g2 = bytes(range(48)), bytes(range(96))
    assert wire.unframe_point(wire.frame_point(g1), 48) == g1
    assert wire.unframe_point(wire.frame_point(g2), 96) == g2
    with pytest.raises(wire.WireError):
        wire.unframe_point(wire.frame_point(g1), 96)
