"""The C-ABI library loads on a CPU-only host and exports every symbol include/hbtc.h declares
(no compute calls: there is no GPU here)."""
import os
import re

from hbbft_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "hbtc.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hbtc_\w+)\s*\(", src)))


def test_header_and_binding_agree():
    assert declared_symbols() == sorted(N.SIGNATURES)


def test_library_exports_every_declared_symbol():
    lib = N.load()
    for name in declared_symbols():
        assert hasattr(lib, name), name


def test_no_device_is_reported_cleanly_without_gpu():
    n = N.device_count()
    assert n >= 0
    assert b"gfx950" in N.load().hbtc_version()


def test_rust_ffi_matches_header():
    """rust/hbtc-sys/src/ffi.rs is generated from include/hbtc.h (tools/gen_rust_ffi.py)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    rc = subprocess.call([sys.executable, os.path.join(root, "tools", "gen_rust_ffi.py"), "--check"])
    assert rc == 0, "run tools/gen_rust_ffi.py after changing include/hbtc.h"
