"""The Fq product / squaring instruction lists (tools/gen_fips_asm.py) on the CPU: the generator's
register-file simulator runs the shared-subroutine bodies (fq_fips_sr.h) on random operands,
checks that the inline-asm form (fq_fips_asm.h) is the same list instruction for instruction,
and the committed headers are exactly what the generator emits."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GEN = os.path.join(ROOT, "tools", "gen_fips_asm.py")


def _run(*args):
    return subprocess.run([sys.executable, GEN, *args], check=True, capture_output=True,
                          text=True).stdout


def test_generator_selftests():
    out = _run("--selftest")
    assert "selftest ok" in out and "selftest_sr ok" in out


def test_committed_headers_match_generator():
    for args, name in (((), "fq_fips_asm.h"), (("--sr",), "fq_fips_sr.h")):
        with open(os.path.join(ROOT, "hbbft_amd", "csrc", name)) as f:
            assert f.read() == _run(*args), name + " differs from tools/gen_fips_asm.py output"


def test_one_move_per_column():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    try:
        import gen_fips_asm as g
    finally:
        sys.path.pop(0)
    for square, macs in ((False, 288), (True, 222)):
        body = g.gen_mul(square)
        ops = [line.split(" ", 1)[0] for line in body]
        assert ops.count("v_mad_u64_u32") == macs
        assert ops.count("v_addc_co_u32_e64") == macs
        # 2 zero-inits + 22 next-low-word moves + 12 result limbs
        assert ops.count("v_mov_b32") == 2 + 22 + 12


def test_lazy_reduction_subroutines():
    """hbtc_fqmac_sr / hbtc_fqredc_sr (the double-width accumulator of gt6.h's lazy products) on
    the simulator: sums of up to 12 products of operands < 2p, the worst case included, reduce
    to r < 2p congruent to ACC 2^-384; a MAC is the 144 product MADs, a REDC 144 + 24."""
    assert "selftest_lazy ok" in _run("--selftest-lazy")
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    try:
        import gen_fips_asm as g
    finally:
        sys.path.pop(0)
    mac = [line.split(" ", 1)[0] for line in g.mac_body()]
    redc = [line.split(" ", 1)[0] for line in g.redc_body()]
    assert mac.count("v_mad_u64_u32") == 144
    assert redc.count("v_mad_u64_u32") == 144 + 24  # q_i p_j, and each ACC word entering by 1
