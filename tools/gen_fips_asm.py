#!/usr/bin/env python3
"""Generate hbbft_amd/csrc/fq_fips_asm.h: the Fq Montgomery product and squaring as ONE inline-asm
block each (product scanning, carry-out MACs), for gfx950.

Why one block: hipcc pads every inline-asm statement with an `s_nop 0` (it cannot see the
hazards inside), and the C++-glued form of fq_fips.h issues ~75 statements per product; the
column shifts and the Montgomery digit need the two 32-bit halves of the 64-bit accumulator,
which an asm operand cannot name, so the accumulator, its overflow word and the squaring's
cross-product accumulator are pinned to fixed VGPRs (HBTC_FIPS_*), named literally below; the
carries go through VCC.

Squaring: a^2 = sum_i a_i^2 2^(64i) + sum_i a_i 2^(32i) * 2 a_{>i}, and 2 a_{>i} is written with
limbs that fit 32 bits: t_{i+1} = (2 a_{i+1}) mod 2^32 and t_j = (2 a_j mod 2^32) + (a_{j-1} >> 31)
for j >= i + 2 (the dropped top bit of each doubled limb reappears in the next limb; the row sum
telescopes to exactly 2 a_{>i}).  So the 66 cross products use one of two precomputed doubled
limb vectors (23 shifts / v_alignbit outside the asm), every term is non-negative and the column
accumulation is the product's: 78 + 144 = 222 MACs and ~540 instructions instead of 288 and ~660.
Bounds as fq_fips.h: inputs < 2p, result < 2p; every 96-bit column sum fits.

Usage: tools/gen_fips_asm.py > hbbft_amd/csrc/fq_fips_asm.h
"""

import re

ACC = "v[%d:%d]"


def gen_mul(square):
    # operand numbering: outputs r0..r11 (%0..%11), q0..q11 (%12..%23); inputs a0..a11, then
    # b0..b11 (mul only), then p0..p11 (SGPR), np (SGPR)
    R = lambda i: "%%%d" % i
    Q = lambda i: "%%%d" % (12 + i)
    A = lambda i: "%%%d" % (24 + i)
    if square:
        B = A
        D2 = lambda j: "%%%d" % (36 + j)       # j = 1..11 -> %37..%47 (%36 unused slot: a'' of 0)
        D1 = lambda j: "%%%d" % (48 + j - 2)   # j = 2..11 -> %48..%57
        P = lambda i: "%%%d" % (58 + i)
        NP = "%70"
    else:
        B = lambda i: "%%%d" % (36 + i)
        P = lambda i: "%%%d" % (48 + i)
        NP = "%60"
    # Two even-aligned accumulator pairs, alternating by column: column k accumulates in pair
    # k % 2 and counts its overflow in the HIGH register of the other pair, which is then
    # already the next column's high word; only the next low word needs a move (one v_mov per
    # column instead of two).
    reg = lambda n: "v\" HBTC_XS(HBTC_FIPS_ACC%d) \"" % n
    pair = lambda p: "v[\" HBTC_XS(HBTC_FIPS_ACC%d) \":\" HBTC_XS(HBTC_FIPS_ACC%d) \"]" % (2 * p, 2 * p + 1)
    cc = "vcc"
    lines = []
    emit = lines.append
    cur = {}

    def column(k):
        p = k % 2
        cur.update(acc=pair(p), lo=reg(2 * p), hi=reg(2 * p + 1), c2=reg(2 * (1 - p) + 1),
                   nlo=reg(2 * (1 - p)))

    def mac(x, y, fresh):
        acc, c2 = cur["acc"], cur["c2"]
        emit("v_mad_u64_u32 %s, %s, %s, %s, %s" % (acc, cc, x, y, acc))
        if fresh:
            emit("v_addc_co_u32_e64 %s, %s, 0, 0, %s" % (c2, cc, cc))
        else:
            emit("v_addc_co_u32_e64 %s, %s, %s, 0, %s" % (c2, cc, c2, cc))

    column(0)
    emit("v_mov_b32 %s, 0" % cur["lo"])
    emit("v_mov_b32 %s, 0" % cur["hi"])
    for k in range(23):
        column(k)
        lo = cur["lo"]
        lo_i, hi_i = (0, k) if k < 12 else (k - 11, 11)
        fresh = True
        if square:
            # row i: a_i * (2 a_{>i}) = a_i * sum_{j>i} t_j^(i) 2^(32j), t_{i+1}^(i) = D2(i+1) =
            # (2 a_{i+1}) mod 2^32, t_j^(i) = D1(j) = (2 a_j mod 2^32) + top bit of a_{j-1}
            # for j >= i + 2 (the top bits cancel along the row): every term non-negative
            for i in range(lo_i, hi_i + 1):
                j = k - i
                if i < j:
                    mac(A(i), D2(j) if j == i + 1 else D1(j), fresh)
                    fresh = False
                elif i == j:
                    mac(A(i), A(i), fresh)
                    fresh = False
        else:
            for i in range(lo_i, hi_i + 1):
                mac(A(i), B(k - i), fresh)
                fresh = False
        qhi = k - 1 if k < 12 else 11
        for i in range(lo_i, qhi + 1):
            mac(Q(i), P(k - i), fresh)
            fresh = False
        if k < 12:
            emit("v_mul_lo_u32 %s, %s, %s" % (Q(k), lo, NP))
            mac(Q(k), P(0), fresh)
        else:
            emit("v_mov_b32 %s, %s" % (R(k - 12), lo))
        if k < 22:
            emit("v_mov_b32 %s, %s" % (cur["nlo"], cur["hi"]))
    emit("v_mov_b32 %s, %s" % (R(11), cur["hi"]))  # the last column's overflow word is 0
    return lines


def block(name, square):
    body = gen_mul(square)
    text = "\n".join('      "%s\\n\\t"' % l for l in body)
    outs = ", ".join('"=&v"(r[%d])' % i for i in range(12)) + ",\n        " + \
        ", ".join('"=&v"(q[%d])' % i for i in range(12))
    ins = ", ".join('"v"(a[%d])' % i for i in range(12))
    if square:
        ins += ",\n        " + ", ".join('"v"(d2[%d])' % i for i in range(12))
        ins += ",\n        " + ", ".join('"v"(d1[%d])' % i for i in range(2, 12))
    else:
        ins += ",\n        " + ", ".join('"v"(b[%d])' % i for i in range(12))
    ins += ",\n        " + ", ".join('"s"(FQ_P[%d])' % i for i in range(12)) + ', "s"(FQ_NP)'
    clob = ", ".join('"v" HBTC_XS(HBTC_FIPS_ACC%d)' % n for n in range(4)) + ', "vcc"'
    args = "uint32_t* r, const uint32_t* a" + ("" if square else ", const uint32_t* b")
    prep = ""
    if square:
        prep = """  uint32_t d2[12], d1[12];
#pragma unroll
  for (int j = 0; j < 12; ++j) d2[j] = a[j] << 1;
#pragma unroll
  for (int j = 1; j < 12; ++j) d1[j] = (a[j] << 1) | (a[j - 1] >> 31);
"""
    return """__device__ __forceinline__ void %s(%s) {
  uint32_t q[12];
%s  asm volatile(
%s
      : %s
      : %s
      : %s);
}
""" % (name, args, prep, text, outs, ins, clob)


def main():
    print("""// GENERATED by tools/gen_fips_asm.py -- do not edit.
// Fq Montgomery product and squaring for gfx950, each one inline-asm block (see the generator's
// docstring): product scanning with carry-out MACs, the 64-bit column accumulator, its overflow
// word and the squaring's cross accumulator pinned to HBTC_FIPS_* registers (override before
// including to move them), the modulus limbs in SGPRs.  Only VALU instructions on registers.
#pragma once
#include <cstdint>
#if defined(__HIP_DEVICE_COMPILE__)
#ifndef HBTC_FIPS_ACC0
#define HBTC_FIPS_ACC0 2
#define HBTC_FIPS_ACC1 3
#define HBTC_FIPS_ACC2 4
#define HBTC_FIPS_ACC3 5
#endif
#define HBTC_S(x) #x
#define HBTC_XS(x) HBTC_S(x)
namespace hbtc {
namespace fips {
""")
    print(block("mont_mul_asm", False))
    print(block("mont_sqr_asm", True))
    print("""}  // namespace fips
}  // namespace hbtc
#endif""")



# ------------------------------------------------------------------------------ subroutines
# fq_fips_sr.h: the same two instruction lists as ONE shared subroutine each (module-level asm),
# entered by s_swappc from a short call-site block, for translation units whose hot loops hold
# many product sites (an inlined copy is ~5.6 KB of code: a point doubling plus a mixed addition
# inline ~100 KB, past the 64 KB instruction cache, and the waves then stall on instruction
# fetch).  Calling convention (every register fixed; the call-site asm names them as operands
# and clobbers, so the compiler keeps nothing else there across a call):
#   a: v8..v19 (the result overwrites it: r_j is written at column 12 + j, after the last read
#   of a_j and b_j at column j + 11), b / the squaring's doubled limbs t_j: v20..v31, the
#   squaring's carried doubled limbs: v32..v41, q: v42..v53, accumulators v54..v59, the modulus
#   s48..s59, -p^-1 s60, target s[62:63], return address s[64:65] (below s72: at 8 waves per
#   SIMD the registers from s72 up are reserved).
SR_A, SR_B, SR_D1, SR_Q, SR_ACC, SR_P, SR_NP, SR_TGT, SR_RET = 8, 20, 32, 42, 54, 48, 60, 62, 64
P_MOD = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
NP_MOD = (-pow(P_MOD, -1, 1 << 32)) % (1 << 32)


def sr_body(square):
    """gen_mul's list with every operand on its fixed register."""
    acc = {}
    for p in range(2):
        acc['v[" HBTC_XS(HBTC_FIPS_ACC%d) ":" HBTC_XS(HBTC_FIPS_ACC%d) "]' % (2 * p, 2 * p + 1)] = \
            "v[%d:%d]" % (SR_ACC + 2 * p, SR_ACC + 2 * p + 1)
    for n in range(4):
        acc['v" HBTC_XS(HBTC_FIPS_ACC%d) "' % n] = "v%d" % (SR_ACC + n)

    def reg(n):
        if n < 12:
            return "v%d" % (SR_A + n)            # r (overwrites a)
        if n < 24:
            return "v%d" % (SR_Q + n - 12)       # q
        if n < 36:
            return "v%d" % (SR_A + n - 24)       # a
        if square:
            if n < 48:
                return "v%d" % (SR_B + n - 36)   # t_j (j = n - 36)
            if n < 58:
                return "v%d" % (SR_D1 + n - 48)  # carried doubled limbs, j = n - 46
            if n < 70:
                return "s%d" % (SR_P + n - 58)
            return "s%d" % SR_NP
        if n < 48:
            return "v%d" % (SR_B + n - 36)
        if n < 60:
            return "s%d" % (SR_P + n - 48)
        return "s%d" % SR_NP

    out = []
    for line in gen_mul(square):
        for k in sorted(acc, key=len, reverse=True):
            line = line.replace(k, acc[k])
        out.append(re.sub(r"%(\d+)", lambda m: reg(int(m.group(1))), line))
    return out


def sr_text(label, square):
    lines = [".p2align 8", "%s:" % label]
    lines += ["s_mov_b32 s%d, 0x%08x" % (SR_P + i, (P_MOD >> (32 * i)) & 0xFFFFFFFF) for i in range(12)]
    lines.append("s_mov_b32 s%d, 0x%08x" % (SR_NP, NP_MOD))
    lines += sr_body(square)
    lines.append("s_setpc_b64 s[%d:%d]" % (SR_RET, SR_RET + 1))
    return lines


def sr_call(name, label, square):
    outs = ", ".join('"={v%d}"(r[%d])' % (SR_A + i, i) for i in range(12))
    ins = ", ".join('"{v%d}"(a[%d])' % (SR_A + i, i) for i in range(12))
    if square:
        ins += ",\n        " + ", ".join('"{v%d}"(t[%d])' % (SR_B + j, j) for j in range(1, 12))
        ins += ",\n        " + ", ".join('"{v%d}"(u[%d])' % (SR_D1 + j - 2, j) for j in range(2, 12))
    else:
        ins += ",\n        " + ", ".join('"{v%d}"(b[%d])' % (SR_B + i, i) for i in range(12))
    clob = []
    if square:
        clob += ['"v%d"' % SR_B]  # t_0 is not an input
    clob += ['"v%d"' % v for v in range(SR_Q, SR_ACC + 4)]
    clob += ['"s%d"' % s for s in range(SR_P, SR_RET + 2)]
    clob += ['"vcc"', '"scc"']
    args = "uint32_t* r, const uint32_t* a" + ("" if square else ", const uint32_t* b")
    prep = ""
    if square:
        prep = """  uint32_t t[12], u[12];
#pragma unroll
  for (int j = 1; j < 12; ++j) t[j] = a[j] << 1;
#pragma unroll
  for (int j = 2; j < 12; ++j) u[j] = (a[j] << 1) | (a[j - 1] >> 31);
"""
    call = ('      "s_getpc_b64 s[%d:%d]\\n\\t"\n' % (SR_TGT, SR_TGT + 1) +
            '      "s_add_u32 s%d, s%d, %s@rel32@lo+4\\n\\t"\n' % (SR_TGT, SR_TGT, label) +
            '      "s_addc_u32 s%d, s%d, %s@rel32@hi+12\\n\\t"\n' % (SR_TGT + 1, SR_TGT + 1, label) +
            '      "s_swappc_b64 s[%d:%d], s[%d:%d]"' % (SR_RET, SR_RET + 1, SR_TGT, SR_TGT + 1))
    return """__device__ __forceinline__ void %s(%s) {
%s  asm volatile(
%s
      : %s
      : %s
      : %s);
}
""" % (name, args, prep, call, outs, ins, ", ".join(clob))


# ------------------------------------------------------------------ lazy (double-width) reduction
# hbtc_fqmac_sr: ACC += a * b, a double-width accumulator of 25 words (v60..v84) that survives
# between calls, a and b (v8..v19, v20..v31) preserved; product scanning into the column pair of
# gen_mul with the column digit added into ACC[k] through the carry chain s[66:67].
# hbtc_fqredc_sr: r (v8..v19) = ACC * 2^-384 mod p, r < 2p, for ACC < 48 p^2 (ACC unchanged):
# Montgomery digits q0..q11 over ACC's low half, the quotient (ACC + Q p) / 2^384 < 48 p^2 / 2^384
# + p < 5.6p (12 words), then conditional subtractions of 4p and 2p.  48 p^2 bounds a sum of 12
# products of reduced operands (< 2p each).
SR_MACC, SR_CC = 60, 66
# A second accumulator (v85..v109) with its own pair of subroutines (hbtc_fqmac2_sr,
# hbtc_fqredc2_sr) lets the two Fq halves of an Fq2 sum accumulate in one pass over the terms.
SR_MACC2 = 85


def mac_body(base=SR_MACC, targets=None):
    """Column digits of a * b added into (sign "+") or subtracted from ("-") each target
    accumulator, modulo 2^800, one carry / borrow chain per target (s[66:67], s[68:69])."""
    if targets is None:
        targets = [(base, "+")]
    A = lambda i: "v%d" % (SR_A + i)
    B = lambda i: "v%d" % (SR_B + i)
    reg = lambda n: "v%d" % (SR_ACC + n)
    pair = lambda p: "v[%d:%d]" % (SR_ACC + 2 * p, SR_ACC + 2 * p + 1)
    cc = "vcc"
    chains = ["s[%d:%d]" % (SR_CC + 2 * t, SR_CC + 2 * t + 1) for t in range(len(targets))]

    def fold(k, word):
        for (tb, sign), chain in zip(targets, chains):
            w = "v%d" % (tb + k)
            if sign == "+":
                if k == 0:
                    out.append("v_add_co_u32_e64 %s, %s, %s, %s" % (w, chain, w, word))
                else:
                    out.append("v_addc_co_u32_e64 %s, %s, %s, %s, %s" % (w, chain, w, word, chain))
            else:
                if k == 0:
                    out.append("v_sub_co_u32_e64 %s, %s, %s, %s" % (w, chain, w, word))
                else:
                    out.append("v_subb_co_u32_e64 %s, %s, %s, %s, %s" % (w, chain, w, word, chain))

    out = ["v_mov_b32 %s, 0" % reg(0), "v_mov_b32 %s, 0" % reg(1)]
    for k in range(23):
        p = k % 2
        acc, lo, hi, c2, nlo = pair(p), reg(2 * p), reg(2 * p + 1), reg(2 * (1 - p) + 1), reg(2 * (1 - p))
        lo_i, hi_i = (0, k) if k < 12 else (k - 11, 11)
        for i in range(lo_i, hi_i + 1):
            out.append("v_mad_u64_u32 %s, %s, %s, %s, %s" % (acc, cc, A(i), B(k - i), acc))
            out.append("v_addc_co_u32_e64 %s, %s, %s, 0, %s" % (c2, cc, "0" if i == lo_i else c2, cc))
        fold(k, lo)
        if k < 22:
            out.append("v_mov_b32 %s, %s" % (nlo, hi))
    # column 22's high word is digit 23 (its overflow word is 0: a * b < 2^768)
    fold(23, reg(1))
    fold(24, "0")
    return out


def redc_body(base=SR_MACC):
    Q = lambda i: "v%d" % (SR_Q + i)
    R = lambda i: "v%d" % (SR_A + i)
    P = lambda i: "s%d" % (SR_P + i)
    ACCW = lambda i: "v%d" % (base + i)
    reg = lambda n: "v%d" % (SR_ACC + n)
    pair = lambda p: "v[%d:%d]" % (SR_ACC + 2 * p, SR_ACC + 2 * p + 1)
    cc = "vcc"
    out = ["v_mov_b32 %s, 0" % reg(0), "v_mov_b32 %s, 0" % reg(1)]
    for k in range(24):
        p = k % 2
        acc, lo, hi, c2, nlo = pair(p), reg(2 * p), reg(2 * p + 1), reg(2 * (1 - p) + 1), reg(2 * (1 - p))
        # the accumulator word enters the column as a product by 1
        out.append("v_mad_u64_u32 %s, %s, %s, 1, %s" % (acc, cc, ACCW(k), acc))
        out.append("v_addc_co_u32_e64 %s, %s, 0, 0, %s" % (c2, cc, cc))
        lo_i, hi_i = (0, k - 1) if k < 12 else (k - 11, 11)
        for i in range(lo_i, hi_i + 1):
            out.append("v_mad_u64_u32 %s, %s, %s, %s, %s" % (acc, cc, Q(i), P(k - i), acc))
            out.append("v_addc_co_u32_e64 %s, %s, %s, 0, %s" % (c2, cc, c2, cc))
        if k < 12:
            out.append("v_mul_lo_u32 %s, %s, s%d" % (Q(k), lo, SR_NP))
            out.append("v_mad_u64_u32 %s, %s, %s, %s, %s" % (acc, cc, Q(k), P(0), acc))
            out.append("v_addc_co_u32_e64 %s, %s, %s, 0, %s" % (c2, cc, c2, cc))
        else:
            out.append("v_mov_b32 %s, %s" % (R(k - 12), lo))
        out.append("v_mov_b32 %s, %s" % (nlo, hi))
    # r < 2^384: column 23's high word and ACC[24] are 0 for ACC < 48 p^2 (see above).  r < 5.6p:
    # subtract 4p, then 2p, where they fit (r - mp into Q, keep r on a borrow).  The multiple's
    # words go through a VGPR: a literal and the VCC carry-in together exceed the constant bus.
    for m in (4, 2):
        mp = m * P_MOD
        for i in range(12):
            w = "0x%08x" % ((mp >> (32 * i)) & 0xFFFFFFFF)
            t = "v%d" % (SR_Q + i)
            out.append("v_mov_b32 %s, %s" % (t, w))
            if i == 0:
                out.append("v_sub_co_u32_e32 %s, vcc, %s, %s" % (t, R(i), t))
            else:
                out.append("v_subb_co_u32_e32 %s, vcc, %s, %s, vcc" % (t, R(i), t))
        for i in range(12):
            out.append("v_cndmask_b32_e32 %s, %s, %s, vcc" % (R(i), "v%d" % (SR_Q + i), R(i)))
    return out


def lazy_text(label, body):
    lines = [".p2align 8", "%s:" % label]
    lines += ["s_mov_b32 s%d, 0x%08x" % (SR_P + i, (P_MOD >> (32 * i)) & 0xFFFFFFFF) for i in range(12)]
    lines.append("s_mov_b32 s%d, 0x%08x" % (SR_NP, NP_MOD))
    lines += body
    lines.append("s_setpc_b64 s[%d:%d]" % (SR_RET, SR_RET + 1))
    return lines


def lazy_calls():
    call = lambda label: (
        '      "s_getpc_b64 s[%d:%d]\\n\\t"\n' % (SR_TGT, SR_TGT + 1) +
        '      "s_add_u32 s%d, s%d, %s@rel32@lo+4\\n\\t"\n' % (SR_TGT, SR_TGT, label) +
        '      "s_addc_u32 s%d, s%d, %s@rel32@hi+12\\n\\t"\n' % (SR_TGT + 1, SR_TGT + 1, label) +
        '      "s_swappc_b64 s[%d:%d], s[%d:%d]"' % (SR_RET, SR_RET + 1, SR_TGT, SR_TGT + 1))
    text = ""
    for sfx, base in (("", SR_MACC), ("2", SR_MACC2)):
        accio = ", ".join('"+{v%d}"(acc[%d])' % (base + i, i) for i in range(25))
        ins = ", ".join('"{v%d}"(a[%d])' % (SR_A + i, i) for i in range(12))
        ins += ",\n        " + ", ".join('"{v%d}"(b[%d])' % (SR_B + i, i) for i in range(12))
        clob = ['"v%d"' % v for v in range(SR_ACC, SR_ACC + 4)]
        clob += ['"s%d"' % s for s in range(SR_P, SR_CC + 2)]
        clob += ['"vcc"', '"scc"']
        text += """__device__ __forceinline__ void fq_mac%s_sr(uint32_t* acc, const uint32_t* a, const uint32_t* b) {
  asm volatile(
%s
      : %s
      : %s
      : %s);
}
""" % (sfx, call("hbtc_fqmac%s_sr" % sfx), accio, ins, ", ".join(clob))
        outs = ", ".join('"={v%d}"(r[%d])' % (SR_A + i, i) for i in range(12))
        ains = ", ".join('"{v%d}"(acc[%d])' % (base + i, i) for i in range(25))
        rclob = ['"v%d"' % v for v in range(SR_Q, SR_ACC + 4)]
        rclob += ['"s%d"' % s for s in range(SR_P, SR_RET + 2)]
        rclob += ['"vcc"', '"scc"']
        text += """__device__ __forceinline__ void fq_redc%s_sr(uint32_t* r, const uint32_t* acc) {
  asm volatile(
%s
      : %s
      : %s
      : %s);
}
""" % (sfx, call("hbtc_fqredc%s_sr" % sfx), outs, ains, ", ".join(rclob))
    # the Karatsuba pair: both accumulators at once
    accio = ", ".join('"+{v%d}"(x[%d])' % (SR_MACC + i, i) for i in range(25))
    accio += ",\n        " + ", ".join('"+{v%d}"(y[%d])' % (SR_MACC2 + i, i) for i in range(25))
    ins = ", ".join('"{v%d}"(a[%d])' % (SR_A + i, i) for i in range(12))
    ins += ",\n        " + ", ".join('"{v%d}"(b[%d])' % (SR_B + i, i) for i in range(12))
    clob = ['"v%d"' % v for v in range(SR_ACC, SR_ACC + 4)]
    clob += ['"s%d"' % s for s in range(SR_P, SR_CC + 4)]
    clob += ['"vcc"', '"scc"']
    for name in ("macsub", "subsub"):
        text += """__device__ __forceinline__ void fq_%s_sr(uint32_t* x, uint32_t* y, const uint32_t* a, const uint32_t* b) {
  asm volatile(
%s
      : %s
      : %s
      : %s);
}
""" % (name, call("hbtc_fq%s_sr" % name), accio, ins, ", ".join(clob))
    return text


# hbtc_fqmacsub_sr: X += a b, Y -= a b;  hbtc_fqsubsub_sr: X -= a b, Y -= a b (X = v60.., Y = v85..,
# modulo 2^800).  With hbtc_fqmac2_sr (Y += a b) they accumulate an Fq2 product by Karatsuba:
# X += a0 b0 - a1 b1, Y += (a0 + a1)(b0 + b1) - a0 b0 - a1 b1, three half products per term.
KARA_BODIES = (("hbtc_fqmacsub_sr", ((SR_MACC, "+"), (SR_MACC2, "-"))),
               ("hbtc_fqsubsub_sr", ((SR_MACC, "-"), (SR_MACC2, "-"))))


# ------------------------------------------------------------------ lane-pair Fq2 product (pair.h)
# hbtc_fqmul2_sr: r = (a b + c d) 2^-384 mod p in ONE product scanning, for operands < 2p (a b +
# c d < 8p^2, so r < 2p): the component of a lane-pair Fq2 product (lane 0: a0 b0 + (-a1) b1,
# lane 1: a0 b1 + a1 b0).  144 + 144 + 144 MACs + 12 digits against 2 x 144 + 168 for two lazy MACs
# and a reduction, and no 25-word accumulator.  Registers: a / r v8..v19, b v20..v31, c v32..v43,
# d v44..v55, q v56..v67, column accumulators v68..v71 (r_j is written at column 12 + j, after the
# last reads of a_j, b_j, c_j, d_j at column j + 11).
M2_A, M2_B, M2_C, M2_D, M2_Q, M2_ACC = 8, 20, 32, 44, 56, 68


def mul2_body():
    A = lambda i: "v%d" % (M2_A + i)
    B = lambda i: "v%d" % (M2_B + i)
    C = lambda i: "v%d" % (M2_C + i)
    D = lambda i: "v%d" % (M2_D + i)
    Q = lambda i: "v%d" % (M2_Q + i)
    P = lambda i: "s%d" % (SR_P + i)
    reg = lambda n: "v%d" % (M2_ACC + n)
    pair = lambda p: "v[%d:%d]" % (M2_ACC + 2 * p, M2_ACC + 2 * p + 1)
    out = ["v_mov_b32 %s, 0" % reg(0), "v_mov_b32 %s, 0" % reg(1)]
    for k in range(23):
        p = k % 2
        acc, lo, hi, c2, nlo = pair(p), reg(2 * p), reg(2 * p + 1), reg(2 * (1 - p) + 1), reg(2 * (1 - p))
        lo_i, hi_i = (0, k) if k < 12 else (k - 11, 11)
        terms = [(A(i), B(k - i)) for i in range(lo_i, hi_i + 1)]
        terms += [(C(i), D(k - i)) for i in range(lo_i, hi_i + 1)]
        terms += [(Q(i), P(k - i)) for i in range(lo_i, (k - 1 if k < 12 else 11) + 1)]
        for n, (x, y) in enumerate(terms):
            out.append("v_mad_u64_u32 %s, vcc, %s, %s, %s" % (acc, x, y, acc))
            out.append("v_addc_co_u32_e64 %s, vcc, %s, 0, vcc" % (c2, "0" if n == 0 else c2))
        if k < 12:
            out.append("v_mul_lo_u32 %s, %s, s%d" % (Q(k), lo, SR_NP))
            out.append("v_mad_u64_u32 %s, vcc, %s, %s, %s" % (acc, Q(k), P(0), acc))
            out.append("v_addc_co_u32_e64 %s, vcc, %s, 0, vcc" % (c2, c2))
        else:
            out.append("v_mov_b32 %s, %s" % (A(k - 12), lo))
        if k < 22:
            out.append("v_mov_b32 %s, %s" % (nlo, hi))
    out.append("v_mov_b32 %s, %s" % (A(11), reg(1)))  # column 22's high word; its overflow is 0
    return out


def mul2_call():
    call = ('      "s_getpc_b64 s[%d:%d]\\n\\t"\n' % (SR_TGT, SR_TGT + 1) +
            '      "s_add_u32 s%d, s%d, hbtc_fqmul2_sr@rel32@lo+4\\n\\t"\n' % (SR_TGT, SR_TGT) +
            '      "s_addc_u32 s%d, s%d, hbtc_fqmul2_sr@rel32@hi+12\\n\\t"\n' % (SR_TGT + 1, SR_TGT + 1) +
            '      "s_swappc_b64 s[%d:%d], s[%d:%d]"' % (SR_RET, SR_RET + 1, SR_TGT, SR_TGT + 1))
    outs = ", ".join('"={v%d}"(r[%d])' % (M2_A + i, i) for i in range(12))
    ins = []
    for base, nm in ((M2_A, "a"), (M2_B, "b"), (M2_C, "c"), (M2_D, "d")):
        ins.append(", ".join('"{v%d}"(%s[%d])' % (base + i, nm, i) for i in range(12)))
    clob = ['"v%d"' % v for v in range(M2_Q, M2_ACC + 4)]
    clob += ['"s%d"' % s for s in range(SR_P, SR_RET + 2)]
    clob += ['"vcc"', '"scc"']
    return """__device__ __forceinline__ void mont_mul2_sr(uint32_t* r, const uint32_t* a, const uint32_t* b,
                                             const uint32_t* c, const uint32_t* d) {
  asm volatile(
%s
      : %s
      : %s
      : %s);
}
""" % (call, outs, ",\n        ".join(ins), ", ".join(clob))


def selftest_mul2(trials=300):
    """hbtc_fqmul2_sr on the register-file simulator: r < 2p and r = (a b + c d) 2^-384 mod p,
    with the extreme operands 2p - 1 first."""
    import random
    M32 = (1 << 32) - 1
    rng = random.Random(11)
    prog = lazy_text("x", mul2_body())[2:-1]
    for t in range(trials):
        ops = [2 * P_MOD - 1] * 4 if t == 0 else [rng.randrange(2 * P_MOD) for _ in range(4)]
        regs = {}
        for base, v in zip((M2_A, M2_B, M2_C, M2_D), ops):
            for i in range(12):
                regs["v%d" % (base + i)] = (v >> (32 * i)) & M32
        run_prog(prog, regs)
        r = sum(regs["v%d" % (M2_A + i)] << (32 * i) for i in range(12))
        a, b, c, d = ops
        assert r < 2 * P_MOD and r % P_MOD == (a * b + c * d) * pow(2, -384, P_MOD) % P_MOD, t
        for base, v in zip((M2_B, M2_C, M2_D), ops[1:]):
            assert sum(regs["v%d" % (base + i)] << (32 * i) for i in range(12)) == v
    print("selftest_mul2 ok (%d instructions)" % len(prog))


def main_sr():
    print("""// GENERATED by tools/gen_fips_asm.py --sr -- do not edit.
// The Fq Montgomery product and squaring of fq_fips_asm.h as ONE shared subroutine each, called
// with s_swappc from a four-instruction call-site block (see the generator: calling convention,
// and why: code size of the hot loops vs the instruction cache).  Device builds that define
// HBTC_FQMUL_SR only.  Only VALU instructions on registers, plus the SALU modulus setup and the
// branches.
#pragma once
#include <cstdint>
#if defined(__HIP_DEVICE_COMPILE__)""")
    # The subroutines live in the code of a never-launched kernel of each translation unit
    # (file-scope asm is not emitted in the device compilation): an s_endpgm, then the bodies.
    print('static __global__ void __launch_bounds__(64) hbtc_fq_sr_holder() {')
    print('  asm volatile(')
    print('    "s_endpgm\\n"')
    for label, square in (("hbtc_fqmul_sr", False), ("hbtc_fqsqr_sr", True)):
        for l in sr_text(label, square):
            print('    "%s\\n"' % l)
    for label, body in (("hbtc_fqmac_sr", mac_body()), ("hbtc_fqredc_sr", redc_body()),
                        ("hbtc_fqmac2_sr", mac_body(SR_MACC2)), ("hbtc_fqredc2_sr", redc_body(SR_MACC2))) + tuple(
                            (label, mac_body(targets=list(t))) for label, t in KARA_BODIES) + (
                                ("hbtc_fqmul2_sr", mul2_body()),):
        for l in lazy_text(label, body):
            print('    "%s\\n"' % l)
    print('    ::: "memory");')
    print('}')
    print("""namespace hbtc {
namespace fips {
""")
    print(sr_call("mont_mul_sr", "hbtc_fqmul_sr", False))
    print(sr_call("mont_sqr_sr", "hbtc_fqsqr_sr", True))
    print(lazy_calls())
    print(mul2_call())
    print("""}  // namespace fips
}  // namespace hbtc
#endif""")


def selftest_sr(trials=200):
    """Run the subroutine bodies on a concrete register file (VCC as one lane's carry bit)."""
    import random
    M32 = (1 << 32) - 1
    rng = random.Random(9)
    for square in (False, True):
        prog = sr_text("x", square)[2:-1]
        for _ in range(trials):
            a = rng.randrange(2 * P_MOD)
            b = a if square else rng.randrange(2 * P_MOD)
            regs = {}
            for i in range(12):
                regs["v%d" % (SR_A + i)] = (a >> (32 * i)) & M32
            al = [(a >> (32 * i)) & M32 for i in range(12)]
            if square:
                for j in range(1, 12):
                    regs["v%d" % (SR_B + j)] = (al[j] << 1) & M32
                for j in range(2, 12):
                    regs["v%d" % (SR_D1 + j - 2)] = ((al[j] << 1) | (al[j - 1] >> 31)) & M32
            else:
                for i in range(12):
                    regs["v%d" % (SR_B + i)] = (b >> (32 * i)) & M32
            vcc = 0

            def val(t):
                t = t.strip()
                if t.startswith("0x") or t.isdigit():
                    return int(t, 0)
                m = re.fullmatch(r"v\[(\d+):(\d+)\]", t)
                if m:
                    return regs["v" + m.group(1)] | (regs["v" + m.group(2)] << 32)
                return regs[t]

            def store(t, v):
                t = t.strip()
                m = re.fullmatch(r"v\[(\d+):(\d+)\]", t)
                if m:
                    regs["v" + m.group(1)] = v & M32
                    regs["v" + m.group(2)] = (v >> 32) & M32
                else:
                    regs[t] = v & M32

            for line in prog:
                op, rest = line.split(" ", 1)
                args = re.split(r",(?![^\[]*\])", rest)
                if op in ("s_mov_b32", "v_mov_b32"):
                    store(args[0], val(args[1]))
                elif op == "v_mad_u64_u32":
                    d, _, x, y, z = args
                    s = val(x) * val(y) + val(z)
                    vcc = s >> 64
                    store(d, s & ((1 << 64) - 1))
                elif op == "v_addc_co_u32_e64":
                    d, _, x, y, _c = args
                    s = val(x) + val(y) + vcc
                    vcc = s >> 32
                    store(d, s)
                elif op == "v_mul_lo_u32":
                    d, x, y = args
                    store(d, val(x) * val(y))
                else:
                    raise ValueError(op)
            r = sum(regs["v%d" % (SR_A + i)] << (32 * i) for i in range(12))
            want = a * b * pow(2, -384, P_MOD) % P_MOD
            assert r < 2 * P_MOD and r % P_MOD == want, ("sr square" if square else "sr mul", hex(a), hex(b))
    print("selftest_sr ok")


if __name__ == "__main__" and len(__import__("sys").argv) > 1 and __import__("sys").argv[1] == "--sr":
    main_sr()

if __name__ == "__main__" and len(__import__("sys").argv) == 1:
    main()


def selftest(trials=300):
    """The inline-asm form: its instruction list IS sr_body's with other register names, so
    check that the two lists agree name for name (sr_body maps every operand and accumulator
    to a fixed register), then selftest_sr executes the list."""
    for square in (False, True):
        a, b = gen_mul(square), sr_body(square)
        assert len(a) == len(b) and all(x.split(" ", 1)[0] == y.split(" ", 1)[0] for x, y in zip(a, b))
        assert not any("HBTC_" in y or "%" in y for y in b), "unmapped operand"
    print("selftest ok (%d / %d instructions)" % (len(gen_mul(False)), len(gen_mul(True))))


if __name__ == "__main__" and len(__import__("sys").argv) > 1 and __import__("sys").argv[1] == "--selftest":
    selftest()
    selftest_sr()


def run_prog(prog, regs):
    """Execute a subroutine body on one lane's register file; carry bits by register name."""
    M32 = (1 << 32) - 1
    carry = {}

    def val(t):
        t = t.strip()
        if t.startswith("0x") or t.isdigit():
            return int(t, 0)
        m = re.fullmatch(r"v\[(\d+):(\d+)\]", t)
        if m:
            return regs["v" + m.group(1)] | (regs["v" + m.group(2)] << 32)
        return regs[t]

    def store(t, v):
        t = t.strip()
        m = re.fullmatch(r"v\[(\d+):(\d+)\]", t)
        if m:
            regs["v" + m.group(1)] = v & M32
            regs["v" + m.group(2)] = (v >> 32) & M32
        else:
            regs[t] = v & M32

    for line in prog:
        op, rest = line.split(" ", 1)
        args = [x.strip() for x in re.split(r",(?![^\[]*\])", rest)]
        if op in ("s_mov_b32", "v_mov_b32"):
            store(args[0], val(args[1]))
        elif op == "v_mad_u64_u32":
            d, c, x, y, z = args
            s = val(x) * val(y) + val(z)
            carry[c] = s >> 64
            store(d, s)
        elif op == "v_add_co_u32_e64":
            d, c, x, y = args
            s = val(x) + val(y)
            carry[c] = s >> 32
            store(d, s)
        elif op == "v_addc_co_u32_e64":
            d, c, x, y, ci = args
            s = val(x) + val(y) + carry[ci]
            carry[c] = s >> 32
            store(d, s)
        elif op == "v_add_u32_e32":
            d, x, y = args
            store(d, val(x) + val(y))
        elif op == "v_subrev_co_u32_e32":
            d, c, x, y = args
            s = val(y) - val(x)
            carry[c] = 1 if s < 0 else 0
            store(d, s)
        elif op == "v_subbrev_co_u32_e32":
            d, c, x, y, ci = args
            s = val(y) - val(x) - carry[ci]
            carry[c] = 1 if s < 0 else 0
            store(d, s)
        elif op in ("v_sub_co_u32_e32", "v_sub_co_u32_e64"):
            d, c, x, y = args
            s = val(x) - val(y)
            carry[c] = 1 if s < 0 else 0
            store(d, s)
        elif op in ("v_subb_co_u32_e32", "v_subb_co_u32_e64"):
            d, c, x, y, ci = args
            s = val(x) - val(y) - carry[ci]
            carry[c] = 1 if s < 0 else 0
            store(d, s)
        elif op == "v_cndmask_b32_e32":
            d, x, y, c = args
            store(d, val(y) if carry[c] else val(x))
        elif op == "v_mul_lo_u32":
            d, x, y = args
            store(d, val(x) * val(y))
        else:
            raise ValueError(op)


def selftest_lazy(trials=200):
    """ACC = sum of up to 12 products of operands < 2p through hbtc_fqmac_sr, then
    hbtc_fqredc_sr: r < 2p and r = ACC 2^-384 mod p; a and b survive the MAC.  The same for the
    second accumulator's pair, and neither pair touches the other accumulator."""
    import random
    M32 = (1 << 32) - 1
    rng = random.Random(10)
    for base, other in ((SR_MACC, SR_MACC2), (SR_MACC2, SR_MACC)):
        mac = lazy_text("x", mac_body(base))[2:-1]
        redc = lazy_text("x", redc_body(base))[2:-1]
        for t in range(trials):
            regs = {"v%d" % (base + i): 0 for i in range(25)}
            guard = [rng.getrandbits(32) for _ in range(25)]
            regs.update({"v%d" % (other + i): guard[i] for i in range(25)})
            total = 0
            n = [1, 2, 12][t % 3] if t >= 3 else 12
            for _ in range(n):
                a = rng.randrange(2 * P_MOD) if t else 2 * P_MOD - 1
                b = rng.randrange(2 * P_MOD) if t else 2 * P_MOD - 1
                for i in range(12):
                    regs["v%d" % (SR_A + i)] = (a >> (32 * i)) & M32
                    regs["v%d" % (SR_B + i)] = (b >> (32 * i)) & M32
                run_prog(mac, regs)
                total += a * b
                assert sum(regs["v%d" % (SR_A + i)] << (32 * i) for i in range(12)) == a
                assert sum(regs["v%d" % (SR_B + i)] << (32 * i) for i in range(12)) == b
            assert sum(regs["v%d" % (base + i)] << (32 * i) for i in range(25)) == total
            run_prog(redc, regs)
            r = sum(regs["v%d" % (SR_A + i)] << (32 * i) for i in range(12))
            assert r < 2 * P_MOD and r % P_MOD == total * pow(2, -384, P_MOD) % P_MOD, (t, n)
            assert sum(regs["v%d" % (base + i)] << (32 * i) for i in range(25)) == total
            assert [regs["v%d" % (other + i)] for i in range(25)] == guard
    # Karatsuba accumulation: X starts at K = 24 p^2, up to 6 terms of operands < 2p
    K = 24 * P_MOD * P_MOD
    macsub = lazy_text("x", mac_body(targets=list(KARA_BODIES[0][1])))[2:-1]
    subsub = lazy_text("x", mac_body(targets=list(KARA_BODIES[1][1])))[2:-1]
    mac2 = lazy_text("x", mac_body(SR_MACC2))[2:-1]
    redc1 = lazy_text("x", redc_body(SR_MACC))[2:-1]
    redc2 = lazy_text("x", redc_body(SR_MACC2))[2:-1]
    M800 = (1 << 800) - 1

    def load(v, base, words):
        for i in range(words):
            regs["v%d" % (base + i)] = (v >> (32 * i)) & M32

    def read(base, words):
        return sum(regs["v%d" % (base + i)] << (32 * i) for i in range(words))

    for t in range(trials):
        regs = {}
        load(K, SR_MACC, 25)
        load(0, SR_MACC2, 25)
        c0 = c1 = 0
        for _ in range(1 + t % 6 if t else 6):
            a0, a1, b0, b1 = (rng.randrange(2 * P_MOD) if t else 2 * P_MOD - 1 for _ in range(4))
            for f, x, y in ((macsub, a0, b0), (subsub, a1, b1), (mac2, a0 + a1, b0 + b1)):
                load(x, SR_A, 12)
                load(y, SR_B, 12)
                run_prog(f, regs)
            c0 += a0 * b0 - a1 * b1
            c1 += a0 * b1 + a1 * b0
        assert read(SR_MACC, 25) == (K + c0) & M800 and read(SR_MACC2, 25) == c1 & M800
        assert 0 <= K + c0 < 48 * P_MOD * P_MOD and 0 <= c1 < 48 * P_MOD * P_MOD
        run_prog(redc1, regs)
        r0 = read(SR_A, 12)
        run_prog(redc2, regs)
        r1 = read(SR_A, 12)
        Ri = pow(2, -384, P_MOD)
        assert r0 < 2 * P_MOD and r0 % P_MOD == c0 * Ri % P_MOD, t
        assert r1 < 2 * P_MOD and r1 % P_MOD == c1 * Ri % P_MOD, t
    print("selftest_lazy ok (%d / %d instructions; Karatsuba pair %d)" % (len(mac), len(redc), len(macsub)))


if __name__ == "__main__" and len(__import__("sys").argv) > 1 and __import__("sys").argv[1] == "--selftest-lazy":
    selftest_lazy()
    selftest_mul2()
