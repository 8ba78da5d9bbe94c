"""BLS12-381 restated in plain Python big-int arithmetic — TEST ORACLE ONLY.

Restates the parts of ``pairing 0.14.2`` (crate ``pairing``, module ``bls12_381``;
NOT vendored under /root/reference — hbbft declares it at Cargo.toml:27 and uses it
directly at src/sync_key_gen.rs:173-174,430,493) that hbbft's crypto hot path
touches [EXT-UNVERIFIED: written from the published BLS12-381 / zcash
serialization specification, not from the crate's source]:

  * Fq (381-bit prime), Fq2 = Fq[u]/(u^2+1), Fq12 (flat: Fq[w]/(w^12 - 2w^6 + 2),
    with u = w^6 - 1 so that w^6 = u + 1 = xi);
  * G1: y^2 = x^3 + 4 over Fq; G2: y^2 = x^3 + 4(u+1) over Fq2;
  * optimal ate pairing with x = -0xd201000000010000 (Miller loop on the twist,
    lines multiplied by w^3, conjugated for negative x) + final exponentiation
    (p^12 - 1)/r.  The Fq12 *value* follows the standard convention; hbbft only
    ever compares pairings for equality (threshold_crypto verify*), so accept /
    reject decisions are independent of the Miller-loop variant;
  * zcash compressed / uncompressed point encodings with the pairing-0.14 decode
    checks (compression bit, infinity bit, lexicographically-largest-y bit,
    coordinate < p, on-curve, subgroup via multiplication by r).

Points are affine tuples ``(x, y)`` (G2 coordinates are ``(c0, c1)`` tuples) and
``None`` is the point at infinity.  Speed: a pairing takes ~0.1-0.3 s; use this
module only for small cases (the C restatement in ``oracle/c`` is the fast oracle).
"""

# ----------------------------------------------------------------------------- constants
X = -0xD201000000010000  # BLS parameter; |X| has Hamming weight 6
R = X ** 4 - X ** 2 + 1  # subgroup order (255 bit)
P = (X - 1) ** 2 * R // 3 + X  # base field modulus (381 bit)
H1 = (X - 1) ** 2 // 3  # G1 cofactor
H2 = (X ** 8 - 4 * X ** 7 + 5 * X ** 6 - 4 * X ** 4 + 6 * X ** 3 - 4 * X ** 2 - 4 * X + 13) // 9  # G2 cofactor

assert R == 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
assert P == 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
# pairing 0.14 hard-codes this constant in G2Affine::scale_by_cofactor [EXT-UNVERIFIED]
assert H2 == 0x5D543A95414E7F1091D50792876A202CD91DE4547085ABAA68A205B2E5A7DDFA628F1CB4D9E82EF21537E293A6691AE1616EC6E786F0C70CF1C38E31C7238E5

G1_GEN = (
    0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB,
    0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1,
)
G2_GEN = (
    (0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
     0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E),
    (0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
     0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE),
)


# ----------------------------------------------------------------------------- Fq
def fq_inv(a):
    a %= P
    if a == 0:
        raise ZeroDivisionError("Fq inverse of 0")
    return pow(a, P - 2, P)


def fq_sqrt(a):
    """Square root for p = 3 mod 4; None if a is not a square."""
    a %= P
    y = pow(a, (P + 1) // 4, P)
    return y if y * y % P == a else None


def fq_is_square(a):
    a %= P
    return a == 0 or pow(a, (P - 1) // 2, P) == 1


# ----------------------------------------------------------------------------- Fq2
F2_ZERO = (0, 0)
F2_ONE = (1, 0)


def f2_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2_neg(a):
    return ((-a[0]) % P, (-a[1]) % P)


def f2_mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def f2_sqr(a):
    return ((a[0] + a[1]) * (a[0] - a[1]) % P, 2 * a[0] * a[1] % P)


def f2_scale(a, k):
    return (a[0] * k % P, a[1] * k % P)


def f2_inv(a):
    n = fq_inv(a[0] * a[0] + a[1] * a[1])
    return (a[0] * n % P, (-a[1]) * n % P)


def f2_conj(a):
    return (a[0], (-a[1]) % P)


def f2_sqrt(a):
    """Some square root of a in Fq2 (u^2 = -1), or None if a is a non-square."""
    a0, a1 = a[0] % P, a[1] % P
    if a1 == 0:
        s = fq_sqrt(a0)
        if s is not None:
            return (s, 0)
        s = fq_sqrt(-a0)
        return (0, s)  # (s*u)^2 = -s^2 = a0
    norm = (a0 * a0 + a1 * a1) % P
    s = fq_sqrt(norm)
    if s is None:
        return None
    inv2 = fq_inv(2)
    for d in ((a0 + s) * inv2 % P, (a0 - s) * inv2 % P):
        x0 = fq_sqrt(d)
        if x0 is not None and x0 != 0:
            x1 = a1 * fq_inv(2 * x0) % P
            r = (x0, x1)
            if f2_sqr(r) == (a0, a1):
                return r
    return None


def fq_lt(a, b):
    return (a % P) < (b % P)


def f2_lt(a, b):
    """pairing 0.14 ``Ord for Fq2``: compare c1 first, then c0 (canonical values)."""
    if a[1] != b[1]:
        return a[1] < b[1]
    return a[0] < b[0]


# ----------------------------------------------------------------------------- curves
class _Field:
    """Operation table so one Jacobian implementation serves G1 (Fq) and G2 (Fq2)."""

    def __init__(self, add, sub, mul, sqr, inv, neg, zero, one, b):
        self.add, self.sub, self.mul, self.sqr, self.inv, self.neg = add, sub, mul, sqr, inv, neg
        self.zero, self.one, self.b = zero, one, b


FQ = _Field(lambda a, b: (a + b) % P, lambda a, b: (a - b) % P, lambda a, b: a * b % P,
            lambda a: a * a % P, fq_inv, lambda a: (-a) % P, 0, 1, 4)
FQ2 = _Field(f2_add, f2_sub, f2_mul, f2_sqr, f2_inv, f2_neg, F2_ZERO, F2_ONE, (4, 4))


def on_curve(F, pt):
    if pt is None:
        return True
    x, y = pt
    return F.sqr(y) == F.add(F.mul(F.sqr(x), x), F.b)


def _to_jac(F, pt):
    return (F.one, F.one, F.zero) if pt is None else (pt[0], pt[1], F.one)


def _jac_is_inf(F, J):
    return J[2] == F.zero


def _from_jac(F, J):
    if _jac_is_inf(F, J):
        return None
    zi = F.inv(J[2])
    zi2 = F.sqr(zi)
    return (F.mul(J[0], zi2), F.mul(J[1], F.mul(zi2, zi)))


def _jac_dbl(F, J):
    X1, Y1, Z1 = J
    if Z1 == F.zero or Y1 == F.zero:
        return (F.one, F.one, F.zero)
    A = F.sqr(X1)
    B = F.sqr(Y1)
    C = F.sqr(B)
    D = F.sub(F.sqr(F.add(X1, B)), F.add(A, C))
    D = F.add(D, D)
    E = F.add(F.add(A, A), A)
    Fv = F.sqr(E)
    X3 = F.sub(Fv, F.add(D, D))
    C8 = F.add(C, C)
    C8 = F.add(C8, C8)
    C8 = F.add(C8, C8)
    Y3 = F.sub(F.mul(E, F.sub(D, X3)), C8)
    Z3 = F.mul(F.add(Y1, Y1), Z1)
    return (X3, Y3, Z3)


def _jac_add(F, J1, J2):
    if _jac_is_inf(F, J1):
        return J2
    if _jac_is_inf(F, J2):
        return J1
    X1, Y1, Z1 = J1
    X2, Y2, Z2 = J2
    Z1Z1 = F.sqr(Z1)
    Z2Z2 = F.sqr(Z2)
    U1 = F.mul(X1, Z2Z2)
    U2 = F.mul(X2, Z1Z1)
    S1 = F.mul(Y1, F.mul(Z2, Z2Z2))
    S2 = F.mul(Y2, F.mul(Z1, Z1Z1))
    if U1 == U2:
        if S1 == S2:
            return _jac_dbl(F, J1)
        return (F.one, F.one, F.zero)
    H = F.sub(U2, U1)
    I = F.sqr(F.add(H, H))
    J = F.mul(H, I)
    rr = F.sub(S2, S1)
    rr = F.add(rr, rr)
    V = F.mul(U1, I)
    X3 = F.sub(F.sub(F.sqr(rr), J), F.add(V, V))
    S1J = F.mul(S1, J)
    Y3 = F.sub(F.mul(rr, F.sub(V, X3)), F.add(S1J, S1J))
    Z3 = F.mul(F.sub(F.sqr(F.add(Z1, Z2)), F.add(Z1Z1, Z2Z2)), H)
    return (X3, Y3, Z3)


def _mul(F, pt, k):
    if pt is None or k == 0:
        return None
    if k < 0:
        pt = (pt[0], F.neg(pt[1]))
        k = -k
    acc = (F.one, F.one, F.zero)
    base = _to_jac(F, pt)
    for bit in bin(k)[2:]:
        acc = _jac_dbl(F, acc)
        if bit == "1":
            acc = _jac_add(F, acc, base)
    return _from_jac(F, acc)


def _add(F, a, b):
    return _from_jac(F, _jac_add(F, _to_jac(F, a), _to_jac(F, b)))


def _neg(F, a):
    return None if a is None else (a[0], F.neg(a[1]))


def g1_add(a, b):
    return _add(FQ, a, b)


def g1_neg(a):
    return _neg(FQ, a)


def g1_mul(pt, k):
    """Scalar multiplication by an arbitrary integer (no reduction mod r)."""
    return _mul(FQ, pt, k)


def g2_add(a, b):
    return _add(FQ2, a, b)


def g2_neg(a):
    return _neg(FQ2, a)


def g2_mul(pt, k):
    return _mul(FQ2, pt, k)


def g1_sum(points):
    acc = (1, 1, 0)
    for q in points:
        acc = _jac_add(FQ, acc, _to_jac(FQ, q))
    return _from_jac(FQ, acc)


def g2_sum(points):
    acc = (F2_ONE, F2_ONE, F2_ZERO)
    for q in points:
        acc = _jac_add(FQ2, acc, _to_jac(FQ2, q))
    return _from_jac(FQ2, acc)


def g1_in_subgroup(pt):
    """pairing 0.14 ``is_in_correct_subgroup_assuming_on_curve``: r * P == O."""
    return g1_mul(pt, R) is None


def g2_in_subgroup(pt):
    return g2_mul(pt, R) is None


# ----------------------------------------------------------------------------- codec (zcash)
def _fq_to_be(a):
    return int(a).to_bytes(48, "big")


def g1_compress(pt):
    """``G1Compressed::from_affine``: x big-endian, flags 0x80 | 0x40 (inf) | 0x20 (y > -y)."""
    if pt is None:
        b = bytearray(48)
        b[0] = 0xC0
        return bytes(b)
    x, y = pt
    b = bytearray(_fq_to_be(x))
    if y > (-y) % P:
        b[0] |= 0x20
    b[0] |= 0x80
    return bytes(b)


def g1_uncompress_bytes(pt):
    """``G1Uncompressed::from_affine`` (96 bytes, x||y, 0x40 for infinity)."""
    if pt is None:
        b = bytearray(96)
        b[0] = 0x40
        return bytes(b)
    return _fq_to_be(pt[0]) + _fq_to_be(pt[1])


def g2_compress(pt):
    """``G2Compressed::from_affine``: x.c1 || x.c0, flags as G1 with Fq2 ordering."""
    if pt is None:
        b = bytearray(96)
        b[0] = 0xC0
        return bytes(b)
    x, y = pt
    b = bytearray(_fq_to_be(x[1]) + _fq_to_be(x[0]))
    if f2_lt(f2_neg(y), y):
        b[0] |= 0x20
    b[0] |= 0x80
    return bytes(b)


def g2_uncompress_bytes(pt):
    """``G2Uncompressed::from_affine`` (192 bytes: x.c1||x.c0||y.c1||y.c0)."""
    if pt is None:
        b = bytearray(192)
        b[0] = 0x40
        return bytes(b)
    x, y = pt
    return _fq_to_be(x[1]) + _fq_to_be(x[0]) + _fq_to_be(y[1]) + _fq_to_be(y[0])


class DecodeError(ValueError):
    pass


def g1_point_from_x(x, greatest):
    """``G1Affine::get_point_from_x``."""
    y = fq_sqrt(x * x * x + 4)
    if y is None:
        return None
    negy = (-y) % P
    return (x, y if (y < negy) ^ greatest else negy)


def g2_point_from_x(x, greatest):
    """``G2Affine::get_point_from_x`` (Fq2 order: c1, then c0)."""
    y = f2_sqrt(f2_add(f2_mul(f2_sqr(x), x), (4, 4)))
    if y is None:
        return None
    negy = f2_neg(y)
    return (x, y if f2_lt(y, negy) ^ greatest else negy)


def g1_decompress(data, check_subgroup=True):
    """``G1Compressed::into_affine`` — raises DecodeError exactly where pairing 0.14 errs."""
    if len(data) != 48:
        raise DecodeError("length")
    c = bytearray(data)
    if not c[0] & 0x80:
        raise DecodeError("UnexpectedCompressionMode")
    if c[0] & 0x40:
        c[0] &= 0x3F
        if any(c):
            raise DecodeError("UnexpectedInformation")
        return None
    greatest = bool(c[0] & 0x20)
    c[0] &= 0x1F
    x = int.from_bytes(c, "big")
    if x >= P:
        raise DecodeError("CoordinateDecodingError")
    pt = g1_point_from_x(x, greatest)
    if pt is None:
        raise DecodeError("NotOnCurve")
    if check_subgroup and not g1_in_subgroup(pt):
        raise DecodeError("NotInSubgroup")
    return pt


def g2_decompress(data, check_subgroup=True):
    """``G2Compressed::into_affine``."""
    if len(data) != 96:
        raise DecodeError("length")
    c = bytearray(data)
    if not c[0] & 0x80:
        raise DecodeError("UnexpectedCompressionMode")
    if c[0] & 0x40:
        c[0] &= 0x3F
        if any(c):
            raise DecodeError("UnexpectedInformation")
        return None
    greatest = bool(c[0] & 0x20)
    c[0] &= 0x1F
    x1 = int.from_bytes(c[:48], "big")
    x0 = int.from_bytes(c[48:], "big")
    if x0 >= P or x1 >= P:
        raise DecodeError("CoordinateDecodingError")
    pt = g2_point_from_x((x0, x1), greatest)
    if pt is None:
        raise DecodeError("NotOnCurve")
    if check_subgroup and not g2_in_subgroup(pt):
        raise DecodeError("NotInSubgroup")
    return pt


# ----------------------------------------------------------------------------- Fq12 (flat)
# Elements: lists of 12 ints, sum c_i w^i, modulus w^12 = 2 w^6 - 2.
_KS = 768  # Kronecker slot width: 12 * p^2 < 2^766
_KMASK = (1 << _KS) - 1


def f12_one():
    return [1] + [0] * 11


def _pack(a):
    v = 0
    for c in reversed(a):
        v = (v << _KS) | c
    return v


def f12_mul(a, b):
    prod = _pack(a) * _pack(b)
    c = []
    for _ in range(23):
        c.append(prod & _KMASK)
        prod >>= _KS
    for k in range(22, 11, -1):  # w^k = 2 w^(k-6) - 2 w^(k-12)
        t = c[k]
        if t:
            c[k - 6] += 2 * t
            c[k - 12] -= 2 * t
    return [v % P for v in c[:12]]


def f12_sqr(a):
    return f12_mul(a, a)


def f2_to_f12(a, k=0):
    """Embed a0 + a1 u (u = w^6 - 1) times w^k."""
    out = [0] * 12
    out[k % 12] = (a[0] - a[1]) % P
    out[(k + 6) % 12] = a[1] % P
    assert k < 6
    return out


def _poly_divmod(num, den):
    num = list(num)
    dl = len(den) - 1
    while dl >= 0 and den[dl] == 0:
        dl -= 1
    inv_lead = fq_inv(den[dl])
    q = [0] * max(1, len(num) - dl)
    for i in range(len(num) - 1, dl - 1, -1):
        coef = num[i] * inv_lead % P
        if coef:
            q[i - dl] = coef
            for j in range(dl + 1):
                num[i - dl + j] = (num[i - dl + j] - coef * den[j]) % P
    return q, num[:dl] if dl > 0 else [0]


def _poly_trim(a):
    a = list(a)
    while len(a) > 1 and a[-1] == 0:
        a.pop()
    return a


def _poly_mul(a, b):
    out = [0] * (len(a) + len(b) - 1)
    for i, x in enumerate(a):
        if x:
            for j, y in enumerate(b):
                out[i + j] = (out[i + j] + x * y) % P
    return out


def _poly_sub(a, b):
    n = max(len(a), len(b))
    return [((a[i] if i < len(a) else 0) - (b[i] if i < len(b) else 0)) % P for i in range(n)]


_MODULUS = [2] + [0] * 5 + [P - 2] + [0] * 5 + [1]  # w^12 - 2w^6 + 2


def f12_inv(a):
    """Extended Euclid over Fq[w]."""
    lm, hm = [1], [0]
    low, high = _poly_trim(a), list(_MODULUS)
    while len(_poly_trim(low)) > 1 or _poly_trim(low)[0] != 1:
        low = _poly_trim(low)
        if len(low) == 1:
            inv = fq_inv(low[0])
            lm = [c * inv % P for c in lm]
            break
        q, rem = _poly_divmod(high, low)
        nm = _poly_sub(hm, _poly_mul(lm, q))
        lm, low, hm, high = nm, rem, lm, low
    out = [0] * 12
    for i, c in enumerate(lm[:12]):
        out[i] = c % P
    return out


# Frobenius: (sum a_i w^i)^p = sum a_i (w^p)^i ; precompute w^(p*i) mod modulus.
def _f12_pow(a, e):
    res = f12_one()
    for bit in bin(e)[2:]:
        res = f12_sqr(res)
        if bit == "1":
            res = f12_mul(res, a)
    return res


_W = [0, 1] + [0] * 10
_WP = _f12_pow(_W, P)
_FROB = [f12_one()]
for _i in range(1, 12):
    _FROB.append(f12_mul(_FROB[-1], _WP))


def f12_frob(a):
    out = [0] * 12
    for i, c in enumerate(a):
        if c:
            row = _FROB[i]
            for j in range(12):
                out[j] += c * row[j]
    return [v % P for v in out]


def f12_conj(a):
    """a^(p^6): negate odd powers of w (w^(p^6) = -w since w^6 = xi and xi^((p^6-1)/6)... )."""
    r = a
    for _ in range(6):
        r = f12_frob(r)
    return r


_HARD = (P ** 4 - P ** 2 + 1) // R
assert (P ** 4 - P ** 2 + 1) % R == 0


def final_exponentiation(f):
    """f^((p^12 - 1)/r) = f^((p^6 - 1)(p^2 + 1) * (p^4 - p^2 + 1)/r)."""
    t = f12_mul(f12_conj(f), f12_inv(f))  # f^(p^6 - 1)
    t = f12_mul(f12_frob(f12_frob(t)), t)  # ^(p^2 + 1)
    return _f12_pow(t, _HARD)


def _line(lam, xr, yr, P1):
    """Line through R on E' with slope lam, evaluated at P1 and scaled by w^3:
    (lam*xr - yr) + (-lam*xP) w^2 + yP w^3."""
    xp, yp = P1
    c0 = f2_sub(f2_mul(lam, xr), yr)
    c2 = f2_scale(lam, (-xp) % P)
    out = f2_to_f12(c0, 0)
    o2 = f2_to_f12(c2, 2)
    for i in range(12):
        out[i] = (out[i] + o2[i]) % P
    out[3] = (out[3] + yp) % P
    return out


def miller_loop(P1, Q2):
    """f_{|x|,Q}(P) conjugated (x < 0); 1 if either input is the identity."""
    if P1 is None or Q2 is None:
        return f12_one()
    f = f12_one()
    Rx, Ry = Q2
    for bit in bin(-X)[3:]:
        lam = f2_mul(f2_scale(f2_sqr(Rx), 3), f2_inv(f2_add(Ry, Ry)))
        f = f12_mul(f12_sqr(f), _line(lam, Rx, Ry, P1))
        nx = f2_sub(f2_sqr(lam), f2_add(Rx, Rx))
        Ry = f2_sub(f2_mul(lam, f2_sub(Rx, nx)), Ry)
        Rx = nx
        if bit == "1":
            lam = f2_mul(f2_sub(Q2[1], Ry), f2_inv(f2_sub(Q2[0], Rx)))
            f = f12_mul(f, _line(lam, Rx, Ry, P1))
            nx = f2_sub(f2_sub(f2_sqr(lam), Rx), Q2[0])
            Ry = f2_sub(f2_mul(lam, f2_sub(Rx, nx)), Ry)
            Rx = nx
    return f12_conj(f)


def pairing(P1, Q2):
    """``Bls12::pairing(p, q)`` = final_exponentiation(miller_loop(p, q))."""
    return final_exponentiation(miller_loop(P1, Q2))


def f12_is_one(a):
    return a == f12_one()
