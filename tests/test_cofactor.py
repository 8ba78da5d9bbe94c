"""The G2 cofactor clearing of hash_g2 / hash_g1_g2 (hbbft_amd/csrc/curve.h g2_clear_cofactor)
restated on the oracle's curve arithmetic: for points of E'(Fq2) OUTSIDE G2 (G2::rand's
candidates), the psi chain equals pairing 0.14's literal [h2] multiplication.  CPU only."""
import random

from oracle import bls12_381 as B

P, R, X, H2 = B.P, B.R, B.X, B.H2
C0 = 0x72D91800AAABC2AC00000000AAAAAAAA  # bls_constants.h G2_CLEAR_C0


def _f2_pow(a, e):
    r = (1, 0)
    while e:
        if e & 1:
            r = B.f2_mul(r, a)
        a = B.f2_sqr(a)
        e >>= 1
    return r


CX = B.f2_inv(_f2_pow((1, 1), (P - 1) // 3))
CY = B.f2_inv(_f2_pow((1, 1), (P - 1) // 2))
ZETA = B.f2_mul(CX, B.f2_conj(CX))[0]


def psi(pt):
    x, y = pt
    return (B.f2_mul(B.f2_conj(x), CX), B.f2_mul(B.f2_conj(y), CY))


def mul(pt, k):
    """[k] pt for any integer k on the whole curve E'(Fq2)."""
    if k < 0:
        return B.g2_neg(B._mul(B.FQ2, pt, -k))
    return B._mul(B.FQ2, pt, k)


def clear_cofactor_psi(pt):
    """curve.h g2_clear_cofactor: Q = [x^2 - x - 1] P + [x - 1] psi(P) + psi^2(2P), then
    [c0] (Q + m(Q)) + m(Q) with m(x, y) = (zeta x, y)."""
    t1 = mul(pt, X)
    t2 = psi(pt)
    t3 = B.g2_add(psi(psi(mul(pt, 2))), B.g2_neg(t2))
    t2 = mul(B.g2_add(t1, t2), X)
    q = B.g2_add(B.g2_add(B.g2_add(t3, t2), B.g2_neg(t1)), B.g2_neg(pt))
    if q is None:
        return None
    mq = (B.f2_mul(q[0], (ZETA, 0)), q[1])
    return B.g2_add(mul(B.g2_add(q, mq), C0), mq)


def test_decomposition_constant():
    mu = (-X * X) % R
    s = pow((3 * X * X - 3) % R, -1, R)
    assert (C0 + (C0 + 1) * mu - s) % R == 0 and C0 < 1 << 127
    g = B.g2_mul(B.G2_GEN, 77)
    assert (B.f2_mul(g[0], (ZETA, 0)), g[1]) == B.g2_mul(g, mu)


def test_psi_chain_equals_h2_multiplication():
    rng = random.Random(11)
    done = 0
    while done < 2:
        x = (rng.randrange(P), rng.randrange(P))
        y = B.f2_sqrt(B.f2_add(B.f2_mul(B.f2_sqr(x), x), (4, 4)))
        if y is None:
            continue
        pt = (x, y)
        assert not B.g2_in_subgroup(pt)  # a G2::rand candidate: off the subgroup
        assert clear_cofactor_psi(pt) == mul(pt, H2)
        done += 1
