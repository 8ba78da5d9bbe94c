"""Why the G1 decode keeps Scott's membership test (VERDICT r05 "Missing 1" / "Next 2").

Every DecryptionShare is deserialised with pairing 0.14's subgroup check before hbbft sees it
(/root/reference/src/honey_badger/epoch_state.rs:246-261), so k_rlc_decode tests membership per
share, exactly.  It computes t1 = [|x|] d (kept: the x-adic table's second entry) and t2 = [|x|] t1
and checks phi(d) == -[x^2] d.  These tests pin the facts DESIGN.md §8 uses to conclude that no
cheaper exact test exists for BLS12-381's G1:

1. Any test of the form alpha(P) == O with alpha = a0 + a1 phi (every published endomorphism test
   for G1, Dai-Lin-Zhao-Zhou ePrint 2022/348 included, is of this form, with a1 possibly
   composed of |x|-chains) must kill all of G1, i.e. a0 + a1 lambda == 0 (mod r) for phi's
   eigenvalue lambda.  Such (a0, a1) form a lattice of determinant r whose shortest vectors have
   max(|a0|, |a1|) ~ 2^127.5: evaluating alpha needs >= 126 doublings.  Scott's alpha = phi +
   [x^2] is such a shortest vector (norm exactly r) and costs two sparse |x|-chains: 126 doublings
   + 10 additions -- the bound.  With t1 shared, the test's own cost is one chain (~520 Fqm).
2. It is exact on E(Fp): ker(alpha) has order N(alpha) = r, so it is G1; in particular it rejects
   points with a component of every prime order dividing the cofactor h1 = 3 m^2,
   m = (|x| + 1) / 3 = 11 * 10177 * 859267 * 52437899 (checked on constructed torsion points).
3. A random linear combination of the shares' membership tests is NOT exact (why the test stays
   per share): a 3-torsion component survives a random combination with probability 1/3.
"""
import random

from oracle import bls12_381 as B

X, R, P = B.X, B.R, B.P
U = abs(X)
H1 = (X - 1) ** 2 // 3
M = (U + 1) // 3
PRIMES = [3, 11, 10177, 859267, 52437899]


def _lam():
    """phi(x, y) = (beta x, y) acts on G1 as [lambda]: the eigenvalue the decode's test uses,
    phi(P) = -[x^2] P, i.e. lambda = -x^2 mod r."""
    return (-X * X) % R


def _beta():
    # beta: the cube root of unity in Fq with phi = [-x^2] on G1 (pinned below on a point)
    for g in range(2, 50):
        b = pow(g, (P - 1) // 3, P)
        if b != 1:
            G = B.g1_mul(B.G1_GEN, 12345)
            for c in (b, b * b % P):
                if (c * G[0] % P, G[1]) == B.g1_mul(G, _lam()):
                    return c
    raise AssertionError("no beta")


def _phi(pt, beta):
    return None if pt is None else (beta * pt[0] % P, pt[1])


def _random_curve_point(rng):
    while True:
        x = rng.randrange(P)
        y2 = (x ** 3 + 4) % P
        if B.fq_is_square(y2):
            return (x, B.fq_sqrt(y2))


def _scott(pt, beta):
    """The decode's test: phi(P) == -[x^2] P (two |x|-chains)."""
    t1 = B.g1_mul(pt, U)
    t2 = B.g1_mul(t1, U)
    return _phi(pt, beta) == B.g1_neg(t2)


def test_cofactor_structure():
    assert H1 == 3 * M * M and M == 11 * 10177 * 859267 * 52437899
    assert (P - 1) % (U + 1) == 0  # the Tate-pairing route (Koshelev) needs mu_(|x|+1) in Fq
    assert P + 1 - (X + 1) == H1 * R  # #E(Fq) = p + 1 - t with trace t = x + 1: h1 r


def test_shortest_killing_vector_needs_126_doublings():
    """Gauss-reduce the lattice {(a0, a1): a0 + a1 lambda == 0 mod r}: its shortest vectors have
    coefficients of 127-128 bits, so alpha = a0 + a1 phi costs >= 126 doublings; Scott's (x^2, 1)
    is one of them (norm a0^2 - a0 a1 + a1^2 = r exactly)."""
    lam = _lam()
    # Lagrange-Gauss reduction in the Euclidean norm
    u, v = (R, 0), ((-lam) % R, 1)
    dot = lambda a, b: a[0] * b[0] + a[1] * b[1]
    if dot(u, u) < dot(v, v):
        u, v = v, u
    while dot(v, v) < dot(u, u):
        q = round(dot(u, v) / dot(v, v)) if dot(v, v) else 0
        u = (u[0] - q * v[0], u[1] - q * v[1])
        u, v = v, u
    short = min((u, v), key=lambda w: max(abs(w[0]), abs(w[1])))
    for w in (u, v):
        assert (w[0] + w[1] * lam) % R == 0
    assert max(abs(short[0]), abs(short[1])).bit_length() >= 127
    # every killing vector has norm >= r (r | N(alpha), N > 0): here the reduced basis' norms
    norm = lambda w: w[0] * w[0] - w[0] * w[1] + w[1] * w[1]
    assert all(norm(w) % R == 0 and norm(w) >= R for w in (u, v))
    # Scott's vector: (x^2, 1), norm x^4 - x^2 + 1 = r
    assert (X * X + lam) % R == 0 and norm((X * X, 1)) == R
    # ... evaluated as two |x| chains: popcount(|x|) = 6 -> 2 x 63 doublings + 2 x 5 additions
    assert bin(U).count("1") == 6 and U.bit_length() == 64


def test_scott_test_is_exact_on_every_cofactor_prime():
    rng = random.Random(2024)
    beta = _beta()
    for _ in range(3):
        g = B.g1_mul(B.G1_GEN, rng.randrange(1, R))
        assert _scott(g, beta)
    # points with a component of order l for every prime l | h1: [h1 r / l^e] Q (l^e || h1) for a
    # random Q on E(Fq) lies in the l-part, then scaled down to order l; added to a G1 point it
    # must fail the test
    for l in PRIMES:
        e = 0
        while H1 % l ** (e + 1) == 0:
            e += 1
        for _ in range(8):
            T = B.g1_mul(_random_curve_point(rng), H1 * R // l ** e)
            while T is not None and B.g1_mul(T, l) is not None:
                T = B.g1_mul(T, l)
            if T is not None:
                break
        assert T is not None and B.g1_mul(T, l) is None
        g = B.g1_mul(B.G1_GEN, rng.randrange(1, R))
        assert not _scott(B.g1_add(g, T), beta), l
        assert not B.g1_in_subgroup(B.g1_add(g, T))


def test_random_combination_of_tests_is_not_exact():
    """Why the test cannot be batched exactly: alpha(P) = phi(P) + [x^2] P lands in the cofactor
    group, and a random combination sum r_i alpha(P_i) misses a 3-torsion component whenever its
    coefficient is divisible by 3 (probability 1/3)."""
    rng = random.Random(7)
    beta = _beta()
    for _ in range(8):
        T = B.g1_mul(_random_curve_point(rng), H1 * R // 3)  # 3 || h1
        if T is not None:
            break
    assert T is not None and B.g1_mul(T, 3) is None
    bad = B.g1_add(B.g1_mul(B.G1_GEN, 5), T)
    alpha = B.g1_add(_phi(bad, beta), B.g1_mul(B.g1_mul(bad, U), U))  # phi(P) + [x^2] P
    assert alpha is not None  # the per-share test rejects it
    assert B.g1_mul(alpha, 3) is None  # ... but [3 k] alpha = O: a combination coefficient 3k hides it
