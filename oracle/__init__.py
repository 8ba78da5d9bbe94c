"""CPU oracle for the hbbft threshold-crypto hot path — TEST INFRASTRUCTURE ONLY.

This package is a restatement of the arithmetic that hbbft delegates to
``threshold_crypto @ 0.1.0-rng-fix`` and ``pairing 0.14.2`` (neither is vendored
under /root/reference).  It exists only to *check* the product
(``hbbft_amd`` + its HIP library).  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it; the product path never does.

Parity status (also recorded in DESIGN.md):
  * pinned by public known-answer values of the BLS12-381 / zcash-serialization
    specification (compressed generators, group orders, cofactor constant that
    pairing 0.14 hard-codes) and by algebraic identities (bilinearity, r-torsion);
  * accept/reject decisions and combined points are mathematically determined, so
    they match threshold_crypto for any correct implementation;
  * ``hash_g2`` / ``hash_bytes`` byte streams depend on rand-0.4 ChaCha details that
    cannot be checked here (no Rust toolchain, no vendored crate): **parity unpinned**
    for those two byte streams.

Modules:
  bls12_381         Fq/Fq2/Fq12, G1/G2, optimal-ate pairing, zcash codec   (pairing 0.14.2)
  rand04            rand 0.4.2 ChaChaRng + Rand impls used by hash_g2     (rand 0.4.2)
  threshold_crypto  hash_g2, hash_g1_g2, hash_bytes, verify*, interpolate,
                    parity, Poly/Commitment/BivarCommitment              (threshold_crypto 0.1.0-rng-fix)
  hbbft_rules       Coin / ThresholdDecryption / SyncKeyGen decision rules (hbbft src/*.rs)
  c/                the same restated in plain C (fast oracle + CPU baseline)
"""
