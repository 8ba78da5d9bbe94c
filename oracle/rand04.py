"""rand 0.4.2 ``ChaChaRng`` and the ``Rand`` impls that threshold_crypto's hashes use —
TEST ORACLE ONLY.

The crate (``rand = "0.4.2"``, /root/reference/Cargo.toml:28) is not vendored; this is
a restatement of its published behaviour [EXT-UNVERIFIED]:

  * ``ChaChaRng::from_seed(&[u32])``: state = "expand 32-byte k" constants, key words
    from the seed (missing words zero), 128-bit block counter in words 12..15 starting
    at 0; 20 rounds; ``next_u32`` returns the output block words in order 0..15 and
    refills (counter += 1) when exhausted.
  * ``Rng::next_u64`` default: ``(next_u32() << 32) | next_u32()`` — the FIRST word is the
    HIGH half (``U64_HIGH_FIRST``; rand >= 0.5 reversed this).  This ordering, and thus
    the exact bytes of hash_g2 / hash_bytes, is **parity unpinned** here.
  * ``u8::rand`` = ``next_u32() as u8``; ``bool::rand`` = ``u8::rand & 1 == 1``;
    ``[u64; 6]::rand`` fills limbs 0..5 in order.
"""

U64_HIGH_FIRST = True

_MASK = 0xFFFFFFFF


def _rotl(v, c):
    return ((v << c) & _MASK) | (v >> (32 - c))


def _quarter(s, a, b, c, d):
    s[a] = (s[a] + s[b]) & _MASK
    s[d] = _rotl(s[d] ^ s[a], 16)
    s[c] = (s[c] + s[d]) & _MASK
    s[b] = _rotl(s[b] ^ s[c], 12)
    s[a] = (s[a] + s[b]) & _MASK
    s[d] = _rotl(s[d] ^ s[a], 8)
    s[c] = (s[c] + s[d]) & _MASK
    s[b] = _rotl(s[b] ^ s[c], 7)


def chacha20_block(state):
    s = list(state)
    for _ in range(10):
        _quarter(s, 0, 4, 8, 12)
        _quarter(s, 1, 5, 9, 13)
        _quarter(s, 2, 6, 10, 14)
        _quarter(s, 3, 7, 11, 15)
        _quarter(s, 0, 5, 10, 15)
        _quarter(s, 1, 6, 11, 12)
        _quarter(s, 2, 7, 8, 13)
        _quarter(s, 3, 4, 9, 14)
    return [(s[i] + state[i]) & _MASK for i in range(16)]


class ChaChaRng:
    def __init__(self, seed_words):
        st = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574] + [0] * 12
        for i, w in enumerate(list(seed_words)[:8]):
            st[4 + i] = w & _MASK
        self.state = st
        self.buf = None
        self.index = 16

    def _update(self):
        self.buf = chacha20_block(self.state)
        self.index = 0
        for i in range(12, 16):  # 128-bit counter
            self.state[i] = (self.state[i] + 1) & _MASK
            if self.state[i] != 0:
                break

    def next_u32(self):
        if self.index == 16:
            self._update()
        v = self.buf[self.index]
        self.index += 1
        return v

    def next_u64(self):
        a = self.next_u32()
        b = self.next_u32()
        return (a << 32) | b if U64_HIGH_FIRST else (b << 32) | a

    def gen_u8(self):
        return self.next_u32() & 0xFF

    def gen_bool(self):
        return (self.gen_u8() & 1) == 1
