"""ctypes binding of the hbtc C ABI (include/hbtc.h) — the product's only compute path.

The library is ``hbbft_amd/libhbtc.so``, built in-tree by ``make lib`` (hipcc, gfx950).  If it is
missing or fails to load, every entry point raises ``NativeUnavailable``: there is no CPU
fallback, by design (the oracle under ``oracle/`` is test infrastructure only).
"""
import ctypes
import os

import numpy as np

# HBTC_LIB_PATH selects another build of the same library (kernel-variant experiments)
LIB_PATH = os.environ.get("HBTC_LIB_PATH") or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "libhbtc.so")

# ---- status codes (include/hbtc.h) ------------------------------------------------------------
ACCEPT = 0
REJECT = 1
DECODE_ERR = 2
UNKNOWN_SENDER = 3
INSTANCE_ERR = 4
NOT_ENOUGH_SHARES = 5
DUPLICATE_ENTRY = 6
MODE_PER_SHARE = 0
MODE_RLC = 1
CHECK_AUTO, CHECK_PLAIN_FIRST, CHECK_PAIR_SUBS, CHECK_PAIR_LEAVES = -1, 0, 1, 2
STATUS_NAMES = {ACCEPT: "ACCEPT", REJECT: "REJECT", DECODE_ERR: "DECODE_ERR",
                UNKNOWN_SENDER: "UNKNOWN_SENDER", INSTANCE_ERR: "INSTANCE_ERR",
                NOT_ENOUGH_SHARES: "NOT_ENOUGH_SHARES", DUPLICATE_ENTRY: "DUPLICATE_ENTRY"}


class NativeUnavailable(RuntimeError):
    """libhbtc.so is not built or cannot be loaded (no fallback exists)."""


class HbtcError(RuntimeError):
    pass


_P = ctypes.c_void_p
_U32 = ctypes.c_uint32
_I32 = ctypes.c_int
_SZ = ctypes.c_size_t

# name -> (restype, argtypes); every symbol declared in include/hbtc.h
SIGNATURES = {
    "hbtc_device_count": (_I32, []),
    "hbtc_version": (ctypes.c_char_p, []),
    "hbtc_ctx_create": (_I32, [_I32, ctypes.POINTER(_P)]),
    "hbtc_ctx_destroy": (None, [_P]),
    "hbtc_last_error": (ctypes.c_char_p, [_P]),
    "hbtc_keyset_load": (_I32, [_P, _P, _U32, ctypes.POINTER(_U32), ctypes.POINTER(_U32)]),
    "hbtc_keyset_free": (_I32, [_P, _U32]),
    "hbtc_verify_sig_shares": (_I32, [_P, _U32, _U32, _P, _P, _P, _P, _P]),
    "hbtc_keyset_set_master": (_I32, [_P, _U32, _P]),
    "hbtc_prepare_g2": (_I32, [_P, _U32, _P, _P]),
    "hbtc_unprepare_g2": (_I32, [_P, _U32, _P]),
    "hbtc_prepared_g2_count": (_I32, [_P, _P]),
    "hbtc_coin_decide": (_I32, [_P, _U32, _U32, _P, _P, _P, _P, _U32, _P, _P, _P, _P]),
    "hbtc_verify_sigs": (_I32, [_P, _U32, _P, _P, _P, _P]),
    "hbtc_combine_sigs": (_I32, [_P, _U32, _P, _P, _P, _U32, _P, _P, _P]),
    "hbtc_verify_dec_shares": (_I32, [_P, _U32, _U32, _P, _P, _P, _P, _P, _P]),
    "hbtc_combine_dec": (_I32, [_P, _U32, _P, _P, _P, _U32, _P, _P]),
    "hbtc_verify_ciphertexts": (_I32, [_P, _U32, _P, _P, _P, _P]),
    "hbtc_g1_mul": (_I32, [_P, _U32, _P, _U32, _P, _P, _P]),
    "hbtc_g2_mul": (_I32, [_P, _U32, _P, _U32, _P, _P, _P]),
    "hbtc_dev_alloc": (_I32, [_P, _SZ, ctypes.POINTER(_P)]),
    "hbtc_dev_free": (_I32, [_P, _P]),
    "hbtc_dev_upload": (_I32, [_P, _P, _P, _SZ]),
    "hbtc_dev_download": (_I32, [_P, _P, _P, _SZ]),
    "hbtc_sync": (_I32, [_P]),
    "hbtc_verify_dec_shares_dev": (_I32, [_P, _U32, _U32, _P, _P, _P, _P, _P, _P]),
    "hbtc_verify_sig_shares_dev": (_I32, [_P, _U32, _U32, _P, _P, _P, _P, _P]),
    "hbtc_combine_dec_dev": (_I32, [_P, _U32, _P, _P, _P, _U32, _P, _P]),
    "hbtc_combine_sigs_dev": (_I32, [_P, _U32, _P, _P, _P, _U32, _P, _P, _P]),
    "hbtc_combine_dec_verified_dev": (_I32, [_P, _U32, _P, _P, _P, _P, _U32, _P, _P]),
    "hbtc_combine_sigs_verified_dev": (_I32, [_P, _U32, _P, _P, _P, _P, _U32, _P, _P, _P]),
    "hbtc_g1_msm": (_I32, [_P, _U32, _U32, _P, _P, _P, _P]),
    "hbtc_g2_msm": (_I32, [_P, _U32, _U32, _P, _P, _P, _P]),
    "hbtc_skg_check_parts": (_I32, [_P, _U32, _U32, _U32, _P, _P, _P]),
    "hbtc_skg_check_acks": (_I32, [_P, _U32, _U32, _U32, _P, _P, _P, _U32, _P, _P, _P, _P]),
    "hbtc_set_verify_mode": (_I32, [_P, _I32]),
    "hbtc_set_rlc_bits": (_I32, [_P, _U32]),
    "hbtc_get_rlc_bits": (_I32, [_P, ctypes.POINTER(_U32)]),
    "hbtc_set_exact_below": (_I32, [_P, _U32]),
    "hbtc_trim_workspace": (_I32, [_P]),
    "hbtc_check_schedule_for": (_I32, [_P, _U32, ctypes.POINTER(_I32)]),
    "hbtc_sha3_256": (_I32, [_P, _SZ, _P]),
    "hbtc_hash_g2": (_I32, [_P, _SZ, _P]),
    "hbtc_hash_g1_g2": (_I32, [_P, _P, _SZ, _P]),
    "hbtc_hash_g2_batch": (_I32, [_U32, _P, _P, _P]),
    "hbtc_hash_g1_g2_batch": (_I32, [_U32, _P, _P, _P, _P]),
    "hbtc_hash_g2_batch_gpu": (_I32, [_P, _U32, _P, _P, _P]),
    "hbtc_hash_g1_g2_batch_gpu": (_I32, [_P, _U32, _P, _P, _P, _P]),
    "hbtc_chacha04_words": (_I32, [_P, _U32, _P]),
    "hbtc_chacha04_words_gpu": (_I32, [_P, _P, _U32, _P]),
    "hbtc_rlc_last_leaves": (_I32, [_P, ctypes.POINTER(_U32)]),
    "hbtc_timing_enable": (_I32, [_P, _I32]),
    "hbtc_timing_read": (_I32, [_P, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double),
                                ctypes.POINTER(ctypes.c_uint64)]),
    "hbtc_timing_reset": (_I32, [_P]),
    "hbtc_set_sender_tracking": (_I32, [_P, _I32]),
    "hbtc_set_check_schedule": (_I32, [_P, _I32]),
    "hbtc_rs_encode": (_I32, [_P, _U32, _U32, _U32, _U32, _P]),
    "hbtc_rs_reconstruct": (_I32, [_P, _U32, _U32, _U32, _U32, _P, _P, _P]),
    "hbtc_merkle_digest_count": (_U32, [_U32]),
    "hbtc_merkle_trees": (_I32, [_P, _U32, _U32, _U32, _P, _P]),
    "hbtc_merkle_validate": (_I32, [_P, _U32, _U32, _P, _P, _P, _P, _P, _P, _P]),
    "hbtc_rs_encode_dev": (_I32, [_P, _U32, _U32, _U32, _U32, _P]),
    "hbtc_rs_reconstruct_dev": (_I32, [_P, _U32, _U32, _U32, _U32, _P, _P, _P]),
    "hbtc_merkle_trees_dev": (_I32, [_P, _U32, _U32, _U32, _P, _P]),
    "hbtc_merkle_validate_dev": (_I32, [_P, _U32, _U32, _P, _P, _P, _P, _P, _P, _P]),
    "hbtc_hash_bytes": (_I32, [_P, _SZ, _P]),
    "hbtc_xor_hash_bytes_batch": (_I32, [_U32, _P, _P, _P, _P]),
    "hbtc_commitment_evaluate": (_I32, [_P, _U32, _P, _U32, _P, _P, _P]),
    "hbtc_decrypt": (_I32, [_P, _U32, _P, _P, _P, _P, _P, _P, _P]),
    "hbtc_unframe_points_dev": (_I32, [_P, _U32, _U32, _P, _P]),
    "hbtc_stream_wait_ctx": (_I32, [_P, _P]),
    "hbtc_ctx_wait_stream": (_I32, [_P, _P]),
    "hbtc_shard_items": (_I32, [_U32, _U32, _U32, _P, ctypes.POINTER(_U32), ctypes.POINTER(_U32),
                                ctypes.POINTER(_U32), _P, _P]),
    "hbtc_shard_instances": (_I32, [_U32, _U32, _P, _P]),
    "hbtc_node_create": (_I32, [_I32, _P, ctypes.POINTER(_P)]),
    "hbtc_node_destroy": (None, [_P]),
    "hbtc_node_last_error": (ctypes.c_char_p, [_P]),
    "hbtc_node_devices": (_I32, [_P]),
    "hbtc_node_context": (_P, [_P, _I32]),
    "hbtc_node_set_verify_mode": (_I32, [_P, _I32]),
    "hbtc_node_set_rlc_bits": (_I32, [_P, _U32]),
    "hbtc_node_keyset_load": (_I32, [_P, _P, _U32, ctypes.POINTER(_U32), ctypes.POINTER(_U32)]),
    "hbtc_node_keyset_free": (_I32, [_P, _U32]),
    "hbtc_node_verify_dec_shares": (_I32, [_P, _U32, _U32, _P, _P, _P, _P, _P, _P]),
    "hbtc_node_verify_sig_shares": (_I32, [_P, _U32, _U32, _P, _P, _P, _P, _P]),
    "hbtc_node_combine_dec": (_I32, [_P, _U32, _P, _P, _P, _U32, _P, _P]),
    "hbtc_node_combine_sigs": (_I32, [_P, _U32, _P, _P, _P, _U32, _P, _P, _P]),
    "hbtc_dec_epoch_submit": (_I32, [_P, _U32, _U32, _P, _P, _P, _P, _P, _U32, _P, _P, _P,
                                     ctypes.POINTER(ctypes.c_uint64)]),
    "hbtc_sig_epoch_submit": (_I32, [_P, _U32, _U32, _P, _P, _P, _P, _U32, _P, _P, _P, _P,
                                     ctypes.POINTER(ctypes.c_uint64)]),
    "hbtc_wait": (_I32, [_P, ctypes.c_uint64]),
    "hbtc_node_verify_sig_shares_dev": (_I32, [_P, _U32, _P]),
    "hbtc_node_verify_dec_shares_dev": (_I32, [_P, _U32, _P]),
    "hbtc_node_combine_sigs_verified_dev": (_I32, [_P, _P, _U32]),
    "hbtc_node_combine_dec_verified_dev": (_I32, [_P, _P, _U32]),
    "hbtc_node_sync": (_I32, [_P]),
}


class NodePart(ctypes.Structure):
    """include/hbtc.h hbtc_node_part: one device's part of a device-resident node batch."""
    _fields_ = [("n_inst", _U32), ("offsets", _P), ("d_H_c96", _P), ("d_w_c96", _P),
                ("d_idx", _P), ("d_items", _P), ("d_status", _P), ("d_out", _P),
                ("d_out_parity", _P), ("d_inst_status", _P)]

_lib = None


def load():
    """Load libhbtc.so once; raise NativeUnavailable when it is absent or broken."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeUnavailable("%s is not built: run `make -j8 lib` (hipcc --offload-arch=gfx950)"
                                % LIB_PATH)
    try:
        lib = ctypes.CDLL(LIB_PATH)
    except OSError as e:
        raise NativeUnavailable("cannot load %s: %s" % (LIB_PATH, e))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def device_count():
    return load().hbtc_device_count()


def sha3_256(msg):
    """SHA3-256 through the library (host code; no context or GPU needed)."""
    m = bytes(msg)
    out = ctypes.create_string_buffer(32)
    if load().hbtc_sha3_256(m, len(m), out) != 0:
        raise HbtcError("hbtc_sha3_256 failed")
    return out.raw


def chacha04_words(seed, n):
    """The first n words of rand 0.4's ChaChaRng::from_seed(seed) (8 u32 seed words) from the
    host hashes' ChaCha code (no GPU): the ChaCha20 known-answer tests' entry point."""
    s = np.ascontiguousarray(np.asarray(seed, dtype=np.uint32))
    if s.shape != (8,):
        raise ValueError("seed must be 8 u32 words")
    out = np.zeros(n, np.uint32)
    if load().hbtc_chacha04_words(_ptr(s), n, _ptr(out)) != 0:
        raise HbtcError("hbtc_chacha04_words failed")
    return out


def hash_g2(msg):
    """threshold_crypto's hash_g2(msg) as compressed G2 bytes (host code, no GPU)."""
    m = bytes(msg)
    out = ctypes.create_string_buffer(96)
    if load().hbtc_hash_g2(m, len(m), out) != 0:
        raise HbtcError("hbtc_hash_g2 failed")
    return out.raw


def hash_g1_g2(g1_c48, msg):
    """threshold_crypto's hash_g1_g2(g1, msg) as compressed G2 bytes (host code, no GPU)."""
    g, m = bytes(g1_c48), bytes(msg)
    if len(g) != 48:
        raise ValueError("g1 must be 48 compressed bytes")
    out = ctypes.create_string_buffer(96)
    if load().hbtc_hash_g1_g2(g, m, len(m), out) != 0:
        raise HbtcError("hbtc_hash_g1_g2 failed")
    return out.raw


def hash_bytes(g1_c48, length):
    """threshold_crypto's hash_bytes(g, len): the encrypt / decrypt XOR pad (host code)."""
    g = bytes(g1_c48)
    if len(g) != 48:
        raise ValueError("g1 must be 48 compressed bytes")
    out = ctypes.create_string_buffer(max(1, length))
    if load().hbtc_hash_bytes(g, length, out) != 0:
        raise HbtcError("hbtc_hash_bytes failed")
    return out.raw[:length]


def xor_hash_bytes_batch(gs, msgs):
    """msgs[i] XOR hash_bytes(gs[i], |msgs[i]|) for every i, over the host's cores."""
    buf, off = _msg_batch(msgs)
    n = off.size - 1
    g = _join(gs, 48)
    if g.size != 48 * n:
        raise ValueError("one 48-byte g per message")
    out = np.zeros(max(1, int(off[-1])), np.uint8)
    if load().hbtc_xor_hash_bytes_batch(n, _ptr(g), _ptr(buf), _ptr(off), _ptr(out)) != 0:
        raise HbtcError("hbtc_xor_hash_bytes_batch failed")
    return [bytes(out[off[i]:off[i + 1]]) for i in range(n)]


def _msg_batch(msgs):
    ms = [bytes(m) for m in msgs]
    off = np.zeros(len(ms) + 1, np.uint32)
    off[1:] = np.cumsum([len(m) for m in ms])
    buf = np.frombuffer(b"".join(ms) or b"\0", np.uint8).copy()
    return buf, off


def hash_g2_batch(msgs):
    """hash_g2 of every message, over the host's cores; returns a list of 96-byte encodings."""
    buf, off = _msg_batch(msgs)
    n = off.size - 1
    out = np.zeros(96 * max(n, 1), np.uint8)
    if load().hbtc_hash_g2_batch(n, _ptr(buf), _ptr(off), _ptr(out)) != 0:
        raise HbtcError("hbtc_hash_g2_batch failed")
    return [bytes(out[96 * i:96 * i + 96]) for i in range(n)]


def hash_g1_g2_batch(us, msgs):
    """hash_g1_g2(u_i, v_i) for every ciphertext, over the host's cores."""
    buf, off = _msg_batch(msgs)
    n = off.size - 1
    u = _join(us, 48)
    if u.size != 48 * n:
        raise ValueError("one 48-byte u per message")
    out = np.zeros(96 * max(n, 1), np.uint8)
    if load().hbtc_hash_g1_g2_batch(n, _ptr(u), _ptr(buf), _ptr(off), _ptr(out)) != 0:
        raise HbtcError("hbtc_hash_g1_g2_batch failed")
    return [bytes(out[96 * i:96 * i + 96]) for i in range(n)]


def _u8(buf, item_bytes=None):
    a = np.frombuffer(bytes(buf), dtype=np.uint8) if isinstance(buf, (bytes, bytearray)) else \
        np.ascontiguousarray(buf, dtype=np.uint8).reshape(-1)
    if item_bytes is not None and a.size % item_bytes:
        raise ValueError("buffer length %d is not a multiple of %d" % (a.size, item_bytes))
    return np.ascontiguousarray(a)


def _join(items, size):
    """list of byte strings (or one packed buffer) -> contiguous uint8 array."""
    if isinstance(items, (list, tuple)):
        for it in items:
            if len(it) != size:
                raise ValueError("expected %d-byte items" % size)
        return np.frombuffer(b"".join(bytes(i) for i in items), dtype=np.uint8).copy() \
            if items else np.zeros(0, np.uint8)
    return _u8(items, size)


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None and a.size else ctypes.c_void_p(0)


def _offsets(counts_or_offsets, is_offsets):
    if is_offsets:
        off = np.ascontiguousarray(counts_or_offsets, dtype=np.uint32)
    else:
        c = np.asarray(counts_or_offsets, dtype=np.uint64).reshape(-1)
        off = np.zeros(c.size + 1, dtype=np.uint32)
        off[1:] = np.cumsum(c)
    return off


class Context:
    """One hbtc context (one GPU).  Methods take host data (bytes / numpy) and return numpy."""

    @classmethod
    def borrowed(cls, handle, device):
        """A non-owning view of a context created elsewhere (a node's device slot)."""
        c = cls.__new__(cls)
        c.lib = load()
        c.h = ctypes.c_void_p(handle)
        c.device = device
        c._borrowed = True
        return c

    def __init__(self, device=0):
        self.lib = load()
        h = ctypes.c_void_p()
        rc = self.lib.hbtc_ctx_create(int(device), ctypes.byref(h))
        if rc != 0:
            raise HbtcError("hbtc_ctx_create(device=%d) failed: %d" % (device, rc))
        self.h = h
        self.device = device

    def close(self):
        if getattr(self, "h", None):
            if not getattr(self, "_borrowed", False):
                self.lib.hbtc_ctx_destroy(self.h)  # completes in-flight tickets into their outputs
            self.h = None
            self._inflight.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            msg = self.lib.hbtc_last_error(self.h)
            raise HbtcError("%s failed (%d): %s" % (what, rc, msg.decode() if msg else ""))

    # ---- hashes (cofactor clearing on this context's GPU)
    def hash_g2_batch(self, msgs):
        buf, off = _msg_batch(msgs)
        n = off.size - 1
        out = np.zeros(96 * max(n, 1), np.uint8)
        self._check(self.lib.hbtc_hash_g2_batch_gpu(self.h, n, _ptr(buf), _ptr(off), _ptr(out)),
                    "hbtc_hash_g2_batch_gpu")
        return [bytes(out[96 * i:96 * i + 96]) for i in range(n)]

    def hash_g1_g2_batch(self, us, msgs):
        buf, off = _msg_batch(msgs)
        n = off.size - 1
        u = _join(us, 48)
        if u.size != 48 * n:
            raise ValueError("one 48-byte u per message")
        out = np.zeros(96 * max(n, 1), np.uint8)
        self._check(self.lib.hbtc_hash_g1_g2_batch_gpu(self.h, n, _ptr(u), _ptr(buf), _ptr(off),
                                                       _ptr(out)), "hbtc_hash_g1_g2_batch_gpu")
        return [bytes(out[96 * i:96 * i + 96]) for i in range(n)]

    def chacha04_words(self, seed, n):
        """chacha04_words on this context's GPU (the ChaCha code of k_hash_cand)."""
        s = np.ascontiguousarray(np.asarray(seed, dtype=np.uint32))
        if s.shape != (8,):
            raise ValueError("seed must be 8 u32 words")
        out = np.zeros(max(n, 1), np.uint32)
        self._check(self.lib.hbtc_chacha04_words_gpu(self.h, _ptr(s), n, _ptr(out)),
                    "hbtc_chacha04_words_gpu")
        return out[:n]

    # ---- key sets
    def keyset_load(self, pk_shares):
        pk = _join(pk_shares, 48)
        n = pk.size // 48
        kid, bad = _U32(), _U32()
        self._check(self.lib.hbtc_keyset_load(self.h, _ptr(pk), n, ctypes.byref(kid),
                                              ctypes.byref(bad)), "hbtc_keyset_load")
        return kid.value, bad.value

    def keyset_free(self, kid):
        self._check(self.lib.hbtc_keyset_free(self.h, kid), "hbtc_keyset_free")

    def keyset_set_master(self, kid, master_pk):
        mp = _join([master_pk], 48)
        self._check(self.lib.hbtc_keyset_set_master(self.h, kid, _ptr(mp)), "hbtc_keyset_set_master")

    def prepare_g2(self, points):
        """hbtc.h hbtc_prepare_g2: the G2 tables of these compressed points (a coin's H, a
        ciphertext's H and w) built ahead of the shares; per-point ACCEPT / DECODE_ERR."""
        pb = _join(points, 96)
        st = np.zeros(max(len(points), 1), np.int32)
        self._check(self.lib.hbtc_prepare_g2(self.h, len(points), _ptr(pb), _ptr(st)), "hbtc_prepare_g2")
        return st[:len(points)]

    def unprepare_g2(self, points):
        pb = _join(points, 96)
        self._check(self.lib.hbtc_unprepare_g2(self.h, len(points), _ptr(pb)), "hbtc_unprepare_g2")

    def prepared_g2_count(self):
        n = np.zeros(1, np.uint32)
        self._check(self.lib.hbtc_prepared_g2_count(self.h, _ptr(n)), "hbtc_prepared_g2_count")
        return int(n[0])

    # ---- verification
    def coin_decide(self, keyset, H, counts, idx, sigs, t, offsets=None):
        """One Threshold Coin round (hbtc.h hbtc_coin_decide): item statuses, combined signatures,
        parity bits and coin statuses (ACCEPT = the combined signature passed the master check)."""
        off = _offsets(offsets if offsets is not None else counts, offsets is not None)
        n_inst = off.size - 1
        Hb, sb = _join(H, 96), _join(sigs, 96)
        ix = np.ascontiguousarray(idx, dtype=np.uint32)
        st = np.empty(max(int(off[-1]), 1), dtype=np.int32)
        sig = np.zeros(96 * max(n_inst, 1), np.uint8)
        par = np.zeros(max(n_inst, 1), np.uint8)
        cst = np.zeros(max(n_inst, 1), np.int32)
        self._check(self.lib.hbtc_coin_decide(self.h, keyset, n_inst, _ptr(Hb), _ptr(off), _ptr(ix),
                                              _ptr(sb), t, _ptr(st), _ptr(sig), _ptr(par), _ptr(cst)),
                    "hbtc_coin_decide")
        return (st[:int(off[-1])], [bytes(sig[96 * k:96 * k + 96]) for k in range(n_inst)],
                par[:n_inst], cst[:n_inst])

    def verify_sig_shares(self, keyset, H, counts, idx, sigs, offsets=None):
        off = _offsets(offsets if offsets is not None else counts, offsets is not None)
        n_inst = off.size - 1
        Hb, sb = _join(H, 96), _join(sigs, 96)
        ix = np.ascontiguousarray(idx, dtype=np.uint32)
        st = np.empty(int(off[-1]), dtype=np.int32)
        self._check(self.lib.hbtc_verify_sig_shares(self.h, keyset, n_inst, _ptr(Hb), _ptr(off),
                                                    _ptr(ix), _ptr(sb), _ptr(st)),
                    "hbtc_verify_sig_shares")
        return st

    def verify_dec_shares(self, keyset, H, w, counts, idx, shares, offsets=None):
        off = _offsets(offsets if offsets is not None else counts, offsets is not None)
        n_ct = off.size - 1
        Hb, wb, sb = _join(H, 96), _join(w, 96), _join(shares, 48)
        ix = np.ascontiguousarray(idx, dtype=np.uint32)
        st = np.empty(int(off[-1]), dtype=np.int32)
        self._check(self.lib.hbtc_verify_dec_shares(self.h, keyset, n_ct, _ptr(Hb), _ptr(wb),
                                                    _ptr(off), _ptr(ix), _ptr(sb), _ptr(st)),
                    "hbtc_verify_dec_shares")
        return st

    # ---- pipelined host-buffer epochs (hbtc_*_epoch_submit / hbtc_wait)
    class Pending:
        """A submitted epoch: its output arrays (filled by wait()) and the inputs kept alive.

        The C side writes into the output arrays when the ticket completes — at wait(), or
        unasked when a later submit reuses the ticket's lane, or at hbtc_ctx_destroy — so the
        Context, not this object, owns them until then (a dropped Pending cannot leave the
        library writing into freed memory)."""

        def __init__(self, ctx, ticket, outs, keep):
            self.ctx, self.ticket, self.outs, self._keep = ctx, ticket, outs, keep

        def wait(self):
            self.ctx._check(self.ctx.lib.hbtc_wait(self.ctx.h, self.ticket), "hbtc_wait")
            self.ctx._inflight.pop(self.ticket, None)
            return self.outs

    # tickets whose buffers the Context holds before it completes the oldest itself
    MAX_HELD_TICKETS = 16

    def _hold(self, ticket, outs, keep):
        held = self._inflight
        held[ticket] = (outs, keep)
        while len(held) > self.MAX_HELD_TICKETS:  # complete (normally long finished) old epochs
            old = min(held)
            self._check(self.lib.hbtc_wait(self.h, old), "hbtc_wait")
            held.pop(old, None)
        return Context.Pending(self, ticket, outs, keep)

    @property
    def _inflight(self):
        return self.__dict__.setdefault("_inflight_d", {})

    def dec_epoch_submit(self, keyset, H, w, offsets, idx, shares, t, outs=None):
        """Submit one epoch of DecryptionShares (verification + combine of the first t verified
        shares per ciphertext, t = 0: verification only); returns a Pending whose wait() gives
        (status, g [n_ct, 48], combine status).  `outs` reuses output arrays."""
        off = np.ascontiguousarray(offsets, dtype=np.uint32)
        n_ct, n = off.size - 1, int(off[-1])
        Hb, wb, sb = _join(H, 96), _join(w, 96), _join(shares, 48)
        ix = np.ascontiguousarray(idx, dtype=np.uint32)
        if outs is None:
            outs = (np.empty(max(n, 1), np.int32), np.empty((max(n_ct, 1), 48), np.uint8),
                    np.empty(max(n_ct, 1), np.int32))
        tk = ctypes.c_uint64()
        self._check(self.lib.hbtc_dec_epoch_submit(self.h, keyset, n_ct, _ptr(Hb), _ptr(wb), _ptr(off), _ptr(ix),
                                                   _ptr(sb), t, _ptr(outs[0]), _ptr(outs[1]), _ptr(outs[2]),
                                                   ctypes.byref(tk)), "hbtc_dec_epoch_submit")
        return self._hold(tk.value, outs, (off,))

    def sig_epoch_submit(self, keyset, H, offsets, idx, sigs, t, outs=None):
        """The SignatureShare epoch (coins): wait() gives (status, sig [n, 96], parity, combine status)."""
        off = np.ascontiguousarray(offsets, dtype=np.uint32)
        n_inst, n = off.size - 1, int(off[-1])
        Hb, sb = _join(H, 96), _join(sigs, 96)
        ix = np.ascontiguousarray(idx, dtype=np.uint32)
        if outs is None:
            outs = (np.empty(max(n, 1), np.int32), np.empty((max(n_inst, 1), 96), np.uint8),
                    np.empty(max(n_inst, 1), np.uint8), np.empty(max(n_inst, 1), np.int32))
        tk = ctypes.c_uint64()
        self._check(self.lib.hbtc_sig_epoch_submit(self.h, keyset, n_inst, _ptr(Hb), _ptr(off), _ptr(ix), _ptr(sb),
                                                   t, _ptr(outs[0]), _ptr(outs[1]), _ptr(outs[2]),
                                                   _ptr(outs[3]), ctypes.byref(tk)), "hbtc_sig_epoch_submit")
        return self._hold(tk.value, outs, (off,))

    def verify_sigs(self, pks, H, sigs):
        pk, Hb, sb = _join(pks, 48), _join(H, 96), _join(sigs, 96)
        n = pk.size // 48
        st = np.empty(n, dtype=np.int32)
        self._check(self.lib.hbtc_verify_sigs(self.h, n, _ptr(pk), _ptr(Hb), _ptr(sb), _ptr(st)),
                    "hbtc_verify_sigs")
        return st

    def verify_ciphertexts(self, us, H, ws):
        u, Hb, wb = _join(us, 48), _join(H, 96), _join(ws, 96)
        n = u.size // 48
        st = np.empty(n, dtype=np.int32)
        self._check(self.lib.hbtc_verify_ciphertexts(self.h, n, _ptr(u), _ptr(Hb), _ptr(wb),
                                                     _ptr(st)), "hbtc_verify_ciphertexts")
        return st

    # ---- combines
    def combine_sigs(self, counts, idx, sigs, t, offsets=None):
        off = _offsets(offsets if offsets is not None else counts, offsets is not None)
        n = off.size - 1
        ix = np.ascontiguousarray(idx, dtype=np.uint32)
        sb = _join(sigs, 96)
        out = np.zeros(96 * n, np.uint8)
        par = np.zeros(n, np.uint8)
        st = np.empty(n, np.int32)
        self._check(self.lib.hbtc_combine_sigs(self.h, n, _ptr(off), _ptr(ix), _ptr(sb), t,
                                               _ptr(out), _ptr(par), _ptr(st)), "hbtc_combine_sigs")
        return [bytes(out[96 * k:96 * k + 96]) for k in range(n)], par, st

    def combine_dec(self, counts, idx, shares, t, offsets=None):
        off = _offsets(offsets if offsets is not None else counts, offsets is not None)
        n = off.size - 1
        ix = np.ascontiguousarray(idx, dtype=np.uint32)
        sb = _join(shares, 48)
        out = np.zeros(48 * n, np.uint8)
        st = np.empty(n, np.int32)
        self._check(self.lib.hbtc_combine_dec(self.h, n, _ptr(off), _ptr(ix), _ptr(sb), t,
                                              _ptr(out), _ptr(st)), "hbtc_combine_dec")
        return [bytes(out[48 * k:48 * k + 48]) for k in range(n)], st

    # ---- scalar multiplication
    def _mul(self, fn, size, bases, scalars):
        sc = np.frombuffer(b"".join(int(k).to_bytes(32, "little") for k in scalars),
                           dtype=np.uint8).copy() if not isinstance(scalars, np.ndarray) else \
            np.ascontiguousarray(scalars, dtype=np.uint8).reshape(-1)
        n = sc.size // 32
        if isinstance(bases, (bytes, bytearray)) and len(bases) == size:
            b, stride = np.frombuffer(bytes(bases), dtype=np.uint8).copy(), 0
        else:
            b, stride = _join(bases, size), 1
        out = np.zeros(size * n, np.uint8)
        st = np.empty(n, np.int32)
        self._check(fn(self.h, n, _ptr(b), stride, _ptr(sc), _ptr(out), _ptr(st)), "point mul")
        return out, st

    def g1_mul(self, bases, scalars):
        """k_i * P_i (bases: one 48-byte point shared by all, or a list); returns (uint8[n*48], status)."""
        return self._mul(self.lib.hbtc_g1_mul, 48, bases, scalars)

    def g2_mul(self, bases, scalars):
        return self._mul(self.lib.hbtc_g2_mul, 96, bases, scalars)

    # ---- multi-scalar multiplication
    def _msm(self, fn, size, n_msm, n, points, scalars):
        pts = _join(points, size)
        sc = np.frombuffer(b"".join(int(k).to_bytes(32, "little") for k in scalars),
                           dtype=np.uint8).copy() if not isinstance(scalars, np.ndarray) else \
            np.ascontiguousarray(scalars, dtype=np.uint8).reshape(-1)
        if pts.size != size * n_msm * n or sc.size != 32 * n_msm * n:
            raise ValueError("expected %d points and scalars" % (n_msm * n))
        out = np.zeros(size * n_msm, np.uint8)
        st = np.empty(n_msm, np.int32)
        self._check(fn(self.h, n_msm, n, _ptr(pts), _ptr(sc), _ptr(out), _ptr(st)), "msm")
        return [bytes(out[size * m:size * m + size]) for m in range(n_msm)], st

    # ---- Reliable Broadcast coding (include/hbtc.h, src/broadcast/)
    def rs_encode(self, k, p, shard_len, shards):
        """ReedSolomon::encode of every instance, in place on the uint8 array `shards`
        (n_inst * (k + p) * shard_len bytes, parity rows overwritten); returns it."""
        a = np.ascontiguousarray(shards, dtype=np.uint8).reshape(-1)
        per = (k + p) * shard_len
        if per == 0 or a.size % per:
            raise ValueError("shards: a multiple of (k + p) * shard_len bytes")
        self._check(self.lib.hbtc_rs_encode(self.h, k, p, shard_len, a.size // per, _ptr(a)), "rs_encode")
        return a

    def rs_reconstruct(self, k, p, shard_len, shards, present):
        """ReedSolomon::reconstruct_shards per instance (present: n_inst * (k + p) flags); fills
        the missing shards in place; returns the per-instance status."""
        a = np.ascontiguousarray(shards, dtype=np.uint8).reshape(-1)
        pr = np.ascontiguousarray(present, dtype=np.uint8).reshape(-1)
        per = (k + p) * shard_len
        if per == 0 or a.size % per or pr.size != (a.size // per) * (k + p):
            raise ValueError("shards / present sizes")
        n_inst = a.size // per
        st = np.empty(n_inst, np.int32)
        self._check(self.lib.hbtc_rs_reconstruct(self.h, k, p, shard_len, n_inst, _ptr(a), _ptr(pr),
                                                 _ptr(st)), "rs_reconstruct")
        return a, st

    def merkle_trees(self, n_leaves, leaf_len, leaves):
        """MerkleTree::from_vec of every instance: uint8[n_inst, digest_count, 32] (level 0
        first, the root last)."""
        a = np.ascontiguousarray(leaves, dtype=np.uint8).reshape(-1)
        per = n_leaves * leaf_len
        if per == 0 or a.size % per:
            raise ValueError("leaves: a multiple of n_leaves * leaf_len bytes")
        n_inst = a.size // per
        nd = self.lib.hbtc_merkle_digest_count(n_leaves)
        out = np.zeros(n_inst * nd * 32, np.uint8)
        self._check(self.lib.hbtc_merkle_trees(self.h, n_leaves, leaf_len, n_inst, _ptr(a), _ptr(out)),
                    "merkle_trees")
        return out.reshape(n_inst, nd, 32)

    def merkle_validate(self, n_nodes, values, index, digests, roots):
        """Proof::validate(n_nodes) of each (values[i], index[i], digests[i] (list of 32-byte
        digests), roots[i]); returns the status array (ACCEPT = valid)."""
        n = len(values)
        voff = np.zeros(n + 1, np.uint64)
        voff[1:] = np.cumsum([len(v) for v in values]) if n else []
        vals = np.frombuffer(b"".join(bytes(v) for v in values) or b"\0", np.uint8).copy()
        doff = np.zeros(n + 1, np.uint32)
        doff[1:] = np.cumsum([len(d) for d in digests]) if n else []
        dig = np.frombuffer(b"".join(bytes(x) for d in digests for x in d) or bytes(32), np.uint8).copy()
        rts = np.frombuffer(b"".join(bytes(r) for r in roots) or bytes(32), np.uint8).copy()
        ix = np.ascontiguousarray(index, dtype=np.uint32)
        st = np.empty(max(n, 1), np.int32)
        self._check(self.lib.hbtc_merkle_validate(self.h, n, n_nodes, _ptr(voff), _ptr(vals), _ptr(ix),
                                                  _ptr(doff), _ptr(dig), _ptr(rts), _ptr(st)),
                    "merkle_validate")
        return st[:n]

    def g1_msm(self, n_msm, n, points, scalars):
        """n_msm MSMs of n terms (points/scalars item-major [m][i]); returns ([48 B], status)."""
        return self._msm(self.lib.hbtc_g1_msm, 48, n_msm, n, points, scalars)

    def g2_msm(self, n_msm, n, points, scalars):
        return self._msm(self.lib.hbtc_g2_msm, 96, n_msm, n, points, scalars)

    # ---- SyncKeyGen
    @staticmethod
    def _fr_bytes(vals):
        if isinstance(vals, np.ndarray):
            return np.ascontiguousarray(vals, dtype=np.uint8).reshape(-1)
        return np.frombuffer(b"".join(int(v).to_bytes(32, "little") for v in vals),
                             dtype=np.uint8).copy()

    def skg_check_parts(self, t, our_idx, commits, rows):
        """commits: per Part the (t+1)(t+2)/2 compressed G1 points (coeff_pos order, packed);
        rows: per Part t+1 Fr ints.  Returns the per-Part status array."""
        m = (t + 1) * (t + 2) // 2
        cm = _join(commits, 48)
        n_parts = cm.size // (48 * m)
        rb = self._fr_bytes([v for r in rows for v in r])
        if rb.size != 32 * n_parts * (t + 1):
            raise ValueError("expected %d row coefficients" % (n_parts * (t + 1)))
        st = np.empty(n_parts, np.int32)
        self._check(self.lib.hbtc_skg_check_parts(self.h, n_parts, t, our_idx, _ptr(cm), _ptr(rb),
                                                  _ptr(st)), "hbtc_skg_check_parts")
        return st

    def skg_check_acks(self, t, our_idx, commits, rows, row_ok, ack_part, ack_sender, vals):
        m = (t + 1) * (t + 2) // 2
        cm = _join(commits, 48)
        n_parts = cm.size // (48 * m)
        rb = self._fr_bytes([v for r in rows for v in r]) if rows is not None else None
        ok = np.ascontiguousarray(row_ok, dtype=np.uint8)
        ap = np.ascontiguousarray(ack_part, dtype=np.uint32)
        sd = np.ascontiguousarray(ack_sender, dtype=np.uint32)
        vb = self._fr_bytes(vals)
        st = np.empty(ap.size, np.int32)
        self._check(self.lib.hbtc_skg_check_acks(self.h, n_parts, t, our_idx, _ptr(cm), _ptr(rb),
                                                 _ptr(ok), ap.size, _ptr(ap), _ptr(sd), _ptr(vb),
                                                 _ptr(st)), "hbtc_skg_check_acks")
        return st

    # ---- SecretKey::decrypt
    def decrypt(self, sk, us, ws, vs):
        """[plaintext or None] and status for ciphertexts (u_i, v_i, w_i) under secret key sk."""
        buf, off = _msg_batch(vs)
        n = off.size - 1
        if n == 0:
            return [], np.zeros(0, np.int32)
        u, w = _join(us, 48), _join(ws, 96)
        out = np.zeros(max(1, int(off[-1])), np.uint8)
        st = np.zeros(n, np.int32)
        k = np.frombuffer(int(sk).to_bytes(32, "little"), np.uint8).copy()
        self._check(self.lib.hbtc_decrypt(self.h, n, _ptr(k), _ptr(u), _ptr(w), _ptr(buf), _ptr(off),
                                          _ptr(out), _ptr(st)), "hbtc_decrypt")
        return [bytes(out[off[i]:off[i + 1]]) if st[i] == ACCEPT else None for i in range(n)], st

    # ---- commitments
    def commitment_evaluate(self, commit, xs):
        """Commitment::evaluate(x) for every x in xs (compressed G1 coefficients)."""
        cm = _join(commit, 48)
        x = np.ascontiguousarray(xs, dtype=np.uint32)
        out = np.zeros(48 * max(1, x.size), np.uint8)
        st = np.zeros(max(1, x.size), np.int32)
        self._check(self.lib.hbtc_commitment_evaluate(self.h, cm.size // 48, _ptr(cm), x.size, _ptr(x),
                                                      _ptr(out), _ptr(st)), "hbtc_commitment_evaluate")
        return [bytes(out[48 * k:48 * k + 48]) for k in range(x.size)], st[:x.size]

    # ---- device memory (benchmarks)
    def dev_alloc(self, nbytes):
        p = ctypes.c_void_p()
        self._check(self.lib.hbtc_dev_alloc(self.h, nbytes, ctypes.byref(p)), "hbtc_dev_alloc")
        return p

    def dev_free(self, p):
        self._check(self.lib.hbtc_dev_free(self.h, p), "hbtc_dev_free")

    def dev_upload(self, p, arr):
        a = np.ascontiguousarray(arr)
        self._check(self.lib.hbtc_dev_upload(self.h, p, _ptr(a), a.nbytes), "hbtc_dev_upload")

    def dev_download(self, arr, p):
        self._check(self.lib.hbtc_dev_download(self.h, _ptr(arr), p, arr.nbytes), "hbtc_dev_download")

    def sync(self):
        self._check(self.lib.hbtc_sync(self.h), "hbtc_sync")

    def stream_wait_ctx(self, hip_stream):
        """Work enqueued later on `hip_stream` (a raw HIP stream handle, e.g.
        torch.cuda.Stream.cuda_stream) waits for everything already enqueued on this context."""
        self._check(self.lib.hbtc_stream_wait_ctx(self.h, ctypes.c_void_p(hip_stream)),
                    "hbtc_stream_wait_ctx")

    def ctx_wait_stream(self, hip_stream):
        """This context's later work waits for everything already enqueued on `hip_stream`."""
        self._check(self.lib.hbtc_ctx_wait_stream(self.h, ctypes.c_void_p(hip_stream)),
                    "hbtc_ctx_wait_stream")

    def set_verify_mode(self, mode):
        """MODE_RLC (default): batched random-linear-combination checks with exact fallback;
        MODE_PER_SHARE: one pairing check per share."""
        self._check(self.lib.hbtc_set_verify_mode(self.h, int(mode)), "hbtc_set_verify_mode")

    def set_rlc_bits(self, bits):
        """RLC scalar size: 128 (default, <= 2^-128 per group check) or 64 (<= 2^-64)."""
        self._check(self.lib.hbtc_set_rlc_bits(self.h, int(bits)), "hbtc_set_rlc_bits")

    def set_exact_below(self, n_items):
        """RLC share calls with fewer than n_items shares get exact cooperative checks of every
        share instead of the group sums (default 256; 0 = always batch)."""
        self._check(self.lib.hbtc_set_exact_below(self.h, int(n_items)), "hbtc_set_exact_below")

    def trim_workspace(self):
        """Free the context's cached device workspace (hbtc_trim_workspace)."""
        self._check(self.lib.hbtc_trim_workspace(self.h), "hbtc_trim_workspace")

    def rlc_bits(self):
        b = _U32()
        self._check(self.lib.hbtc_get_rlc_bits(self.h, ctypes.byref(b)), "hbtc_get_rlc_bits")
        return b.value

    def check_schedule_for(self, n_tiles):
        """The group-check schedule (CHECK_*) an RLC call of n_tiles 64-share tiles gets."""
        s = _I32()
        self._check(self.lib.hbtc_check_schedule_for(self.h, int(n_tiles), ctypes.byref(s)),
                    "hbtc_check_schedule_for")
        return s.value

    def set_check_schedule(self, schedule):
        """HBTC_CHECK_* (include/hbtc.h): -1 auto, 0 plain-first, 1 paired + sub-tiles, 2 paired -> leaves."""
        self._check(self.lib.hbtc_set_check_schedule(self.h, int(schedule)), "hbtc_set_check_schedule")

    def set_sender_tracking(self, on):
        """Sender tracking (default on): recent liars' shares are checked one by one."""
        self._check(self.lib.hbtc_set_sender_tracking(self.h, 1 if on else 0),
                    "hbtc_set_sender_tracking")

    def rlc_last_leaves(self):
        n = _U32()
        self._check(self.lib.hbtc_rlc_last_leaves(self.h, ctypes.byref(n)), "hbtc_rlc_last_leaves")
        return n.value

    def timing_enable(self, on=True):
        self._check(self.lib.hbtc_timing_enable(self.h, 1 if on else 0), "hbtc_timing_enable")

    def timing_reset(self):
        self._check(self.lib.hbtc_timing_reset(self.h), "hbtc_timing_reset")

    def timing_read(self, family):
        ms, n = ctypes.c_double(), ctypes.c_uint64()
        self._check(self.lib.hbtc_timing_read(self.h, family.encode(), ctypes.byref(ms),
                                              ctypes.byref(n)), "hbtc_timing_read")
        return ms.value, n.value


class Node:
    """A multi-device node (include/hbtc.h hbtc_node_*): one epoch's batch split across the
    devices (strong scaling), the same host-buffer interface and statuses as Context."""

    def __init__(self, devices):
        self.lib = load()
        devs = np.ascontiguousarray(devices, dtype=np.int32)
        h = ctypes.c_void_p()
        rc = self.lib.hbtc_node_create(int(devs.size), _ptr(devs), ctypes.byref(h))
        if rc != 0:
            raise HbtcError("hbtc_node_create(%s) failed: %d" % (list(devices), rc))
        self.h = h
        self.devices = list(devices)

    def close(self):
        if getattr(self, "h", None):
            self.lib.hbtc_node_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            msg = self.lib.hbtc_node_last_error(self.h)
            raise HbtcError("%s failed (%d): %s" % (what, rc, msg.decode() if msg else ""))

    def set_verify_mode(self, mode):
        self._check(self.lib.hbtc_node_set_verify_mode(self.h, int(mode)), "hbtc_node_set_verify_mode")

    def set_rlc_bits(self, bits):
        self._check(self.lib.hbtc_node_set_rlc_bits(self.h, int(bits)), "hbtc_node_set_rlc_bits")

    def keyset_load(self, pk_shares):
        pk = _join(pk_shares, 48)
        kid, bad = _U32(), _U32()
        self._check(self.lib.hbtc_node_keyset_load(self.h, _ptr(pk), pk.size // 48, ctypes.byref(kid),
                                                   ctypes.byref(bad)), "hbtc_node_keyset_load")
        return kid.value, bad.value

    def keyset_free(self, kid):
        self._check(self.lib.hbtc_node_keyset_free(self.h, kid), "hbtc_node_keyset_free")

    def verify_dec_shares(self, keyset, H, w, counts, idx, shares, offsets=None):
        off = _offsets(offsets if offsets is not None else counts, offsets is not None)
        Hb, wb = _join(H, 96), _join(w, 96)
        ix = np.ascontiguousarray(idx, dtype=np.uint32)
        sh = _join(shares, 48)
        st = np.zeros(max(int(off[-1]), 1), np.int32)
        self._check(self.lib.hbtc_node_verify_dec_shares(self.h, keyset, off.size - 1, _ptr(Hb), _ptr(wb),
                                                         _ptr(off), _ptr(ix), _ptr(sh), _ptr(st)),
                    "hbtc_node_verify_dec_shares")
        return st[:int(off[-1])]

    def verify_sig_shares(self, keyset, H, counts, idx, sigs, offsets=None):
        off = _offsets(offsets if offsets is not None else counts, offsets is not None)
        Hb = _join(H, 96)
        ix = np.ascontiguousarray(idx, dtype=np.uint32)
        sg = _join(sigs, 96)
        st = np.zeros(max(int(off[-1]), 1), np.int32)
        self._check(self.lib.hbtc_node_verify_sig_shares(self.h, keyset, off.size - 1, _ptr(Hb), _ptr(off),
                                                         _ptr(ix), _ptr(sg), _ptr(st)),
                    "hbtc_node_verify_sig_shares")
        return st[:int(off[-1])]

    def combine_dec(self, counts, idx, shares, t, offsets=None):
        off = _offsets(offsets if offsets is not None else counts, offsets is not None)
        n = off.size - 1
        ix = np.ascontiguousarray(idx, dtype=np.uint32)
        sh = _join(shares, 48)
        out = np.zeros(48 * max(n, 1), np.uint8)
        st = np.zeros(max(n, 1), np.int32)
        self._check(self.lib.hbtc_node_combine_dec(self.h, n, _ptr(off), _ptr(ix), _ptr(sh), t, _ptr(out),
                                                   _ptr(st)), "hbtc_node_combine_dec")
        return [bytes(out[48 * k:48 * k + 48]) for k in range(n)], st[:n]

    def combine_sigs(self, counts, idx, sigs, t, offsets=None):
        off = _offsets(offsets if offsets is not None else counts, offsets is not None)
        n = off.size - 1
        ix = np.ascontiguousarray(idx, dtype=np.uint32)
        sg = _join(sigs, 96)
        out = np.zeros(96 * max(n, 1), np.uint8)
        par = np.zeros(max(n, 1), np.uint8)
        st = np.zeros(max(n, 1), np.int32)
        self._check(self.lib.hbtc_node_combine_sigs(self.h, n, _ptr(off), _ptr(ix), _ptr(sg), t, _ptr(out),
                                                    _ptr(par), _ptr(st)), "hbtc_node_combine_sigs")
        return [bytes(out[96 * k:96 * k + 96]) for k in range(n)], par[:n], st[:n]

    # ---- device-resident parts (one per device slot; include/hbtc.h hbtc_node_part)
    def context(self, slot):
        """Device slot `slot`'s context (owned by the node) for allocation and copies."""
        h = self.lib.hbtc_node_context(self.h, int(slot))
        if not h:
            raise HbtcError("hbtc_node_context(%d): no such slot" % slot)
        return Context.borrowed(h, self.devices[slot])

    @staticmethod
    def parts(specs):
        """specs: per slot a dict of NodePart fields (device pointers as ints / c_void_p, the
        host `offsets` as a uint32 array, kept alive by the returned tuple)."""
        arr = (NodePart * len(specs))()
        keep = []
        for i, sp in enumerate(specs):
            off = sp.get("offsets")
            if off is not None:
                off = np.ascontiguousarray(off, dtype=np.uint32)
                keep.append(off)
                arr[i].offsets = off.ctypes.data
                arr[i].n_inst = off.size - 1
            for k, v in sp.items():
                if k in ("offsets", "n_inst"):
                    continue
                setattr(arr[i], k, v.value if isinstance(v, ctypes.c_void_p) else v)
        return arr, keep

    def verify_sig_shares_dev(self, keyset, parts):
        self._check(self.lib.hbtc_node_verify_sig_shares_dev(self.h, keyset, parts),
                    "hbtc_node_verify_sig_shares_dev")

    def verify_dec_shares_dev(self, keyset, parts):
        self._check(self.lib.hbtc_node_verify_dec_shares_dev(self.h, keyset, parts),
                    "hbtc_node_verify_dec_shares_dev")

    def combine_sigs_verified_dev(self, parts, t):
        self._check(self.lib.hbtc_node_combine_sigs_verified_dev(self.h, parts, t),
                    "hbtc_node_combine_sigs_verified_dev")

    def combine_dec_verified_dev(self, parts, t):
        self._check(self.lib.hbtc_node_combine_dec_verified_dev(self.h, parts, t),
                    "hbtc_node_combine_dec_verified_dev")

    def sync(self):
        self._check(self.lib.hbtc_node_sync(self.h), "hbtc_node_sync")
