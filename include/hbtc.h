/* hbtc — MI355X-native batched threshold-crypto verifier for hbbft's per-epoch hot path.
 *
 * C ABI (plain pointers and sizes; no torch / HIP types in the signatures).  Each entry point
 * replaces calls the reference makes into the `threshold_crypto` crate (re-exported as
 * `crypto` at /root/reference/src/lib.rs:136), batched over a whole epoch:
 *
 *   hbtc_verify_sig_shares   PublicKeyShare::verify(&SignatureShare, nonce)   src/coin.rs:151
 *   hbtc_verify_sigs         PublicKey::verify(&Signature, msg)               src/coin.rs:192-197,
 *                              src/dynamic_honey_badger/votes.rs:154, dynamic_honey_badger.rs:439
 *   hbtc_combine_sigs        PublicKeySet::combine_signatures + Signature::parity
 *                                                                             src/coin.rs:185-191,173
 *   hbtc_verify_dec_shares   PublicKeyShare::verify_decryption_share          src/threshold_decryption.rs:159
 *   hbtc_combine_dec         PublicKeySet::decrypt, the G1 interpolation      src/threshold_decryption.rs:181-185
 *                            (plaintext = v XOR hash_bytes(g, |v|) stays with the caller)
 *   hbtc_verify_ciphertexts  Ciphertext::verify inside SecretKeyShare::decrypt_share
 *                                                                             src/threshold_decryption.rs:98
 *   hbtc_keyset_load         the public_key_share(idx) table of NetworkInfo::new
 *                                                                             src/messaging.rs:253-256
 *   hbtc_g1_mul/hbtc_g2_mul  batched scalar multiplication (Poly::commitment src/sync_key_gen.rs:366,
 *                            SecretKeyShare::sign src/coin.rs:142, decrypt_share src/threshold_decryption.rs:98)
 *   hbtc_skg_check_parts     SyncKeyGen::handle_part: row.commitment() == commit.row(x)
 *                                                                             src/sync_key_gen.rs:366
 *   hbtc_skg_check_acks      SyncKeyGen::handle_ack_or_err: commit.evaluate(x, y) == val * G1
 *                                                                             src/sync_key_gen.rs:493
 *   hbtc_g1_msm/hbtc_g2_msm  batched Pippenger MSMs (BivarCommitment::row / Commitment::evaluate,
 *                            src/sync_key_gen.rs:345,366,493); the combines run on the same kernels
 *
 * Encodings are hbbft's wire encodings of the points (zcash compressed: G1 = 48 bytes, G2 =
 * 96 bytes with x.c1 first; flag bits 0x80 compressed, 0x40 infinity, 0x20 lexicographically
 * largest y).  Decoding and the r-order subgroup check run on the GPU; an encoding that
 * pairing 0.14's `into_affine` would reject yields HBTC_DECODE_ERR for that item (the
 * reference would have rejected the message in serde before calling the verifier).
 *
 * Batches are CSR-shaped: instance k (a coin instance or a ciphertext) owns items
 * [offsets[k], offsets[k+1]) with offsets[0] == 0.  `idx` is the sender's node index
 * (NetworkInfo::node_index, src/messaging.rs:334): it selects pk_idx from the loaded key set
 * and gives x = idx + 1 in the Lagrange interpolation.  Item arrays are item-major
 * (48 or 96 bytes per item, 16-byte aligned base).
 *
 * Threading: one context per GPU; calls on one context are serialised by an internal mutex.
 * Host entry points block until the results are on the host; *_dev entry points take
 * device pointers (from hbtc_dev_alloc) and are ordered as issued: combines run on a side
 * stream, concurrently with the verification issued after them, and any later call that
 * writes a device range a pending combine still reads (a status array, an upload into the
 * share buffer) first waits for that combine.
 * The caller owns every buffer; nothing is retained after a call returns.
 */
#ifndef HBTC_H
#define HBTC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- return codes (< 0: API / device error) ---------------------------------------------- */
#define HBTC_OK 0
#define HBTC_ERR_ARG (-1)
#define HBTC_ERR_DEVICE (-2)
#define HBTC_ERR_NO_KEYSET (-3)
#define HBTC_ERR_OOM (-4)

/* ---- per-item / per-instance status ------------------------------------------------------- */
#define HBTC_ACCEPT 0            /* verifies (combine: combined)                               */
#define HBTC_REJECT 1            /* well-formed, but the pairing equation fails                */
#define HBTC_DECODE_ERR 2        /* encoding rejected (serde would have refused the message)   */
#define HBTC_UNKNOWN_SENDER 3    /* idx >= key-set size (public_key_share(id) == None)          */
#define HBTC_INSTANCE_ERR 4      /* the instance's own H / w failed to decode                  */
#define HBTC_NOT_ENOUGH_SHARES 5 /* combine: fewer than t items (crypto Error::NotEnoughShares) */
#define HBTC_DUPLICATE_ENTRY 6   /* combine: repeated index among the first t (DuplicateEntry) */

typedef struct hbtc_ctx hbtc_ctx;

/* Number of visible HIP devices (0 without a GPU); does not create a context. */
int hbtc_device_count(void);
/* Build identification string (static storage). */
const char* hbtc_version(void);

/* Create a context on HIP device `device`. */
int hbtc_ctx_create(int device, hbtc_ctx** out);
void hbtc_ctx_destroy(hbtc_ctx* ctx);
/* Description of the last error on this context (valid until the next call). */
const char* hbtc_last_error(hbtc_ctx* ctx);

/* ---- key sets ------------------------------------------------------------------------------ */
/* Upload and decode n compressed G1 public-key shares (pk_0 .. pk_{n-1}, node-index order).
 * *n_bad counts shares that failed to decode (their senders can never be ACCEPTed). */
int hbtc_keyset_load(hbtc_ctx* ctx, const uint8_t* pk_shares_c48, uint32_t n,
                     uint32_t* keyset_id, uint32_t* n_bad);
int hbtc_keyset_free(hbtc_ctx* ctx, uint32_t keyset_id);

/* ---- signature shares (Coin) ---------------------------------------------------------------- */
/* H_k = hash_g2(nonce_k) (compressed G2, one per instance).  Item i of instance k is checked as
 * e(pk_{idx_i}, H_k) == e(G1, sig_i).  status[i] receives an HBTC_* item status. */
int hbtc_verify_sig_shares(hbtc_ctx* ctx, uint32_t keyset_id, uint32_t n_inst,
                           const uint8_t* H_c96, const uint32_t* offsets, const uint32_t* idx,
                           const uint8_t* sig_c96, int32_t* status);

/* Non-threshold verify: e(pk_i, H_i) == e(G1, sig_i) for n independent items. */
int hbtc_verify_sigs(hbtc_ctx* ctx, uint32_t n, const uint8_t* pk_c48, const uint8_t* H_c96,
                     const uint8_t* sig_c96, int32_t* status);

/* The key set's master public key (NetworkInfo::public_key, src/messaging.rs:253; compressed
 * G1), decoded once with the subgroup check and kept resident for hbtc_coin_decide.  Returns
 * HBTC_OK, or HBTC_ERR_ARG when it fails to decode (the key set keeps no master key then). */
int hbtc_keyset_set_master(hbtc_ctx* ctx, uint32_t keyset_id, const uint8_t* master_pk_c48);

/* Per-instance G2 preparation ahead of the shares.  hbbft knows a coin's nonce when it creates
 * the Coin (src/binary_agreement/binary_agreement.rs:320; H = hash_g2(nonce)) and a ciphertext
 * at set_ciphertext (src/threshold_decryption.rs:94-113; H = hash_g1_g2(u, v) and w), before most
 * shares arrive.  hbtc_prepare_g2 decodes n compressed G2 points (subgroup-checked) and builds
 * their Miller-line tables, kept resident and keyed by the 96 bytes.  A later
 * hbtc_verify_sig_shares / hbtc_coin_decide / hbtc_verify_dec_shares / *_epoch_submit call whose
 * per-instance G2 arguments are ALL prepared copies their tables instead of building them; the
 * outputs are identical either way.  out_status[i] (optional): HBTC_ACCEPT, or HBTC_DECODE_ERR
 * for a point that fails to decode (a call with it reports the instance error as usual).  Points
 * already prepared are not rebuilt.  Entries stay until hbtc_unprepare_g2 (unknown points are
 * ignored) or hbtc_ctx_destroy.  Both calls wait for the context's calls in flight. */
int hbtc_prepare_g2(hbtc_ctx* ctx, uint32_t n, const uint8_t* g2_c96, int32_t* out_status);
int hbtc_unprepare_g2(hbtc_ctx* ctx, uint32_t n, const uint8_t* g2_c96);
int hbtc_prepared_g2_count(hbtc_ctx* ctx, uint32_t* count);

/* A Threshold Coin round of n_inst coin instances in ONE call (the batch queue of src/coin.rs:
 * 149-207): every SignatureShare verified as hbtc_verify_sig_shares (status[i], coin.rs:151),
 * the first t ACCEPTed shares of each instance combined (combine_signatures, coin.rs:185-191:
 * sig_c96[k], parity[k] = Signature::parity, coin.rs:173), and the combined signature checked
 * against the master key (PublicKey::verify, coin.rs:192-197).  coin_status[k]: HBTC_ACCEPT (the
 * coin value is parity[k]), the combine's failure (NOT_ENOUGH_SHARES, DUPLICATE_ENTRY,
 * DECODE_ERR), or HBTC_REJECT when the combined signature fails the master check.
 * The master check is exact without a pairing: every combined share passed e(pk_i, H) ==
 * e(G1, sig_i), so e(G1, sum l_i sig_i) == e(sum l_i pk_i, H), and PublicKey::verify holds iff
 * sum l_i pk_i == master pk in G1 (H != O, e non-degenerate) -- a G1 combine of the key set's
 * resident shares.  So the master check is exactly as sound as the share checks under it: exact
 * in HBTC_MODE_PER_SHARE and for calls below hbtc_set_exact_below (256 shares: every coin of up
 * to N = 255), and otherwise wrong with probability <= 2^-k per RLC group for k-bit scalars
 * (hbtc_set_rlc_bits: 2^-128 by default, the curve's level; 2^-64 when set to 64), where the
 * reference's separate pairing check (coin.rs:192-197) would be exact.  Small calls (n_inst * (t + 1) <= 256, t < 64) combine speculatively while the
 * shares are checked: every leave-one-out subset of each instance's first t + 1 items, committed
 * when the verified selection is one of them (at most one of the first t + 1 rejected), else
 * combined again from the statuses.  Needs hbtc_keyset_set_master; t in 1..64. */
int hbtc_coin_decide(hbtc_ctx* ctx, uint32_t keyset_id, uint32_t n_inst, const uint8_t* H_c96,
                     const uint32_t* offsets, const uint32_t* idx, const uint8_t* sig_items_c96,
                     uint32_t t, int32_t* status, uint8_t* sig_c96, uint8_t* parity,
                     int32_t* coin_status);

/* Lagrange combine of the first t items of each instance (x = idx + 1) in G2: the compressed
 * signature, Signature::parity() (0/1) and an instance status (ACCEPT, NOT_ENOUGH_SHARES,
 * DUPLICATE_ENTRY, DECODE_ERR). */
int hbtc_combine_sigs(hbtc_ctx* ctx, uint32_t n_inst, const uint32_t* offsets,
                      const uint32_t* idx, const uint8_t* sig_c96, uint32_t t,
                      uint8_t* out_sig_c96, uint8_t* out_parity, int32_t* inst_status);

/* ---- decryption shares (ThresholdDecryption / HoneyBadger) -------------------------------- */
/* Ciphertext k = (u_k, v_k, w_k); the caller passes H_k = hash_g1_g2(u_k, v_k) and w_k.  Item i
 * of ciphertext k is checked as e(share_i, H_k) == e(pk_{idx_i}, w_k). */
int hbtc_verify_dec_shares(hbtc_ctx* ctx, uint32_t keyset_id, uint32_t n_ct,
                           const uint8_t* H_c96, const uint8_t* w_c96, const uint32_t* offsets,
                           const uint32_t* idx, const uint8_t* share_c48, int32_t* status);

/* G1 Lagrange combine of the first t decryption shares of each ciphertext (compressed g). */
int hbtc_combine_dec(hbtc_ctx* ctx, uint32_t n_ct, const uint32_t* offsets, const uint32_t* idx,
                     const uint8_t* share_c48, uint32_t t, uint8_t* out_g_c48,
                     int32_t* inst_status);

/* SecretKey::decrypt for n ciphertexts (u_i, v_i, w_i) under ONE secret key (32-byte LE scalar):
 * the row / value a node decrypts from every SyncKeyGen Part and Ack (src/sync_key_gen.rs:358,
 * 481-484; 10^6 Acks per era at N = 1000).  Per item: H = hash_g1_g2(u, v) (host candidates, GPU
 * cofactor clearing), Ciphertext::verify e(G1, w) == e(u, H) and g = sk u on the GPU, then
 * out = v XOR hash_bytes(g, |v|) on the host's cores.  v_i = msgs[offsets[i] .. offsets[i+1]),
 * out has the same layout.  status[i] = ACCEPT (decrypted), REJECT (Ciphertext::verify failed:
 * decrypt returns None, Fault::ValueDecryption), DECODE_ERR (u or w does not decode). */
int hbtc_decrypt(hbtc_ctx* ctx, uint32_t n, const uint8_t* sk_le32, const uint8_t* u_c48,
                 const uint8_t* w_c96, const uint8_t* msgs, const uint32_t* offsets, uint8_t* out,
                 int32_t* status);
/* Ciphertext::verify: e(G1, w_i) == e(u_i, H_i) with H_i = hash_g1_g2(u_i, v_i). */
int hbtc_verify_ciphertexts(hbtc_ctx* ctx, uint32_t n, const uint8_t* u_c48,
                            const uint8_t* H_c96, const uint8_t* w_c96, int32_t* status);

/* ---- host hashes (no context, no GPU) ----------------------------------------------------- */
/* threshold_crypto's crate-internal hash_g2(msg) -> compressed G2 (96 B), and hash_g1_g2(g1, msg)
 * = hash_g2((|msg| > 64 ? sha3_256(msg) : msg) || g1_c48).  These produce the H that
 * PublicKeyShare::verify (src/coin.rs:151: H = hash_g2(nonce)) and verify_decryption_share /
 * Ciphertext::verify (src/threshold_decryption.rs:98,159: H = hash_g1_g2(u, v)) compute per
 * call; the batch queue computes it once per instance and passes it to the verifiers.  Byte
 * stream follows rand 0.4's ChaChaRng (parity unpinned). */
int hbtc_sha3_256(const uint8_t* msg, size_t len, uint8_t* out32);
int hbtc_hash_g2(const uint8_t* msg, size_t len, uint8_t* out_c96);
int hbtc_hash_g1_g2(const uint8_t* g1_c48, const uint8_t* msg, size_t len, uint8_t* out_c96);
/* threshold_crypto's hash_bytes(g, len) (crate-internal): the XOR pad of PublicKey::encrypt and
 * SecretKey::decrypt (v = msg XOR hash_bytes(r * pk, |msg|); src/sync_key_gen.rs:321,358,377,483).
 * rand 0.4 ChaChaRng seeded with sha3_256(compressed g), the low byte of one next_u32 per byte.
 * The batch form XORs item i's pad into msgs[offsets[i] .. offsets[i+1]) -> out (same layout),
 * i.e. it encrypts or decrypts n messages given g_i, over the host's cores. */
int hbtc_hash_bytes(const uint8_t* g1_c48, size_t len, uint8_t* out);
int hbtc_xor_hash_bytes_batch(uint32_t n, const uint8_t* g1_c48, const uint8_t* msgs,
                              const uint32_t* offsets, uint8_t* out);
/* Batches over the host's cores: message i = msgs[offsets[i] .. offsets[i+1]) (offsets[0] == 0,
 * non-decreasing); ciphertext i's u is g1_c48[48 i ..]. */
int hbtc_hash_g2_batch(uint32_t n, const uint8_t* msgs, const uint32_t* offsets,
                       uint8_t* out_c96);
int hbtc_hash_g1_g2_batch(uint32_t n, const uint8_t* g1_c48, const uint8_t* msgs,
                          const uint32_t* offsets, uint8_t* out_c96);
/* The same batches with the whole draw on the context's GPU: one lane per message runs the SHA3
 * seed, the ChaCha stream and G2::rand's candidate loop (k_hash_cand), then [h2] P by the psi
 * chain (k_g2_clear_cofactor); the host only redraws in the (never observed) case
 * [h2] P = O. */
int hbtc_hash_g2_batch_gpu(hbtc_ctx* ctx, uint32_t n, const uint8_t* msgs, const uint32_t* offsets,
                           uint8_t* out_c96);
int hbtc_hash_g1_g2_batch_gpu(hbtc_ctx* ctx, uint32_t n, const uint8_t* g1_c48,
                              const uint8_t* msgs, const uint32_t* offsets, uint8_t* out_c96);
/* Diagnostics for the ChaCha20 known-answer tests: the first n words of rand 0.4's
 * ChaChaRng::from_seed(seed8) (key = the 8 seed words, 128-bit block counter from 0, output words
 * in block order), computed by the ChaCha code of the host hashes (hbtc_chacha04_words) and of
 * the GPU candidate kernel (hbtc_chacha04_words_gpu). */
int hbtc_chacha04_words(const uint32_t* seed8, uint32_t n, uint32_t* out);
int hbtc_chacha04_words_gpu(hbtc_ctx* ctx, const uint32_t* seed8, uint32_t n, uint32_t* out);

/* ---- pipelined host-buffer epochs ------------------------------------------------------------ */
/* The batch queue's epoch call without blocking (hbbft keeps the current epoch and up to
 * max_future_epochs = 3 more in flight, src/honey_badger/builder.rs:37; the batch points are
 * ThresholdDecryption::remove_invalid_shares, src/threshold_decryption.rs:136-149, and the
 * epoch's coin / decryption queues).  A submit copies the inputs into pinned staging of the next
 * verification lane and enqueues, on that lane: H2D, the verification (as hbtc_verify_*_shares),
 * then, for t > 0, the combine of the FIRST t ACCEPTed items of every instance (as
 * hbtc_combine_*_verified_dev: the shares hbbft keeps, coin.rs:185-191, td.rs:184), and D2H of
 * every result; it returns a ticket at once.  hbtc_wait(ticket) blocks until that epoch's results
 * are in the caller's output buffers, which must stay valid until then (inputs may be reused as
 * soon as submit returns).  At most four epochs are in flight per context: a fifth submit first
 * completes the oldest (its outputs written as by hbtc_wait).  Waiting on a completed ticket
 * returns HBTC_OK. */
int hbtc_dec_epoch_submit(hbtc_ctx* ctx, uint32_t keyset_id, uint32_t n_ct, const uint8_t* H_c96,
                          const uint8_t* w_c96, const uint32_t* offsets, const uint32_t* idx,
                          const uint8_t* share_c48, uint32_t t, int32_t* status, uint8_t* out_g_c48,
                          int32_t* inst_status, uint64_t* ticket);
int hbtc_sig_epoch_submit(hbtc_ctx* ctx, uint32_t keyset_id, uint32_t n_inst, const uint8_t* H_c96,
                          const uint32_t* offsets, const uint32_t* idx, const uint8_t* sig_c96,
                          uint32_t t, int32_t* status, uint8_t* out_sig_c96, uint8_t* out_parity,
                          int32_t* inst_status, uint64_t* ticket);
int hbtc_wait(hbtc_ctx* ctx, uint64_t ticket);

/* ---- batched scalar multiplication -------------------------------------------------------- */
/* out_i = k_i * P_i with 32-byte little-endian scalars (any value < 2^256).  base_stride is 1
 * for one base per item or 0 for a single shared base.  status[i] = ACCEPT or DECODE_ERR. */
int hbtc_g1_mul(hbtc_ctx* ctx, uint32_t n, const uint8_t* base_c48, uint32_t base_stride,
                const uint8_t* scalars_le32, uint8_t* out_c48, int32_t* status);
int hbtc_g2_mul(hbtc_ctx* ctx, uint32_t n, const uint8_t* base_c96, uint32_t base_stride,
                const uint8_t* scalars_le32, uint8_t* out_c96, int32_t* status);

/* ---- device-resident variants (benchmarks, pipelined callers) ----------------------------- */
int hbtc_dev_alloc(hbtc_ctx* ctx, size_t bytes, void** d_ptr);
int hbtc_dev_free(hbtc_ctx* ctx, void* d_ptr);
int hbtc_dev_upload(hbtc_ctx* ctx, void* d_dst, const void* h_src, size_t bytes);
int hbtc_dev_download(hbtc_ctx* ctx, void* h_dst, const void* d_src, size_t bytes);
int hbtc_sync(hbtc_ctx* ctx);
/* Ordering with a caller's HIP stream (e.g. the stream an RCCL all-gather runs on):
 * hbtc_stream_wait_ctx  work enqueued on `stream` after this call waits for everything already
 *                       enqueued on the context (verification, preparation, combines);
 * hbtc_ctx_wait_stream  the context's later work waits for everything already on `stream`
 *                       (before overwriting a buffer the caller's stream still reads). */
int hbtc_stream_wait_ctx(hbtc_ctx* ctx, void* hip_stream);
int hbtc_ctx_wait_stream(hbtc_ctx* ctx, void* hip_stream);
/* bincode-framed wire points (a SignatureShare / DecryptionShare as serialized: u64 LE length
 * || 96 / 48 compressed bytes, back to back) -> the 16-aligned item array the *_dev verifiers
 * read, on the context's main stream.  A frame whose length is not point_size yields an item
 * that decodes to HBTC_DECODE_ERR (the message serde would refuse). */
int hbtc_unframe_points_dev(hbtc_ctx* ctx, uint32_t n, uint32_t point_size, const uint8_t* d_framed,
                            uint8_t* d_items);
/* Same semantics as the host entry points; every d_* argument is a device pointer from
 * hbtc_dev_alloc and `offsets` stays a HOST array (it shapes the launch).  Work is enqueued on
 * the context's stream; call hbtc_sync before reading results. */
int hbtc_verify_dec_shares_dev(hbtc_ctx* ctx, uint32_t keyset_id, uint32_t n_ct,
                               const uint8_t* d_H_c96, const uint8_t* d_w_c96,
                               const uint32_t* offsets, const uint32_t* d_idx,
                               const uint8_t* d_share_c48, int32_t* d_status);
int hbtc_verify_sig_shares_dev(hbtc_ctx* ctx, uint32_t keyset_id, uint32_t n_inst,
                               const uint8_t* d_H_c96, const uint32_t* offsets,
                               const uint32_t* d_idx, const uint8_t* d_sig_c96,
                               int32_t* d_status);
int hbtc_combine_dec_dev(hbtc_ctx* ctx, uint32_t n_ct, const uint32_t* offsets,
                         const uint32_t* d_idx, const uint8_t* d_share_c48, uint32_t t,
                         uint8_t* d_out_g_c48, int32_t* d_inst_status);
int hbtc_combine_sigs_dev(hbtc_ctx* ctx, uint32_t n_inst, const uint32_t* offsets,
                          const uint32_t* d_idx, const uint8_t* d_sig_c96, uint32_t t,
                          uint8_t* d_out_sig_c96, uint8_t* d_out_parity, int32_t* d_inst_status);

/* Combine from the verified shares: as hbtc_combine_dec_dev / hbtc_combine_sigs_dev, but over the
 * first t items of each instance whose d_status (written by hbtc_verify_*_dev on the same
 * context) is HBTC_ACCEPT — the shares hbbft keeps after verification (coin.rs:185-191 combines
 * `received_shares`, threshold_decryption.rs:184 `shares`; both hold verified shares only).
 * Ordered after the verification on the context's streams; no host synchronisation. */
int hbtc_combine_dec_verified_dev(hbtc_ctx* ctx, uint32_t n_ct, const uint32_t* offsets,
                                  const uint32_t* d_idx, const uint8_t* d_share_c48,
                                  const int32_t* d_status, uint32_t t, uint8_t* d_out_g_c48,
                                  int32_t* d_inst_status);
int hbtc_combine_sigs_verified_dev(hbtc_ctx* ctx, uint32_t n_inst, const uint32_t* offsets,
                                   const uint32_t* d_idx, const uint8_t* d_sig_c96,
                                   const int32_t* d_status, uint32_t t, uint8_t* d_out_sig_c96,
                                   uint8_t* d_out_parity, int32_t* d_inst_status);

/* ---- commitments ------------------------------------------------------------------------ */
/* Commitment::evaluate(x) for n_x points at once: out_k = sum_j xs[k]^j C_j over the n_coeff
 * compressed G1 coefficients (Poly::commitment order, constant term first).  This is the
 * per-era public-key-share table: NetworkInfo::new evaluates public_key_share(i) =
 * commitment.evaluate(i + 1) for every node (src/messaging.rs:253-256, PublicKeySet from
 * SyncKeyGen::generate, src/sync_key_gen.rs:428-447).  status[k] = ACCEPT or DECODE_ERR. */
int hbtc_commitment_evaluate(hbtc_ctx* ctx, uint32_t n_coeff, const uint8_t* commit_c48,
                             uint32_t n_x, const uint32_t* xs, uint8_t* out_c48, int32_t* status);

/* ---- batched multi-scalar multiplication (Pippenger) -------------------------------------- */
/* n_msm independent MSMs of n terms: out_m = sum_i k_{m,i} P_{m,i} (points item-major
 * [m][i], 32-byte little-endian scalars, reduced mod r).  Used for commitments and bivariate
 * commitment rows (BivarCommitment::row, Commitment::evaluate: src/sync_key_gen.rs:345,366,493)
 * and by the combines.  status[m] = ACCEPT or DECODE_ERR (a point failed to decode). */
int hbtc_g1_msm(hbtc_ctx* ctx, uint32_t n_msm, uint32_t n, const uint8_t* pts_c48,
                const uint8_t* scalars_le32, uint8_t* out_c48, int32_t* status);
int hbtc_g2_msm(hbtc_ctx* ctx, uint32_t n_msm, uint32_t n, const uint8_t* pts_c96,
                const uint8_t* scalars_le32, uint8_t* out_c96, int32_t* status);

/* ---- SyncKeyGen (DynamicHoneyBadger era change) ------------------------------------------- */
/* A node's Part checks (SyncKeyGen::handle_part, src/sync_key_gen.rs:338-369): for every Part p,
 * commit_c48[p] holds the (t+1)(t+2)/2 compressed G1 coefficients of its BivarCommitment in
 * coeff_pos order (pos(i, j) = j(j+1)/2 + i, i <= j) and rows_le32[p] the t+1 coefficients
 * (32-byte little-endian Fr) of the row this node decrypted from it.  part_status[p] = ACCEPT
 * iff row.commitment() == commit.row(our_idx + 1) (:366), REJECT otherwise (InvalidPartMessage;
 * also for a row coefficient >= r, which bincode's Fr decoding refuses), DECODE_ERR if a
 * commitment point does not decode (serde would refuse the Part).  One random linear
 * combination of the t+1 coefficient equations per Part (one Pippenger MSM, error <= 1/r). */
int hbtc_skg_check_parts(hbtc_ctx* ctx, uint32_t n_parts, uint32_t t, uint32_t our_idx,
                         const uint8_t* commit_c48, const uint8_t* rows_le32,
                         int32_t* part_status);
/* A node's Ack value checks (handle_ack_or_err, :493): Ack a (for Part ack_part[a], from node
 * ack_sender[a], decrypted value vals_le32[a]) is ACCEPT iff
 * commit.evaluate(our_idx + 1, ack_sender + 1) == val * G1, REJECT otherwise (ValueInvalid),
 * DECODE_ERR for a value >= r (ValueDeserialization).  For a Part with row_ok[p] != 0 (its row
 * passed hbtc_skg_check_parts) the check is the identical scalar equation val == row(y); the
 * other Parts' Acks are checked by one random linear combination per Part with an exact per-Ack
 * fallback.  The caller applies the checks that precede the value (NodeCount, SenderExist,
 * DuplicateAck, ValueDecryption: :467-482) and calls this for the Acks that reach :493. */
int hbtc_skg_check_acks(hbtc_ctx* ctx, uint32_t n_parts, uint32_t t, uint32_t our_idx,
                        const uint8_t* commit_c48, const uint8_t* rows_le32,
                        const uint8_t* row_ok, uint32_t n_acks, const uint32_t* ack_part,
                        const uint32_t* ack_sender, const uint8_t* vals_le32,
                        int32_t* ack_status);

/* ---- multi-device node ------------------------------------------------------------------- */
/* One hbbft node (one process, /root/reference/src/messaging.rs:188) driving several GPUs: a
 * context per device, each call's batch split across them (strong scaling of ONE epoch).
 * Verification cuts the item range into equal contiguous slices (an instance crossing a cut is
 * verified as one sub-instance per side with the same H / w: the RLC groups are tiles inside an
 * instance, so no exchange is needed); combines take whole instances, balanced by share count.
 * Host buffers, blocking, the same semantics and statuses as the single-context calls.
 * devices == NULL means 0 .. n_devices-1; a device may repeat (several contexts on one GPU). */
typedef struct hbtc_node hbtc_node;
int hbtc_node_create(int n_devices, const int* devices, hbtc_node** out);
void hbtc_node_destroy(hbtc_node* node);
const char* hbtc_node_last_error(hbtc_node* node);
int hbtc_node_devices(hbtc_node* node);
hbtc_ctx* hbtc_node_context(hbtc_node* node, int device_slot);
int hbtc_node_set_verify_mode(hbtc_node* node, int mode);
/* hbtc_set_rlc_bits on every device of the node. */
int hbtc_node_set_rlc_bits(hbtc_node* node, uint32_t bits);
int hbtc_node_keyset_load(hbtc_node* node, const uint8_t* pk_shares_c48, uint32_t n,
                          uint32_t* keyset_id, uint32_t* n_bad);
int hbtc_node_keyset_free(hbtc_node* node, uint32_t keyset_id);
int hbtc_node_verify_dec_shares(hbtc_node* node, uint32_t keyset_id, uint32_t n_ct,
                                const uint8_t* H_c96, const uint8_t* w_c96,
                                const uint32_t* offsets, const uint32_t* idx,
                                const uint8_t* share_c48, int32_t* status);
int hbtc_node_verify_sig_shares(hbtc_node* node, uint32_t keyset_id, uint32_t n_inst,
                                const uint8_t* H_c96, const uint32_t* offsets,
                                const uint32_t* idx, const uint8_t* sig_c96, int32_t* status);
int hbtc_node_combine_dec(hbtc_node* node, uint32_t n_ct, const uint32_t* offsets,
                          const uint32_t* idx, const uint8_t* share_c48, uint32_t t,
                          uint8_t* out_g_c48, int32_t* inst_status);
int hbtc_node_combine_sigs(hbtc_node* node, uint32_t n_inst, const uint32_t* offsets,
                           const uint32_t* idx, const uint8_t* sig_c96, uint32_t t,
                           uint8_t* out_sig_c96, uint8_t* out_parity, int32_t* inst_status);

/* Device-resident node calls: the batch is already split over the node's devices, part d living
 * on device slot d (one hbtc_node_part per slot, in slot order; a part with n_inst == 0 is
 * skipped).  The shard plans below give the parts: whole instances per device
 * (hbtc_shard_instances), or item slices whose sub-instances share their parent's H / w
 * (hbtc_shard_items).  Every device's call is enqueued on its own context from its own host
 * thread and the call returns without waiting for the GPUs (hbtc_node_sync waits); semantics
 * and statuses are those of the single-context *_dev calls.  The combines read the statuses the
 * verification of the SAME parts wrote, so their parts must hold whole instances (a split
 * instance's sub-instances are gathered onto one device by the caller first). */
typedef struct {
  uint32_t n_inst;          /* instances (or sub-instances) of this part                      */
  const uint32_t* offsets;  /* HOST array, n_inst + 1 entries, offsets[0] == 0                 */
  const uint8_t* d_H_c96;   /* device: H per instance (verification only)                    */
  const uint8_t* d_w_c96;   /* device: w per ciphertext (decryption shares only)             */
  const uint32_t* d_idx;    /* device: node index per item                                    */
  const uint8_t* d_items;   /* device: compressed items (48 B decryption, 96 B signature)     */
  int32_t* d_status;        /* device: item statuses (written by verification, read by combine) */
  uint8_t* d_out;           /* device: combined points (48 / 96 B per instance; combine only)  */
  uint8_t* d_out_parity;    /* device: Signature::parity per instance (signature combine only) */
  int32_t* d_inst_status;   /* device: combine status per instance (combine only)              */
} hbtc_node_part;
int hbtc_node_verify_sig_shares_dev(hbtc_node* node, uint32_t keyset_id, const hbtc_node_part* parts);
int hbtc_node_verify_dec_shares_dev(hbtc_node* node, uint32_t keyset_id, const hbtc_node_part* parts);
int hbtc_node_combine_sigs_verified_dev(hbtc_node* node, const hbtc_node_part* parts, uint32_t t);
int hbtc_node_combine_dec_verified_dev(hbtc_node* node, const hbtc_node_part* parts, uint32_t t);
/* Wait for every device's enqueued work. */
int hbtc_node_sync(hbtc_node* node);

/* The node's shard plans (host code, no GPU), for callers that run one process per GPU and
 * merge with their own collective (bench.py: RCCL all-gather of statuses and combined points).
 * hbtc_shard_items: device `dev`'s verification slice [*lo, *hi) of the item range and its
 *   *n_sub sub-instances: parent[s] (capacity n_inst) is the instance of sub-instance s,
 *   sub_offsets (capacity n_inst + 1) their item offsets relative to *lo.
 * hbtc_shard_instances: the combine plan, device d takes instances [first[d], first[d+1])
 *   (first has n_dev + 1 entries), balanced by share count. */
int hbtc_shard_items(uint32_t n_dev, uint32_t dev, uint32_t n_inst, const uint32_t* offsets,
                     uint32_t* lo, uint32_t* hi, uint32_t* n_sub, uint32_t* parent,
                     uint32_t* sub_offsets);
int hbtc_shard_instances(uint32_t n_dev, uint32_t n_inst, const uint32_t* offsets, uint32_t* first);

/* ---- verification strategy ----------------------------------------------------------------- */
/* HBTC_MODE_RLC (default): shares of one instance are checked together by a random linear
 * combination (fresh ChaCha20 scalars per call, 128-bit by default, 64-bit with
 * hbtc_set_rlc_bits; prime-order points only) in groups of
 * 64 consecutive shares; failing groups are split 64 -> 32 -> 8 -> 1 share (plain-first) or
 * 64 -> 8 -> 1 (paired schedules); a group with exactly one
 * wrong share is resolved by a position-weighted second combination (the wrong share located
 * without per-share pairings), the rest get the exact pairing check.  The decisions equal the
 * per-share decisions except with probability <= 2^-128 per group check (<= 2^-122 per located
 * group); <= 2^-64 (2^-58) with 64-bit scalars.
 * HBTC_MODE_PER_SHARE: every share gets its own 2-pair pairing check (the reference's count).
 * Applies to hbtc_verify_dec_shares[_dev]. */
#define HBTC_MODE_PER_SHARE 0
#define HBTC_MODE_RLC 1
int hbtc_set_verify_mode(hbtc_ctx* ctx, int mode);
/* In RLC mode, hbtc_verify_dec_shares[_dev] / hbtc_verify_sig_shares[_dev] calls with fewer than
 * n_items shares skip the group sums: the item pass only decodes, and every share gets the exact
 * cooperative pairing check of the leaf level.  Two or three dependent launches instead of the
 * item pass plus its group-check levels, for calls too small to fill the GPU (a single N = 10
 * coin).  hbtc_verify_sigs / hbtc_verify_ciphertexts / hbtc_decrypt calls with fewer than n_items
 * items take the same exact checks in the SignatureShare form (e(A, Q) = e(G1, W)) instead of
 * the pair batch.  Default 256; 0 = always batch.  The decisions are the same either way. */
int hbtc_set_exact_below(hbtc_ctx* ctx, uint32_t n_items);
/* Size of the RLC scalars r_i = d0 + d1 x + d2 mu + d3 mu x (x the BLS parameter, mu = -x^2 mod r;
 * four digits of bits/4 bits; DESIGN.md §4, "x-adic scalars" and "Soundness"): 128 (default:
 * 2^128 distinct scalars: a wrong share survives a group check with probability <= 2^-128,
 * <= 2^-122 per located group, matching BLS12-381's ~2^-128 security level, as SURVEY.md §7
 * step 5 specifies) or 64 (16-bit digits: <= 2^-64 per group check, <= 2^-58 per located group;
 * the item passes do half the doublings and table additions).  Any other value: HBTC_ERR_ARG.  Applies to the RLC calls of
 * hbtc_verify_dec_shares[_dev] and hbtc_verify_sig_shares[_dev]. */
int hbtc_set_rlc_bits(hbtc_ctx* ctx, uint32_t bits);
int hbtc_get_rlc_bits(hbtc_ctx* ctx, uint32_t* bits);
/* Free every cached device workspace buffer of the context (after completing its work; key sets
 * stay loaded).  Calls size their workspace to the largest batch seen and keep it; buffers up to
 * 256 MB grow on all four verification lanes at once (one that grew mid-pipeline would stall
 * every lane in flight).  The peak is set by hbtc_verify_ciphertexts / hbtc_verify_sigs /
 * hbtc_decrypt batches, which run in chunks of 2^18 items with 19.6 KB of G2 line tables per
 * item (~5.8 GB per chunk, on the lanes that ran one; HBTC_PB_CHUNK = a smaller multiple of 64
 * lowers it), and by RLC verification of n shares (~0.15 KB per share and lane). */
int hbtc_trim_workspace(hbtc_ctx* ctx);
/* Sender tracking (default on, RLC mode): a sender with many shares REJECTed (at least 1/8 of
 * the call's average shares per sender) by one of the last 16 RLC calls on a key set has its
 * shares checked one by one, outside the group sums, so f Byzantine senders who lie in every
 * epoch cannot make the honest shares' groups fail.  The
 * decisions are exactly those of the per-share check either way; only the work differs. */
int hbtc_set_sender_tracking(hbtc_ctx* ctx, int enable);
/* Group-check schedule of RLC calls (DecryptionShares).  HBTC_CHECK_AUTO (default) picks by the
 * call's tile count against the device's SIMDs: the plain-first schedule (plain checks of every
 * tile, weighted checks only of failing ones: tiles, tiles_w, halves, halves_w, sub-tiles,
 * sub-tiles_w, leaves = 7 dependent check levels, the least work) for calls that fill the chip,
 * the paired schedules (plain and weighted value of a group in one check launch: tiles ->
 * sub-tiles -> leaves, or tiles -> leaves) for small calls, which are bound by the chain of check
 * latencies (a rank's slice of an epoch under strong scaling).  Decisions are identical under
 * every schedule.  hbtc_check_schedule_for reports the schedule a call of n_tiles 64-share tiles
 * gets (the forced one, if any). */
#define HBTC_CHECK_AUTO (-1)
#define HBTC_CHECK_PLAIN_FIRST 0
#define HBTC_CHECK_PAIR_SUBS 1
#define HBTC_CHECK_PAIR_LEAVES 2
int hbtc_set_check_schedule(hbtc_ctx* ctx, int schedule);
int hbtc_check_schedule_for(hbtc_ctx* ctx, uint32_t n_tiles, int* schedule);
/* Number of shares that needed the exact single-share check in the last RLC call (syncs). */
int hbtc_rlc_last_leaves(hbtc_ctx* ctx, uint32_t* leaves);

/* ---- Reliable Broadcast coding (hbbft src/broadcast/) ------------------------------------- */
/* Reed-Solomon erasure code of reed-solomon-erasure 3.1 over GF(2^8) (0x11D), as hbbft's
 * Coding wraps it (broadcast.rs:395-459): k data + p parity shards, k + p <= 256 (ReedSolomon::new
 * refuses more: HBTC_ERR_ARG), every shard shard_len bytes.  Shards of one instance are
 * contiguous ((k + p) * shard_len bytes, shard i at i * shard_len: hbbft's padded value buffer,
 * broadcast.rs:171-178), instances back to back.
 * hbtc_rs_encode: ReedSolomon::encode — the p parity shards of every instance (in place).
 * hbtc_rs_reconstruct: ReedSolomon::reconstruct_shards — present[i * (k + p) + j] != 0 marks
 *   shard j of instance i present; the missing ones are computed from the first k present
 *   (in index order) and written in place; status[i] = HBTC_ACCEPT, or HBTC_NOT_ENOUGH_SHARES
 *   (TooFewShardsPresent: fewer than k present; the instance's bytes are left unchanged). */
int hbtc_rs_encode(hbtc_ctx* ctx, uint32_t data_shards, uint32_t parity_shards, uint32_t shard_len,
                   uint32_t n_inst, uint8_t* shards);
int hbtc_rs_reconstruct(hbtc_ctx* ctx, uint32_t data_shards, uint32_t parity_shards,
                        uint32_t shard_len, uint32_t n_inst, uint8_t* shards, const uint8_t* present,
                        int32_t* status);
/* Merkle trees of merkle.rs (MerkleTree::from_vec, merkle.rs:19-32): SHA3-256 leaves, pair
 * digests, an odd last digest carried up.  Per instance hbtc_merkle_digest_count(n_leaves)
 * digests of 32 bytes: level 0 (the n_leaves leaf digests), level 1, ..., the root last (the
 * levels MerkleTree::proof reads).  leaves: n_inst * n_leaves * leaf_len bytes. */
uint32_t hbtc_merkle_digest_count(uint32_t n_leaves);
int hbtc_merkle_trees(hbtc_ctx* ctx, uint32_t n_leaves, uint32_t leaf_len, uint32_t n_inst,
                      const uint8_t* leaves, uint8_t* digests);
/* Proof::validate(n_nodes) (merkle.rs:82-102) of n proofs: proof i has the value bytes
 * values[value_off[i] .. value_off[i + 1]), index[i], the digests
 * digests[32 * digest_off[i] .. 32 * digest_off[i + 1]) and root roots[32 * i ..].  status[i] =
 * HBTC_ACCEPT (valid) or HBTC_REJECT.  (The caller's index == sender check,
 * broadcast.rs:366, stays with the caller.) */
int hbtc_merkle_validate(hbtc_ctx* ctx, uint32_t n, uint32_t n_nodes, const uint64_t* value_off,
                         const uint8_t* values, const uint32_t* index, const uint32_t* digest_off,
                         const uint8_t* digests, const uint8_t* roots, int32_t* status);
/* Device-pointer forms (ordered on the context's streams like the other *_dev calls; present,
 * status of hbtc_rs_reconstruct_dev and the offsets' last entries stay host-side where noted:
 * present / status are HOST arrays, everything else device memory, digests 8-byte aligned). */
int hbtc_rs_encode_dev(hbtc_ctx* ctx, uint32_t data_shards, uint32_t parity_shards,
                       uint32_t shard_len, uint32_t n_inst, uint8_t* d_shards);
int hbtc_rs_reconstruct_dev(hbtc_ctx* ctx, uint32_t data_shards, uint32_t parity_shards,
                            uint32_t shard_len, uint32_t n_inst, uint8_t* d_shards,
                            const uint8_t* present, int32_t* status);
int hbtc_merkle_trees_dev(hbtc_ctx* ctx, uint32_t n_leaves, uint32_t leaf_len, uint32_t n_inst,
                          const uint8_t* d_leaves, uint8_t* d_digests);
int hbtc_merkle_validate_dev(hbtc_ctx* ctx, uint32_t n, uint32_t n_nodes, const uint64_t* d_value_off,
                             const uint8_t* d_values, const uint32_t* d_index,
                             const uint32_t* d_digest_off, const uint8_t* d_digests,
                             const uint8_t* d_roots, int32_t* d_status);

/* ---- kernel timing (HIP events on the context's stream) ---------------------------------- */
/* Families: "prepare", "dec_verify", "sig_verify", "pair_verify", "lagrange" (selection +
 * Lagrange coefficients), "comb_decode", "comb_digits", "combine" (MSM bucket reduction), "skg_scalars", "skg_ack_rows",
 * "mul", "rlc_items", "chk_tiles", "chk_tiles_w", "chk_halves", "chk_halves_w", "chk_subs",
 * "chk_subs_w", "chk_leaves", "rlc_finalize", "rs", "merkle",
 * "merkle_validate".  Reading
 * synchronises the stream. */
int hbtc_timing_enable(hbtc_ctx* ctx, int enable);
int hbtc_timing_read(hbtc_ctx* ctx, const char* family, double* total_ms, uint64_t* launches);
int hbtc_timing_reset(hbtc_ctx* ctx);

#ifdef __cplusplus
}
#endif

#endif /* HBTC_H */
