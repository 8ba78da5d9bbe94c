//! Rust binding of libhbtc, the MI355X batched verifier behind hbbft's threshold-crypto calls.
//!
//! `ffi` is generated from `include/hbtc.h` (tools/gen_rust_ffi.py; tests/test_abi.py fails when
//! it drifts).  The safe layer below is what hbbft's batch queues use: a `Context` per GPU (or a
//! `Node` over several), key sets loaded once per era, and CSR-shaped batches of compressed
//! points exactly as they arrive on the wire (G1 48 bytes, G2 96 bytes).
//!
//! Call-site mapping:
//!   Coin::handle_share -> PublicKeyShare::verify          verify_sig_shares   (src/coin.rs:151)
//!   Coin::try_output   -> combine_signatures + parity     combine_sigs        (src/coin.rs:185-191)
//!   ThresholdDecryption -> verify_decryption_share        verify_dec_shares   (src/threshold_decryption.rs:159)
//!   ThresholdDecryption -> PublicKeySet::decrypt          combine_dec         (src/threshold_decryption.rs:181-185)
//!   SyncKeyGen::handle_part / handle_ack                  skg_check_parts / skg_check_acks / decrypt
#![allow(clippy::too_many_arguments)]
pub mod ffi;
#[cfg(feature = "experimental-queues")]
pub mod queues;

use std::ffi::CStr;
use std::os::raw::c_int;
use std::ptr;

pub const ACCEPT: i32 = 0;
pub const REJECT: i32 = 1;
pub const DECODE_ERR: i32 = 2;
pub const UNKNOWN_SENDER: i32 = 3;
pub const INSTANCE_ERR: i32 = 4;
pub const NOT_ENOUGH_SHARES: i32 = 5;
pub const DUPLICATE_ENTRY: i32 = 6;

pub const MODE_PER_SHARE: c_int = 0;
pub const MODE_RLC: c_int = 1;

#[derive(Debug, Clone)]
pub struct Error {
    pub code: i32,
    pub message: String,
}

pub type Result<T> = std::result::Result<T, Error>;

/// A CSR batch: instance k owns items offsets[k] .. offsets[k + 1].
pub struct Batch<'a> {
    pub offsets: &'a [u32],
    pub idx: &'a [u32],
    pub items: &'a [u8],
}

impl<'a> Batch<'a> {
    fn check(&self, item_size: usize) {
        assert!(!self.offsets.is_empty() && self.offsets[0] == 0, "offsets[0] must be 0");
        assert!(self.offsets.windows(2).all(|w| w[0] <= w[1]), "offsets must be non-decreasing");
        let n = *self.offsets.last().unwrap() as usize;
        assert_eq!(self.idx.len(), n, "one node index per item");
        assert_eq!(self.items.len(), n * item_size, "item bytes");
    }
    fn n_inst(&self) -> u32 {
        (self.offsets.len() - 1) as u32
    }
    fn n_items(&self) -> usize {
        *self.offsets.last().unwrap() as usize
    }
}

/// One context on one GPU.  Calls are serialised inside the library (one mutex per context).
pub struct Context {
    raw: *mut ffi::hbtc_ctx,
}

unsafe impl Send for Context {}
unsafe impl Sync for Context {}

impl Context {
    pub fn new(device: i32) -> Result<Context> {
        let mut raw = ptr::null_mut();
        let rc = unsafe { ffi::hbtc_ctx_create(device, &mut raw) };
        if rc != 0 {
            return Err(Error { code: rc, message: format!("hbtc_ctx_create({})", device) });
        }
        Ok(Context { raw })
    }

    fn err(&self, rc: c_int) -> Error {
        let msg = unsafe { CStr::from_ptr(ffi::hbtc_last_error(self.raw)) };
        Error { code: rc, message: msg.to_string_lossy().into_owned() }
    }

    fn ok(&self, rc: c_int) -> Result<()> {
        if rc == 0 { Ok(()) } else { Err(self.err(rc)) }
    }

    /// NetworkInfo's public_key_share table (src/messaging.rs:253-256): (key set id, undecodable).
    pub fn keyset_load(&self, pk_shares_c48: &[u8]) -> Result<(u32, u32)> {
        assert_eq!(pk_shares_c48.len() % 48, 0);
        let (mut id, mut bad) = (0u32, 0u32);
        let n = (pk_shares_c48.len() / 48) as u32;
        self.ok(unsafe { ffi::hbtc_keyset_load(self.raw, pk_shares_c48.as_ptr(), n, &mut id, &mut bad) })?;
        Ok((id, bad))
    }

    pub fn keyset_free(&self, id: u32) -> Result<()> {
        self.ok(unsafe { ffi::hbtc_keyset_free(self.raw, id) })
    }

    pub fn set_verify_mode(&self, mode: c_int) -> Result<()> {
        self.ok(unsafe { ffi::hbtc_set_verify_mode(self.raw, mode) })
    }

    /// RLC scalar size: 128 (default) or 64 bits (soundness 2^-128 / 2^-64 per group check).
    pub fn set_rlc_bits(&self, bits: u32) -> Result<()> {
        self.ok(unsafe { ffi::hbtc_set_rlc_bits(self.raw, bits) })
    }

    /// Calls with fewer than `n_items` items get exact checks only, no RLC batch (default 256;
    /// 0 = always batch).  The decisions are the same either way.
    pub fn set_exact_below(&self, n_items: u32) -> Result<()> {
        self.ok(unsafe { ffi::hbtc_set_exact_below(self.raw, n_items) })
    }

    /// PublicKeyShare::verify for every SignatureShare of every coin instance (H = hash_g2(nonce)).
    pub fn verify_sig_shares(&self, keyset: u32, h_c96: &[u8], b: &Batch) -> Result<Vec<i32>> {
        b.check(96);
        assert_eq!(h_c96.len(), 96 * b.n_inst() as usize);
        let mut st = vec![0i32; b.n_items()];
        self.ok(unsafe {
            ffi::hbtc_verify_sig_shares(self.raw, keyset, b.n_inst(), h_c96.as_ptr(), b.offsets.as_ptr(),
                                        b.idx.as_ptr(), b.items.as_ptr(), st.as_mut_ptr())
        })?;
        Ok(st)
    }

    /// verify_decryption_share for every DecryptionShare (H = hash_g1_g2(u, v), w per ciphertext).
    pub fn verify_dec_shares(&self, keyset: u32, h_c96: &[u8], w_c96: &[u8], b: &Batch) -> Result<Vec<i32>> {
        b.check(48);
        assert_eq!(h_c96.len(), 96 * b.n_inst() as usize);
        assert_eq!(w_c96.len(), 96 * b.n_inst() as usize);
        let mut st = vec![0i32; b.n_items()];
        self.ok(unsafe {
            ffi::hbtc_verify_dec_shares(self.raw, keyset, b.n_inst(), h_c96.as_ptr(), w_c96.as_ptr(),
                                        b.offsets.as_ptr(), b.idx.as_ptr(), b.items.as_ptr(), st.as_mut_ptr())
        })?;
        Ok(st)
    }

    /// PublicKey::verify for n (pk, H, sigma) triples: e(pk, H) == e(G1, sigma) (src/coin.rs:192-197).
    pub fn verify_sigs(&self, pk_c48: &[u8], h_c96: &[u8], sig_c96: &[u8]) -> Result<Vec<i32>> {
        assert_eq!(pk_c48.len() % 48, 0);
        let n = pk_c48.len() / 48;
        assert_eq!(h_c96.len(), 96 * n, "one H per signature");
        assert_eq!(sig_c96.len(), 96 * n, "one signature per key");
        let mut st = vec![0i32; n];
        self.ok(unsafe {
            ffi::hbtc_verify_sigs(self.raw, n as u32, pk_c48.as_ptr(), h_c96.as_ptr(), sig_c96.as_ptr(),
                                  st.as_mut_ptr())
        })?;
        Ok(st)
    }

    /// Ciphertext::verify for n (u, H, w) triples: e(G1, w) == e(u, H) (src/threshold_decryption.rs:98).
    pub fn verify_ciphertexts(&self, u_c48: &[u8], h_c96: &[u8], w_c96: &[u8]) -> Result<Vec<i32>> {
        assert_eq!(u_c48.len() % 48, 0);
        let n = u_c48.len() / 48;
        assert_eq!(h_c96.len(), 96 * n, "one H per ciphertext");
        assert_eq!(w_c96.len(), 96 * n, "one w per ciphertext");
        let mut st = vec![0i32; n];
        self.ok(unsafe {
            ffi::hbtc_verify_ciphertexts(self.raw, n as u32, u_c48.as_ptr(), h_c96.as_ptr(), w_c96.as_ptr(),
                                         st.as_mut_ptr())
        })?;
        Ok(st)
    }

    /// BivarCommitment::row(x) == row.commitment() for every Part (x = our_idx + 1): commits holds
    /// per Part the (t+1)(t+2)/2 compressed points, rows per Part t+1 Fr (32-byte LE each).
    pub fn skg_check_parts(&self, t: u32, our_idx: u32, commits_c48: &[u8], rows_le32: &[u8]) -> Result<Vec<i32>> {
        let m = ((t + 1) * (t + 2) / 2) as usize;
        assert_eq!(commits_c48.len() % (48 * m), 0);
        let n_parts = commits_c48.len() / (48 * m);
        assert_eq!(rows_le32.len(), 32 * (t as usize + 1) * n_parts, "t + 1 row coefficients per Part");
        let mut st = vec![0i32; n_parts];
        self.ok(unsafe {
            ffi::hbtc_skg_check_parts(self.raw, n_parts as u32, t, our_idx, commits_c48.as_ptr(), rows_le32.as_ptr(),
                                      st.as_mut_ptr())
        })?;
        Ok(st)
    }

    /// BivarCommitment::evaluate(x, y) == val G1 for every Ack value (x = our_idx + 1, y = sender
    /// + 1), against Part ack_part[i]'s commitment; row_ok[p] != 0: Part p's verified row (rows)
    /// gives the scalar fast path.
    pub fn skg_check_acks(&self, t: u32, our_idx: u32, commits_c48: &[u8], rows_le32: &[u8], row_ok: &[u8],
                          ack_part: &[u32], ack_sender: &[u32], vals_le32: &[u8]) -> Result<Vec<i32>> {
        let m = ((t + 1) * (t + 2) / 2) as usize;
        assert_eq!(commits_c48.len() % (48 * m), 0);
        let n_parts = commits_c48.len() / (48 * m);
        assert_eq!(rows_le32.len(), 32 * (t as usize + 1) * n_parts);
        assert_eq!(row_ok.len(), n_parts);
        let n = ack_part.len();
        assert!(ack_part.iter().all(|&p| (p as usize) < n_parts), "ack_part out of range");
        assert_eq!(ack_sender.len(), n);
        assert_eq!(vals_le32.len(), 32 * n);
        let mut st = vec![0i32; n];
        self.ok(unsafe {
            ffi::hbtc_skg_check_acks(self.raw, n_parts as u32, t, our_idx, commits_c48.as_ptr(), rows_le32.as_ptr(),
                                     row_ok.as_ptr(), n as u32, ack_part.as_ptr(), ack_sender.as_ptr(),
                                     vals_le32.as_ptr(), st.as_mut_ptr())
        })?;
        Ok(st)
    }

    /// combine_signatures over the first t shares of every instance: (signatures, parities, status).
    pub fn combine_sigs(&self, b: &Batch, t: u32) -> Result<(Vec<u8>, Vec<u8>, Vec<i32>)> {
        b.check(96);
        let n = b.n_inst() as usize;
        let (mut out, mut par, mut st) = (vec![0u8; 96 * n], vec![0u8; n], vec![0i32; n]);
        self.ok(unsafe {
            ffi::hbtc_combine_sigs(self.raw, b.n_inst(), b.offsets.as_ptr(), b.idx.as_ptr(), b.items.as_ptr(), t,
                                   out.as_mut_ptr(), par.as_mut_ptr(), st.as_mut_ptr())
        })?;
        Ok((out, par, st))
    }

    /// PublicKeySet::decrypt's interpolation: g per ciphertext (plaintext = v ^ hash_bytes(g)).
    pub fn combine_dec(&self, b: &Batch, t: u32) -> Result<(Vec<u8>, Vec<i32>)> {
        b.check(48);
        let n = b.n_inst() as usize;
        let (mut out, mut st) = (vec![0u8; 48 * n], vec![0i32; n]);
        self.ok(unsafe {
            ffi::hbtc_combine_dec(self.raw, b.n_inst(), b.offsets.as_ptr(), b.idx.as_ptr(), b.items.as_ptr(), t,
                                  out.as_mut_ptr(), st.as_mut_ptr())
        })?;
        Ok((out, st))
    }

    /// SecretKey::decrypt for a batch under one key: (plaintexts in the msgs layout, status).
    pub fn decrypt(&self, sk_le32: &[u8; 32], u_c48: &[u8], w_c96: &[u8], msgs: &[u8], offsets: &[u32])
        -> Result<(Vec<u8>, Vec<i32>)> {
        assert!(!offsets.is_empty() && offsets[0] == 0, "offsets[0] must be 0");
        assert!(offsets.windows(2).all(|w| w[0] <= w[1]), "offsets must be non-decreasing");
        let n = offsets.len() - 1;
        assert!(offsets[n] as usize <= msgs.len(), "offsets past the message bytes");
        assert_eq!(u_c48.len(), 48 * n, "one compressed G1 u per ciphertext");
        assert_eq!(w_c96.len(), 96 * n, "one compressed G2 w per ciphertext");
        let (mut out, mut st) = (vec![0u8; msgs.len()], vec![0i32; n]);
        self.ok(unsafe {
            ffi::hbtc_decrypt(self.raw, n as u32, sk_le32.as_ptr(), u_c48.as_ptr(), w_c96.as_ptr(), msgs.as_ptr(),
                              offsets.as_ptr(), out.as_mut_ptr(), st.as_mut_ptr())
        })?;
        Ok((out, st))
    }
}

impl Drop for Context {
    fn drop(&mut self) {
        unsafe { ffi::hbtc_ctx_destroy(self.raw) }
    }
}

/// One hbbft node over several GPUs (strong scaling of one epoch).
pub struct Node {
    raw: *mut ffi::hbtc_node,
}

unsafe impl Send for Node {}
unsafe impl Sync for Node {}

impl Node {
    pub fn new(devices: &[i32]) -> Result<Node> {
        let mut raw = ptr::null_mut();
        let rc = unsafe { ffi::hbtc_node_create(devices.len() as c_int, devices.as_ptr(), &mut raw) };
        if rc != 0 {
            return Err(Error { code: rc, message: "hbtc_node_create".into() });
        }
        Ok(Node { raw })
    }

    fn ok(&self, rc: c_int) -> Result<()> {
        if rc == 0 {
            return Ok(());
        }
        let msg = unsafe { CStr::from_ptr(ffi::hbtc_node_last_error(self.raw)) };
        Err(Error { code: rc, message: msg.to_string_lossy().into_owned() })
    }

    pub fn keyset_load(&self, pk_shares_c48: &[u8]) -> Result<(u32, u32)> {
        assert_eq!(pk_shares_c48.len() % 48, 0);
        let (mut id, mut bad) = (0u32, 0u32);
        self.ok(unsafe {
            ffi::hbtc_node_keyset_load(self.raw, pk_shares_c48.as_ptr(), (pk_shares_c48.len() / 48) as u32, &mut id,
                                       &mut bad)
        })?;
        Ok((id, bad))
    }

    pub fn verify_dec_shares(&self, keyset: u32, h_c96: &[u8], w_c96: &[u8], b: &Batch) -> Result<Vec<i32>> {
        b.check(48);
        assert_eq!(h_c96.len(), 96 * b.n_inst() as usize);
        assert_eq!(w_c96.len(), 96 * b.n_inst() as usize);
        let mut st = vec![0i32; b.n_items()];
        self.ok(unsafe {
            ffi::hbtc_node_verify_dec_shares(self.raw, keyset, b.n_inst(), h_c96.as_ptr(), w_c96.as_ptr(),
                                             b.offsets.as_ptr(), b.idx.as_ptr(), b.items.as_ptr(), st.as_mut_ptr())
        })?;
        Ok(st)
    }

    pub fn verify_sig_shares(&self, keyset: u32, h_c96: &[u8], b: &Batch) -> Result<Vec<i32>> {
        b.check(96);
        assert_eq!(h_c96.len(), 96 * b.n_inst() as usize);
        let mut st = vec![0i32; b.n_items()];
        self.ok(unsafe {
            ffi::hbtc_node_verify_sig_shares(self.raw, keyset, b.n_inst(), h_c96.as_ptr(), b.offsets.as_ptr(),
                                             b.idx.as_ptr(), b.items.as_ptr(), st.as_mut_ptr())
        })?;
        Ok(st)
    }
}

impl Drop for Node {
    fn drop(&mut self) {
        unsafe { ffi::hbtc_node_destroy(self.raw) }
    }
}

/// threshold_crypto's hash_g2(msg) (host).
pub fn hash_g2(msg: &[u8]) -> [u8; 96] {
    let mut out = [0u8; 96];
    unsafe { ffi::hbtc_hash_g2(msg.as_ptr(), msg.len(), out.as_mut_ptr()) };
    out
}
