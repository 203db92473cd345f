//! `ic-verify-bls-signature` (utils/verify-bls-signatures/src/lib.rs) for
//! node-side (std) callers, backed by the MI355X batch verifier through the C
//! ABI in include/cess_bls.h.  Same public names and error behaviour as the
//! reference crate, plus `verify_batch` and the multi-GPU entry points.  The
//! no_std wasm runtime keeps the original crate.
//!
//! NOT COMPILED in this repository's image (cargo/rustc are absent there);
//! every call maps 1:1 onto a C entry point that the repository's ctypes
//! mirror (cess_amd/bls.py) and C test program (tests/c/cabi_golden.c)
//! exercise on MI355X.
//!
//! There is no CPU fallback: without a HIP device `Verifier::new` returns
//! `Error::NoDevice` and the free functions panic (a node configured for GPU
//! verification must not silently degrade).

mod ffi;

use core::ffi::{c_int, c_void, CStr};
use std::sync::{Mutex, OnceLock};

/// Infrastructure failure (never a verdict).
#[derive(Clone, Copy, Debug, Eq, PartialEq)]
pub enum Error {
    InvalidArg,
    NoDevice,
    Hip,
    OutOfMemory,
    Rccl,
    Busy,
    BadKey,
    BadSig,
    NoComm,
    /// shared-memory communicator: a peer timed out / the transport failed
    Comm,
    /// RSA: the key parses (the reference accepts it) but the GPU cannot
    /// verify it (even modulus, n < 3, non-NULL SPKI parameters); the
    /// caller's own path decides (include/cess_rsa.h)
    Unsupported,
    Other(i32),
}

impl Error {
    fn from_status(st: c_int) -> Self {
        match st {
            ffi::CESS_BLS_E_INVALID_ARG => Error::InvalidArg,
            ffi::CESS_BLS_E_NO_DEVICE => Error::NoDevice,
            ffi::CESS_BLS_E_HIP => Error::Hip,
            ffi::CESS_BLS_E_OOM => Error::OutOfMemory,
            ffi::CESS_BLS_E_RCCL => Error::Rccl,
            ffi::CESS_BLS_E_BUSY => Error::Busy,
            ffi::CESS_BLS_E_BAD_KEY => Error::BadKey,
            ffi::CESS_BLS_E_BAD_SIG => Error::BadSig,
            ffi::CESS_BLS_E_NO_COMM => Error::NoComm,
            ffi::CESS_BLS_E_COMM => Error::Comm,
            ffi::CESS_RSA_E_UNSUPPORTED => Error::Unsupported,
            s => Error::Other(s),
        }
    }
    pub fn message(self) -> String {
        let st = match self {
            Error::InvalidArg => ffi::CESS_BLS_E_INVALID_ARG,
            Error::NoDevice => ffi::CESS_BLS_E_NO_DEVICE,
            Error::Hip => ffi::CESS_BLS_E_HIP,
            Error::OutOfMemory => ffi::CESS_BLS_E_OOM,
            Error::Rccl => ffi::CESS_BLS_E_RCCL,
            Error::Busy => ffi::CESS_BLS_E_BUSY,
            Error::BadKey => ffi::CESS_BLS_E_BAD_KEY,
            Error::BadSig => ffi::CESS_BLS_E_BAD_SIG,
            Error::NoComm => ffi::CESS_BLS_E_NO_COMM,
            Error::Comm => ffi::CESS_BLS_E_COMM,
            Error::Unsupported => ffi::CESS_RSA_E_UNSUPPORTED,
            Error::Other(s) => s,
        };
        unsafe { CStr::from_ptr(ffi::cess_bls_status_string(st)) }.to_string_lossy().into_owned()
    }
}

fn check(st: c_int) -> Result<(), Error> {
    if st == ffi::CESS_BLS_OK {
        Ok(())
    } else {
        Err(Error::from_status(st))
    }
}

/// Per-record verdict codes (include/cess_bls.h): 0 OK, 1 SIG_LEN, 2 SIG_POINT,
/// 3 PK_LEN, 4 PK_POINT, 5 PAIRING_FAIL; precedence signature, key, pairing
/// (src/lib.rs:244-246).  Codes 1..5 are the reference's `Err(())`.
#[derive(Clone, Debug, Eq, PartialEq)]
pub struct Verdicts {
    /// bit i % 64 of word i / 64 (LSB first) = record i verified
    pub bitmap: Vec<u64>,
    pub codes: Vec<u8>,
}

impl Verdicts {
    pub fn ok(&self, i: usize) -> bool {
        (self.bitmap[i / 64] >> (i % 64)) & 1 == 1
    }
    pub fn all_ok(&self) -> bool {
        self.codes.iter().all(|&c| c == ffi::CODE_OK)
    }
}

/// Context configuration (cess_bls_config).
#[derive(Clone, Debug)]
pub struct Config {
    pub device: i32,
    pub max_batch: u64,
    pub profile: bool,
    /// reject identity public keys (IETF KeyValidate); off = reference behaviour
    pub strict_identity: bool,
    /// what `verify_batch` runs: per-signature (default) or RLC with bisection
    pub rlc: bool,
    /// RLC for batches of distinct keys: one pairing per record, the Miller
    /// values kept for bisection (CESS_BLS_F_RLC_DISTINCT)
    pub rlc_distinct: bool,
    /// several GPUs of this process (host batches sharded across them)
    pub devices: Vec<i32>,
}

impl Default for Config {
    fn default() -> Self {
        Config { device: 0, max_batch: 1 << 20, profile: false, strict_identity: false, rlc: false, rlc_distinct: false,
                 devices: vec![] }
    }
}

/// One context (one GPU, or several with `Config::devices`).  A context is
/// used by one thread at a time: `Verifier` is `Send`, not `Sync`.
pub struct Verifier {
    ctx: *mut ffi::cess_bls_ctx,
    _devices: Vec<c_int>,
    // rank count given to comm_init / comm_init_shm (0: no communicator): the
    // C side writes that many bus ids in cess_bls_comm_info
    comm_nranks: i32,
}

unsafe impl Send for Verifier {}

fn offsets<'a, I: Iterator<Item = &'a [u8]>>(parts: I, data: &mut Vec<u8>) -> Vec<u64> {
    let mut o = vec![0u64];
    for p in parts {
        data.extend_from_slice(p);
        o.push(data.len() as u64);
    }
    o
}

impl Verifier {
    pub fn new(cfg: &Config) -> Result<Self, Error> {
        let devices: Vec<c_int> = cfg.devices.iter().map(|&d| d as c_int).collect();
        let c = ffi::cess_bls_config {
            device: cfg.device as c_int,
            max_batch: cfg.max_batch,
            flags: (if cfg.profile { ffi::CESS_BLS_F_PROFILE } else { 0 })
                | (if cfg.strict_identity { ffi::CESS_BLS_F_STRICT_IDENTITY } else { 0 })
                | (if cfg.rlc_distinct { ffi::CESS_BLS_F_RLC_DISTINCT } else { 0 }),
            mode: if cfg.rlc { ffi::CESS_BLS_MODE_RLC } else { ffi::CESS_BLS_MODE_PER_SIG },
            n_devices: if devices.len() > 1 { devices.len() as c_int } else { 0 },
            devices: if devices.len() > 1 { devices.as_ptr() } else { core::ptr::null() },
        };
        let mut p = core::ptr::null_mut();
        check(unsafe { ffi::cess_bls_ctx_create(&c, &mut p) })?;
        Ok(Verifier { ctx: p, _devices: devices, comm_nranks: 0 })
    }

    /// `verify_bls_signature(sig, msg, key)` (src/lib.rs:243-247) -> verdict code.
    pub fn verify_code(&mut self, sig: &[u8], msg: &[u8], key: &[u8]) -> Result<u8, Error> {
        let mut code = 0xffu8;
        check(unsafe {
            ffi::cess_bls_verify(self.ctx, sig.as_ptr(), sig.len(), msg.as_ptr(), msg.len(), key.as_ptr(), key.len(),
                                 &mut code)
        })?;
        Ok(code)
    }

    /// New: one call for a batch of (sig, msg, key) records of any lengths.
    pub fn verify_batch(&mut self, records: &[(&[u8], &[u8], &[u8])]) -> Result<Verdicts, Error> {
        let n = records.len();
        let mut v = Verdicts { bitmap: vec![0; (n + 63) / 64], codes: vec![0; n] };
        if n == 0 {
            return Ok(v);
        }
        let fixed = records.iter().all(|r| r.0.len() == 48 && r.2.len() == 96);
        let (mut sd, mut pd, mut md) = (Vec::new(), Vec::new(), Vec::new());
        let mo = offsets(records.iter().map(|r| r.1), &mut md);
        if fixed {
            for r in records {
                sd.extend_from_slice(r.0);
                pd.extend_from_slice(r.2);
            }
            check(unsafe {
                ffi::cess_bls_verify_batch(self.ctx, n, sd.as_ptr(), pd.as_ptr(), md.as_ptr(), mo.as_ptr(),
                                           v.codes.as_mut_ptr(), v.bitmap.as_mut_ptr())
            })?;
        } else {
            let so = offsets(records.iter().map(|r| r.0), &mut sd);
            let po = offsets(records.iter().map(|r| r.2), &mut pd);
            check(unsafe {
                ffi::cess_bls_verify_batch_var(self.ctx, n, sd.as_ptr(), so.as_ptr(), pd.as_ptr(), po.as_ptr(),
                                               md.as_ptr(), mo.as_ptr(), v.codes.as_mut_ptr(), v.bitmap.as_mut_ptr())
            })?;
        }
        Ok(v)
    }

    /// RLC batch mode over fixed-stride records; the library draws the seed
    /// from the OS CSPRNG (it must be secret and unpredictable to the signers).
    pub fn verify_batch_rlc(&mut self, sigs: &[u8], pks: &[u8], msgs: &[u8], msg_offsets: &[u64])
                            -> Result<Verdicts, Error> {
        let n = sigs.len() / 48;
        assert!(sigs.len() == 48 * n && pks.len() == 96 * n && msg_offsets.len() == n + 1);
        let mut v = Verdicts { bitmap: vec![0; (n + 63) / 64], codes: vec![0; n] };
        check(unsafe {
            ffi::cess_bls_verify_batch_rlc(self.ctx, n, sigs.as_ptr(), pks.as_ptr(), msgs.as_ptr(),
                                           msg_offsets.as_ptr(), core::ptr::null(), v.codes.as_mut_ptr(),
                                           v.bitmap.as_mut_ptr(), core::ptr::null_mut())
        })?;
        Ok(v)
    }

    /// Distinct-key table: decode + G2Prepared once per key; per-key codes.
    pub fn load_keys(&mut self, keys: &[[u8; 96]]) -> Result<Vec<u8>, Error> {
        let flat: Vec<u8> = keys.iter().flat_map(|k| k.iter().copied()).collect();
        let mut codes = vec![0u8; keys.len()];
        check(unsafe { ffi::cess_bls_keys_load(self.ctx, keys.len(), flat.as_ptr(), codes.as_mut_ptr()) })?;
        Ok(codes)
    }

    /// Per-signature verdicts against loaded keys (same codes as verify_batch).
    pub fn verify_batch_keyed(&mut self, sigs: &[u8], key_idx: &[u32], msgs: &[u8], msg_offsets: &[u64])
                              -> Result<Verdicts, Error> {
        let n = key_idx.len();
        assert!(sigs.len() == 48 * n && msg_offsets.len() == n + 1);
        let mut v = Verdicts { bitmap: vec![0; (n + 63) / 64], codes: vec![0; n] };
        check(unsafe {
            ffi::cess_bls_verify_batch_keyed(self.ctx, n, sigs.as_ptr(), key_idx.as_ptr(), msgs.as_ptr(),
                                             msg_offsets.as_ptr(), v.codes.as_mut_ptr(), v.bitmap.as_mut_ptr())
        })?;
        Ok(v)
    }

    // --- one process per GPU (RCCL communicator in the context) ---------------
    /// ncclGetUniqueId on one rank; distribute the bytes to all ranks out of band.
    pub fn comm_id() -> Result<[u8; ffi::CESS_BLS_COMM_ID_BYTES], Error> {
        let mut id = [0u8; ffi::CESS_BLS_COMM_ID_BYTES];
        check(unsafe { ffi::cess_bls_comm_id(id.as_mut_ptr()) })?;
        Ok(id)
    }
    /// ncclCommInitRank on this context's GPU (collective).
    pub fn comm_init(&mut self, nranks: i32, rank: i32, id: &[u8; ffi::CESS_BLS_COMM_ID_BYTES]) -> Result<(), Error> {
        check(unsafe { ffi::cess_bls_comm_init(self.ctx, nranks, rank, id.as_ptr()) })?;
        self.comm_nranks = nranks;
        Ok(())
    }
    /// Every rank passes the whole fixed-stride batch and gets all verdicts.
    pub fn verify_batch_sharded(&mut self, sigs: &[u8], pks: &[u8], msgs: &[u8], msg_offsets: &[u64])
                                -> Result<Verdicts, Error> {
        let n = sigs.len() / 48;
        assert!(sigs.len() == 48 * n && pks.len() == 96 * n && msg_offsets.len() == n + 1);
        let mut v = Verdicts { bitmap: vec![0; (n + 63) / 64], codes: vec![0; n] };
        check(unsafe {
            ffi::cess_bls_verify_batch_sharded(self.ctx, n, sigs.as_ptr(), pks.as_ptr(), msgs.as_ptr(),
                                               msg_offsets.as_ptr(), v.codes.as_mut_ptr(), v.bitmap.as_mut_ptr())
        })?;
        Ok(v)
    }
    /// `verify_batch` over the communicator for records of any lengths: this
    /// rank verifies its index shard, every rank receives all verdicts.
    pub fn verify_batch_var_sharded(&mut self, records: &[(&[u8], &[u8], &[u8])]) -> Result<Verdicts, Error> {
        let n = records.len();
        let mut v = Verdicts { bitmap: vec![0; (n + 63) / 64], codes: vec![0; n] };
        let (mut sd, mut pd, mut md) = (Vec::new(), Vec::new(), Vec::new());
        let so = offsets(records.iter().map(|r| r.0), &mut sd);
        let po = offsets(records.iter().map(|r| r.2), &mut pd);
        let mo = offsets(records.iter().map(|r| r.1), &mut md);
        check(unsafe {
            ffi::cess_bls_verify_batch_var_sharded(self.ctx, n, sd.as_ptr(), so.as_ptr(), pd.as_ptr(), po.as_ptr(),
                                                   md.as_ptr(), mo.as_ptr(), v.codes.as_mut_ptr(),
                                                   v.bitmap.as_mut_ptr())
        })?;
        Ok(v)
    }
    /// What the communicator reports: (rank count, own rank, each rank's PCI
    /// bus id in rank order).  Collective: call it on every rank.  ONE call to
    /// cess_bls_comm_info with the buffer sized from the rank count given at
    /// init (what the C side writes), so a rank whose local query fails still
    /// joins the collective and its peers never wait for it until the comm
    /// deadline.
    pub fn comm_info(&mut self) -> Result<(i32, i32, Vec<String>), Error> {
        if self.comm_nranks <= 0 {
            return Err(Error::NoComm);
        }
        let (mut nr, mut rk) = (0 as c_int, 0 as c_int);
        let mut buf = vec![0 as core::ffi::c_char; self.comm_nranks as usize * ffi::CESS_BLS_BUS_ID_BYTES];
        check(unsafe { ffi::cess_bls_comm_info(self.ctx, &mut nr, &mut rk, buf.as_mut_ptr()) })?;
        let ids = buf
            .chunks(ffi::CESS_BLS_BUS_ID_BYTES)
            .map(|c| unsafe { CStr::from_ptr(c.as_ptr()) }.to_string_lossy().into_owned())
            .collect();
        Ok((nr, rk, ids))
    }
    /// Host shared-memory transport instead of RCCL (ranks on one host, which
    /// may share a GPU); `name` from `Verifier::comm_shm_name` on one rank.
    pub fn comm_init_shm(&mut self, nranks: i32, rank: i32, name: &CStr) -> Result<(), Error> {
        check(unsafe { ffi::cess_bls_comm_init_shm(self.ctx, nranks, rank, name.as_ptr()) })?;
        self.comm_nranks = nranks;
        Ok(())
    }
    pub fn comm_shm_name() -> Result<std::ffi::CString, Error> {
        let mut buf = [0 as core::ffi::c_char; ffi::CESS_BLS_COMM_NAME_BYTES];
        check(unsafe { ffi::cess_bls_comm_shm_name(buf.as_mut_ptr()) })?;
        Ok(unsafe { CStr::from_ptr(buf.as_ptr()) }.to_owned())
    }
    /// Records [begin, end) of `rank`'s shard and the bitmap words per rank.
    pub fn shard_range(n: u64, nranks: i32, rank: i32) -> Result<(u64, u64, u64), Error> {
        let (mut b, mut e, mut w) = (0u64, 0u64, 0u64);
        check(unsafe { ffi::cess_bls_shard_range(n, nranks, rank, &mut b, &mut e, &mut w) })?;
        Ok((b, e, w))
    }

    /// Signature::deserialize / PublicKey::deserialize over a batch, decode
    /// kernels only (no pairing): codes 0, SIG_LEN / SIG_POINT or PK_LEN / PK_POINT.
    pub fn deserialize_codes(&mut self, kind: c_int, encodings: &[&[u8]]) -> Result<Vec<u8>, Error> {
        let mut data = Vec::new();
        let o = offsets(encodings.iter().copied(), &mut data);
        let mut codes = vec![0u8; encodings.len()];
        if encodings.is_empty() {
            return Ok(codes);
        }
        check(unsafe {
            ffi::cess_bls_deserialize_batch(self.ctx, kind, encodings.len(), data.as_ptr(), o.as_ptr(),
                                            codes.as_mut_ptr())
        })?;
        Ok(codes)
    }

    /// `cp_enclave_verify::verify_bls(key, msg, sig)` without the panics.
    pub fn enclave_verify_bls(&mut self, key: &[u8], msg: &[u8], sig: &[u8]) -> Result<bool, Error> {
        let mut ok: c_int = 0;
        check(unsafe {
            ffi::cess_bls_enclave_verify_bls(self.ctx, key.as_ptr(), key.len(), msg.as_ptr(), msg.len(), sig.as_ptr(),
                                             sig.len(), &mut ok)
        })?;
        Ok(ok != 0)
    }

    // --- RSA PKCS#1 v1.5 raw (include/cess_rsa.h) ------------------------------
    /// `cp_enclave_verify::verify_rsa(key, msg, sig)` (primitives/enclave-verify/
    /// src/lib.rs:221-228) without the panic: `Err(Error::BadKey)` where
    /// `from_public_key_der(key).unwrap()` would panic.
    pub fn verify_rsa(&mut self, key_der: &[u8], msg: &[u8], sig: &[u8]) -> Result<bool, Error> {
        let mut ok: c_int = 0;
        check(unsafe {
            ffi::cess_rsa_verify(self.ctx, key_der.as_ptr(), key_der.len(), msg.as_ptr(), msg.len(), sig.as_ptr(),
                                 sig.len(), &mut ok)
        })?;
        Ok(ok != 0)
    }

    /// Load a distinct-key table of DER keys (`format`: ffi::CESS_RSA_KEY_SPKI or
    /// ffi::CESS_RSA_KEY_PKCS1, the latter for Podr2Key = [u8; 270]); returns
    /// the per-key load status.
    pub fn rsa_keys_load(&mut self, ders: &[&[u8]], format: i32) -> Result<Vec<i32>, Error> {
        let mut data = Vec::new();
        let o = offsets(ders.iter().copied(), &mut data);
        let mut st = vec![0 as c_int; ders.len()];
        check(unsafe {
            ffi::cess_rsa_keys_load(self.ctx, ders.len(), data.as_ptr(), o.as_ptr(), format as c_int, st.as_mut_ptr())
        })?;
        Ok(st.into_iter().map(|x| x as i32).collect())
    }

    /// verify_rsa over a batch against the loaded key table: record i =
    /// (key key_idx[i], msgs[i], sigs[i]); codes 0 OK, 1 SIG_LEN, 2 SIG_RANGE,
    /// 3 MSG_LEN, 4 MISMATCH, 5 KEY (codes 1..5 are the reference's `false`).
    pub fn verify_rsa_batch(&mut self, key_idx: &[u32], msgs: &[&[u8]], sigs: &[&[u8]]) -> Result<Verdicts, Error> {
        assert!(key_idx.len() == msgs.len() && msgs.len() == sigs.len());
        let n = key_idx.len();
        let (mut md, mut sd) = (Vec::new(), Vec::new());
        let mo = offsets(msgs.iter().copied(), &mut md);
        let so = offsets(sigs.iter().copied(), &mut sd);
        let mut codes = vec![0u8; n];
        let mut bitmap = vec![0u64; (n + 63) / 64];
        check(unsafe {
            ffi::cess_rsa_verify_batch(self.ctx, n, key_idx.as_ptr(), sd.as_ptr(), so.as_ptr(), md.as_ptr(),
                                       mo.as_ptr(), codes.as_mut_ptr(), bitmap.as_mut_ptr())
        })?;
        Ok(Verdicts { bitmap, codes })
    }

    // --- generators (PrivateKey::public_key / sign, src/lib.rs:226-236) -------
    pub fn public_keys(&mut self, sks: &[[u8; 32]]) -> Result<Vec<[u8; 96]>, Error> {
        let flat: Vec<u8> = sks.iter().flat_map(|k| k.iter().copied()).collect();
        let mut out = vec![0u8; 96 * sks.len()];
        check(unsafe { ffi::cess_bls_public_key_batch(self.ctx, sks.len(), flat.as_ptr(), out.as_mut_ptr()) })?;
        Ok(out.chunks(96).map(|c| c.try_into().unwrap()).collect())
    }
    pub fn sign(&mut self, sks: &[[u8; 32]], msgs: &[&[u8]]) -> Result<Vec<[u8; 48]>, Error> {
        let flat: Vec<u8> = sks.iter().flat_map(|k| k.iter().copied()).collect();
        let mut md = Vec::new();
        let mo = offsets(msgs.iter().copied(), &mut md);
        let mut out = vec![0u8; 48 * sks.len()];
        check(unsafe {
            ffi::cess_bls_sign_batch(self.ctx, sks.len(), flat.as_ptr(), md.as_ptr(), mo.as_ptr(), out.as_mut_ptr())
        })?;
        Ok(out.chunks(48).map(|c| c.try_into().unwrap()).collect())
    }

    /// Device memory on this context's GPU, for device-resident batches.
    pub fn device_alloc(&mut self, bytes: usize) -> Result<*mut c_void, Error> {
        let mut p = core::ptr::null_mut();
        check(unsafe { ffi::cess_bls_device_alloc(self.ctx, bytes, &mut p) })?;
        Ok(p)
    }
}

impl Drop for Verifier {
    fn drop(&mut self) {
        unsafe { ffi::cess_bls_ctx_destroy(self.ctx) }
    }
}

// ---------------------------------------------------------------------------
// The reference crate's API (src/lib.rs), over one process-wide context.
// ---------------------------------------------------------------------------
static DEFAULT: OnceLock<Mutex<Verifier>> = OnceLock::new();

fn with_default<R>(f: impl FnOnce(&mut Verifier) -> R) -> R {
    let m = DEFAULT.get_or_init(|| {
        Mutex::new(Verifier::new(&Config::default()).expect("MI355X verifier: no HIP device (no CPU fallback)"))
    });
    let mut v = m.lock().unwrap();
    f(&mut v)
}

#[derive(Copy, Clone, Debug, Eq, PartialEq)]
pub enum InvalidPublicKey {
    WrongLength,
    InvalidPoint,
}

#[derive(Copy, Clone, Debug, Eq, PartialEq)]
pub enum InvalidSignature {
    WrongLength,
    InvalidPoint,
}

#[derive(Copy, Clone, Debug, Eq, PartialEq)]
pub enum InvalidPrivateKey {
    WrongLength,
    OutOfRange,
}

/// `PublicKey` (src/lib.rs:33-101): a checked 96-byte compressed G2 point.
#[derive(Clone, Eq, PartialEq)]
pub struct PublicKey {
    raw: [u8; 96],
}

impl PublicKey {
    pub const BYTES: usize = 96;
    /// PublicKey::deserialize (src/lib.rs:68-82): decode + subgroup check on the GPU.
    pub fn deserialize(bytes: &[u8]) -> Result<Self, InvalidPublicKey> {
        if bytes.len() != Self::BYTES {
            return Err(InvalidPublicKey::WrongLength);
        }
        // decode kernels only (cess_bls_deserialize_batch): a decode's latency,
        // not a whole verification's
        let code = with_default(|v| v.deserialize_codes(ffi::CESS_BLS_KIND_PK, &[bytes])).expect("verifier")[0];
        if code == ffi::CODE_PK_POINT {
            return Err(InvalidPublicKey::InvalidPoint);
        }
        Ok(PublicKey { raw: bytes.try_into().unwrap() })
    }
    pub fn serialize(&self) -> [u8; 96] {
        self.raw
    }
    /// PublicKey::verify (src/lib.rs:85-100)
    pub fn verify(&self, message: &[u8], signature: &Signature) -> Result<(), ()> {
        verify_bls_signature(&signature.raw, message, &self.raw)
    }
}

impl core::fmt::Debug for PublicKey {
    fn fmt(&self, f: &mut core::fmt::Formatter<'_>) -> core::fmt::Result {
        write!(f, "PublicKey(")?;
        for b in self.raw.iter() {
            write!(f, "{b:02x}")?;
        }
        write!(f, ")")
    }
}

/// `Signature` (src/lib.rs:113-153): a checked 48-byte compressed G1 point.
#[derive(Copy, Clone, Eq, PartialEq)]
pub struct Signature {
    raw: [u8; 48],
}

impl Signature {
    pub const BYTES: usize = 48;
    /// Signature::deserialize (src/lib.rs:138-152)
    pub fn deserialize(bytes: &[u8]) -> Result<Self, InvalidSignature> {
        if bytes.len() != Self::BYTES {
            return Err(InvalidSignature::WrongLength);
        }
        let code = with_default(|v| v.deserialize_codes(ffi::CESS_BLS_KIND_SIG, &[bytes])).expect("verifier")[0];
        if code == ffi::CODE_SIG_POINT {
            return Err(InvalidSignature::InvalidPoint);
        }
        Ok(Signature { raw: bytes.try_into().unwrap() })
    }
    pub fn serialize(&self) -> [u8; 48] {
        self.raw
    }
}

impl core::fmt::Debug for Signature {
    fn fmt(&self, f: &mut core::fmt::Formatter<'_>) -> core::fmt::Result {
        write!(f, "Signature(")?;
        for b in self.raw.iter() {
            write!(f, "{b:02x}")?;
        }
        write!(f, ")")
    }
}

const R_ORDER_BE: [u8; 32] = [
    0x73, 0xed, 0xa7, 0x53, 0x29, 0x9d, 0x7d, 0x48, 0x33, 0x39, 0xd8, 0x08, 0x09, 0xa1, 0xd8, 0x05, 0x53, 0xbd, 0xa4,
    0x02, 0xff, 0xfe, 0x5b, 0xfe, 0xff, 0xff, 0xff, 0xff, 0x00, 0x00, 0x00, 0x01,
];

/// `PrivateKey` (src/lib.rs:166-237): a 32-byte big-endian scalar < r.
#[derive(Copy, Clone, Eq, PartialEq)]
pub struct PrivateKey {
    sk: [u8; 32],
}

impl PrivateKey {
    pub const BYTES: usize = 32;
    /// PrivateKey::random (src/lib.rs:185-198): 32 bytes from the OS CSPRNG
    /// (getrandom), redrawn until the big-endian value is below r -- the
    /// reference's rejection sampling through `Scalar::from_bytes`.  Zero is
    /// accepted, as there (it yields the identity key).
    pub fn random() -> Self {
        loop {
            let mut sk = [0u8; 32];
            getrandom::getrandom(&mut sk).expect("getrandom");
            if let Ok(k) = Self::deserialize(&sk) {
                return k;
            }
        }
    }
    /// PrivateKey::deserialize (src/lib.rs:208-223)
    pub fn deserialize(bytes: &[u8]) -> Result<Self, InvalidPrivateKey> {
        if bytes.len() != Self::BYTES {
            return Err(InvalidPrivateKey::WrongLength);
        }
        let sk: [u8; 32] = bytes.try_into().unwrap();
        if sk >= R_ORDER_BE {
            return Err(InvalidPrivateKey::OutOfRange);
        }
        Ok(PrivateKey { sk })
    }
    pub fn serialize(&self) -> [u8; 32] {
        self.sk
    }
    /// PrivateKey::public_key (src/lib.rs:226-228)
    pub fn public_key(&self) -> PublicKey {
        let pk = with_default(|v| v.public_keys(&[self.sk])).expect("verifier");
        PublicKey { raw: pk[0] }
    }
    /// PrivateKey::sign (src/lib.rs:233-236)
    pub fn sign(&self, message: &[u8]) -> Signature {
        let s = with_default(|v| v.sign(&[self.sk], &[message])).expect("verifier");
        Signature { raw: s[0] }
    }
}

impl core::fmt::Debug for PrivateKey {
    fn fmt(&self, f: &mut core::fmt::Formatter<'_>) -> core::fmt::Result {
        write!(f, "PrivateKey(REDACTED)")
    }
}

/// `verify_bls_signature(sig, msg, key)` (src/lib.rs:243-247).
pub fn verify_bls_signature(sig: &[u8], msg: &[u8], key: &[u8]) -> Result<(), ()> {
    let code = with_default(|v| v.verify_code(sig, msg, key)).expect("verifier");
    if code == ffi::CODE_OK {
        Ok(())
    } else {
        Err(())
    }
}

/// New: `verify_batch(&[..]) -> bitmap` (BASELINE north_star).
pub fn verify_batch(records: &[(&[u8], &[u8], &[u8])]) -> Verdicts {
    with_default(|v| v.verify_batch(records)).expect("verifier")
}

/// `cp_enclave_verify::verify_bls(key, msg, sig)` (primitives/enclave-verify/
/// src/lib.rs:230-235) with the reference's semantics: panics if the key, then
/// the signature, does not deserialize.
pub fn verify_bls(key: &[u8], msg: &[u8], sig: &[u8]) -> Result<(), ()> {
    match with_default(|v| v.enclave_verify_bls(key, msg, sig)) {
        Ok(true) => Ok(()),
        Ok(false) => Err(()),
        Err(Error::BadKey) => panic!("called `Result::unwrap()` on an `Err` value: {:?}", InvalidPublicKey::InvalidPoint),
        Err(Error::BadSig) => panic!("called `Result::unwrap()` on an `Err` value: {:?}", InvalidSignature::InvalidPoint),
        Err(e) => panic!("MI355X verifier: {}", e.message()),
    }
}

/// `cp_enclave_verify::verify_rsa(key, msg, sig)` (primitives/enclave-verify/
/// src/lib.rs:221-228) with the reference's semantics: panics if the key does
/// not parse as SubjectPublicKeyInfo DER.
///
/// DIVERGENCE (documented): a key the reference parses but the GPU
/// cannot verify (even modulus, n < 3, non-NULL SPKI parameters;
/// `Error::Unsupported`) also panics here, where the reference returns a
/// verdict.  Callers that must not panic on such keys use `try_verify_rsa` and
/// route `Err(Error::Unsupported)` to their own path (the node hook answers
/// "unavailable" and the runtime's unchanged verifier decides).  This crate
/// links no CPU RSA implementation.
pub fn verify_rsa(key: &[u8], msg: &[u8], sig: &[u8]) -> bool {
    match try_verify_rsa(key, msg, sig) {
        Ok(ok) => ok,
        Err(e) => panic!("called `Result::unwrap()` on an `Err` value: {}", e.message()),
    }
}

/// `verify_rsa` without panics: `Err(BadKey)` where the reference panics,
/// `Err(Unsupported)` where only the GPU cannot decide.
pub fn try_verify_rsa(key: &[u8], msg: &[u8], sig: &[u8]) -> Result<bool, Error> {
    with_default(|v| v.verify_rsa(key, msg, sig))
}

/// Bounded verdict cache of the C library (cess_bls_cache_*): SHA-256 of the
/// length-prefixed (sig, msg, key) -> verdict code; oldest entries evicted
/// first at capacity.  Thread-safe (the library locks it).
pub struct VerdictCache {
    cache: *mut ffi::cess_bls_cache,
}

unsafe impl Send for VerdictCache {}
unsafe impl Sync for VerdictCache {}

/// What `VerdictCache::verify` reports next to the codes.
#[derive(Clone, Copy, Debug, Default, Eq, PartialEq)]
pub struct CacheStats {
    pub hits: u64,
    pub verified: u64,
    pub evicted: u64,
}

impl VerdictCache {
    pub fn new(capacity: usize) -> Result<Self, Error> {
        let mut p = core::ptr::null_mut();
        check(unsafe { ffi::cess_bls_cache_create(capacity, &mut p) })?;
        Ok(VerdictCache { cache: p })
    }
    pub fn len(&self) -> usize {
        unsafe { ffi::cess_bls_cache_size(self.cache) }
    }
    pub fn clear(&self) {
        unsafe { ffi::cess_bls_cache_clear(self.cache) };
    }
    /// Codes for records of any lengths: cached verdicts, the misses verified
    /// in one batch on `verifier` and cached.  With no verifier, or when that
    /// batch fails, the misses are `ffi::CODE_UNAVAILABLE` (never cached) and
    /// the batch's error is returned beside the codes.
    pub fn verify(&self, verifier: Option<&mut Verifier>, records: &[(&[u8], &[u8], &[u8])])
                  -> (Vec<u8>, CacheStats, Result<(), Error>) {
        let n = records.len();
        let mut codes = vec![ffi::CODE_UNAVAILABLE; n];
        if n == 0 {
            return (codes, CacheStats::default(), Ok(()));
        }
        let (mut sd, mut pd, mut md) = (Vec::new(), Vec::new(), Vec::new());
        let so = offsets(records.iter().map(|r| r.0), &mut sd);
        let mo = offsets(records.iter().map(|r| r.1), &mut md);
        let po = offsets(records.iter().map(|r| r.2), &mut pd);
        let ctx = verifier.map(|v| v.ctx).unwrap_or(core::ptr::null_mut());
        let mut st3 = [0u64; 3];
        let st = unsafe {
            ffi::cess_bls_cache_verify_var(self.cache, ctx, n, sd.as_ptr(), so.as_ptr(), pd.as_ptr(), po.as_ptr(),
                                           md.as_ptr(), mo.as_ptr(), codes.as_mut_ptr(), st3.as_mut_ptr())
        };
        (codes, CacheStats { hits: st3[0], verified: st3[1], evicted: st3[2] }, check(st))
    }
    /// Insert verdicts obtained elsewhere (e.g. gathered codes of a sharded batch).
    pub fn insert(&self, records: &[(&[u8], &[u8], &[u8])], codes: &[u8]) -> Result<(), Error> {
        assert_eq!(records.len(), codes.len());
        let (mut sd, mut pd, mut md) = (Vec::new(), Vec::new(), Vec::new());
        let so = offsets(records.iter().map(|r| r.0), &mut sd);
        let mo = offsets(records.iter().map(|r| r.1), &mut md);
        let po = offsets(records.iter().map(|r| r.2), &mut pd);
        check(unsafe {
            ffi::cess_bls_cache_insert_var(self.cache, records.len(), sd.as_ptr(), so.as_ptr(), pd.as_ptr(),
                                           po.as_ptr(), md.as_ptr(), mo.as_ptr(), codes.as_ptr())
        })
    }
}

impl Drop for VerdictCache {
    fn drop(&mut self) {
        unsafe { ffi::cess_bls_cache_destroy(self.cache) }
    }
}

#[cfg(test)]
mod tests {
    // The reference's KATs (utils/verify-bls-signatures/tests/tests.rs) run
    // against this crate in tests/kat.rs on a box with cargo and an MI355X.
    use super::*;

    #[test]
    fn batch_equals_single() {
        let sk = PrivateKey::deserialize(&[7u8; 32]).unwrap();
        let pk = sk.public_key();
        let sig = sk.sign(b"cess");
        assert!(pk.verify(b"cess", &sig).is_ok());
        let v = verify_batch(&[(&sig.serialize()[..], b"cess", &pk.serialize()[..]),
                               (&sig.serialize()[..], b"xess", &pk.serialize()[..])]);
        assert_eq!(v.codes, vec![0, 5]);
        assert!(v.ok(0) && !v.ok(1));
    }
}
