"""Host-side mirror of the reference crate `ic-verify-bls-signature`
(/root/reference/utils/verify-bls-signatures/src/lib.rs) over the C ABI in
include/cess_bls.h, plus the new batch entry point.

Same names, argument meaning and error behaviour as the reference:
  verify_bls_signature(sig, msg, key) -> Ok/Err            src/lib.rs:243-247
  PublicKey.{BYTES, deserialize, serialize, verify}        src/lib.rs:33-101
  Signature.{BYTES, deserialize, serialize}                src/lib.rs:113-153
  PrivateKey.{BYTES, random, deserialize, serialize,
              public_key, sign}                            src/lib.rs:166-237
  InvalidPublicKey / InvalidSignature / InvalidPrivateKey  src/lib.rs:45-52, 104-110, 156-162
New: verify_batch(records) -> Verdicts(bitmap, codes)      

All arithmetic runs in the gfx950 kernels of libcess_bls.so.  There is no CPU
fallback: without a HIP device every call raises DeviceUnavailable.
"""
from __future__ import annotations

import ctypes
import enum
import os
import secrets
import threading
from dataclasses import dataclass
from typing import Iterable, Optional, Sequence, Tuple

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CESS_BLS_LIB", os.path.join(_HERE, "lib", "libcess_bls.so"))

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001

CODE_OK, CODE_SIG_LEN, CODE_SIG_POINT, CODE_PK_LEN, CODE_PK_POINT, CODE_PAIRING_FAIL = range(6)
CODE_NAMES = {0: "OK", 1: "SIG_LEN", 2: "SIG_POINT", 3: "PK_LEN", 4: "PK_POINT", 5: "PAIRING_FAIL"}

# the exported C symbols (tests check the library exports all of them)
EXPORTS = (
    "cess_bls_ctx_create", "cess_bls_ctx_destroy", "cess_bls_verify", "cess_bls_verify_batch",
    "cess_bls_verify_batch_var", "cess_bls_verify_batch_device", "cess_bls_public_key_batch",
    "cess_bls_sign_batch", "cess_bls_sign_batch_device", "cess_bls_hash_to_g1_batch", "cess_bls_gt_batch", "cess_bls_stage_times",
    "cess_bls_status_string", "cess_bls_version", "cess_bls_device_count",
    "cess_bls_verify_batch_rlc", "cess_bls_rlc_begin", "cess_bls_gt_product_is_one", "cess_bls_rlc_finish",
    "cess_bls_keys_load", "cess_bls_verify_batch_keyed", "cess_bls_verify_batch_keyed_device",
    "cess_bls_comm_id", "cess_bls_comm_init", "cess_bls_shard_range", "cess_bls_verify_batch_sharded",
    "cess_bls_verify_batch_sharded_device", "cess_bls_verify_batch_rlc_sharded", "cess_bls_comm_barrier",
    "cess_bls_comm_max_f64", "cess_bls_device_alloc", "cess_bls_device_free", "cess_bls_copy_to_device",
    "cess_bls_copy_from_device", "cess_bls_synchronize", "cess_bls_enclave_verify_bls",
    "cess_bls_stage_stats", "cess_bls_launch_records",
    # transport seam of the sharded entry points (RCCL or host shared memory)
    "cess_bls_comm_kind", "cess_bls_comm_shm_name", "cess_bls_comm_init_shm", "cess_bls_comm_open_shm",
    "cess_bls_comm_close", "cess_bls_comm_agree", "cess_bls_comm_gather_verdicts", "cess_bls_comm_info",
    "cess_bls_verify_batch_var_sharded",
    # node-side services: decode-only batches, the bounded verdict cache
    "cess_bls_deserialize_batch", "cess_bls_cache_create", "cess_bls_cache_destroy", "cess_bls_cache_clear",
    "cess_bls_cache_size", "cess_bls_cache_verify_var", "cess_bls_cache_insert_var", "cess_bls_sha256",
    # include/cess_rsa.h (RSA PKCS#1 v1.5 raw verify, cp_enclave_verify::verify_rsa)
    "cess_rsa_parse_key", "cess_rsa_keys_load", "cess_rsa_verify_batch", "cess_rsa_verify_batch_device",
    "cess_rsa_verify",
)
RSA_E_UNSUPPORTED = -10
RSA_KEY_SPKI, RSA_KEY_PKCS1 = 0, 1
RSA_CODE_NAMES = {0: "OK", 1: "SIG_LEN", 2: "SIG_RANGE", 3: "MSG_LEN", 4: "MISMATCH", 5: "KEY"}

# infrastructure status codes (include/cess_bls.h)
E_INVALID_ARG, E_NO_DEVICE, E_HIP, E_OOM, E_RCCL, E_BUSY, E_BAD_KEY, E_BAD_SIG, E_NO_COMM = range(-1, -10, -1)
E_COMM = -11
KIND_SIG, KIND_PK = 0, 1
CODE_UNAVAILABLE = 0xFF
F_PROFILE, F_STRICT_IDENTITY, F_RLC_DISTINCT = 1, 2, 4   # include/cess_bls.h CESS_BLS_F_*
MODE_PER_SIG, MODE_RLC = 0, 1


class DeviceUnavailable(RuntimeError):
    """No usable HIP device / library: the verifier has no CPU fallback."""


class BlsInfraError(RuntimeError):
    def __init__(self, msg, status=None):
        super().__init__(msg)
        self.status = status


class _Config(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("max_batch", ctypes.c_uint64), ("flags", ctypes.c_uint32),
                ("mode", ctypes.c_uint32), ("n_devices", ctypes.c_int), ("devices", ctypes.POINTER(ctypes.c_int))]


_u8p = ctypes.POINTER(ctypes.c_uint8)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_lib = None
_lib_lock = threading.Lock()


def load_library(path: str = LIB_PATH):
    """Load libcess_bls.so and declare its C signatures (no device access)."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise DeviceUnavailable(f"{path} not built (run __graft_entry__.build())")
        lib = ctypes.CDLL(path)
        vp = ctypes.c_void_p
        sz = ctypes.c_size_t
        lib.cess_bls_ctx_create.argtypes = [ctypes.POINTER(_Config), ctypes.POINTER(vp)]
        lib.cess_bls_ctx_destroy.argtypes = [vp]
        lib.cess_bls_ctx_destroy.restype = None
        lib.cess_bls_verify.argtypes = [vp, _u8p, sz, _u8p, sz, _u8p, sz, _u8p]
        lib.cess_bls_verify_batch.argtypes = [vp, sz, _u8p, _u8p, _u8p, _u64p, _u8p, _u64p]
        lib.cess_bls_verify_batch_var.argtypes = [vp, sz, _u8p, _u64p, _u8p, _u64p, _u8p, _u64p, _u8p, _u64p]
        lib.cess_bls_verify_batch_device.argtypes = [vp, sz, vp, vp, vp, vp, vp, vp, vp]
        lib.cess_bls_keys_load.argtypes = [vp, sz, _u8p, _u8p]
        lib.cess_bls_verify_batch_keyed.argtypes = [vp, sz, _u8p, ctypes.POINTER(ctypes.c_uint32), _u8p, _u64p,
                                                    _u8p, _u64p]
        lib.cess_bls_verify_batch_keyed_device.argtypes = [vp, sz, vp, vp, vp, vp, vp, vp, vp]
        lib.cess_bls_public_key_batch.argtypes = [vp, sz, _u8p, _u8p]
        lib.cess_bls_sign_batch.argtypes = [vp, sz, _u8p, _u8p, _u64p, _u8p]
        lib.cess_bls_sign_batch_device.argtypes = [vp, sz, vp, vp, vp, vp, vp]
        lib.cess_bls_hash_to_g1_batch.argtypes = [vp, sz, _u8p, _u64p, _u8p]
        lib.cess_bls_gt_batch.argtypes = [vp, sz, _u8p, _u8p, _u8p, _u64p, _u8p, _u8p]
        lib.cess_bls_rlc_begin.argtypes = [vp, sz, _u8p, _u8p, _u8p, _u64p, _u8p, _u8p]
        lib.cess_bls_gt_product_is_one.argtypes = [vp, sz, _u8p, ctypes.POINTER(ctypes.c_int)]
        lib.cess_bls_rlc_finish.argtypes = [vp, ctypes.c_int, _u8p, _u64p, _u64p]
        lib.cess_bls_verify_batch_rlc.argtypes = [vp, sz, _u8p, _u8p, _u8p, _u64p, _u8p, _u8p, _u64p, _u64p]
        lib.cess_bls_comm_id.argtypes = [_u8p]
        lib.cess_bls_comm_init.argtypes = [vp, ctypes.c_int, ctypes.c_int, _u8p]
        lib.cess_bls_shard_range.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, _u64p, _u64p, _u64p]
        lib.cess_bls_verify_batch_sharded.argtypes = [vp, sz, _u8p, _u8p, _u8p, _u64p, _u8p, _u64p]
        lib.cess_bls_verify_batch_sharded_device.argtypes = [vp, sz, vp, vp, vp, vp, vp, vp, vp]
        lib.cess_bls_verify_batch_rlc_sharded.argtypes = [vp, sz, _u8p, _u8p, _u8p, _u64p, _u8p, _u8p, _u64p, _u64p,
                                                          ctypes.POINTER(ctypes.c_int)]
        lib.cess_bls_comm_init_shm.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_char_p]
        lib.cess_bls_comm_kind.argtypes = [vp]
        lib.cess_bls_comm_info.argtypes = [vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                           ctypes.c_char_p]
        lib.cess_bls_verify_batch_var_sharded.argtypes = [vp, sz, _u8p, _u64p, _u8p, _u64p, _u8p, _u64p, _u8p, _u64p]
        lib.cess_bls_comm_kind.restype = ctypes.c_char_p
        lib.cess_bls_comm_shm_name.argtypes = [ctypes.c_char_p]
        lib.cess_bls_comm_open_shm.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]
        lib.cess_bls_comm_close.argtypes = [vp]
        lib.cess_bls_comm_close.restype = None
        lib.cess_bls_comm_agree.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        lib.cess_bls_comm_gather_verdicts.argtypes = [vp, ctypes.c_uint64, _u8p, _u8p, _u64p]
        lib.cess_bls_deserialize_batch.argtypes = [vp, ctypes.c_int, sz, _u8p, _u64p, _u8p]
        lib.cess_bls_cache_create.argtypes = [sz, ctypes.POINTER(vp)]
        lib.cess_bls_cache_destroy.argtypes = [vp]
        lib.cess_bls_cache_destroy.restype = None
        lib.cess_bls_cache_clear.argtypes = [vp]
        lib.cess_bls_cache_size.argtypes = [vp]
        lib.cess_bls_cache_size.restype = ctypes.c_size_t
        lib.cess_bls_cache_verify_var.argtypes = [vp, vp, sz, _u8p, _u64p, _u8p, _u64p, _u8p, _u64p, _u8p, _u64p]
        lib.cess_bls_cache_insert_var.argtypes = [vp, sz, _u8p, _u64p, _u8p, _u64p, _u8p, _u64p, _u8p]
        lib.cess_bls_sha256.argtypes = [_u8p, sz, _u8p]
        lib.cess_bls_comm_barrier.argtypes = [vp]
        lib.cess_bls_comm_max_f64.argtypes = [vp, ctypes.POINTER(ctypes.c_double)]
        lib.cess_bls_device_alloc.argtypes = [vp, sz, ctypes.POINTER(vp)]
        lib.cess_bls_device_free.argtypes = [vp, vp]
        lib.cess_bls_copy_to_device.argtypes = [vp, vp, vp, sz]
        lib.cess_bls_copy_from_device.argtypes = [vp, vp, vp, sz]
        lib.cess_bls_synchronize.argtypes = [vp]
        lib.cess_bls_enclave_verify_bls.argtypes = [vp, _u8p, sz, _u8p, sz, _u8p, sz, ctypes.POINTER(ctypes.c_int)]
        lib.cess_rsa_parse_key.argtypes = [_u8p, sz, ctypes.c_int, _u8p, sz, ctypes.POINTER(ctypes.c_size_t), _u64p]
        lib.cess_rsa_keys_load.argtypes = [vp, sz, _u8p, _u64p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        lib.cess_rsa_verify_batch.argtypes = [vp, sz, ctypes.POINTER(ctypes.c_uint32), _u8p, _u64p, _u8p, _u64p, _u8p,
                                              _u64p]
        lib.cess_rsa_verify_batch_device.argtypes = [vp, sz, vp, vp, vp, vp, vp, vp, vp]
        lib.cess_rsa_verify.argtypes = [vp, _u8p, sz, _u8p, sz, _u8p, sz, ctypes.POINTER(ctypes.c_int)]
        lib.cess_bls_stage_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_double),
                                             _u64p, ctypes.c_int, ctypes.c_int]
        lib.cess_bls_launch_records.argtypes = [vp]
        lib.cess_bls_launch_records.restype = ctypes.c_uint64
        lib.cess_bls_stage_times.argtypes = [vp, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_double),
                                             ctypes.c_int, ctypes.c_int]
        lib.cess_bls_status_string.restype = ctypes.c_char_p
        lib.cess_bls_status_string.argtypes = [ctypes.c_int]
        lib.cess_bls_version.restype = ctypes.c_char_p
        if hasattr(lib, "cess_bls_device_count"):   # (absent from pre-round-5 builds used in A/B sweeps)
            lib.cess_bls_device_count.restype = ctypes.c_int
            lib.cess_bls_device_count.argtypes = []
        _lib = lib
        return lib


def _buf(b: bytes):
    if not b:
        return ctypes.cast(ctypes.c_char_p(b"\0"), _u8p)
    return ctypes.cast(ctypes.c_char_p(bytes(b)), _u8p)


def _u64arr(x):
    """uint64 array argument: numpy arrays are passed without a copy (the
    caller keeps them alive for the call), sequences are converted."""
    if hasattr(x, "ctypes") and getattr(x, "dtype", None) is not None:
        import numpy as np
        a = np.ascontiguousarray(x, dtype=np.uint64)
        return (ctypes.c_uint64 * len(a)).from_buffer(a) if a.flags.writeable else \
            (ctypes.c_uint64 * len(a)).from_buffer_copy(a)
    return (ctypes.c_uint64 * len(x))(*x)


def _offsets(lengths: Sequence[int]):
    arr = (ctypes.c_uint64 * (len(lengths) + 1))()
    acc = 0
    for i, n in enumerate(lengths):
        arr[i] = acc
        acc += n
    arr[len(lengths)] = acc
    return arr


class Context:
    """One GPU: device buffers, stream and the -G2 prepared table."""

    def __init__(self, device: int = 0, max_batch: int = 1 << 20, profile: bool = False,
                 strict_identity: bool = False, mode: int = MODE_PER_SIG, devices: Optional[Sequence[int]] = None,
                 rlc_distinct: bool = False):
        """devices: a list of >1 ordinals makes one context over several GPUs of
        this process (host-buffer batches sharded by index across them)."""
        lib = load_library()
        self._lib = lib
        flags = (F_PROFILE if profile else 0) | (F_STRICT_IDENTITY if strict_identity else 0) | \
            (F_RLC_DISTINCT if rlc_distinct else 0)
        ndev = len(devices) if devices is not None and len(devices) > 1 else 0
        self._devs = (ctypes.c_int * max(ndev, 1))(*(devices if ndev else [0]))
        cfg = _Config(device, max_batch, flags, mode, ndev, self._devs if ndev else None)
        self._keys_owner = None      # None | "user" | "verify_batch": who loaded the key table
        h = ctypes.c_void_p()
        st = lib.cess_bls_ctx_create(ctypes.byref(cfg), ctypes.byref(h))
        if st != 0:
            msg = lib.cess_bls_status_string(st).decode()
            if st == -2:
                raise DeviceUnavailable(msg)
            raise BlsInfraError(msg)
        self._h = h
        self.device = device
        self.max_batch = max_batch

    def close(self):
        if getattr(self, "_h", None):
            self._lib.cess_bls_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, st):
        if st != 0:
            raise BlsInfraError(self._lib.cess_bls_status_string(st).decode(), st)

    @property
    def handle(self):
        return self._h

    # --- verification ---------------------------------------------------
    def verify_codes(self, records: Sequence[Tuple[bytes, bytes, bytes]]) -> bytes:
        """Per-record verdict codes for (sig, msg, key) triples of any lengths."""
        n = len(records)
        if n == 0:
            return b""
        sigs = [bytes(r[0]) for r in records]
        msgs = [bytes(r[1]) for r in records]
        keys = [bytes(r[2]) for r in records]
        codes = (ctypes.c_uint8 * n)()
        bitmap = (ctypes.c_uint64 * ((n + 63) // 64))()
        if all(len(s) == 48 for s in sigs) and all(len(k) == 96 for k in keys):
            self._chk(self._lib.cess_bls_verify_batch(
                self._h, n, _buf(b"".join(sigs)), _buf(b"".join(keys)), _buf(b"".join(msgs)),
                _offsets([len(m) for m in msgs]), codes, bitmap))
        else:
            self._chk(self._lib.cess_bls_verify_batch_var(
                self._h, n, _buf(b"".join(sigs)), _offsets([len(s) for s in sigs]),
                _buf(b"".join(keys)), _offsets([len(k) for k in keys]),
                _buf(b"".join(msgs)), _offsets([len(m) for m in msgs]), codes, bitmap))
        return bytes(codes)

    def verify_fixed(self, sigs: bytes, pks: bytes, msgs: bytes, msg_offsets) -> Tuple[bytes, list]:
        """Fixed-stride batch over packed host buffers; returns (codes, bitmap words)."""
        n = len(sigs) // 48
        assert len(sigs) == 48 * n and len(pks) == 96 * n
        offs = _u64arr(msg_offsets)
        codes = (ctypes.c_uint8 * max(n, 1))()
        bitmap = (ctypes.c_uint64 * max((n + 63) // 64, 1))()
        self._chk(self._lib.cess_bls_verify_batch(self._h, n, _buf(sigs), _buf(pks), _buf(msgs), offs, codes, bitmap))
        return bytes(codes)[:n], list(bitmap)[: (n + 63) // 64]

    def gt(self, records) -> Tuple[bytes, list]:
        n = len(records)
        sigs, msgs, keys = (b"".join(bytes(r[j]) for r in records) for j in (0, 1, 2))
        codes = (ctypes.c_uint8 * n)()
        gt = (ctypes.c_uint8 * (576 * n))()
        self._chk(self._lib.cess_bls_gt_batch(self._h, n, _buf(sigs), _buf(keys), _buf(msgs),
                                              _offsets([len(r[1]) for r in records]), codes, gt))
        raw = bytes(gt)
        return bytes(codes), [raw[576 * i:576 * (i + 1)] for i in range(n)]

    def sign_device(self, n, d_sks, d_msgs, d_offs, d_sigs_out, stream=0):
        """cess_bls_sign_batch_device: enqueue PrivateKey::sign over device buffers."""
        self._chk(self._lib.cess_bls_sign_batch_device(self._h, n, d_sks, d_msgs, d_offs, d_sigs_out,
                                                       stream or None))

    def verify_device(self, n, d_sigs, d_pks, d_msgs, d_offs, d_codes, d_bitmap, stream=0):
        """Device-resident batch (HBM pointers as ints); enqueued on `stream`, not synchronised."""
        self._chk(self._lib.cess_bls_verify_batch_device(self._h, n, d_sigs, d_pks, d_msgs, d_offs, d_codes,
                                                         d_bitmap, stream or None))

    # --- distinct-key table (per-key decode + G2Prepared done once) -------
    def load_keys(self, keys: Sequence[bytes], _owner: str = "user") -> bytes:
        """Decode and prepare each distinct 96-byte key once (PublicKey::deserialize,
        src/lib.rs:68-82, and G2Prepared::from, :88); returns the per-key codes
        (0, or 4 = PK_POINT).  Replaces any previously loaded table."""
        self._keys_owner = _owner
        k = len(keys)
        assert all(len(bytes(x)) == 96 for x in keys)
        kc = (ctypes.c_uint8 * max(k, 1))()
        self._chk(self._lib.cess_bls_keys_load(self._h, k, _buf(b"".join(bytes(x) for x in keys)), kc))
        return bytes(kc)[:k]

    def verify_keyed(self, sigs: bytes, key_idx: Sequence[int], msgs: bytes, msg_offsets) -> Tuple[bytes, list]:
        """Per-signature verdicts where signature i is checked against loaded key
        key_idx[i]; same codes as the per-record path on the expanded records."""
        n = len(sigs) // 48
        assert len(sigs) == 48 * n and len(key_idx) == n
        if self._keys_owner != "user":
            raise BlsInfraError("no user-loaded key table on this context (load_keys first; verify_batch's "
                                "internal table is never used for caller indices)", E_INVALID_ARG)
        idx = (ctypes.c_uint32 * max(n, 1))(*key_idx)
        offs = _u64arr(msg_offsets)
        codes = (ctypes.c_uint8 * max(n, 1))()
        bitmap = (ctypes.c_uint64 * max((n + 63) // 64, 1))()
        self._chk(self._lib.cess_bls_verify_batch_keyed(self._h, n, _buf(sigs), idx, _buf(msgs), offs, codes, bitmap))
        return bytes(codes)[:n], list(bitmap)[: (n + 63) // 64]

    def _verify_keyed_any(self, sigs, key_idx, msgs, msg_offsets):
        n = len(sigs) // 48
        idx = (ctypes.c_uint32 * max(n, 1))(*key_idx)
        offs = _u64arr(msg_offsets)
        codes = (ctypes.c_uint8 * max(n, 1))()
        bitmap = (ctypes.c_uint64 * max((n + 63) // 64, 1))()
        self._chk(self._lib.cess_bls_verify_batch_keyed(self._h, n, _buf(sigs), idx, _buf(msgs), offs, codes, bitmap))
        return bytes(codes)[:n], list(bitmap)[: (n + 63) // 64]

    def verify_keyed_device(self, n, d_sigs, d_key_idx, d_msgs, d_offs, d_codes, d_bitmap, stream=0):
        """Device-resident keyed batch (HBM pointers as ints); not synchronised."""
        if self._keys_owner != "user":
            raise BlsInfraError("no user-loaded key table on this context", E_INVALID_ARG)
        self._chk(self._lib.cess_bls_verify_batch_keyed_device(self._h, n, d_sigs, d_key_idx, d_msgs, d_offs,
                                                               d_codes, d_bitmap, stream or None))

    # --- RLC batch mode (random linear combination + bisection) ----------
    def rlc_begin(self, sigs: bytes, pks: bytes, msgs: bytes, msg_offsets, seed: Optional[bytes] = None) -> bytes:
        """Decode, hash and scale a fixed-stride batch, run its RLC check and
        return this shard's Gt partial (576 canonical bytes).  The buffers are
        kept alive until rlc_finish."""
        n = len(sigs) // 48
        assert len(sigs) == 48 * n and len(pks) == 96 * n and (seed is None or len(seed) == 32)
        keep = (_buf(sigs), _buf(pks), _buf(msgs), _u64arr(msg_offsets),
                _buf(seed) if seed is not None else None)
        self._rlc_keep = keep
        self._rlc_n = n
        gt = (ctypes.c_uint8 * 576)()
        self._chk(self._lib.cess_bls_rlc_begin(self._h, n, keep[0], keep[1], keep[2], keep[3], keep[4], gt))
        return bytes(gt)

    def gt_product_is_one(self, gts: bytes) -> bool:
        """prod of m canonical Gt values (m*576 bytes) == 1, computed on the device."""
        m = len(gts) // 576
        ok = ctypes.c_int()
        self._chk(self._lib.cess_bls_gt_product_is_one(self._h, m, _buf(gts), ctypes.byref(ok)))
        return bool(ok.value)

    def rlc_finish(self, global_ok: bool):
        """Per-record codes of the batch given the (cross-shard) verdict of the
        combined check; a failing shard is bisected.  -> (codes, bitmap, stats)"""
        n = self._rlc_n
        codes = (ctypes.c_uint8 * max(n, 1))()
        bitmap = (ctypes.c_uint64 * max((n + 63) // 64, 1))()
        st = (ctypes.c_uint64 * 4)()
        self._chk(self._lib.cess_bls_rlc_finish(self._h, 1 if global_ok else 0, codes, bitmap, st))
        self._rlc_keep = None
        stats = {"checks": st[0], "leaves": st[1], "leaf_sigs": st[2], "distinct_keys": st[3]}
        return bytes(codes)[:n], list(bitmap)[: (n + 63) // 64], stats

    def verify_rlc(self, sigs: bytes, pks: bytes, msgs: bytes, msg_offsets, seed: Optional[bytes] = None):
        """Single-GPU RLC batch verification -> (codes, bitmap, stats); codes equal
        verify_fixed's (soundness error 2^-127 per check)."""
        n = len(sigs) // 48
        offs = _u64arr(msg_offsets)
        codes = (ctypes.c_uint8 * max(n, 1))()
        bitmap = (ctypes.c_uint64 * max((n + 63) // 64, 1))()
        st = (ctypes.c_uint64 * 4)()
        # seed None: the library draws it from the OS CSPRNG (it must be secret
        # and unpredictable to the signers, include/cess_bls.h)
        sd = _buf(seed) if seed is not None else None
        self._chk(self._lib.cess_bls_verify_batch_rlc(self._h, n, _buf(sigs), _buf(pks), _buf(msgs), offs,
                                                      sd, codes, bitmap, st))
        stats = {"checks": st[0], "leaves": st[1], "leaf_sigs": st[2], "distinct_keys": st[3]}
        return bytes(codes)[:n], list(bitmap)[: (n + 63) // 64], stats

    # --- RCCL communicator (one process per GPU) ------------------------
    def comm_init(self, nranks: int, rank: int, comm_id: bytes):
        """ncclCommInitRank on this context's device (collective)."""
        assert len(comm_id) == 128
        self._chk(self._lib.cess_bls_comm_init(self._h, nranks, rank, _buf(comm_id)))
        self.nranks, self.rank = nranks, rank

    def comm_init_shm(self, nranks: int, rank: int, name: str):
        """Host shared-memory transport (ranks on one host, may share a GPU;
        collective, same name on every rank: comm_shm_name())."""
        self._chk(self._lib.cess_bls_comm_init_shm(self._h, nranks, rank, name.encode()))
        self.nranks, self.rank = nranks, rank

    @property
    def comm_kind(self) -> str:
        return self._lib.cess_bls_comm_kind(self._h).decode()

    def verify_sharded(self, sigs: bytes, pks: bytes, msgs: bytes, msg_offsets) -> Tuple[bytes, list]:
        """Every rank passes the whole fixed-stride batch; returns the verdicts
        of all records (each rank verifies its shard, RCCL all-gathers)."""
        n = len(sigs) // 48
        offs = _u64arr(msg_offsets)
        codes = (ctypes.c_uint8 * max(n, 1))()
        bitmap = (ctypes.c_uint64 * max((n + 63) // 64, 1))()
        self._chk(self._lib.cess_bls_verify_batch_sharded(self._h, n, _buf(sigs), _buf(pks), _buf(msgs), offs, codes,
                                                          bitmap))
        return bytes(codes)[:n], list(bitmap)[: (n + 63) // 64]

    def verify_var_sharded(self, records) -> Tuple[bytes, list]:
        """Every rank passes the whole batch of (sig, msg, key) triples of any
        lengths; returns the verdicts of all records (cess_bls_verify_batch_var_sharded)."""
        n = len(records)
        sigs = [bytes(r[0]) for r in records]
        msgs = [bytes(r[1]) for r in records]
        keys = [bytes(r[2]) for r in records]
        codes = (ctypes.c_uint8 * max(n, 1))()
        bitmap = (ctypes.c_uint64 * max((n + 63) // 64, 1))()
        self._chk(self._lib.cess_bls_verify_batch_var_sharded(
            self._h, n, _buf(b"".join(sigs)), _offsets([len(x) for x in sigs]), _buf(b"".join(keys)),
            _offsets([len(k) for k in keys]), _buf(b"".join(msgs)), _offsets([len(m) for m in msgs]), codes, bitmap))
        return bytes(codes)[:n], list(bitmap)[: (n + 63) // 64]

    def comm_info(self, bus_ids: bool = True) -> dict:
        """What the communicator reports: its rank count and this rank
        (ncclCommCount / ncclCommUserRank over RCCL) and, when bus_ids (a
        collective: pass it on every rank), every rank's GPU PCI bus id."""
        nr, rk = ctypes.c_int(), ctypes.c_int()
        buf = ctypes.create_string_buffer(32 * max(self.nranks if hasattr(self, "nranks") else 1, 1)) \
            if bus_ids else None
        self._chk(self._lib.cess_bls_comm_info(self._h, ctypes.byref(nr), ctypes.byref(rk), buf))
        out = {"nranks": nr.value, "rank": rk.value}
        if bus_ids:
            raw = buf.raw
            out["bus_ids"] = [raw[32 * q:32 * q + 32].split(b"\0", 1)[0].decode() for q in range(nr.value)]
        return out

    def verify_sharded_device(self, n_total, d_sigs, d_pks, d_msgs, d_offs, d_codes_all, d_bitmap_all, stream=0):
        """Device-resident sharded batch (this rank's shard in HBM); returns
        after the final status agreement (every rank sees any rank's failure)."""
        self._chk(self._lib.cess_bls_verify_batch_sharded_device(self._h, n_total, d_sigs, d_pks, d_msgs, d_offs,
                                                                 d_codes_all or None, d_bitmap_all, stream or None))

    def verify_rlc_sharded(self, sigs: bytes, pks: bytes, msgs: bytes, msg_offsets, seed: Optional[bytes] = None):
        """RLC over the communicator for this rank's shard -> (codes, bitmap, stats)."""
        n = len(sigs) // 48
        offs = _u64arr(msg_offsets)
        codes = (ctypes.c_uint8 * max(n, 1))()
        bitmap = (ctypes.c_uint64 * max((n + 63) // 64, 1))()
        st = (ctypes.c_uint64 * 4)()
        g = ctypes.c_int()
        self._chk(self._lib.cess_bls_verify_batch_rlc_sharded(self._h, n, _buf(sigs), _buf(pks), _buf(msgs), offs,
                                                              _buf(seed) if seed is not None else None, codes, bitmap,
                                                              st, ctypes.byref(g)))
        stats = {"checks": st[0], "leaves": st[1], "leaf_sigs": st[2], "distinct_keys": st[3], "global_ok": bool(g.value)}
        return bytes(codes)[:n], list(bitmap)[: (n + 63) // 64], stats

    def comm_barrier(self):
        self._chk(self._lib.cess_bls_comm_barrier(self._h))

    def comm_max(self, v: float) -> float:
        d = ctypes.c_double(v)
        self._chk(self._lib.cess_bls_comm_max_f64(self._h, ctypes.byref(d)))
        return d.value

    # --- deserialize only (Signature/PublicKey::deserialize, no pairing) ---
    def deserialize_codes(self, kind: int, encodings: Sequence[bytes]) -> bytes:
        """Per-encoding codes: 0 or SIG_LEN/SIG_POINT (kind KIND_SIG), PK_LEN/PK_POINT (KIND_PK)."""
        n = len(encodings)
        if n == 0:
            return b""
        codes = (ctypes.c_uint8 * n)()
        self._chk(self._lib.cess_bls_deserialize_batch(self._h, kind, n, _buf(b"".join(bytes(e) for e in encodings)),
                                                       _offsets([len(e) for e in encodings]), codes))
        return bytes(codes)

    # --- device memory on this context's GPU -------------------------------
    def device_alloc(self, nbytes: int) -> int:
        p = ctypes.c_void_p()
        self._chk(self._lib.cess_bls_device_alloc(self._h, nbytes, ctypes.byref(p)))
        return p.value

    def device_free(self, d: int):
        self._chk(self._lib.cess_bls_device_free(self._h, d))

    def to_device(self, data, d: Optional[int] = None) -> int:
        """Copy a bytes-like / numpy buffer to HBM (allocating when d is None)."""
        mv = memoryview(data).cast("B")
        if d is None:
            d = self.device_alloc(len(mv))
        if len(mv):
            src = (ctypes.c_uint8 * len(mv)).from_buffer_copy(mv) if mv.readonly else (ctypes.c_uint8 * len(mv)).from_buffer(mv)
            self._chk(self._lib.cess_bls_copy_to_device(self._h, d, src, len(mv)))
        return d

    def from_device(self, d: int, nbytes: int) -> bytes:
        out = (ctypes.c_uint8 * max(nbytes, 1))()
        self._chk(self._lib.cess_bls_copy_from_device(self._h, out, d, nbytes))
        return bytes(out)[:nbytes]

    def synchronize(self):
        self._chk(self._lib.cess_bls_synchronize(self._h))

    # --- cp_enclave_verify::verify_bls (primitives/enclave-verify/src/lib.rs:230-235)
    def enclave_verify_bls(self, key: bytes, msg: bytes, sig: bytes) -> bool:
        """Reversed argument order as the reference; raises BlsInfraError with
        status E_BAD_KEY / E_BAD_SIG where the reference panics (key first)."""
        ok = ctypes.c_int()
        key, msg, sig = bytes(key), bytes(msg), bytes(sig)
        self._chk(self._lib.cess_bls_enclave_verify_bls(self._h, _buf(key), len(key), _buf(msg), len(msg), _buf(sig),
                                                        len(sig), ctypes.byref(ok)))
        return bool(ok.value)

    # --- RSA PKCS#1 v1.5 raw verify (include/cess_rsa.h) -------------------
    def rsa_keys_load(self, ders: Sequence[bytes], fmt: int = RSA_KEY_SPKI) -> list:
        """Load the RSA key table (DER keys); returns per-key status (0, E_BAD_KEY, RSA_E_UNSUPPORTED)."""
        k = len(ders)
        st = (ctypes.c_int * max(k, 1))()
        self._chk(self._lib.cess_rsa_keys_load(self._h, k, _buf(b"".join(bytes(d) for d in ders)),
                                               _offsets([len(d) for d in ders]), fmt, st))
        return list(st)[:k]

    def rsa_verify_batch(self, key_idx: Sequence[int], msgs: Sequence[bytes], sigs: Sequence[bytes]) -> bytes:
        """verify_rsa over records (key key_idx[i] of the loaded table): per-record codes."""
        n = len(key_idx)
        idx = (ctypes.c_uint32 * max(n, 1))(*key_idx)
        codes = (ctypes.c_uint8 * max(n, 1))()
        bitmap = (ctypes.c_uint64 * max((n + 63) // 64, 1))()
        self._chk(self._lib.cess_rsa_verify_batch(self._h, n, idx, _buf(b"".join(sigs)), _offsets([len(x) for x in sigs]),
                                                  _buf(b"".join(msgs)), _offsets([len(m) for m in msgs]), codes,
                                                  bitmap))
        return bytes(codes)[:n]

    def rsa_verify_batch_device(self, n, d_key_idx, d_sigs, d_sig_offs, d_msgs, d_msg_offs, d_codes, stream=0):
        self._chk(self._lib.cess_rsa_verify_batch_device(self._h, n, d_key_idx, d_sigs, d_sig_offs, d_msgs, d_msg_offs,
                                                         d_codes, stream or None))

    def verify_rsa(self, key_der: bytes, msg: bytes, sig: bytes) -> bool:
        """cp_enclave_verify::verify_rsa (enclave-verify/src/lib.rs:221-228); raises
        BlsInfraError(E_BAD_KEY) where from_public_key_der(key).unwrap() panics."""
        ok = ctypes.c_int()
        key_der, msg, sig = bytes(key_der), bytes(msg), bytes(sig)
        self._chk(self._lib.cess_rsa_verify(self._h, _buf(key_der), len(key_der), _buf(msg), len(msg), _buf(sig),
                                            len(sig), ctypes.byref(ok)))
        return bool(ok.value)

    # --- generator side -------------------------------------------------
    def public_keys_raw(self, sks: bytes) -> bytes:
        """n concatenated 32-byte secret keys -> n concatenated 96-byte keys."""
        n = len(sks) // 32
        out = (ctypes.c_uint8 * (96 * max(n, 1)))()
        self._chk(self._lib.cess_bls_public_key_batch(self._h, n, _buf(sks), out))
        return bytes(out)[: 96 * n]

    def sign_raw(self, sks: bytes, msgs: bytes, msg_offsets) -> bytes:
        """Fixed arrays in, 48-byte signatures out (concatenated)."""
        n = len(sks) // 32
        offs = _u64arr(msg_offsets)
        out = (ctypes.c_uint8 * (48 * max(n, 1)))()
        self._chk(self._lib.cess_bls_sign_batch(self._h, n, _buf(sks), _buf(msgs), offs, out))
        return bytes(out)[: 48 * n]

    def public_keys(self, sks: Sequence[bytes]) -> list:
        n = len(sks)
        out = (ctypes.c_uint8 * (96 * max(n, 1)))()
        self._chk(self._lib.cess_bls_public_key_batch(self._h, n, _buf(b"".join(sks)), out))
        raw = bytes(out)
        return [raw[96 * i:96 * (i + 1)] for i in range(n)]

    def sign(self, sks: Sequence[bytes], msgs: Sequence[bytes]) -> list:
        n = len(sks)
        out = (ctypes.c_uint8 * (48 * max(n, 1)))()
        self._chk(self._lib.cess_bls_sign_batch(self._h, n, _buf(b"".join(sks)), _buf(b"".join(msgs)),
                                                _offsets([len(m) for m in msgs]), out))
        raw = bytes(out)
        return [raw[48 * i:48 * (i + 1)] for i in range(n)]

    def hash_to_g1(self, msgs: Sequence[bytes]) -> list:
        n = len(msgs)
        out = (ctypes.c_uint8 * (48 * max(n, 1)))()
        self._chk(self._lib.cess_bls_hash_to_g1_batch(self._h, n, _buf(b"".join(msgs)),
                                                      _offsets([len(m) for m in msgs]), out))
        raw = bytes(out)
        return [raw[48 * i:48 * (i + 1)] for i in range(n)]

    def stage_stats(self, reset=True) -> dict:
        """{stage: (ms summed over launches, launches)} since the last reset."""
        names = (ctypes.c_char_p * 16)()
        ms = (ctypes.c_double * 16)()
        ln = (ctypes.c_uint64 * 16)()
        k = self._lib.cess_bls_stage_stats(self._h, names, ms, ln, 16, 1 if reset else 0)
        return {names[i].decode(): (ms[i], ln[i]) for i in range(k)}

    @property
    def launch_records(self) -> int:
        return int(self._lib.cess_bls_launch_records(self._h))

    def stage_times(self, reset=True) -> dict:
        names = (ctypes.c_char_p * 16)()
        ms = (ctypes.c_double * 16)()
        k = self._lib.cess_bls_stage_times(self._h, names, ms, 16, 1 if reset else 0)
        return {names[i].decode(): ms[i] for i in range(k)}


_default: Optional[Context] = None


def shard_range(n: int, nranks: int, rank: int) -> Tuple[int, int, int]:
    """(begin, end, words_per_rank) of rank's shard (cess_bls_shard_range)."""
    lib = load_library()
    b, e, w = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    st = lib.cess_bls_shard_range(n, nranks, rank, ctypes.byref(b), ctypes.byref(e), ctypes.byref(w))
    if st != 0:
        raise BlsInfraError(lib.cess_bls_status_string(st).decode(), st)
    return b.value, e.value, w.value


def rsa_parse_key(der: bytes, fmt: int = RSA_KEY_SPKI) -> Tuple[bytes, int]:
    """(modulus big-endian, e) of a DER RSA public key (host-side parse)."""
    lib = load_library()
    der = bytes(der)
    out = (ctypes.c_uint8 * 512)()
    ln, e = ctypes.c_size_t(), ctypes.c_uint64()
    st = lib.cess_rsa_parse_key(_buf(der), len(der), fmt, out, 512, ctypes.byref(ln), ctypes.byref(e))
    if st != 0:
        raise BlsInfraError(lib.cess_bls_status_string(st).decode(), st)
    return bytes(out)[: ln.value], e.value


def comm_id() -> bytes:
    """ncclGetUniqueId (128 bytes) for cess_bls_comm_init; call on one rank."""
    lib = load_library()
    out = (ctypes.c_uint8 * 128)()
    st = lib.cess_bls_comm_id(out)
    if st != 0:
        raise BlsInfraError(lib.cess_bls_status_string(st).decode(), st)
    return bytes(out)


def comm_shm_name() -> str:
    """A fresh job name for the shared-memory transport; make it on one rank
    and distribute it out of band (as comm_id for RCCL)."""
    lib = load_library()
    out = ctypes.create_string_buffer(64)
    st = lib.cess_bls_comm_shm_name(out)
    if st != 0:
        raise BlsInfraError(lib.cess_bls_status_string(st).decode(), st)
    return out.value.decode()


class Comm:
    """Context-free shared-memory communicator (cess_bls_comm_open_shm): the
    merge step of the sharded entry points.  Needs no GPU."""

    def __init__(self, name: str, nranks: int, rank: int):
        self._lib = load_library()
        h = ctypes.c_void_p()
        st = self._lib.cess_bls_comm_open_shm(name.encode(), nranks, rank, ctypes.byref(h))
        if st != 0:
            raise BlsInfraError(self._lib.cess_bls_status_string(st).decode(), st)
        self._h = h
        self.nranks, self.rank = nranks, rank

    def close(self):
        if getattr(self, "_h", None):
            self._lib.cess_bls_comm_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, st):
        if st != 0:
            raise BlsInfraError(self._lib.cess_bls_status_string(st).decode(), st)

    def agree(self, status: int) -> int:
        out = ctypes.c_int()
        self._chk(self._lib.cess_bls_comm_agree(self._h, status, ctypes.byref(out)))
        return out.value

    def gather_verdicts(self, n_total: int, shard_codes: bytes) -> Tuple[bytes, list]:
        """(codes, bitmap words) of the whole batch from this rank's shard codes."""
        codes = (ctypes.c_uint8 * max(n_total, 1))()
        bitmap = (ctypes.c_uint64 * max((n_total + 63) // 64, 1))()
        self._chk(self._lib.cess_bls_comm_gather_verdicts(self._h, n_total, _buf(shard_codes), codes, bitmap))
        return bytes(codes)[:n_total], list(bitmap)[: (n_total + 63) // 64]


def sha256(data: bytes) -> bytes:
    """The library's host SHA-256 (the verdict cache's key derivation)."""
    lib = load_library()
    out = (ctypes.c_uint8 * 32)()
    data = bytes(data)
    st = lib.cess_bls_sha256(_buf(data), len(data), out)
    if st != 0:
        raise BlsInfraError(lib.cess_bls_status_string(st).decode(), st)
    return bytes(out)


class VerdictCache:
    """Bounded verdict cache (cess_bls_cache_*): what the node host function
    reads and the node batcher fills.  Needs no GPU for lookups and inserts."""

    def __init__(self, capacity: int):
        self._lib = load_library()
        h = ctypes.c_void_p()
        st = self._lib.cess_bls_cache_create(capacity, ctypes.byref(h))
        if st != 0:
            raise BlsInfraError(self._lib.cess_bls_status_string(st).decode(), st)
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._lib.cess_bls_cache_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self):
        return int(self._lib.cess_bls_cache_size(self._h))

    def clear(self):
        self._lib.cess_bls_cache_clear(self._h)

    @staticmethod
    def _flat(records):
        sigs = [bytes(r[0]) for r in records]
        msgs = [bytes(r[1]) for r in records]
        keys = [bytes(r[2]) for r in records]
        return (_buf(b"".join(sigs)), _offsets([len(x) for x in sigs]), _buf(b"".join(keys)),
                _offsets([len(x) for x in keys]), _buf(b"".join(msgs)), _offsets([len(x) for x in msgs]))

    def verify(self, records, ctx: Optional[Context] = None):
        """(status, codes, stats) for (sig, msg, key) records: hits from the cache,
        misses verified in one batch on ctx (None: reported CODE_UNAVAILABLE)."""
        n = len(records)
        codes = (ctypes.c_uint8 * max(n, 1))()
        st3 = (ctypes.c_uint64 * 3)()
        st = self._lib.cess_bls_cache_verify_var(self._h, ctx.handle if ctx is not None else None, n,
                                                 *self._flat(records), codes, st3)
        return st, bytes(codes)[:n], {"hits": st3[0], "verified": st3[1], "evicted": st3[2]}

    def insert(self, records, codes: bytes):
        n = len(records)
        st = self._lib.cess_bls_cache_insert_var(self._h, n, *self._flat(records), _buf(bytes(codes)))
        if st != 0:
            raise BlsInfraError(self._lib.cess_bls_status_string(st).decode(), st)


def default_context() -> Context:
    global _default
    if _default is None:
        _default = Context()
    return _default


# ---------------------------------------------------------------------------
# reference API mirror
# ---------------------------------------------------------------------------
class Result:
    """Rust Result<(), ()> stand-in: truthy iff Ok."""

    __slots__ = ("ok",)

    def __init__(self, ok: bool):
        self.ok = ok

    def is_ok(self):
        return self.ok

    def is_err(self):
        return not self.ok

    def __bool__(self):
        return self.ok

    def __repr__(self):
        return "Ok(())" if self.ok else "Err(())"


class InvalidPublicKey(enum.Enum):
    WrongLength = 0
    InvalidPoint = 1


class InvalidSignature(enum.Enum):
    WrongLength = 0
    InvalidPoint = 1


class InvalidPrivateKey(enum.Enum):
    WrongLength = 0
    OutOfRange = 1


class DeserializeError(ValueError):
    def __init__(self, kind):
        super().__init__(kind.name)
        self.kind = kind


# a fixed valid (sig, pk) pair lets the GPU classify one half of a record alone
_ID_SIG = bytes([0xC0]) + bytes(47)
_ID_PK = bytes([0xC0]) + bytes(95)


class PublicKey:
    BYTES = 96

    def __init__(self, raw: bytes):
        self._raw = bytes(raw)

    @classmethod
    def deserialize(cls, b: bytes) -> "PublicKey":
        b = bytes(b)
        if len(b) != cls.BYTES:
            raise DeserializeError(InvalidPublicKey.WrongLength)
        code = default_context().deserialize_codes(KIND_PK, [b])[0]      # decode kernels only
        if code == CODE_PK_POINT:
            raise DeserializeError(InvalidPublicKey.InvalidPoint)
        return cls(b)

    def serialize(self) -> bytes:
        return self._raw

    def verify(self, message: bytes, signature: "Signature") -> Result:
        code = default_context().verify_codes([(signature.serialize(), message, self._raw)])[0]
        return Result(code == CODE_OK)

    def __eq__(self, other):
        return isinstance(other, PublicKey) and other._raw == self._raw

    def __repr__(self):
        return f"PublicKey({self._raw.hex()})"


class Signature:
    BYTES = 48

    def __init__(self, raw: bytes):
        self._raw = bytes(raw)

    @classmethod
    def deserialize(cls, b: bytes) -> "Signature":
        b = bytes(b)
        if len(b) != cls.BYTES:
            raise DeserializeError(InvalidSignature.WrongLength)
        code = default_context().deserialize_codes(KIND_SIG, [b])[0]     # decode kernels only
        if code == CODE_SIG_POINT:
            raise DeserializeError(InvalidSignature.InvalidPoint)
        return cls(b)

    def serialize(self) -> bytes:
        return self._raw

    def __eq__(self, other):
        return isinstance(other, Signature) and other._raw == self._raw

    def __repr__(self):
        return f"Signature({self._raw.hex()})"


class PrivateKey:
    BYTES = 32

    def __init__(self, k: int):
        self._k = k

    @classmethod
    def random(cls) -> "PrivateKey":
        while True:   # rejection sampling, src/lib.rs:185-198
            k = int.from_bytes(secrets.token_bytes(32), "big")
            if k < R_ORDER:
                return cls(k)

    @classmethod
    def deserialize(cls, b: bytes) -> "PrivateKey":
        b = bytes(b)
        if len(b) != cls.BYTES:
            raise DeserializeError(InvalidPrivateKey.WrongLength)
        k = int.from_bytes(b, "big")
        if k >= R_ORDER:
            raise DeserializeError(InvalidPrivateKey.OutOfRange)
        return cls(k)

    def serialize(self) -> bytes:
        return self._k.to_bytes(32, "big")

    def public_key(self) -> PublicKey:
        return PublicKey(default_context().public_keys([self.serialize()])[0])

    def sign(self, message: bytes) -> Signature:
        return Signature(default_context().sign([self.serialize()], [bytes(message)])[0])

    def __eq__(self, other):
        return isinstance(other, PrivateKey) and other._k == self._k

    def __repr__(self):
        return "PrivateKey(REDACTED)"


def verify_bls_signature(sig: bytes, msg: bytes, key: bytes) -> Result:
    """verify_bls_signature (src/lib.rs:243-247)."""
    return Result(default_context().verify_codes([(sig, msg, key)])[0] == CODE_OK)


@dataclass
class Verdicts:
    bitmap: list      # u64 words, bit i%64 of word i//64 = record i verified
    codes: bytes      # per-record code (0 OK, 1..5 see CODE_NAMES)

    def ok(self, i: int) -> bool:
        return bool((self.bitmap[i >> 6] >> (i & 63)) & 1)


def verify_batch(records: Iterable[Tuple[bytes, bytes, bytes]], ctx: Optional[Context] = None,
                 dedup_keys: bool = True) -> Verdicts:
    """New batch entry point: records of (sig, msg, key) -> Verdicts.

    With dedup_keys, a fixed-size batch whose records share few keys (at most
    one distinct key per 8 records, e.g. TEE-signed audit verdicts) runs the
    keyed path: each distinct key is decoded and prepared once
    (cess_bls_keys_load).  A context whose key table a caller loaded
    (Context.load_keys) is never overwritten: then the batch runs the
    per-record path.  Codes are the same either way (tests/test_gpu_keyed.py)."""
    records = list(records)
    ctx = ctx or default_context()
    n = len(records)
    codes = None
    if dedup_keys and ctx._keys_owner != "user" and n >= 256 and all(len(r[0]) == 48 and len(r[2]) == 96 for r in records):
        kid = {}
        for r in records:
            kid.setdefault(bytes(r[2]), len(kid))
            if 8 * len(kid) > n:
                break
        if 8 * len(kid) <= n:
            ctx.load_keys(list(kid), _owner="verify_batch")
            msgs = [bytes(r[1]) for r in records]
            offs = [0]
            for m in msgs:
                offs.append(offs[-1] + len(m))
            codes, _ = ctx._verify_keyed_any(b"".join(bytes(r[0]) for r in records), [kid[bytes(r[2])] for r in records],
                                        b"".join(msgs), offs)
    if codes is None:
        codes = ctx.verify_codes(records)
    words = [0] * ((len(records) + 63) // 64)
    for i, c in enumerate(codes):
        if c == CODE_OK:
            words[i >> 6] |= 1 << (i & 63)
    return Verdicts(words, codes)
