"""CPU oracle (TEST INFRASTRUCTURE ONLY) for SURVEY §8(f) rank 4: the RSA
PKCS#1 v1.5 raw signature check behind cp_enclave_verify::verify_rsa
(/root/reference/primitives/enclave-verify/src/lib.rs:221-228):

    let pk = rsa::RsaPublicKey::from_public_key_der(key).unwrap();
    match pk.verify(Pkcs1v15Sign::new_raw(), msg, sig) { Ok(()) => true, Err(_) => false }

The arithmetic lives in the third-party crate `rsa` 0.8.2
(/root/reference/Cargo.lock:6538-6541), which is NOT vendored in the reference
and not in this image, so this module restates its published behaviour:

* from_public_key_der: SubjectPublicKeyInfo DER (RFC 5280) with algorithm
  rsaEncryption (1.2.840.113549.1.1.1) wrapping an RFC 8017 RSAPublicKey
  SEQUENCE { INTEGER n, INTEGER e }; the key checks of rsa 0.8
  (RsaPublicKey::new -> check_public: n at most 4096 bits, 2 <= e <= 2^33 - 1).
  Failure -> the reference panics.  The crate's check_public has no parity or
  size-floor check on n and its AlgorithmIdentifier handling asserts the OID
  only, so even moduli, n = 1 and non-NULL parameters parse here (unpinned:
  the GPU library reports such keys CESS_RSA_E_UNSUPPORTED, never BAD_KEY).
* Pkcs1v15Sign::new_raw(): no DigestInfo prefix and no hash-length check, so
  the signed "hashed" value is the message bytes themselves.
* verify (RFC 8017 RSASSA-PKCS1-v1_5-VERIFY with an empty T prefix):
  k = byte length of n; sig.len() == k and s < n, else Err; m = s^e mod n;
  EM = I2OSP(m, k); require k >= len(msg) + 11 and
  EM == 0x00 || 0x01 || 0xff * (k - len(msg) - 3) || 0x00 || msg.

PARITY UNPINNED: the reference's only test of this path
(enclave-verify/src/lib.rs:242-255, `cryptos_rsa`) signs with a freshly
generated random key and prints the result (no assertion, no fixed vector),
and the crate cannot be built here (no Rust toolchain).  The golden fixtures
(tests/golden/rsa_vectors.json, tests/golden/gen_rsa.py) are produced by this
restatement; they include the reference test's own message ("hello world!").

Codes (mirrored by the GPU kernel and include/cess_rsa.h):
  0 OK, 1 SIG_LEN (len != k), 2 SIG_RANGE (s >= n), 3 MSG_LEN (k < len + 11),
  4 MISMATCH (EM is not the raw PKCS#1 v1.5 encoding of msg).
"""
from __future__ import annotations

RSA_OID = bytes.fromhex("2a864886f70d010101")      # 1.2.840.113549.1.1.1
MAX_BITS = 4096
MIN_E, MAX_E = 2, (1 << 33) - 1

OK, SIG_LEN, SIG_RANGE, MSG_LEN, MISMATCH = range(5)


class KeyError_(ValueError):
    """from_public_key_der(key).unwrap() would panic."""


# --- minimal DER (definite lengths only, as DER requires) ---------------------
def _tlv(b: bytes, pos: int):
    if pos + 2 > len(b):
        raise KeyError_("truncated")
    tag = b[pos]
    ln = b[pos + 1]
    pos += 2
    if ln & 0x80:
        nb = ln & 0x7F
        if nb == 0 or nb > 4 or pos + nb > len(b):
            raise KeyError_("bad length")
        ln = int.from_bytes(b[pos:pos + nb], "big")
        if ln < 0x80 or b[pos] == 0:
            raise KeyError_("non-minimal length")
        pos += nb
    if pos + ln > len(b):
        raise KeyError_("truncated value")
    return tag, b[pos:pos + ln], pos + ln


def _uint(v: bytes) -> int:
    if not v or v[0] & 0x80:
        raise KeyError_("negative or empty INTEGER")
    if len(v) > 1 and v[0] == 0 and not v[1] & 0x80:
        raise KeyError_("non-minimal INTEGER")
    return int.from_bytes(v, "big")


def parse_pkcs1(der: bytes):
    """RSAPublicKey ::= SEQUENCE { modulus INTEGER, publicExponent INTEGER }"""
    tag, body, end = _tlv(der, 0)
    if tag != 0x30 or end != len(der):
        raise KeyError_("not a SEQUENCE")
    t1, vn, p = _tlv(body, 0)
    t2, ve, p = _tlv(body, p)
    if t1 != 0x02 or t2 != 0x02 or p != len(body):
        raise KeyError_("bad RSAPublicKey")
    return _check(_uint(vn), _uint(ve))


def parse_spki(der: bytes):
    """SubjectPublicKeyInfo with rsaEncryption (what from_public_key_der accepts)."""
    tag, body, end = _tlv(der, 0)
    if tag != 0x30 or end != len(der):
        raise KeyError_("not a SEQUENCE")
    ta, alg, p = _tlv(body, 0)
    tb, bits, p = _tlv(body, p)
    if ta != 0x30 or tb != 0x03 or p != len(body):
        raise KeyError_("bad SubjectPublicKeyInfo")
    to, oid, q = _tlv(alg, 0)
    if to != 0x06 or oid != RSA_OID:
        raise KeyError_("not rsaEncryption")
    if q != len(alg):
        tn, nul, q = _tlv(alg, q)       # any single parameters element (OID checked only)
        if q != len(alg):
            raise KeyError_("bad parameters")
    if not bits or bits[0] != 0:
        raise KeyError_("unused bits")
    return parse_pkcs1(bits[1:])


def _check(n: int, e: int):
    if n.bit_length() > MAX_BITS or n == 0:
        raise KeyError_("modulus")
    if not MIN_E <= e <= MAX_E:
        raise KeyError_("exponent")
    return n, e


def der_len(n: int) -> bytes:
    if n < 0x80:
        return bytes([n])
    b = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([0x80 | len(b)]) + b


def der_int(v: int) -> bytes:
    b = v.to_bytes(max(1, (v.bit_length() + 8) // 8), "big")
    return b"\x02" + der_len(len(b)) + b


def encode_pkcs1(n: int, e: int) -> bytes:
    body = der_int(n) + der_int(e)
    return b"\x30" + der_len(len(body)) + body


def encode_spki(n: int, e: int) -> bytes:
    alg = b"\x06" + der_len(len(RSA_OID)) + RSA_OID + b"\x05\x00"
    alg = b"\x30" + der_len(len(alg)) + alg
    bits = b"\x00" + encode_pkcs1(n, e)
    body = alg + b"\x03" + der_len(len(bits)) + bits
    return b"\x30" + der_len(len(body)) + body


# --- verify (rsa 0.8.2 pkcs1v15 verify with Pkcs1v15Sign::new_raw()) ----------
# The crate answers every failure below with Error::Verification (verify_rsa:
# false); the distinct codes are this build's refinement, in the precedence the
# GPU path applies them: lengths first (k_rsa_classify), then the range and the
# encoded message (k_rsa_verify_*).
def verify_code(n: int, e: int, msg: bytes, sig: bytes) -> int:
    k = (n.bit_length() + 7) // 8
    if len(sig) != k:
        return SIG_LEN
    if k < len(msg) + 11:
        return MSG_LEN
    s = int.from_bytes(sig, "big")
    if s >= n:
        return SIG_RANGE
    em = pow(s, e, n).to_bytes(k, "big")
    want = b"\x00\x01" + b"\xff" * (k - len(msg) - 3) + b"\x00" + msg
    return OK if em == want else MISMATCH


def verify_rsa(key_der: bytes, msg: bytes, sig: bytes) -> bool:
    """cp_enclave_verify::verify_rsa; raises KeyError_ where the reference panics."""
    n, e = parse_spki(key_der)
    return verify_code(n, e, msg, sig) == OK


def sign_raw(n: int, d: int, msg: bytes) -> bytes:
    """RsaPrivateKey::sign(Pkcs1v15Sign::new_raw(), msg) (fixture generation)."""
    k = (n.bit_length() + 7) // 8
    em = b"\x00\x01" + b"\xff" * (k - len(msg) - 3) + b"\x00" + msg
    return pow(int.from_bytes(em, "big"), d, n).to_bytes(k, "big")


# --- deterministic key generation for fixtures --------------------------------
def _is_probable_prime(m: int, rng) -> bool:
    if m < 2:
        return False
    for p in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        if m % p == 0:
            return m == p
    d, s = m - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for _ in range(24):
        a = rng.randrange(2, m - 2)
        x = pow(a, d, m)
        if x in (1, m - 1):
            continue
        for _ in range(s - 1):
            x = x * x % m
            if x == m - 1:
                break
        else:
            return False
    return True


def gen_key(bits: int, e: int, rng):
    while True:
        ps = []
        for half in (bits // 2, bits - bits // 2):
            while True:
                c = rng.getrandbits(half) | (3 << (half - 2)) | 1
                if _is_probable_prime(c, rng) and (c - 1) % e:
                    ps.append(c)
                    break
        n = ps[0] * ps[1]
        if n.bit_length() == bits and ps[0] != ps[1]:
            phi = (ps[0] - 1) * (ps[1] - 1)
            return n, e, pow(e, -1, phi)
