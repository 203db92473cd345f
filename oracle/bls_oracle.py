"""CPU ORACLE (test infrastructure only) — pure-Python restatement of the
BLS12-381 "minimal-signature-size" verifier used by CESS.

NOT PART OF THE PRODUCT.  Only `tests/`, `__graft_entry__.smoke()` and the
`cpu_baseline` leg of `bench.py` may import this module, and only as the checker.

What it restates
----------------
Reference crate: /root/reference/utils/verify-bls-signatures (ic-verify-bls-signature 0.2.0)
  * verify_bls_signature            src/lib.rs:243-247
  * Signature::deserialize          src/lib.rs:138-152  (G1Affine::from_compressed, :144)
  * PublicKey::deserialize          src/lib.rs:68-82    (G2Affine::from_compressed, :74)
  * PublicKey::verify               src/lib.rs:85-100   (multi_miller_loop + final_exponentiation)
  * hash_to_g1 / DST                src/lib.rs:23-31
  * G2PREPARED_NEG_G                src/lib.rs:19-21
  * PrivateKey::{deserialize,serialize,public_key,sign}  src/lib.rs:200-236
The arithmetic lives in the third-party crate `bls12_381` 0.7.1 (Cargo.lock:576-587,
not vendored, not in this container).  Its published algorithms are restated here:
  * ZCash compressed point encoding (flags c/i/s in the top 3 bits of byte 0)
  * RFC 9380 hash_to_curve BLS12381G1_XMD:SHA-256_SSWU_RO_ (expand_message_xmd,
    simple SWU on the 11-isogenous curve E', 11-isogeny, h_eff = 0xd201000000010001)
  * optimal-ate Miller loop over |x| with Jacobian G2 line coefficients
    (Costello-Lange-Naehrig, eprint 2010/354 Alg. 26/27) and mul_by_014
  * final exponentiation: easy part (p^6-1)(p^2+1), hard part built from five
    cyclotomic exponentiations by x  ==>  Gt = (textbook reduced pairing)^3
Parity pinning: every KAT in utils/verify-bls-signatures/tests/tests.rs is checked
in tests/test_oracle_kat.py (verdicts, G1 subgroup rejection, G2 off-curve rejection,
exact signature bytes — which pins hash_to_g1 bit-for-bit).  Gt values are not pinned
by any reference test ("parity unpinned" for Gt; verdicts are pinned).
"""
import hashlib

# ---------------------------------------------------------------------------
# Curve parameters (all derived from the BLS parameter x; nothing recalled)
# ---------------------------------------------------------------------------
BLS_X = 0xd201000000010000          # |x|, x is negative
X = -BLS_X
R = X**4 - X**2 + 1                 # subgroup order r (255 bits)
P = (X - 1) ** 2 * R // 3 + X       # base field modulus p (381 bits)
assert P.bit_length() == 381 and R.bit_length() == 255
assert P % 4 == 3 and P % 6 == 1
H1 = (X - 1) ** 2 // 3              # G1 cofactor
H_EFF_G1 = 1 - X                    # = 0xd201000000010001 (RFC 9380 h_eff for G1)

DST = b"BLS_SIG_BLS12381G1_XMD:SHA-256_SSWU_RO_NUL_"   # src/lib.rs:23
assert len(DST) == 43

# verdict codes of the build, precedence sig → key → pairing
OK, SIG_LEN, SIG_POINT, PK_LEN, PK_POINT, PAIRING_FAIL = range(6)


# ---------------------------------------------------------------------------
# Fp
# ---------------------------------------------------------------------------
def fp_inv(a):
    return pow(a, P - 2, P)


def fp_sqrt(a):
    """Square root for p = 3 mod 4, or None."""
    y = pow(a, (P + 1) // 4, P)
    return y if y * y % P == a % P else None


def fp_lex_largest(a):
    return a > (P - 1) // 2


# ---------------------------------------------------------------------------
# Fp2 = Fp[u]/(u^2+1): tuples (c0, c1)
# ---------------------------------------------------------------------------
F2_ZERO = (0, 0)
F2_ONE = (1, 0)


def f2_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2_neg(a):
    return ((-a[0]) % P, (-a[1]) % P)


def f2_mul(a, b):
    a0, a1 = a
    b0, b1 = b
    return ((a0 * b0 - a1 * b1) % P, (a0 * b1 + a1 * b0) % P)


def f2_sqr(a):
    a0, a1 = a
    return ((a0 + a1) * (a0 - a1) % P, 2 * a0 * a1 % P)


def f2_muls(a, s):
    return (a[0] * s % P, a[1] * s % P)


def f2_conj(a):
    return (a[0], (-a[1]) % P)


def f2_inv(a):
    t = fp_inv((a[0] * a[0] + a[1] * a[1]) % P)
    return (a[0] * t % P, (-a[1]) * t % P)


def f2_mul_nr(a):
    """multiply by the Fp6 non-residue xi = u + 1"""
    return ((a[0] - a[1]) % P, (a[0] + a[1]) % P)


def f2_pow(a, e):
    r = F2_ONE
    base = a
    while e:
        if e & 1:
            r = f2_mul(r, base)
        base = f2_sqr(base)
        e >>= 1
    return r


def f2_is_square(a):
    # a is a square in Fp2 iff its norm is a square in Fp
    n = (a[0] * a[0] + a[1] * a[1]) % P
    return n == 0 or pow(n, (P - 1) // 2, P) == 1


def f2_sqrt(a):
    """Some square root of a in Fp2, or None (which root does not matter:
    the caller fixes the sign by the lexicographic rule)."""
    if a == F2_ZERO:
        return F2_ZERO
    if not f2_is_square(a):
        return None
    # p^2 = 9 mod 16: use the generic (p^2+7)/16 exponent with a correction
    # by a fourth/eighth root of unity search — simple and exact.
    c = f2_pow(a, (P * P + 7) // 16)
    # candidates: c * zeta for zeta in 8th roots of unity
    for z in _EIGHTH_ROOTS:
        y = f2_mul(c, z)
        if f2_sqr(y) == a:
            return y
    raise AssertionError("f2_sqrt failed on a square")


def _find_eighth_roots():
    # a primitive 8th root of unity in Fp2: (1+u)^((p^2-1)/8) is not always
    # primitive; search small elements.
    e = (P * P - 1) // 8
    for c0 in range(1, 50):
        for c1 in range(0, 50):
            g = f2_pow((c0, c1), e)
            if f2_pow(g, 4) != F2_ONE:       # primitive 8th root
                roots = [F2_ONE]
                for _ in range(7):
                    roots.append(f2_mul(roots[-1], g))
                return roots
    raise AssertionError


_EIGHTH_ROOTS = _find_eighth_roots()


def f2_lex_largest(a):
    return fp_lex_largest(a[1]) or (a[1] == 0 and fp_lex_largest(a[0]))


# ---------------------------------------------------------------------------
# Fp6 = Fp2[v]/(v^3 - xi), Fp12 = Fp6[w]/(w^2 - v)
# ---------------------------------------------------------------------------
F6_ZERO = (F2_ZERO, F2_ZERO, F2_ZERO)
F6_ONE = (F2_ONE, F2_ZERO, F2_ZERO)
F12_ONE = (F6_ONE, F6_ZERO)


def f6_add(a, b):
    return (f2_add(a[0], b[0]), f2_add(a[1], b[1]), f2_add(a[2], b[2]))


def f6_sub(a, b):
    return (f2_sub(a[0], b[0]), f2_sub(a[1], b[1]), f2_sub(a[2], b[2]))


def f6_neg(a):
    return (f2_neg(a[0]), f2_neg(a[1]), f2_neg(a[2]))


def f6_mul(a, b):
    a0, a1, a2 = a
    b0, b1, b2 = b
    t0 = f2_mul(a0, b0)
    t1 = f2_mul(a1, b1)
    t2 = f2_mul(a2, b2)
    c0 = f2_add(t0, f2_mul_nr(f2_add(f2_mul(a1, b2), f2_mul(a2, b1))))
    c1 = f2_add(f2_add(f2_mul(a0, b1), f2_mul(a1, b0)), f2_mul_nr(t2))
    c2 = f2_add(f2_add(f2_mul(a0, b2), f2_mul(a2, b0)), t1)
    return (c0, c1, c2)


def f6_mul_by_v(a):
    """a * v"""
    return (f2_mul_nr(a[2]), a[0], a[1])


def f6_inv(a):
    a0, a1, a2 = a
    c0 = f2_sub(f2_sqr(a0), f2_mul_nr(f2_mul(a1, a2)))
    c1 = f2_sub(f2_mul_nr(f2_sqr(a2)), f2_mul(a0, a1))
    c2 = f2_sub(f2_sqr(a1), f2_mul(a0, a2))
    t = f2_add(f2_mul(a0, c0), f2_mul_nr(f2_add(f2_mul(a2, c1), f2_mul(a1, c2))))
    t = f2_inv(t)
    return (f2_mul(c0, t), f2_mul(c1, t), f2_mul(c2, t))


def f12_mul(a, b):
    a0, a1 = a
    b0, b1 = b
    t0 = f6_mul(a0, b0)
    t1 = f6_mul(a1, b1)
    c1 = f6_sub(f6_sub(f6_mul(f6_add(a0, a1), f6_add(b0, b1)), t0), t1)
    c0 = f6_add(t0, f6_mul_by_v(t1))
    return (c0, c1)


def f12_sqr(a):
    return f12_mul(a, a)


def f12_conj(a):
    return (a[0], f6_neg(a[1]))


def f12_inv(a):
    a0, a1 = a
    t = f6_sub(f6_mul(a0, a0), f6_mul_by_v(f6_mul(a1, a1)))
    t = f6_inv(t)
    return (f6_mul(a0, t), f6_neg(f6_mul(a1, t)))


def f12_pow(a, e):
    r = F12_ONE
    base = a
    while e:
        if e & 1:
            r = f12_mul(r, base)
        base = f12_sqr(base)
        e >>= 1
    return r


# Frobenius: element = sum_i a_i w^i (i = 0..5, a_i in Fp2); w^6 = xi.
# (sum a_i w^i)^p = sum conj(a_i) * gamma_i * w^i, gamma_i = xi^(i(p-1)/6).
_XI = (1, 1)
_GAMMA1 = [f2_pow(_XI, i * (P - 1) // 6) for i in range(6)]


def _f12_to_w(a):
    (c00, c01, c02), (c10, c11, c12) = a
    return [c00, c10, c01, c11, c02, c12]


def _f12_from_w(v):
    return ((v[0], v[2], v[4]), (v[1], v[3], v[5]))


def f12_frob(a):
    v = _f12_to_w(a)
    return _f12_from_w([f2_mul(f2_conj(v[i]), _GAMMA1[i]) for i in range(6)])


def f12_mul_by_014(f, c0, c1, c4):
    """f * (c0 + c1*v + c4*v*w)  — sparse line multiplication (bls12_381 mul_by_014)."""
    line = ((c0, c1, F2_ZERO), (F2_ZERO, c4, F2_ZERO))
    return f12_mul(f, line)


# ---------------------------------------------------------------------------
# Curves: G1: y^2 = x^3 + 4 over Fp, G2: y^2 = x^3 + 4(u+1) over Fp2.
# Affine points are tuples (x, y) or None for the identity.
# ---------------------------------------------------------------------------
B1 = 4
B2 = (4, 4)

G1_GEN = (
    0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB,
    0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1,
)
G2_GEN = (
    (0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
     0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E),
    (0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
     0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE),
)


# generic affine group law over a field given as ops (used for G1, E' and G2)
class _Field:
    def __init__(self, add, sub, mul, sqr, inv, neg, zero, one, muls):
        self.add, self.sub, self.mul, self.sqr = add, sub, mul, sqr
        self.inv, self.neg, self.zero, self.one, self.muls = inv, neg, zero, one, muls


FP = _Field(lambda a, b: (a + b) % P, lambda a, b: (a - b) % P, lambda a, b: a * b % P,
            lambda a: a * a % P, fp_inv, lambda a: (-a) % P, 0, 1, lambda a, s: a * s % P)
FP2 = _Field(f2_add, f2_sub, f2_mul, f2_sqr, f2_inv, f2_neg, F2_ZERO, F2_ONE, f2_muls)


def on_curve(F, pt, a, b):
    if pt is None:
        return True
    x, y = pt
    rhs = F.add(F.add(F.mul(F.sqr(x), x), F.mul(a, x)), b)
    return F.sqr(y) == rhs


def ec_add(F, p1, p2, a=None):
    """Affine addition on y^2 = x^3 + a x + b (a=None means a=0)."""
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    x1, y1 = p1
    x2, y2 = p2
    if x1 == x2:
        if y1 == y2 and y1 != F.zero:
            num = F.muls(F.sqr(x1), 3)
            if a is not None:
                num = F.add(num, a)
            lam = F.mul(num, F.inv(F.muls(y1, 2)))
        else:
            return None
    else:
        lam = F.mul(F.sub(y2, y1), F.inv(F.sub(x2, x1)))
    x3 = F.sub(F.sub(F.sqr(lam), x1), x2)
    y3 = F.sub(F.mul(lam, F.sub(x1, x3)), y1)
    return (x3, y3)


def ec_neg(F, pt):
    return None if pt is None else (pt[0], F.neg(pt[1]))


# Jacobian-coordinate scalar multiplication (a = 0 curves) for speed
def _jac_dbl(F, Pj):
    X1, Y1, Z1 = Pj
    if Z1 == F.zero:
        return Pj
    A = F.sqr(X1)
    Bq = F.sqr(Y1)
    C = F.sqr(Bq)
    D = F.muls(F.sub(F.sub(F.sqr(F.add(X1, Bq)), A), C), 2)
    E = F.muls(A, 3)
    Fq = F.sqr(E)
    X3 = F.sub(Fq, F.muls(D, 2))
    Y3 = F.sub(F.mul(E, F.sub(D, X3)), F.muls(C, 8))
    Z3 = F.muls(F.mul(Y1, Z1), 2)
    return (X3, Y3, Z3)


def _jac_add_aff(F, Pj, Q):
    X1, Y1, Z1 = Pj
    if Q is None:
        return Pj
    if Z1 == F.zero:
        return (Q[0], Q[1], F.one)
    x2, y2 = Q
    Z1Z1 = F.sqr(Z1)
    U2 = F.mul(x2, Z1Z1)
    S2 = F.mul(F.mul(y2, Z1), Z1Z1)
    H = F.sub(U2, X1)
    Rr = F.sub(S2, Y1)
    if H == F.zero:
        if Rr == F.zero:
            return _jac_dbl(F, Pj)
        return (F.one, F.one, F.zero)
    HH = F.sqr(H)
    HHH = F.mul(H, HH)
    V = F.mul(X1, HH)
    X3 = F.sub(F.sub(F.sqr(Rr), HHH), F.muls(V, 2))
    Y3 = F.sub(F.mul(Rr, F.sub(V, X3)), F.mul(Y1, HHH))
    Z3 = F.mul(Z1, H)
    return (X3, Y3, Z3)


def _jac_to_aff(F, Pj):
    X1, Y1, Z1 = Pj
    if Z1 == F.zero:
        return None
    zi = F.inv(Z1)
    zi2 = F.sqr(zi)
    return (F.mul(X1, zi2), F.mul(Y1, F.mul(zi, zi2)))


def ec_mul(F, pt, k):
    """k * pt for a = 0 curves (G1, G2)."""
    if pt is None or k == 0:
        return None
    if k < 0:
        return ec_mul(F, ec_neg(F, pt), -k)
    acc = (F.one, F.one, F.zero)
    for bit in bin(k)[2:]:
        acc = _jac_dbl(F, acc)
        if bit == "1":
            acc = _jac_add_aff(F, acc, pt)
    return _jac_to_aff(F, acc)


def g1_in_subgroup(pt):
    return ec_mul(FP, pt, R) is None


def g2_in_subgroup(pt):
    return ec_mul(FP2, pt, R) is None


# ---------------------------------------------------------------------------
# ZCash compressed encodings (bls12_381 G1Affine/G2Affine::{to,from}_compressed)
# ---------------------------------------------------------------------------
def g1_to_compressed(pt):
    if pt is None:
        out = bytearray(48)
        out[0] = 0xC0
        return bytes(out)
    x, y = pt
    out = bytearray(x.to_bytes(48, "big"))
    out[0] |= 0x80
    if fp_lex_largest(y):
        out[0] |= 0x20
    return bytes(out)


def g2_to_compressed(pt):
    if pt is None:
        out = bytearray(96)
        out[0] = 0xC0
        return bytes(out)
    (x0, x1), y = pt
    out = bytearray(x1.to_bytes(48, "big") + x0.to_bytes(48, "big"))
    out[0] |= 0x80
    if f2_lex_largest(y):
        out[0] |= 0x20
    return bytes(out)


class Invalid(Exception):
    pass


def g1_from_compressed(b):
    """Returns affine point (None = identity) or raises Invalid.
    Acceptance rules: SURVEY Appendix A.1 (bls12_381 G1Affine::from_compressed,
    called at src/lib.rs:144)."""
    assert len(b) == 48
    c, i, s = (b[0] >> 7) & 1, (b[0] >> 6) & 1, (b[0] >> 5) & 1
    x = int.from_bytes(bytes([b[0] & 0x1F]) + b[1:], "big")
    if x >= P:
        raise Invalid("x not canonical")
    if i and c and not s and x == 0:
        return None
    y = fp_sqrt((x * x * x + B1) % P)
    if y is None:
        raise Invalid("not on curve")
    if fp_lex_largest(y) != bool(s):
        y = (-y) % P
    if i or not c:
        raise Invalid("bad flags")
    pt = (x, y)
    if not g1_in_subgroup(pt):
        raise Invalid("not in G1")
    return pt


def g2_from_compressed(b):
    """Rules: SURVEY Appendix A.1 (bls12_381 G2Affine::from_compressed, src/lib.rs:74)."""
    assert len(b) == 96
    c, i, s = (b[0] >> 7) & 1, (b[0] >> 6) & 1, (b[0] >> 5) & 1
    x1 = int.from_bytes(bytes([b[0] & 0x1F]) + b[1:48], "big")
    x0 = int.from_bytes(b[48:96], "big")
    if x1 >= P or x0 >= P:
        raise Invalid("x not canonical")
    x = (x0, x1)
    if i and c and not s and x == F2_ZERO:
        return None
    y = f2_sqrt(f2_add(f2_mul(f2_sqr(x), x), B2))
    if y is None:
        raise Invalid("not on curve")
    if f2_lex_largest(y) != bool(s):
        y = f2_neg(y)
    if i or not c:
        raise Invalid("bad flags")
    pt = (x, y)
    if not g2_in_subgroup(pt):
        raise Invalid("not in G2")
    return pt


# ---------------------------------------------------------------------------
# RFC 9380 hash_to_curve for G1 (src/lib.rs:25-31)
# ---------------------------------------------------------------------------
def expand_message_xmd(msg, dst, len_in_bytes):
    b_in, r_in = 32, 64
    ell = (len_in_bytes + b_in - 1) // b_in
    assert ell <= 255 and len(dst) <= 255
    dst_prime = dst + bytes([len(dst)])
    msg_prime = bytes(r_in) + msg + len_in_bytes.to_bytes(2, "big") + b"\x00" + dst_prime
    b0 = hashlib.sha256(msg_prime).digest()
    b = [hashlib.sha256(b0 + b"\x01" + dst_prime).digest()]
    for i in range(2, ell + 1):
        x = bytes(u ^ v for u, v in zip(b0, b[-1]))
        b.append(hashlib.sha256(x + bytes([i]) + dst_prime).digest())
    return b"".join(b)[:len_in_bytes]


def hash_to_field_fp(msg, count, dst=DST):
    L = 64
    u = expand_message_xmd(msg, dst, count * L)
    return [int.from_bytes(u[i * L:(i + 1) * L], "big") % P for i in range(count)]


from oracle.iso_g1 import ISO_A, ISO_B, ISO_Z, ISO_XNUM, ISO_XDEN, ISO_YNUM, ISO_YDEN  # noqa: E402


def _sgn0(a):
    return a & 1


def map_to_curve_sswu(u):
    """RFC 9380 §6.6.2 simplified SWU onto E': y^2 = x^3 + A'x + B'."""
    A, Bc, Z = ISO_A, ISO_B, ISO_Z
    tv1 = (Z * Z * pow(u, 4, P) + Z * u * u) % P
    tv1 = 0 if tv1 == 0 else fp_inv(tv1)
    if tv1 == 0:
        x1 = Bc * fp_inv(Z * A % P) % P
    else:
        x1 = (-Bc) * fp_inv(A) % P * (1 + tv1) % P
    gx1 = (x1 * x1 * x1 + A * x1 + Bc) % P
    y1 = fp_sqrt(gx1)
    if y1 is not None:
        x, y = x1, y1
    else:
        x = Z * u * u % P * x1 % P
        gx2 = (x * x * x + A * x + Bc) % P
        y = fp_sqrt(gx2)
        assert y is not None
    if _sgn0(u) != _sgn0(y):
        y = (-y) % P
    return (x, y)


def _poly_eval(coeffs, x):
    acc = 0
    for c in reversed(coeffs):
        acc = (acc * x + c) % P
    return acc


def iso_map_g1(pt):
    """11-isogeny E' -> E (coefficients derived by oracle/derive_iso.py)."""
    x, y = pt
    xd = _poly_eval(ISO_XDEN, x)
    yd = _poly_eval(ISO_YDEN, x)
    if xd == 0 or yd == 0:
        return None
    xn = _poly_eval(ISO_XNUM, x)
    yn = _poly_eval(ISO_YNUM, x)
    return (xn * fp_inv(xd) % P, y * yn % P * fp_inv(yd) % P)


def hash_to_g1(msg, dst=DST):
    u0, u1 = hash_to_field_fp(msg, 2, dst)
    q0 = iso_map_g1(map_to_curve_sswu(u0))
    q1 = iso_map_g1(map_to_curve_sswu(u1))
    r = ec_add(FP, q0, q1)
    return ec_mul(FP, r, H_EFF_G1)


# ---------------------------------------------------------------------------
# Pairing: G2Prepared (Jacobian doubling/addition line coefficients) +
# multi Miller loop + final exponentiation  (src/lib.rs:85-100)
# ---------------------------------------------------------------------------
def _doubling_step(r):
    """eprint 2010/354 Alg. 26 adaptation; r = [X, Y, Z] (Jacobian, Fp2); returns (c0, c1, c2)."""
    rx, ry, rz = r
    tmp0 = f2_sqr(rx)
    tmp1 = f2_sqr(ry)
    tmp2 = f2_sqr(tmp1)
    tmp3 = f2_sub(f2_sub(f2_sqr(f2_add(tmp1, rx)), tmp0), tmp2)
    tmp3 = f2_add(tmp3, tmp3)
    tmp4 = f2_add(f2_add(tmp0, tmp0), tmp0)
    tmp6 = f2_add(rx, tmp4)
    tmp5 = f2_sqr(tmp4)
    zsq = f2_sqr(rz)
    nx = f2_sub(f2_sub(tmp5, tmp3), tmp3)
    nz = f2_sub(f2_sub(f2_sqr(f2_add(rz, ry)), tmp1), zsq)
    ny = f2_mul(f2_sub(tmp3, nx), tmp4)
    tmp2 = f2_muls(tmp2, 8)
    ny = f2_sub(ny, tmp2)
    t3 = f2_neg(f2_muls(f2_mul(tmp4, zsq), 2))
    t6 = f2_sub(f2_sub(f2_sqr(tmp6), tmp0), tmp5)
    t6 = f2_sub(t6, f2_muls(tmp1, 4))
    t0 = f2_muls(f2_mul(nz, zsq), 2)
    r[0], r[1], r[2] = nx, ny, nz
    return (t0, t3, t6)


def _addition_step(r, q):
    """eprint 2010/354 Alg. 27 adaptation; q affine G2."""
    rx, ry, rz = r
    qx, qy = q
    zsq = f2_sqr(rz)
    ysq = f2_sqr(qy)
    t0 = f2_mul(zsq, qx)
    t1 = f2_mul(f2_sub(f2_sub(f2_sqr(f2_add(qy, rz)), ysq), zsq), zsq)
    t2 = f2_sub(t0, rx)
    t3 = f2_sqr(t2)
    t4 = f2_muls(t3, 4)
    t5 = f2_mul(t4, t2)
    t6 = f2_sub(f2_sub(t1, ry), ry)
    t9 = f2_mul(t6, qx)
    t7 = f2_mul(t4, rx)
    nx = f2_sub(f2_sub(f2_sub(f2_sqr(t6), t5), t7), t7)
    nz = f2_sub(f2_sub(f2_sqr(f2_add(rz, t2)), zsq), t3)
    t10 = f2_add(qy, nz)
    t8 = f2_mul(f2_sub(t7, nx), t6)
    t0 = f2_muls(f2_mul(ry, t5), 2)
    ny = f2_sub(t8, t0)
    t10 = f2_sub(f2_sub(f2_sqr(t10), ysq), f2_sqr(nz))
    t9 = f2_sub(f2_add(t9, t9), t10)
    t10 = f2_add(nz, nz)
    t6 = f2_neg(t6)
    t1 = f2_add(t6, t6)
    r[0], r[1], r[2] = nx, ny, nz
    return (t10, t1, t9)


# bits of |x| >> 1 below the leading one, MSB first (62 entries, 5 ones)
_LOOP_BITS = [((BLS_X >> 1) >> b) & 1 for b in range(62, -1, -1)]
assert _LOOP_BITS[0] == 1
_LOOP_BITS = _LOOP_BITS[1:]


def g2_prepare(q):
    """G2Prepared::from (src/lib.rs:20, :88): 68 coefficient triples.
    The identity is replaced by the generator and flagged (infinity=True)."""
    infinity = q is None
    if infinity:
        q = G2_GEN
    r = [q[0], q[1], F2_ONE]
    coeffs = []
    for bit in _LOOP_BITS:
        coeffs.append(_doubling_step(r))
        if bit:
            coeffs.append(_addition_step(r, q))
    coeffs.append(_doubling_step(r))
    assert len(coeffs) == 68
    return (infinity, coeffs)


def _ell(f, coeffs, p1):
    c0 = f2_muls(coeffs[0], p1[1])
    c1 = f2_muls(coeffs[1], p1[0])
    return f12_mul_by_014(f, coeffs[2], c1, c0)


def multi_miller_loop(terms):
    """terms: list of (G1 affine or None, prepared G2)."""
    f = F12_ONE
    idx = 0

    def step(f, idx):
        for p1, (inf, coeffs) in terms:
            if p1 is None or inf:
                continue
            f = _ell(f, coeffs[idx], p1)
        return f

    for bit in _LOOP_BITS:
        f = step(f, idx)
        idx += 1
        if bit:
            f = step(f, idx)
            idx += 1
        f = f12_sqr(f)
    f = step(f, idx)
    idx += 1
    assert idx == 68
    return f12_conj(f)   # x is negative


def _cyc_exp(f):
    """f^|x| then conjugate (= f^x in the cyclotomic subgroup)."""
    tmp = F12_ONE
    found = False
    for b in range(63, -1, -1):
        bit = (BLS_X >> b) & 1
        if found:
            tmp = f12_sqr(tmp)
        else:
            found = bool(bit)
        if bit:
            tmp = f12_mul(tmp, f)
    return f12_conj(tmp)


def final_exponentiation(f):
    """bls12_381 MillerLoopResult::final_exponentiation (src/lib.rs:93)."""
    t0 = f
    for _ in range(6):
        t0 = f12_frob(t0)
    t1 = f12_inv(f)
    t2 = f12_mul(t0, t1)
    t1 = t2
    t2 = f12_frob(f12_frob(t2))
    t2 = f12_mul(t2, t1)
    t1 = f12_conj(f12_sqr(t2))
    t3 = _cyc_exp(t2)
    t4 = f12_sqr(t3)
    t5 = f12_mul(t1, t3)
    t1 = _cyc_exp(t5)
    t0 = _cyc_exp(t1)
    t6 = _cyc_exp(t0)
    t6 = f12_mul(t6, t4)
    t4 = _cyc_exp(t6)
    t5 = f12_conj(t5)
    t4 = f12_mul(t4, f12_mul(t5, t2))
    t5 = f12_conj(t2)
    t1 = f12_mul(t1, t2)
    t1 = f12_frob(f12_frob(f12_frob(t1)))
    t6 = f12_mul(t6, t5)
    t6 = f12_frob(t6)
    t3 = f12_mul(t3, t0)
    t3 = f12_frob(f12_frob(t3))
    t3 = f12_mul(t3, t1)
    t3 = f12_mul(t3, t6)
    return f12_mul(t3, t4)


def pairing(p1, q2):
    return final_exponentiation(multi_miller_loop([(p1, g2_prepare(q2))]))


NEG_G2_PREPARED = None


def _neg_g2_prepared():
    global NEG_G2_PREPARED
    if NEG_G2_PREPARED is None:
        NEG_G2_PREPARED = g2_prepare(ec_neg(FP2, G2_GEN))
    return NEG_G2_PREPARED


def gt_to_bytes(f):
    """576 B: 12 big-endian Fp in tower order c0.c0.c0, c0.c0.c1, ..., c1.c2.c1."""
    out = b""
    for c6 in f:
        for c2 in c6:
            for c in c2:
                out += c.to_bytes(48, "big")
    return out


def verify_gt(sig_pt, msg, pk_pt):
    """PublicKey::verify (src/lib.rs:85-100) returning the Gt element."""
    h = hash_to_g1(msg)
    f = multi_miller_loop([(sig_pt, _neg_g2_prepared()), (h, g2_prepare(pk_pt))])
    return final_exponentiation(f)


def verify_code(sig, msg, key):
    """verify_bls_signature (src/lib.rs:243-247) as a build verdict code (A6)."""
    if len(sig) != 48:
        return SIG_LEN
    try:
        s = g1_from_compressed(sig)
    except Invalid:
        return SIG_POINT
    if len(key) != 96:
        return PK_LEN
    try:
        k = g2_from_compressed(key)
    except Invalid:
        return PK_POINT
    gt = verify_gt(s, msg, k)
    return OK if gt == F12_ONE else PAIRING_FAIL


def verify_bls_signature(sig, msg, key):
    return verify_code(sig, msg, key) == OK


# ---------------------------------------------------------------------------
# PrivateKey (src/lib.rs:166-236)
# ---------------------------------------------------------------------------
def sk_deserialize(b):
    """32-B big-endian scalar < r (src/lib.rs:208-223); returns int or raises."""
    if len(b) != 32:
        raise Invalid("WrongLength")
    k = int.from_bytes(b, "big")
    if k >= R:
        raise Invalid("OutOfRange")
    return k


def sk_serialize(k):
    return k.to_bytes(32, "big")


def public_key(k):
    return g2_to_compressed(ec_mul(FP2, G2_GEN, k))


def sign(k, msg):
    return g1_to_compressed(ec_mul(FP, hash_to_g1(msg), k))
