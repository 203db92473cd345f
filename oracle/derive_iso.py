"""ORACLE TOOL (test infrastructure only): derive the RFC 9380 11-isogeny
E' -> E for BLS12381G1_XMD:SHA-256_SSWU_RO_ and write oracle/iso_g1.py.

Why: hash_to_g1 (reference src/lib.rs:25-31) goes through the bls12_381 0.7.1
crate, which is not in the container, and the isogeny coefficient tables of
RFC 9380 Appendix E.2 are not available offline.  They are a function of E'
alone, so they are re-derived here:

  1. E': y^2 = x^3 + A'x + B' (RFC 9380 §8.8.1 constants A', B', Z = 11).
     Sanity: #E'(Fp) must equal #E(Fp) (isogenous curves have equal order).
  2. E'(Fp) has rational 11-torsion (11^2 | #E).  For every order-11 subgroup
     K, Vélu's construction gives an isogeny E' -> E'/K.  Keep those whose
     codomain has j = 0, then compose with the isomorphisms
     (X, Y) -> (c^2 X, c^3 Y) onto y^2 = x^3 + 4.
  3. Among the candidates, the correct map is the one that reproduces the
     reference's signing KAT (tests/tests.rs:99-112, H(m) pinned exactly)
     and its valid-signature KATs.  Only one candidate does.

The map is written as x = xnum(x')/xden(x'), y = y' * ynum(x')/yden(x') with
monic xden (deg 10) and yden (deg 15), which is the normalisation RFC 9380 uses.
"""
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

P = None


def main():
    global P
    import importlib
    # bls_oracle imports iso_g1; write a placeholder first if absent
    here = os.path.dirname(os.path.abspath(__file__))
    iso_path = os.path.join(here, "iso_g1.py")
    A_ = 0x144698A3B8E9433D693A02C96D4982B0EA985383EE66A8D8E8981AEFD881AC98936F8DA0E0F97F5CF428082D584C1D
    B_ = 0x12E2908D11688030018B12E8753EEE3B2016C1F0F24F4070A0B9C14FCEF35EF55A23215A316CEAA5D1CC48E98E172BE0
    Z_ = 11
    if not os.path.exists(iso_path):
        with open(iso_path, "w") as f:
            f.write(f"ISO_A = {A_:#x}\nISO_B = {B_:#x}\nISO_Z = {Z_}\n"
                    "ISO_XNUM = ISO_XDEN = ISO_YNUM = ISO_YDEN = [1]\n")
    o = importlib.import_module("oracle.bls_oracle")
    P = o.P
    N = P + 1 - (o.X + 1)          # #E(Fp): trace t = x + 1
    assert N % o.R == 0
    rng = random.Random(11)

    def rand_point(a, b):
        while True:
            x = rng.randrange(P)
            y = o.fp_sqrt((x * x * x + a * x + b) % P)
            if y is not None:
                return (x, y)

    def mul(pt, k, a):
        acc = None
        for bit in bin(k)[2:]:
            acc = o.ec_add(o.FP, acc, acc, a)
            if bit == "1":
                acc = o.ec_add(o.FP, acc, pt, a)
        return acc

    # 1. order check of E'
    for _ in range(3):
        pt = rand_point(A_, B_)
        assert mul(pt, N, A_) is None, "E' constants inconsistent with #E"
    print("E' order check passed")

    # 2. 11-torsion points
    v11 = 0
    m = N
    while m % 11 == 0:
        m //= 11
        v11 += 1
    print("11-adic valuation of #E:", v11)
    kernels = {}
    for _ in range(40):
        q = mul(rand_point(A_, B_), m, A_)
        if q is None:
            continue
        # reduce to order exactly 11
        while True:
            q2 = mul(q, 11, A_)
            if q2 is None:
                break
            q = q2
        pts = [q]
        for _ in range(9):
            pts.append(o.ec_add(o.FP, pts[-1], q, A_))
        assert o.ec_add(o.FP, pts[-1], q, A_) is None
        key = frozenset(p_[0] for p_ in pts)
        kernels[key] = pts
    print("distinct order-11 kernels found:", len(kernels))

    def velu(pts, a, b):
        # S = one point of each {Q, -Q} pair
        S = []
        seen = set()
        for q in pts:
            if q[0] in seen:
                continue
            seen.add(q[0])
            S.append(q)
        assert len(S) == 5
        v = w = 0
        for (xq, yq) in S:
            gx = (3 * xq * xq + a) % P
            gy = (-2 * yq) % P
            vq = 2 * gx % P
            uq = gy * gy % P
            v = (v + vq) % P
            w = (w + uq + xq * vq) % P
        A2 = (a - 5 * v) % P
        B2 = (b - 7 * w) % P
        return S, A2, B2

    def phi(S, pt, a):
        # definitional Vélu map: x + sum_{Q in K*} (x(P+Q) - x(Q)), same for y
        X_, Y_ = pt
        for q in S:
            for qq in (q, (q[0], (-q[1]) % P)):
                s_ = o.ec_add(o.FP, pt, qq, a)
                X_ = (X_ + s_[0] - qq[0]) % P
                Y_ = (Y_ + s_[1] - qq[1]) % P
        return (X_, Y_)

    def poly_mul(f, g):
        r = [0] * (len(f) + len(g) - 1)
        for i, fi in enumerate(f):
            for j, gj in enumerate(g):
                r[i + j] = (r[i + j] + fi * gj) % P
        return r

    def interp(xs, ys):
        # Lagrange interpolation -> coefficient list (low degree first)
        n = len(xs)
        coeffs = [0] * n
        for i in range(n):
            num = [1]
            den = 1
            for j in range(n):
                if j == i:
                    continue
                num = poly_mul(num, [(-xs[j]) % P, 1])
                den = den * (xs[i] - xs[j]) % P
            s = ys[i] * pow(den, P - 2, P) % P
            for k in range(n):
                coeffs[k] = (coeffs[k] + s * num[k]) % P
        return coeffs

    def peval(c, x):
        acc = 0
        for ci in reversed(c):
            acc = (acc * x + ci) % P
        return acc

    candidates = []
    for pts in kernels.values():
        S, A2, B2 = velu(pts, A_, B_)
        if A2 != 0:
            continue
        # denominators
        xden = [1]
        yden = [1]
        for (xq, _) in S:
            lin = [(-xq) % P, 1]
            xden = poly_mul(xden, poly_mul(lin, lin))
            yden = poly_mul(yden, poly_mul(lin, poly_mul(lin, lin)))
        # sample points, interpolate numerators
        samples = [rand_point(A_, B_) for _ in range(16)]
        imgs = [phi(S, s_, A_) for s_ in samples]
        for (X_, Y_) in imgs:
            assert (Y_ * Y_ - X_ ** 3 - B2) % P == 0
        xs = [s_[0] for s_ in samples]
        xnum = interp(xs[:12], [imgs[i][0] * peval(xden, xs[i]) % P for i in range(12)])
        ynum = interp(xs, [imgs[i][1] * peval(yden, xs[i]) % P * pow(samples[i][1], P - 2, P) % P
                           for i in range(16)])
        # isomorphisms onto y^2 = x^3 + 4: c^6 = 4 / B2
        t = 4 * pow(B2, P - 2, P) % P
        # sixth roots of t
        roots = []
        g = 2
        while pow(g, (P - 1) // 2, P) == 1 or pow(g, (P - 1) // 3, P) == 1:
            g += 1
        zeta6 = pow(g, (P - 1) // 6, P)
        # find one root: t^(1/6) via t^(1/2) then cube root by exhaustive exponent trick
        c2 = o.fp_sqrt(t)
        if c2 is None:
            continue
        for sgn in (c2, (-c2) % P):
            # cube root of sgn (p = 1 mod 3: use Adleman-Manders-Miller-lite via search)
            cr = _cube_root(sgn)
            if cr is None:
                continue
            for k in range(6):
                c = cr * pow(zeta6, k, P) % P
                if pow(c, 6, P) == t and c not in roots:
                    roots.append(c)
        for c in roots:
            c2_, c3_ = c * c % P, c * c * c % P
            candidates.append(([x * c2_ % P for x in xnum], xden,
                               [y * c3_ % P for y in ynum], yden))
    print("candidate maps:", len(candidates))

    # 3. pick the candidate reproducing the reference KATs
    sk = 0x6F3977F6051E184B2C412DAA1B5C0115EF7AB347CAC8D808FFA2C26BD0658243
    msg = bytes.fromhex(
        "50484522ad8aede64ec7f86b9273b7ed3940481acf93cdd40a2b77f2be2734a14012b2492b6363b12adaeaf055c573e4611b"
        "085d2e0fe2153d72453a95eaebf350ac3ba6a26ba0bc79f4c0bf5664dfdf5865f69f7fc6b58ba7d068e8")
    expected = "8f7ad830632657f7b3eae17fd4c3d9ff5c13365eea8d33fd0a1a6d8fbebc5152e066bb0ad61ab64e8a8541c8e3f96de9"
    winners = []
    for cand in candidates:
        o.ISO_XNUM, o.ISO_XDEN, o.ISO_YNUM, o.ISO_YDEN = cand
        # bls_oracle binds the names at import: patch module globals
        o.__dict__["ISO_XNUM"], o.__dict__["ISO_XDEN"] = cand[0], cand[1]
        o.__dict__["ISO_YNUM"], o.__dict__["ISO_YDEN"] = cand[2], cand[3]
        if o.sign(sk, msg).hex() == expected:
            winners.append(cand)
    print("candidates matching the signing KAT:", len(winners))
    assert len(winners) == 1
    xnum, xden, ynum, yden = winners[0]
    assert xden[-1] == 1 and yden[-1] == 1 and len(xnum) == 12 and len(ynum) == 16
    with open(iso_path, "w") as f:
        f.write('"""GENERATED by oracle/derive_iso.py — RFC 9380 11-isogeny E\' -> E for G1.\n'
                'Oracle/test data (also the source of the device constant tables).\n'
                'Coefficient lists are low-degree first; xden/yden are monic."""\n')
        f.write(f"ISO_A = {A_:#x}\nISO_B = {B_:#x}\nISO_Z = {Z_}\n")
        for name, c in (("ISO_XNUM", xnum), ("ISO_XDEN", xden), ("ISO_YNUM", ynum), ("ISO_YDEN", yden)):
            f.write(f"{name} = [\n")
            for ci in c:
                f.write(f"    {ci:#098x},\n")
            f.write("]\n")
    print("wrote", iso_path)


def _cube_root(a):
    # p = 1 mod 3.  Tonelli-Shanks style for cube roots.
    if a == 0:
        return 0
    if pow(a, (P - 1) // 3, P) != 1:
        return None
    s, t = 0, P - 1
    while t % 3 == 0:
        t //= 3
        s += 1
    # find a cubic non-residue
    g = 2
    while pow(g, (P - 1) // 3, P) == 1:
        g += 1
    c = pow(g, t, P)  # generator of the 3-Sylow
    # brute force: x = a^k * c^j; use baby steps since 3^s is small
    k = pow(3, -1, t) if t % 3 else None
    if k is not None:
        x0 = pow(a, k, P)        # x0^3 = a^(3k) = a * a^(3k-1); a^(3k-1) in 3-Sylow
        err = pow(x0, 3, P) * pow(a, P - 2, P) % P
        # find j with (c^j)^3 = err^-1
        inv_err = pow(err, P - 2, P)
        cj = 1
        c3 = pow(c, 3, P)
        acc = 1
        for j in range(3 ** s):
            if acc == inv_err:
                return x0 * cj % P
            acc = acc * c3 % P
            cj = cj * c % P
    return None


if __name__ == "__main__":
    main()
