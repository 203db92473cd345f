"""Generate cess_amd/csrc/bls/consts.hpp: every BLS12-381 constant the HIP
kernels need, in 12 x u32 little-endian limbs (Montgomery form, R = 2^384,
unless the name says RAW).

Everything is computed from the curve parameter x and the RFC 9380 E' curve,
except the 11-isogeny coefficient table (RFC 9380 Appendix E.2), which is given
literally below (low degree first; xden/yden monic).  Run:
    python cess_amd/csrc/gen_consts.py
"""
import hashlib
import os
import struct

BLS_X = 0xd201000000010000
X = -BLS_X
R = X**4 - X**2 + 1
P = (X - 1) ** 2 * R // 3 + X
RM = 1 << 392   # Montgomery radix: 14 x 28-bit compute limbs

ISO_A = 0x144698a3b8e9433d693a02c96d4982b0ea985383ee66a8d8e8981aefd881ac98936f8da0e0f97f5cf428082d584c1d
ISO_B = 0x12e2908d11688030018b12e8753eee3b2016c1f0f24f4070a0b9c14fcef35ef55a23215a316ceaa5d1cc48e98e172be0
ISO_Z = 11
ISO_XNUM = [
    0x11a05f2b1e833340b809101dd99815856b303e88a2d7005ff2627b56cdb4e2c85610c2d5f2e62d6eaeac1662734649b7,
    0x17294ed3e943ab2f0588bab22147a81c7c17e75b2f6a8417f565e33c70d1e86b4838f2a6f318c356e834eef1b3cb83bb,
    0x0d54005db97678ec1d1048c5d10a9a1bce032473295983e56878e501ec68e25c958c3e3d2a09729fe0179f9dac9edcb0,
    0x1778e7166fcc6db74e0609d307e55412d7f5e4656a8dbf25f1b33289f1b330835336e25ce3107193c5b388641d9b6861,
    0x0e99726a3199f4436642b4b3e4118e5499db995a1257fb3f086eeb65982fac18985a286f301e77c451154ce9ac8895d9,
    0x1630c3250d7313ff01d1201bf7a74ab5db3cb17dd952799b9ed3ab9097e68f90a0870d2dcae73d19cd13c1c66f652983,
    0x0d6ed6553fe44d296a3726c38ae652bfb11586264f0f8ce19008e218f9c86b2a8da25128c1052ecaddd7f225a139ed84,
    0x17b81e7701abdbe2e8743884d1117e53356de5ab275b4db1a682c62ef0f2753339b7c8f8c8f475af9ccb5618e3f0c88e,
    0x080d3cf1f9a78fc47b90b33563be990dc43b756ce79f5574a2c596c928c5d1de4fa295f296b74e956d71986a8497e317,
    0x169b1f8e1bcfa7c42e0c37515d138f22dd2ecb803a0c5c99676314baf4bb1b7fa3190b2edc0327797f241067be390c9e,
    0x10321da079ce07e272d8ec09d2565b0dfa7dccdde6787f96d50af36003b14866f69b771f8c285decca67df3f1605fb7b,
    0x06e08c248e260e70bd1e962381edee3d31d79d7e22c837bc23c0bf1bc24c6b68c24b1b80b64d391fa9c8ba2e8ba2d229,
]
ISO_XDEN = [
    0x08ca8d548cff19ae18b2e62f4bd3fa6f01d5ef4ba35b48ba9c9588617fc8ac62b558d681be343df8993cf9fa40d21b1c,
    0x12561a5deb559c4348b4711298e536367041e8ca0cf0800c0126c2588c48bf5713daa8846cb026e9e5c8276ec82b3bff,
    0x0b2962fe57a3225e8137e629bff2991f6f89416f5a718cd1fca64e00b11aceacd6a3d0967c94fedcfcc239ba5cb83e19,
    0x03425581a58ae2fec83aafef7c40eb545b08243f16b1655154cca8abc28d6fd04976d5243eecf5c4130de8938dc62cd8,
    0x13a8e162022914a80a6f1d5f43e7a07dffdfc759a12062bb8d6b44e833b306da9bd29ba81f35781d539d395b3532a21e,
    0x0e7355f8e4e667b955390f7f0506c6e9395735e9ce9cad4d0a43bcef24b8982f7400d24bc4228f11c02df9a29f6304a5,
    0x0772caacf16936190f3e0c63e0596721570f5799af53a1894e2e073062aede9cea73b3538f0de06cec2574496ee84a3a,
    0x14a7ac2a9d64a8b230b3f5b074cf01996e7f63c21bca68a81996e1cdf9822c580fa5b9489d11e2d311f7d99bbdcc5a5e,
    0x0a10ecf6ada54f825e920b3dafc7a3cce07f8d1d7161366b74100da67f39883503826692abba43704776ec3a79a1d641,
    0x095fc13ab9e92ad4476d6e3eb3a56680f682b4ee96f7d03776df533978f31c1593174e4b4b7865002d6384d168ecdd0a,
    0x000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000001,
]
ISO_YNUM = [
    0x090d97c81ba24ee0259d1f094980dcfa11ad138e48a869522b52af6c956543d3cd0c7aee9b3ba3c2be9845719707bb33,
    0x134996a104ee5811d51036d776fb46831223e96c254f383d0f906343eb67ad34d6c56711962fa8bfe097e75a2e41c696,
    0x00cc786baa966e66f4a384c86a3b49942552e2d658a31ce2c344be4b91400da7d26d521628b00523b8dfe240c72de1f6,
    0x01f86376e8981c217898751ad8746757d42aa7b90eeb791c09e4a3ec03251cf9de405aba9ec61deca6355c77b0e5f4cb,
    0x08cc03fdefe0ff135caf4fe2a21529c4195536fbe3ce50b879833fd221351adc2ee7f8dc099040a841b6daecf2e8fedb,
    0x16603fca40634b6a2211e11db8f0a6a074a7d0d4afadb7bd76505c3d3ad5544e203f6326c95a807299b23ab13633a5f0,
    0x04ab0b9bcfac1bbcb2c977d027796b3ce75bb8ca2be184cb5231413c4d634f3747a87ac2460f415ec961f8855fe9d6f2,
    0x0987c8d5333ab86fde9926bd2ca6c674170a05bfe3bdd81ffd038da6c26c842642f64550fedfe935a15e4ca31870fb29,
    0x09fc4018bd96684be88c9e221e4da1bb8f3abd16679dc26c1e8b6e6a1f20cabe69d65201c78607a360370e577bdba587,
    0x0e1bba7a1186bdb5223abde7ada14a23c42a0ca7915af6fe06985e7ed1e4d43b9b3f7055dd4eba6f2bafaaebca731c30,
    0x19713e47937cd1be0dfd0b8f1d43fb93cd2fcbcb6caf493fd1183e416389e61031bf3a5cce3fbafce813711ad011c132,
    0x18b46a908f36f6deb918c143fed2edcc523559b8aaf0c2462e6bfe7f911f643249d9cdf41b44d606ce07c8a4d0074d8e,
    0x0b182cac101b9399d155096004f53f447aa7b12a3426b08ec02710e807b4633f06c851c1919211f20d4c04f00b971ef8,
    0x0245a394ad1eca9b72fc00ae7be315dc757b3b080d4c158013e6632d3c40659cc6cf90ad1c232a6442d9d3f5db980133,
    0x05c129645e44cf1102a159f748c4a3fc5e673d81d7e86568d9ab0f5d396a7ce46ba1049b6579afb7866b1e715475224b,
    0x15e6be4e990f03ce4ea50b3b42df2eb5cb181d8f84965a3957add4fa95af01b2b665027efec01c7704b456be69c8b604,
]
ISO_YDEN = [
    0x16112c4c3a9c98b252181140fad0eae9601a6de578980be6eec3232b5be72e7a07f3688ef60c206d01479253b03663c1,
    0x1962d75c2381201e1a0cbd6c43c348b885c84ff731c4d59ca4a10356f453e01f78a4260763529e3532f6102c2e49a03d,
    0x058df3306640da276faaae7d6e8eb15778c4855551ae7f310c35a5dd279cd2eca6757cd636f96f891e2538b53dbf67f2,
    0x16b7d288798e5395f20d23bf89edb4d1d115c5dbddbcd30e123da489e726af41727364f2c28297ada8d26d98445f5416,
    0x0be0e079545f43e4b00cc912f8228ddcc6d19c9f0f69bbb0542eda0fc9dec916a20b15dc0fd2ededda39142311a5001d,
    0x08d9e5297186db2d9fb266eaac783182b70152c65550d881c5ecd87b6f0f5a6449f38db9dfa9cce202c6477faaf9b7ac,
    0x166007c08a99db2fc3ba8734ace9824b5eecfdfa8d0cf8ef5dd365bc400a0051d5fa9c01a58b1fb93d1a1399126a775c,
    0x16a3ef08be3ea7ea03bcddfabba6ff6ee5a4375efa1f4fd7feb34fd206357132b920f5b00801dee460ee415a15812ed9,
    0x1866c8ed336c61231a1be54fd1d74cc4f9fb0ce4c6af5920abc5750c4bf39b4852cfe2f7bb9248836b233d9d55535d4a,
    0x167a55cda70a6e1cea820597d94a84903216f763e13d87bb5308592e7ea7d4fbc7385ea3d529b35e346ef48bb8913f55,
    0x04d2f259eea405bd48f010a01ad2911d9c6dd039bb61a6290e591b36e636a5c871a5c29f4f83060400f8b49cba8f6aa8,
    0x0accbb67481d033ff5852c1e48c50c477f94ff8aefce42d28c0f9a88cea7913516f968986f7ebbea9684b529e2561092,
    0x0ad6b9514c767fe3c3613144b45f1496543346d98adf02267d5ceef9a00d9b8693000763e3b90ac11e99b138573345cc,
    0x02660400eb2e4f3b628bdd0d53cd76f2bf565b94e72927c1cb748df27942480e420517bd8714cc80d1fadc1326ed06f7,
    0x0e0fa1d816ddc03e6b24255e0d7819c171c40f65e273b853324efcd6356caa205ca2f570f13497804415473a1d634b8f,
    0x000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000001,
]

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
DST = b"BLS_SIG_BLS12381G1_XMD:SHA-256_SSWU_RO_NUL_"


def mont(a):
    return a * RM % P


def limbs(v, n=12):
    return [(v >> (32 * i)) & 0xFFFFFFFF for i in range(n)]


def f2mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def f2pow(a, e):
    r = (1, 0)
    while e:
        if e & 1:
            r = f2mul(r, a)
        a = f2mul(a, a)
        e >>= 1
    return r


def f2inv(a):
    t = pow((a[0] ** 2 + a[1] ** 2) % P, P - 2, P)
    return (a[0] * t % P, -a[1] * t % P)


# --- small affine helpers just for self-checks of the endomorphism constants
def add_aff(pa, pb, mul, sub, inv, zero, three, two):
    if pa is None:
        return pb
    if pb is None:
        return pa
    (x1, y1), (x2, y2) = pa, pb
    if x1 == x2:
        if y1 != y2 or y1 == zero:
            return None
        lam = mul(mul(three, mul(x1, x1)), inv(mul(two, y1)))
    else:
        lam = mul(sub(y2, y1), inv(sub(x2, x1)))
    x3 = sub(sub(mul(lam, lam), x1), x2)
    return (x3, sub(mul(lam, sub(x1, x3)), y1))


def smul(pt, k, ops):
    neg = k < 0
    k = abs(k)
    acc = None
    for bit in bin(k)[2:]:
        acc = add_aff(acc, acc, *ops)
        if bit == "1":
            acc = add_aff(acc, pt, *ops)
    if neg and acc is not None:
        acc = (acc[0], ops[1](ops[3], acc[1]))
    return acc


FP_OPS = (lambda a, b: a * b % P, lambda a, b: (a - b) % P, lambda a: pow(a, P - 2, P), 0, 3, 2)
FP2_OPS = (f2mul, lambda a, b: ((a[0] - b[0]) % P, (a[1] - b[1]) % P), f2inv, (0, 0), (3, 0), (2, 0))


def sha256_compress(state, block):
    k = [
        0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
        0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
        0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
        0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
        0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
        0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
        0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
        0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2]
    M = 0xFFFFFFFF

    def rotr(v, n):
        return ((v >> n) | (v << (32 - n))) & M
    w = list(struct.unpack(">16I", block))
    for i in range(16, 64):
        s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3)
        s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10)
        w.append((w[i - 16] + s0 + w[i - 7] + s1) & M)
    a, b, c, d, e, f, g, h = state
    for i in range(64):
        S1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)
        ch = (e & f) ^ (~e & g)
        t1 = (h + S1 + ch + k[i] + w[i]) & M
        S0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)
        maj = (a & b) ^ (a & c) ^ (b & c)
        t2 = (S0 + maj) & M
        h, g, f, e, d, c, b, a = g, f, e, (d + t1) & M, c, b, a, (t1 + t2) & M
    return [(x + y) & M for x, y in zip(state, (a, b, c, d, e, f, g, h))]


SHA_IV = [0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19]


def main():
    out = []
    w = out.append
    w("// GENERATED by cess_amd/csrc/gen_consts.py — do not edit.")
    w("// BLS12-381 constants, 12 x u32 little-endian limbs; MONT = Montgomery form (R = 2^392).")
    w("#pragma once")
    w("#include <stdint.h>")
    w("#ifndef CESS_CONST")
    w("#define CESS_CONST static constexpr")
    w("#endif")
    w("namespace bls { namespace c {")

    def arr(name, v, n=12):
        w(f"CESS_CONST uint32_t {name}[{n}] = {{" + ", ".join(f"0x{x:08x}u" for x in limbs(v, n)) + "};")

    arr("P_RAW", P)
    arr("P2_RAW", 2 * P)   # field values live in [0, 2p) (field.hpp)
    arr("ONE", mont(1))
    arr("R2", RM * RM % P)
    arr("R2_384", (1 << 384) * RM * RM % P)   # mul(H, .) = H * 2^384 * R
    p28 = [(P >> (28 * i)) & 0xFFFFFFF for i in range(14)]
    w("CESS_CONST uint32_t P28[14] = {" + ", ".join(f"0x{x:07x}u" for x in p28) + "};")
    w(f"CESS_CONST uint32_t PINV28 = 0x{(-pow(P, -1, 1 << 28)) % (1 << 28):07x}u;")
    # lazy Fp2 product: column-wise multiple of p dominating every column of a
    # product of two values < 2^384 in 14 x 28-bit limbs (top limb < 2^20)
    L = [(1 << 28) - 1] * 13 + [(1 << 20) - 1]
    B = [sum(L[i] * L[k - i] for i in range(14) if 0 <= k - i < 14) for k in range(27)]
    D = sum(b << (28 * k) for k, b in enumerate(B))
    adj = (-D) % P
    for k in range(14):
        B[k] += (adj >> (28 * k)) & ((1 << 28) - 1)
    M = sum(b << (28 * k) for k, b in enumerate(B))
    assert M % P == 0 and M < (1 << 770) and max(B) < (1 << 60)
    w("CESS_CONST uint64_t LAZY_M28[27] = {" + ", ".join(f"0x{x:016x}ull" for x in B) + "};")
    # digit-wise negation: K - x with K = 0 mod p and every 28-bit digit of K at
    # least the largest digit of a value < 2^384 (2^28 - 1, top digit 2^20 - 1),
    # so K - x has non-negative digits (< 2^29) and represents -x mod p
    base = [(1 << 28) - 1] * 13 + [(1 << 20) - 1]
    bv = sum(b << (28 * k) for k, b in enumerate(base))
    adj = (-bv) % P
    K = [base[k] + ((adj >> (28 * k)) & ((1 << 28) - 1)) for k in range(14)]
    assert sum(k << (28 * i) for i, k in enumerate(K)) % P == 0 and max(K) < (1 << 29)
    w("CESS_CONST uint32_t NEG_K28[14] = {" + ", ".join(f"0x{x:08x}u" for x in K) + "};")
    arr("HALF", mont((P + 1) // 2))
    arr("P_HALF_RAW", (P - 1) // 2)
    # exponents (raw integers, little-endian words)
    arr("EXP_SQRT", (P + 1) // 4)
    arr("EXP_SQRT_RATIO", (P - 3) // 4)
    arr("EXP_INV", P - 2)
    arr("EXP_LEGENDRE", (P - 1) // 2)
    # safegcd inversion (field.hpp inv): p in 13 x 30-bit limbs, p^-1 mod 2^30,
    # and R^3 mod p, which turns the integer inverse of a Montgomery value aR
    # (a^-1 R^-1) back into Montgomery form a^-1 R with one product
    w("CESS_CONST int32_t P30[13] = {" + ", ".join(str((P >> (30 * i)) & ((1 << 30) - 1)) for i in range(13)) + "};")
    w(f"CESS_CONST uint32_t PINV30 = 0x{pow(P, -1, 1 << 30):08x}u;")
    arr("R3", RM ** 3 % P)
    arr("B1", mont(4))
    arr("B1_3", mont(12))
    arr("ISO_A", mont(ISO_A))
    arr("ISO_B", mont(ISO_B))
    arr("ISO_Z", mont(ISO_Z))
    # c2 = sqrt(-Z) for sqrt_ratio (any root: final sign is fixed by sgn0)
    c2 = pow((-ISO_Z) % P, (P + 1) // 4, P)
    assert c2 * c2 % P == (-ISO_Z) % P
    arr("SSWU_C2", mont(c2))
    for name, lst in (("ISO_XNUM", ISO_XNUM), ("ISO_XDEN", ISO_XDEN), ("ISO_YNUM", ISO_YNUM), ("ISO_YDEN", ISO_YDEN)):
        w(f"CESS_CONST uint32_t {name}[{len(lst)}][12] = {{")
        for v in lst:
            w("  {" + ", ".join(f"0x{x:08x}u" for x in limbs(mont(v))) + "},")
        w("};")
    # G1 endomorphism: phi(x, y) = (beta x, y) acts as [-x^2] on G1
    beta = None
    for cand in range(2, 40):
        b = pow(cand, (P - 1) // 3, P)
        if b == 1:
            continue
        for bb in (b, b * b % P):
            phi = (G1_GEN[0] * bb % P, G1_GEN[1])
            if phi == smul(G1_GEN, -(X * X), FP_OPS):
                beta = bb
        if beta:
            break
    assert beta
    arr("G1_BETA", mont(beta))
    # G2 psi: (conj(x) * PSI_X, conj(y) * PSI_Y) acts as [p] = [x] on G2
    xi = (1, 1)
    psi_x = f2inv(f2pow(xi, (P - 1) // 3))
    psi_y = f2inv(f2pow(xi, (P - 1) // 2))
    gx, gy = G2_GEN
    psi_g = (f2mul((gx[0], -gx[1] % P), psi_x), f2mul((gy[0], -gy[1] % P), psi_y))
    assert psi_g == smul(G2_GEN, X, FP2_OPS), "psi constant check"
    for name, v in (("PSI_X", psi_x), ("PSI_Y", psi_y)):
        arr(name + "_C0", mont(v[0]))
        arr(name + "_C1", mont(v[1]))
    # Frobenius coefficients gamma_{k,i} = xi^(i (p^k - 1)/6), k = 1..3, i = 0..5
    w("CESS_CONST uint32_t FROB[3][6][2][12] = {")
    for k in (1, 2, 3):
        w("  {")
        for i in range(6):
            g = f2pow(xi, i * (P ** k - 1) // 6)
            w("    {{" + ", ".join(f"0x{x:08x}u" for x in limbs(mont(g[0]))) + "}, {" +
              ", ".join(f"0x{x:08x}u" for x in limbs(mont(g[1]))) + "}},")
        w("  },")
    w("};")
    arr("G1_GEN_X", mont(G1_GEN[0]))
    arr("G1_GEN_Y", mont(G1_GEN[1]))
    arr("G2_GEN_X0", mont(G2_GEN[0][0]))
    arr("G2_GEN_X1", mont(G2_GEN[0][1]))
    arr("G2_GEN_Y0", mont(G2_GEN[1][0]))
    arr("G2_GEN_Y1", mont(G2_GEN[1][1]))
    arr("R_RAW", R, 8)
    # SHA-256: midstate after the 64-byte all-zero Z_pad block of expand_message_xmd
    mid = sha256_compress(SHA_IV, bytes(64))
    w("CESS_CONST uint32_t SHA_ZPAD_MID[8] = {" + ", ".join(f"0x{x:08x}u" for x in mid) + "};")
    dstp = DST + bytes([len(DST)])
    w(f"CESS_CONST uint32_t DST_PRIME_LEN = {len(dstp)};")
    w("CESS_CONST uint8_t DST_PRIME[44] = {" + ", ".join(str(b) for b in dstp) + "};")
    w("}}  // namespace bls::c")
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "bls", "consts.hpp")
    with open(path, "w") as f:
        f.write("\n".join(out) + "\n")
    print("wrote", path)


if __name__ == "__main__":
    main()
