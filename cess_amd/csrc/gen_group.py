"""Generate cess_amd/csrc/bls/group_prog.hpp: the lane-group verification
program of the small-batch (latency) path, k_group.hip.

One signature per wavefront: the 64 lanes of a wave cooperate on one pairing
check.  The whole computation after decoding and hashing -- the two-pair
Miller loop of PublicKey::verify (reference utils/verify-bls-signatures/src/
lib.rs:90-93) with the key's line coefficients computed on the fly
(G2Prepared::from, :88), the key's G2 subgroup check on the final point of
that iteration, and the final exponentiation (:93-95) -- is written here as a
data-flow graph of Fp2 operations and scheduled into ROUNDS.  In a round every
lane runs at most one operation of the round's kind:

  MUL   d = A * B         (lazy Fp2 product; A, B: a slot or a constant, or the
                           sum / difference of two slots; optional conjugate)
  SQR   d = A^2           (A as for MUL)
  LIN   d = (sum of +-slots) + xi * (sum of +-slots)   (up to 12 terms)
  INV   d = A^-1          (safegcd; one lane)

Values live in an LDS "register file" of Fp2 slots per wave; the register
allocator below assigns slots from the schedule's live ranges.  The schedule
is list scheduling by critical path, so independent work (the key's next
doubling step, the pair-0 line scalings) fills the lanes of the rounds the
accumulator's critical path needs anyway: a Miller step costs about two
product rounds and two combination rounds of ONE lane's latency each.

Everything is straight-line (no data-dependent branch): a pair whose point is
the identity is evaluated at P = (0, 0), which turns its line into a constant
Fp2 factor (exactly 1 for the normalised -G2 lines); any Fp2 factor of the
Miller value dies in the final exponentiation ((p^2 - 1) | (p^12 - 1)/r), so
the Gt value is unchanged and the (O, O) pair still yields one.

Fp12 elements are kept in the w-basis (f = sum f_i w^i, w^6 = xi = 1 + u); the
tower order of the reference (c_h.c_j, Fp12 = Fp6[w]/(w^2 - v)) is w-index
2j + h.

simulate() runs a program on Python integers (test infrastructure uses it to
pin the generated schedule against the golden Gt bytes before any GPU runs it).
Run:  python cess_amd/csrc/gen_group.py
"""
import heapq
import os

BLS_X = 0xd201000000010000
X = -BLS_X
R_ORD = X**4 - X**2 + 1
P = (X - 1) ** 2 * R_ORD // 3 + X
RM = 1 << 392
XI = (1, 1)

G2_GEN = (
    (0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
     0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E),
    (0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
     0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE),
)

LANES = 32   # operations per round: two lanes per operation (one per Fp2 component)
MAX_LIN_TERMS = 12
OP_MUL, OP_SQR, OP_LIN, OP_INV = 0, 1, 2, 3
OP_NAMES = {OP_MUL: "MUL", OP_SQR: "SQR", OP_LIN: "LIN", OP_INV: "INV"}


# --- Fp2 arithmetic on integers (constants, the -G2 lines, simulate()) --------
def f2add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2neg(a):
    return ((-a[0]) % P, (-a[1]) % P)


def f2mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def f2conj(a):
    return (a[0], (-a[1]) % P)


def f2inv(a):
    t = pow((a[0] * a[0] + a[1] * a[1]) % P, P - 2, P)
    return (a[0] * t % P, (-a[1]) * t % P)


def f2pow(a, e):
    r = (1, 0)
    while e:
        if e & 1:
            r = f2mul(r, a)
        a = f2mul(a, a)
        e >>= 1
    return r


def f2small(a, k):
    return (a[0] * k % P, a[1] * k % P)


# --- the data-flow graph -----------------------------------------------------
class H:
    """A handle: node id with a pending sign (negation is free: it is folded
    into the combinations that consume the value)."""
    __slots__ = ("n", "neg")

    def __init__(self, n, neg=False):
        self.n, self.neg = n, neg

    def __neg__(self):
        return H(self.n, not self.neg)


class Graph:
    def __init__(self, pool=None):
        self.kind = []      # "in", "const", "mul", "sqr", "lin", "inv"
        self.args = []
        self.consts = list(pool) if pool else []   # Fp2 integer values of const nodes (pool order)
        # pool: another program's constant pool, shared (its indices kept)
        self.pool_index = {v: i for i, v in enumerate(self.consts)}
        self.const_of = {}
        self.inputs = {}    # name -> node
        self.outputs = {}   # name -> node (+ sign folded by the caller)

    def _new(self, kind, args):
        self.kind.append(kind)
        self.args.append(args)
        return len(self.kind) - 1

    def inp(self, name):
        n = self._new("in", name)
        self.inputs[name] = n
        return H(n)

    def const(self, v):
        v = (v[0] % P, v[1] % P)
        if v not in self.const_of:
            if v not in self.pool_index:
                self.pool_index[v] = len(self.consts)
                self.consts.append(v)
            self.const_of[v] = self._new("const", self.pool_index[v])
        return H(self.const_of[v])

    # operands of MUL / SQR: a handle, or a 2-term sum of handles
    def _operand(self, x):
        """-> (node_a, node_b or None, sub_b, sign, conj)"""
        if isinstance(x, H):
            return (x.n, None, False, x.neg, False)
        tag = x[0]
        if tag == "conj":
            h = x[1]
            assert isinstance(h, H)
            return (h.n, None, False, h.neg, True)
        a, b = x[1], x[2]      # ("sum", a, b): a + b with handle signs
        if a.neg and b.neg:     # -a - b = -(a + b)
            return (a.n, b.n, False, True, False)
        if a.neg:               # -a + b = b - a
            return (b.n, a.n, True, False, False)
        return (a.n, b.n, b.neg, False, False)

    def mul(self, x, y):
        ox, oy = self._operand(x), self._operand(y)
        assert not (self.kind[ox[0]] == "const" and ox[1] is not None)
        n = self._new("mul", (ox[:3] + (ox[4],), oy[:3] + (oy[4],)))
        return H(n, ox[3] != oy[3])

    def sqr(self, x):
        ox = self._operand(x)
        return H(self._new("sqr", (ox[:3] + (ox[4],),)))   # (+-A)^2 = A^2

    def lin(self, terms, xi_terms=()):
        """sum(terms) + xi * sum(xi_terms); terms are handles (signs honoured);
        longer combinations are split into chained LINs."""
        t = [(h.n, h.neg) for h in terms]
        x = [(h.n, h.neg) for h in xi_terms]
        if not x and len(t) == 1:          # a (signed) copy: no operation
            return H(t[0][0], t[0][1])
        while len(t) + len(x) > MAX_LIN_TERMS:
            if len(x) > 1:
                k = min(len(x), MAX_LIN_TERMS)
                part = self._new("lin", (tuple(x[:k]), ()))
                x = [(part, False)] + x[k:]
            else:
                k = min(len(t), MAX_LIN_TERMS)
                part = self._new("lin", (tuple(t[:k]), ()))
                t = [(part, False)] + t[k:]
        return H(self._new("lin", (tuple(t), tuple(x))))

    def inv(self, x):
        h = x
        n = self._new("inv", (h.n,))
        return H(n, h.neg)

    def out(self, name, h):
        # an output is a positive value computed by the program
        if h.neg or self.kind[h.n] in ("in", "const"):
            h = H(self._new("lin", (((h.n, h.neg),), ())))
        self.outputs[name] = h.n


# --- Fp12 in the w-basis ----------------------------------------------------
def f12_mul(g, a, b):
    """dense a * b: 36 products, one combination per coefficient"""
    pr = {}
    for i in range(6):
        for j in range(6):
            if a[i] is None or b[j] is None:
                continue
            pr[(i, j)] = g.mul(a[i], b[j])
    out = []
    for k in range(6):
        t = [pr[(i, k - i)] for i in range(6) if 0 <= k - i < 6 and (i, k - i) in pr]
        x = [pr[(i, k + 6 - i)] for i in range(6) if 0 <= k + 6 - i < 6 and (i, k + 6 - i) in pr]
        out.append(g.lin(t, x) if (t or x) else None)
    return out


def f12_sqr(g, a):
    """a^2: 21 products (off-diagonal ones counted twice)"""
    pr = {}
    for i in range(6):
        for j in range(i, 6):
            pr[(i, j)] = g.sqr(a[i]) if i == j else g.mul(a[i], a[j])
    out = []
    for k in range(6):
        t, x = [], []
        for i in range(6):
            for j in range(i, 6):
                if i + j == k:
                    t += [pr[(i, j)]] * (1 if i == j else 2)
                elif i + j == k + 6:
                    x += [pr[(i, j)]] * (1 if i == j else 2)
        out.append(g.lin(t, x))
    return out


def f12_conj(a):
    """conj over Fp6: negate the odd w-coefficients (free: a sign)"""
    return [a[i] if i % 2 == 0 else -a[i] for i in range(6)]


def f12_frob(g, a, k):
    """coefficient i -> conj^k(a_i) * gamma_{k,i}, gamma_{k,i} = xi^(i (p^k - 1)/6)"""
    out = []
    for i in range(6):
        gam = f2pow(XI, i * (P ** k - 1) // 6)
        x = ("conj", a[i]) if k & 1 else a[i]
        if gam == (1, 0):
            out.append(g.mul(x, g.const((1, 0))) if k & 1 else a[i])
        else:
            out.append(g.mul(x, g.const(gam)))
    return out


def fp6_mul(g, a, b):
    """Fp6 = Fp2[v]/(v^3 - xi), schoolbook: 9 products"""
    pr = {(i, j): g.mul(a[i], b[j]) for i in range(3) for j in range(3)}
    c0 = g.lin([pr[(0, 0)]], [pr[(1, 2)], pr[(2, 1)]])
    c1 = g.lin([pr[(0, 1)], pr[(1, 0)]], [pr[(2, 2)]])
    c2 = g.lin([pr[(0, 2)], pr[(1, 1)], pr[(2, 0)]])
    return [c0, c1, c2]


def fp6_sqr(g, a):
    s = {(i, j): (g.sqr(a[i]) if i == j else g.mul(a[i], a[j])) for i in range(3) for j in range(i, 3)}
    c0 = g.lin([s[(0, 0)]], [s[(1, 2)], s[(1, 2)]])
    c1 = g.lin([s[(0, 1)], s[(0, 1)]], [s[(2, 2)]])
    c2 = g.lin([s[(0, 2)], s[(0, 2)], s[(1, 1)]])
    return [c0, c1, c2]


def fp6_inv(g, a):
    A = g.lin([g.sqr(a[0])], [-g.mul(a[1], a[2])])
    B = g.lin([-g.mul(a[0], a[1])], [g.sqr(a[2])])
    C = g.lin([g.sqr(a[1]), -g.mul(a[0], a[2])])
    N = g.lin([g.mul(a[0], A)], [g.mul(a[2], B), g.mul(a[1], C)])
    iN = g.inv(N)
    return [g.mul(A, iN), g.mul(B, iN), g.mul(C, iN)]


def f12_inv(g, a):
    """(c0 + c1 w)^-1 = (c0 - c1 w) / (c0^2 - v c1^2)"""
    c0, c1 = [a[0], a[2], a[4]], [a[1], a[3], a[5]]
    s0, s1 = fp6_sqr(g, c0), fp6_sqr(g, c1)
    # v * (x0, x1, x2) = (xi x2, x0, x1)
    t = [g.lin([s0[0]], [-s1[2]]), g.lin([s0[1], -s1[0]]), g.lin([s0[2], -s1[1]])]
    ti = fp6_inv(g, t)
    d0, d1 = fp6_mul(g, c0, ti), fp6_mul(g, c1, ti)
    return [d0[0], -d1[0], d0[1], -d1[1], d0[2], -d1[2]]


def cyc_sqr(g, a):
    """Granger-Scott squaring in the cyclotomic subgroup (field.hpp
    cyclotomic_square): 9 Fp2 squarings in one round, one combination each"""
    z0, z4, z3, z2, z1, z5 = a[0], a[2], a[4], a[1], a[3], a[5]
    sq = {}
    for nm, x in (("a0", z0), ("b0", z1), ("s0", ("sum", z0, z1)),
                  ("a1", z2), ("b1", z3), ("s1", ("sum", z2, z3)),
                  ("a2", z4), ("b2", z5), ("s2", ("sum", z4, z5))):
        sq[nm] = g.sqr(x)
    # fp4 square: c0 = xi b^2 + a^2, c1 = (a + b)^2 - a^2 - b^2
    def c0(q):
        return ([sq["a" + q]], [sq["b" + q]])

    def c1(q):
        return [sq["s" + q], -sq["a" + q], -sq["b" + q]]
    t0, x0 = c0("0")
    z0n = g.lin(t0 * 3 + [-z0] * 2, x0 * 3)            # 3 t0 - 2 z0
    z1n = g.lin(c1("0") * 3 + [z1] * 2)                 # 3 t1 + 2 z1
    t0b, x0b = c0("1")
    z4n = g.lin(t0b * 3 + [-z4] * 2, x0b * 3)          # 3 t0' - 2 z4
    z5n = g.lin(c1("1") * 3 + [z5] * 2)                 # 3 t1' + 2 z5
    z2n = g.lin([z2] * 2, c1("2") * 3)                  # 3 xi t3 + 2 z2
    t2, x2 = c0("2")
    z3n = g.lin(t2 * 3 + [-z3] * 2, x2 * 3)            # 3 t2 - 2 z3
    r = [None] * 6
    r[0], r[2], r[4], r[1], r[3], r[5] = z0n, z4n, z3n, z2n, z1n, z5n
    return r


def cyc_exp(g, a):
    """conj(a^|x|): 63 squarings, products at |x|'s bits 62, 60, 57, 48, 16"""
    t = a
    for b in range(62, -1, -1):
        t = cyc_sqr(g, t)
        if b in (62, 60, 57, 48, 16):
            t = f12_mul(g, t, a)
    return f12_conj(t)


def final_exp(g, f):
    """MillerLoopResult::final_exponentiation (bls12_381 0.7.1; the sequence of
    pairing.hpp final_exponentiation): easy part (p^6 - 1)(p^2 + 1), hard part
    from five cyclotomic exponentiations by x; result = e(..)^3, canonical."""
    t0 = f12_conj(f)
    t1 = f12_inv(g, f)
    t2 = f12_mul(g, t0, t1)
    t1 = t2
    t2 = f12_frob(g, t2, 2)
    t2 = f12_mul(g, t2, t1)
    t1 = f12_conj(cyc_sqr(g, t2))
    t3 = cyc_exp(g, t2)
    t4 = cyc_sqr(g, t3)
    t5 = f12_mul(g, t1, t3)
    t1 = cyc_exp(g, t5)
    t0 = cyc_exp(g, t1)
    t6 = cyc_exp(g, t0)
    t6 = f12_mul(g, t6, t4)
    t4 = cyc_exp(g, t6)
    t5 = f12_conj(t5)
    t5 = f12_mul(g, t5, t2)
    t4 = f12_mul(g, t4, t5)
    t5 = f12_conj(t2)
    t1 = f12_mul(g, t1, t2)
    t1 = f12_frob(g, t1, 3)
    t6 = f12_mul(g, t6, t5)
    t6 = f12_frob(g, t6, 1)
    t3 = f12_mul(g, t3, t0)
    t3 = f12_frob(g, t3, 2)
    t3 = f12_mul(g, t3, t1)
    t3 = f12_mul(g, t3, t6)
    t3 = f12_mul(g, t3, t4)
    return t3


# --- G2 line steps (pairing.hpp doubling_step / addition_step) -------------
def doubling_step(g, T):
    """projective R <- 2R and its tangent line (c0, c1, c2) (y_P, x_P, constant
    coefficients), as pairing.hpp doubling_step up to the factors that a
    projective point and a line may carry"""
    X_, Y_, Z_ = T
    B = g.sqr(Y_)
    YZ = g.mul(Y_, Z_)
    J = g.sqr(X_)
    A2 = g.mul(X_, Y_)                    # 2A
    W = g.sqr(("sum", Z_, Z_))            # 4 Z^2
    E = g.lin([], [W] * 3)                # 12 xi Z^2 = 3 b' Z^2
    F = g.lin([], [W] * 9)                # 3E
    c0 = g.lin([YZ, YZ])                  # H = 2YZ
    c1 = g.lin([-J] * 3)                  # -3 X^2
    c2 = g.lin([B], [-W] * 3)             # B - E
    nx = g.lin([g.mul(A2, ("sum", B, -F))] * 2)
    FE = g.mul(F, E)
    ny = g.lin([g.sqr(("sum", B, F))] + [-FE] * 4)   # (B + F)^2 - 12 E^2
    nz = g.lin([g.mul(B, YZ)] * 8)                   # 4 B H
    return (nx, ny, nz), (c0, c1, c2)


def addition_step(g, T, qx, qy):
    X_, Y_, Z_ = T
    th = g.lin([Y_, -g.mul(qy, Z_)])
    la = g.lin([X_, -g.mul(qx, Z_)])
    D = g.sqr(la)
    E3 = g.mul(la, D)
    G = g.mul(X_, D)
    Hh = g.lin([E3, g.mul(Z_, g.sqr(th)), -G, -G])
    nx = g.mul(la, Hh)
    ny = g.lin([g.mul(th, ("sum", G, -Hh)), -g.mul(Y_, E3)])
    nz = g.mul(Z_, E3)
    c2 = g.lin([g.mul(th, qx), -g.mul(la, qy)])
    return (nx, ny, nz), (la, -th, c2)


def loop_bit(b):
    return b in (61, 59, 56, 47, 15)


def line_steps():
    """the 68 steps of G2Prepared in Miller-loop order: (kind, square_after)"""
    steps = []
    for b in range(61, -1, -1):
        steps.append(["D", True])
        if loop_bit(b):
            steps[-1][1] = False
            steps.append(["A", True])
    steps.append(["D", False])
    return steps


# --- the constant -G2 table (G2PREPARED_NEG_G, src/lib.rs:19-21), normalised --
def neg_g2_lines():
    """68 lines of -G2, each scaled to c2 = 1 (integers).  Computed with the
    same projective steps on integers; any Fp2 multiple of a line gives the
    same Gt, and the normalised triple is unique."""
    qx, qy = G2_GEN[0], f2neg(G2_GEN[1])
    T = (qx, qy, (1, 0))
    out = []

    def dbl(T):
        X_, Y_, Z_ = T
        B, C = f2mul(Y_, Y_), f2mul(Z_, Z_)
        E = f2mul((12, 12), C)
        F = f2small(E, 3)
        H_ = f2small(f2mul(Y_, Z_), 2)
        J = f2mul(X_, X_)
        A2 = f2mul(X_, Y_)
        nx = f2small(f2mul(A2, f2sub(B, F)), 2)
        ny = f2sub(f2mul(f2add(B, F), f2add(B, F)), f2small(f2mul(E, E), 12))
        nz = f2small(f2mul(B, H_), 4)
        return (nx, ny, nz), (H_, f2neg(f2small(J, 3)), f2sub(B, E))

    def add(T):
        X_, Y_, Z_ = T
        th = f2sub(Y_, f2mul(qy, Z_))
        la = f2sub(X_, f2mul(qx, Z_))
        D = f2mul(la, la)
        E3 = f2mul(la, D)
        G = f2mul(X_, D)
        Hh = f2sub(f2add(E3, f2mul(Z_, f2mul(th, th))), f2small(G, 2))
        nx = f2mul(la, Hh)
        ny = f2sub(f2mul(th, f2sub(G, Hh)), f2mul(Y_, E3))
        nz = f2mul(Z_, E3)
        return (nx, ny, nz), (la, f2neg(th), f2sub(f2mul(th, qx), f2mul(la, qy)))

    for kind, _ in line_steps():
        T, c = (dbl(T) if kind == "D" else add(T))
        ic2 = f2inv(c[2])
        out.append((f2mul(c[0], ic2), f2mul(c[1], ic2)))
    return out


def build():
    g = Graph()
    # inputs: G1 points as Fp2 with c1 = 0 (zeros for an unused pair), the key
    p0x, p0y = g.inp("p0x"), g.inp("p0y")     # signature (pair 0, with -G2)
    p1x, p1y = g.inp("p1x"), g.inp("p1y")     # H(m)      (pair 1, with the key)
    qx, qy = g.inp("qx"), g.inp("qy")
    one = g.inp("one")                        # Fp2 one (the first step's Z)
    T = (qx, qy, one)
    f = None
    lines0 = neg_g2_lines()
    for s, (kind, square_after) in enumerate(line_steps()):
        # pair 1: the key's line of this step, from the running point T
        if kind == "D":
            T, (c0, c1, c2) = doubling_step(g, T)
        else:
            T, (c0, c1, c2) = addition_step(g, T, qx, qy)
        # l1 = c2 + (c1 x1) w^2 + (c0 y1) w^3;  l0 = 1 + (a x0) w^2 + (b y0) w^3
        C = g.mul(c1, p1x)
        D = g.mul(c0, p1y)
        a, b = lines0[s]
        A = g.mul(g.const(b), p0x)       # -G2 line (c0, c1, 1): c1 x0 at w^2, c0 y0 at w^3
        B_ = g.mul(g.const(a), p0y)
        # L = l0 l1 = [c + xi B D, 0, c A + C, c B + D, A C, A D + B C]
        L = [g.lin([c2], [g.mul(B_, D)]), None, g.lin([g.mul(c2, A), C]), g.lin([g.mul(c2, B_), D]),
             g.mul(A, C), g.lin([g.mul(A, D), g.mul(B_, C)])]
        if f is None:   # f = 1: f L = L (w^1 stays empty: f12_mul skips it)
            f = L
        else:
            f = f12_mul(g, f, L)
        if square_after:
            f = f12_sqr(g, f)
    f = f12_conj(f)   # x < 0
    # the key's subgroup check: psi(Q) == -[|x|]Q = -T (curve.hpp g2_psi_is_neg_proj)
    psi_x = f2inv(f2pow(XI, (P - 1) // 3))
    psi_y = f2inv(f2pow(XI, (P - 1) // 2))
    px = g.mul(("conj", qx), g.const(psi_x))
    py = g.mul(("conj", qy), g.const(psi_y))
    g.out("tx", T[0])
    g.out("ty", T[1])
    g.out("tz", T[2])
    g.out("pzx", g.mul(px, T[2]))
    g.out("pzy", g.mul(py, T[2]))
    gt = final_exp(g, f)
    for i in range(6):
        g.out(f"gt{i}", gt[i])
    return g


def build_fe(pool):
    """The final exponentiation alone (k_group_fe: one Miller-loop value or
    product per wave, the RLC checks): inputs f0..f5 (w-basis), outputs
    gt0..gt5; constants from the full program's pool (same indices)."""
    g = Graph(pool)
    f = [g.inp(f"f{i}") for i in range(6)]
    gt = final_exp(g, f)
    for i in range(6):
        g.out(f"gt{i}", gt[i])
    return g


# --- scheduling --------------------------------------------------------------
def deps(g, n):
    k, a = g.kind[n], g.args[n]
    if k in ("in", "const"):
        return []
    if k in ("mul", "sqr"):
        d = []
        for o in a:
            d.append(o[0])
            if o[1] is not None:
                d.append(o[1])
        return d
    if k == "lin":
        return [t[0] for t in a[0]] + [t[0] for t in a[1]]
    if k == "inv":
        return [a[0]]
    raise ValueError(k)


OPKIND = {"mul": OP_MUL, "sqr": OP_SQR, "lin": OP_LIN, "inv": OP_INV}
# relative latency of one round of each kind (lone wave, VALU-issue bound)
COST = {OP_MUL: 1.0, OP_SQR: 0.65, OP_LIN: 0.4, OP_INV: 18.0}


def reachable(g):
    seen = set()
    stack = list(g.outputs.values())
    while stack:
        n = stack.pop()
        if n in seen:
            continue
        seen.add(n)
        stack += deps(g, n)
    return seen


def schedule(g):
    live = reachable(g)
    ops = [n for n in sorted(live) if g.kind[n] not in ("in", "const")]
    users = {n: [] for n in live}
    for n in ops:
        for d in deps(g, n):
            users[d].append(n)
    # priority: longest cost path to a sink
    prio = {}
    for n in reversed(ops):
        c = COST[OPKIND[g.kind[n]]]
        prio[n] = c + max((prio[u] for u in users[n]), default=0.0)
    done_round = {n: -1 for n in live if g.kind[n] in ("in", "const")}
    pending = {n: sum(1 for d in deps(g, n) if g.kind[d] not in ("in", "const")) for n in ops}
    ready = {k: [] for k in COST}
    for n in ops:
        if pending[n] == 0:
            heapq.heappush(ready[OPKIND[g.kind[n]]], (-prio[n], n))
    rounds = []
    while any(ready.values()):
        # the kind of the most critical ready op
        best = min((v[0][0], k) for k, v in ready.items() if v)[1]
        take = []
        if best == OP_MUL:
            cap = LANES
            while ready[OP_MUL] and len(take) < cap:
                take.append(heapq.heappop(ready[OP_MUL])[1])
            # squarings ride along as products when lanes are left
            while ready[OP_SQR] and len(take) < cap:
                take.append(heapq.heappop(ready[OP_SQR])[1])
        elif best == OP_INV:
            take.append(heapq.heappop(ready[OP_INV])[1])
        else:
            while ready[best] and len(take) < LANES:
                take.append(heapq.heappop(ready[best])[1])
        r = len(rounds)
        kinds = {OPKIND[g.kind[n]] for n in take}
        rounds.append((OP_MUL if OP_MUL in kinds else best, take))
        for n in take:
            done_round[n] = r
        for n in take:
            for u in users[n]:
                pending[u] -= 1
                if pending[u] == 0:
                    heapq.heappush(ready[OPKIND[g.kind[u]]], (-prio[u], u))
    assert len(done_round) == len(live), "cycle or unreachable"
    return rounds, done_round


def allocate(g, rounds, done_round):
    """LDS slot per value from live ranges; a slot is reused from the round
    after its value's last read (or never, for program outputs)."""
    last = {}
    for r, (_, take) in enumerate(rounds):
        for n in take:
            for d in deps(g, n):
                last[d] = max(last.get(d, -1), r)
    outs = set(g.outputs.values())
    end = len(rounds) + 1
    slot = {}
    free = []
    nslots = 0
    releases = {}
    # inputs first (slots 0..)
    for name in sorted(g.inputs):
        n = g.inputs[name]
        if n not in last and n not in outs:
            continue
        slot[n] = nslots
        nslots += 1
        releases.setdefault(last.get(n, -1) + 1, []).append(slot[n])
    for r, (_, take) in enumerate(rounds):
        for s in releases.pop(r, []):
            heapq.heappush(free, s)
        for n in take:
            if free:
                slot[n] = heapq.heappop(free)
            else:
                slot[n] = nslots
                nslots += 1
            rel = end if n in outs else last.get(n, r) + 1
            releases.setdefault(max(rel, r + 1), []).append(slot[n])
    return slot, nslots


# --- encoding ----------------------------------------------------------------
# MUL/SQR entry (16 bytes): d, a0, a1, b0, b1, flags, 0...
#   flags: 1 a1 present, 2 a1 subtracted, 4 b1 present, 8 b1 subtracted,
#          16 a0 is a constant (pool index), 32 b0 is a constant, 64 conj(A)
# LIN entry: d, n_pos, n_neg, n_xpos, n_xneg (packed: byte1 = n_pos | n_neg << 4,
#   byte2 = n_xpos | n_xneg << 4), then up to 12 term slots in that order
# INV entry: d, a
def encode(g, rounds, slot):
    ents = []
    heads = []
    for kind, take in rounds:
        off = len(ents)
        for n in take:
            k, a = g.kind[n], g.args[n]
            e = [0] * 16
            e[0] = slot[n]
            if kind in (OP_MUL, OP_SQR):
                oa = a[0]
                ob = a[1] if k == "mul" else a[0]
                fl = 0
                for (node, node2, sub2, conj), (i0, i1, fp, fs, fc) in ((oa, (1, 2, 1, 2, 16)), (ob, (3, 4, 4, 8, 32))):
                    if g.kind[node] == "const":
                        e[i0] = g.args[node]
                        fl |= fc
                    else:
                        e[i0] = slot[node]
                    if node2 is not None:
                        e[i1] = slot[node2]
                        fl |= fp
                        if sub2:
                            fl |= fs
                if oa[3]:
                    fl |= 64
                if k == "mul" and ob[3]:
                    raise ValueError("conjugate on the second operand")
                e[5] = fl
            elif kind == OP_LIN:
                t, x = a
                cls = [[s for s, ng in t if not ng], [s for s, ng in t if ng],
                       [s for s, ng in x if not ng], [s for s, ng in x if ng]]
                assert sum(map(len, cls)) <= MAX_LIN_TERMS
                e[1] = len(cls[0]) | (len(cls[1]) << 4)
                e[2] = len(cls[2]) | (len(cls[3]) << 4)
                q = 3
                for c in cls:
                    for s in c:
                        e[q] = slot[s]
                        q += 1
                # LIN terms must be slots (no constants)
                assert all(g.kind[s] not in ("const",) for c in cls for s in c)
            else:
                e[1] = slot[a[0]]
            ents.append(e)
        heads.append((kind, len(take), off))
    return heads, ents


# --- simulation on integers (tests) ------------------------------------------
def simulate(g, rounds, slot, nslots, inputs):
    """Run the scheduled program with the slot allocation on integer Fp2
    values; returns {output name: value}.  Reads see the slot state before
    the round, writes land after it (the kernel's lockstep semantics)."""
    S = [None] * nslots
    for name, n in g.inputs.items():
        if n in slot:
            S[slot[n]] = inputs[name]

    def val(node):
        if g.kind[node] == "const":
            return g.consts[g.args[node]]
        return S[slot[node]]

    def operand(o):
        node, node2, sub2, conj = o
        v = val(node)
        if node2 is not None:
            v = f2sub(v, val(node2)) if sub2 else f2add(v, val(node2))
        return f2conj(v) if conj else v

    for kind, take in rounds:
        wr = []
        for n in take:
            k, a = g.kind[n], g.args[n]
            if k == "mul":
                v = f2mul(operand(a[0]), operand(a[1]))
            elif k == "sqr":
                x = operand(a[0])
                v = f2mul(x, x)
            elif k == "lin":
                acc, accx = (0, 0), (0, 0)
                for s, ng in a[0]:
                    acc = f2sub(acc, val(s)) if ng else f2add(acc, val(s))
                for s, ng in a[1]:
                    accx = f2sub(accx, val(s)) if ng else f2add(accx, val(s))
                v = f2add(acc, f2mul(XI, accx))
            else:
                v = f2inv(val(a[0]))
            wr.append((slot[n], v))
        for s, v in wr:
            S[s] = v
    return {name: S[slot[n]] for name, n in g.outputs.items()}


def generate(g=None):
    g = g or build()
    rounds, done = schedule(g)
    slot, nslots = allocate(g, rounds, done)
    heads, ents = encode(g, rounds, slot)
    return g, rounds, slot, nslots, heads, ents


def write_fe(full):
    """bls/group_fe_prog.hpp: the final-exponentiation program (namespace
    grpfe; its constants are grp::kConsts)."""
    g, rounds, slot, nslots, heads, ents = generate(build_fe(full.consts))
    assert len(g.consts) == len(full.consts), "the FE program needs no new constants"
    out = []
    w = out.append
    w("// GENERATED by cess_amd/csrc/gen_group.py -- do not edit.")
    w("// Lane-group final exponentiation (k_group_fe, k_group.hip): the RLC checks'")
    w(f"// one value per wave.  {len(heads)} rounds, {nslots} LDS Fp2 slots; constants: grp::kConsts.")
    w("#pragma once")
    w('#include "group_prog.hpp"')
    w("namespace grpfe {")
    w(f"constexpr int N_ROUNDS = {len(heads)};")
    w(f"constexpr int N_SLOTS = {nslots};")
    w(f"constexpr int N_ENTS = {len(ents)};")
    for i in range(6):
        w(f"constexpr int IN_F{i} = {slot[g.inputs[f'f{i}']]};")
    for i in range(6):
        w(f"constexpr int OUT_GT{i} = {slot[g.outputs[f'gt{i}']]};")
    w("CESS_GRP_DATA uint32_t kRounds[N_ROUNDS] = {")
    for i in range(0, len(heads), 8):
        w("  " + ", ".join(f"0x{(k | (n << 8) | (off << 16)):08x}u" for k, n, off in heads[i:i + 8]) + ",")
    w("};")
    w("CESS_GRP_DATA uint32_t kEnts[N_ENTS][4] = {")
    for e in ents:
        words = [e[4 * q] | (e[4 * q + 1] << 8) | (e[4 * q + 2] << 16) | (e[4 * q + 3] << 24) for q in range(4)]
        w("  {" + ", ".join(f"0x{x:08x}u" for x in words) + "},")
    w("};")
    w("}  // namespace grpfe")
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "bls", "group_fe_prog.hpp")
    with open(path, "w") as f:
        f.write("\n".join(out) + "\n")
    print("wrote", path, f"({len(heads)} rounds, {nslots} slots, {len(ents)} entries)")


def limbs(v, n=12):
    return [(v >> (32 * i)) & 0xFFFFFFFF for i in range(n)]


def main():
    g, rounds, slot, nslots, heads, ents = generate()
    cnt = {k: 0 for k in OP_NAMES}
    ops = {k: 0 for k in OP_NAMES}
    for kind, n, _ in heads:
        cnt[kind] += 1
        ops[kind] += n
    out = []
    w = out.append
    w("// GENERATED by cess_amd/csrc/gen_group.py -- do not edit.")
    w("// Lane-group program of the small-batch verification path (k_group.hip):")
    w(f"// {len(heads)} rounds (" + ", ".join(f"{OP_NAMES[k]} {cnt[k]} rounds / {ops[k]} ops" for k in OP_NAMES) +
      f"), {nslots} LDS Fp2 slots, {len(g.consts)} constants.")
    w("#pragma once")
    w("#include <stdint.h>")
    w("#if defined(CESS_HOSTEMU)")
    w("#define CESS_GRP_DATA static const")
    w("#else")
    w("#include <hip/hip_runtime.h>")
    w("#define CESS_GRP_DATA __device__ const")
    w("#endif")
    w("namespace grp {")
    w(f"constexpr int N_ROUNDS = {len(heads)};")
    w(f"constexpr int N_SLOTS = {nslots};")
    w(f"constexpr int N_CONSTS = {len(g.consts)};")
    w(f"constexpr int N_ENTS = {len(ents)};")
    for name in ("p0x", "p0y", "p1x", "p1y", "qx", "qy", "one"):
        w(f"constexpr int IN_{name.upper()} = {slot[g.inputs[name]]};")
    for name in ("tx", "ty", "tz", "pzx", "pzy") + tuple(f"gt{i}" for i in range(6)):
        w(f"constexpr int OUT_{name.upper()} = {slot[g.outputs[name]]};")
    w("// round headers: kind | count << 8 | first entry << 16")
    w("CESS_GRP_DATA uint32_t kRounds[N_ROUNDS] = {")
    for i in range(0, len(heads), 8):
        w("  " + ", ".join(f"0x{(k | (n << 8) | (off << 16)):08x}u" for k, n, off in heads[i:i + 8]) + ",")
    w("};")
    w("// 16-byte entries (see gen_group.py encode), 4 little-endian words each")
    w("CESS_GRP_DATA uint32_t kEnts[N_ENTS][4] = {")
    for e in ents:
        words = [e[4 * q] | (e[4 * q + 1] << 8) | (e[4 * q + 2] << 16) | (e[4 * q + 3] << 24) for q in range(4)]
        w("  {" + ", ".join(f"0x{x:08x}u" for x in words) + "},")
    w("};")
    w("// constant pool: Fp2 values in Montgomery form (R = 2^392), c0 then c1")
    w("CESS_GRP_DATA uint32_t kConsts[N_CONSTS][24] = {")
    for v in g.consts:
        w("  {" + ", ".join(f"0x{x:08x}u" for x in limbs(v[0] * RM % P) + limbs(v[1] * RM % P)) + "},")
    w("};")
    w("}  // namespace grp")
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "bls", "group_prog.hpp")
    with open(path, "w") as f:
        f.write("\n".join(out) + "\n")
    print("wrote", path, f"({len(heads)} rounds, {nslots} slots, {len(ents)} entries)")
    print({OP_NAMES[k]: (cnt[k], ops[k]) for k in OP_NAMES})
    write_fe(g)


if __name__ == "__main__":
    main()
