"""TEST INFRASTRUCTURE ONLY — pure-Python restatement of the BLS12-381 arithmetic behind `Bls`.

This is the CPU *oracle* the HIP engine is checked against.  It is never imported by the
product (`lambda_ethereum_consensus_amd`), only by `tests/`, `__graft_entry__.smoke()` and
`bench.py`'s `cpu_baseline` leg (see oracle/__init__.py).

What it restates (the reference's arithmetic is third-party and NOT vendored under
/root/reference: lighthouse `bls` @ e99ba3a14e5f85011ffed081c9c4cb1dabb772fe ->
`blst` 0.3.11, pinned at native/bls_nif/Cargo.lock:86-101,115-123):

* BLS12-381 field tower Fp / Fp2 = Fp[u]/(u^2+1) / Fp6 = Fp2[v]/(v^3-(1+u)) /
  Fp12 = Fp6[w]/(w^2-v); curves E1: y^2 = x^3+4, E2: y^2 = x^3+4(1+u).
* ZCash compressed serialisation (flags 0x80 compressed, 0x40 infinity, 0x20 sign),
  with blst's decode rules (x >= p -> BAD_ENCODING, no sqrt -> POINT_NOT_ON_CURVE,
  G1 x == 0 -> POINT_NOT_IN_GROUP).
* hash_to_curve BLS12381G2_XMD:SHA-256_SSWU_RO_ (RFC 9380 §8.8.2): expand_message_xmd,
  hash_to_field (count 2, L 64), simplified SWU on E2' (A'=240u, B'=1012(1+u), Z=-(2+u)),
  3-isogeny map, clear_cofactor (h_eff).
* Optimal-ate pairing (Miller loop over |x| = 0xd201000000010000, x < 0 -> conjugate,
  final exponentiation (p^12-1)/r computed literally).
* The IETF BLS signature PoP ciphersuite (DST `BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_`,
  reference docs/specs/beacon-chain.md:976-987) wrapped exactly as the reference NIF
  `native/bls_nif/src/lib.rs` wraps lighthouse (error precedence, `{:ok,_}/{:error,_}`).

Everything is plain Python ints; clarity over speed.  Functions cite the reference lines
whose behaviour they restate.
"""
from __future__ import annotations

import hashlib

# --------------------------------------------------------------------------------------
# Parameters (BLS12-381)
# --------------------------------------------------------------------------------------
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
X_ABS = 0xD201000000010000  # BLS parameter x = -X_ABS
X = -X_ABS

DST_POP = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"

G1_X = 0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB
G1_Y = 0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1
G2_X = (
    0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
    0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E,
)
G2_Y = (
    0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
    0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE,
)

# --------------------------------------------------------------------------------------
# Fp
# --------------------------------------------------------------------------------------

def fp_inv(a: int) -> int:
    if a % P == 0:
        raise ZeroDivisionError("fp_inv(0)")
    return pow(a, P - 2, P)


def fp_is_square(a: int) -> bool:
    a %= P
    return a == 0 or pow(a, (P - 1) // 2, P) == 1


def fp_sqrt(a: int):
    """p = 3 mod 4: candidate a^((p+1)/4); None if a is a non-residue (blst sqrt_fp)."""
    a %= P
    s = pow(a, (P + 1) // 4, P)
    return s if s * s % P == a else None


def fp_sgn(a: int) -> int:
    """ZCash/blst 'lexicographically largest' flag: 1 iff a > (p-1)/2."""
    return 1 if (a % P) > (P - 1) // 2 else 0


# --------------------------------------------------------------------------------------
# Fp2 = Fp[u]/(u^2 + 1); elements are tuples (c0, c1) = c0 + c1*u
# --------------------------------------------------------------------------------------
F2_ZERO = (0, 0)
F2_ONE = (1, 0)


def f2(a, b=0):
    return (a % P, b % P)


def f2_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2_neg(a):
    return ((-a[0]) % P, (-a[1]) % P)


def f2_mul(a, b):
    t0 = a[0] * b[0]
    t1 = a[1] * b[1]
    return ((t0 - t1) % P, ((a[0] + a[1]) * (b[0] + b[1]) - t0 - t1) % P)


def f2_sqr(a):
    return ((a[0] + a[1]) * (a[0] - a[1]) % P, 2 * a[0] * a[1] % P)


def f2_muls(a, s: int):
    return (a[0] * s % P, a[1] * s % P)


def f2_conj(a):
    return (a[0], (-a[1]) % P)


def f2_inv(a):
    n = fp_inv(a[0] * a[0] + a[1] * a[1])
    return (a[0] * n % P, (-a[1]) * n % P)


def f2_eq(a, b):
    return a[0] % P == b[0] % P and a[1] % P == b[1] % P


def f2_is_zero(a):
    return a[0] % P == 0 and a[1] % P == 0


def f2_pow(a, e: int):
    r = F2_ONE
    b = a
    while e:
        if e & 1:
            r = f2_mul(r, b)
        b = f2_sqr(b)
        e >>= 1
    return r


def f2_is_square(a) -> bool:
    """a is a square in Fp2 iff its norm a0^2 + a1^2 is a square in Fp."""
    return fp_is_square(a[0] * a[0] + a[1] * a[1])


def f2_sqrt(a):
    """Some square root of a in Fp2, or None (sign fixed by the caller)."""
    a = f2(*a)
    if f2_is_zero(a):
        return F2_ZERO
    if a[1] == 0:
        s = fp_sqrt(a[0])
        if s is not None:
            return (s, 0)
        s = fp_sqrt(-a[0])
        return (0, s) if s is not None else None
    gamma = fp_sqrt(a[0] * a[0] + a[1] * a[1])
    if gamma is None:
        return None
    inv2 = fp_inv(2)
    delta = (a[0] + gamma) * inv2 % P
    x0 = fp_sqrt(delta)
    if x0 is None:
        delta = (a[0] - gamma) * inv2 % P
        x0 = fp_sqrt(delta)
        if x0 is None:
            return None
    x1 = a[1] * fp_inv(2 * x0) % P
    r = (x0, x1)
    return r if f2_eq(f2_sqr(r), a) else None


def f2_sgn_zcash(a) -> int:
    """G2 y-sign flag (blst sgn0_pty_mod_384x bit 1): im != 0 ? im > (p-1)/2 : re > (p-1)/2."""
    return fp_sgn(a[1]) if a[1] % P != 0 else fp_sgn(a[0])


def f2_sgn0_rfc(a) -> int:
    """RFC 9380 §4.1 sgn0 for m = 2."""
    sign_0 = a[0] % 2
    zero_0 = a[0] == 0
    sign_1 = a[1] % 2
    return sign_0 | (zero_0 & sign_1)


XI = (1, 1)  # 1 + u, the Fp6 non-residue


def f2_mul_xi(a):
    # (a0 + a1 u)(1 + u) = (a0 - a1) + (a0 + a1) u
    return ((a[0] - a[1]) % P, (a[0] + a[1]) % P)


# --------------------------------------------------------------------------------------
# Fp6 = Fp2[v]/(v^3 - xi), Fp12 = Fp6[w]/(w^2 - v)
# --------------------------------------------------------------------------------------
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
    c0 = f2_add(t0, f2_mul_xi(f2_sub(f2_mul(f2_add(a1, a2), f2_add(b1, b2)), f2_add(t1, t2))))
    c1 = f2_add(f2_sub(f2_mul(f2_add(a0, a1), f2_add(b0, b1)), f2_add(t0, t1)), f2_mul_xi(t2))
    c2 = f2_add(f2_sub(f2_mul(f2_add(a0, a2), f2_add(b0, b2)), f2_add(t0, t2)), t1)
    return (c0, c1, c2)


def f6_mul_v(a):
    # (a0 + a1 v + a2 v^2) v = xi a2 + a0 v + a1 v^2
    return (f2_mul_xi(a[2]), a[0], a[1])


def f6_inv(a):
    a0, a1, a2 = a
    c0 = f2_sub(f2_sqr(a0), f2_mul_xi(f2_mul(a1, a2)))
    c1 = f2_sub(f2_mul_xi(f2_sqr(a2)), f2_mul(a0, a1))
    c2 = f2_sub(f2_sqr(a1), f2_mul(a0, a2))
    t = f2_add(f2_mul(a0, c0), f2_mul_xi(f2_add(f2_mul(a2, c1), f2_mul(a1, c2))))
    ti = f2_inv(t)
    return (f2_mul(c0, ti), f2_mul(c1, ti), f2_mul(c2, ti))


def f12_mul(a, b):
    a0, a1 = a
    b0, b1 = b
    t0 = f6_mul(a0, b0)
    t1 = f6_mul(a1, b1)
    c0 = f6_add(t0, f6_mul_v(t1))
    c1 = f6_sub(f6_mul(f6_add(a0, a1), f6_add(b0, b1)), f6_add(t0, t1))
    return (c0, c1)


def f12_sqr(a):
    return f12_mul(a, a)


def f12_conj(a):
    return (a[0], f6_neg(a[1]))


def f12_inv(a):
    a0, a1 = a
    t = f6_inv(f6_sub(f6_mul(a0, a0), f6_mul_v(f6_mul(a1, a1))))
    return (f6_mul(a0, t), f6_neg(f6_mul(a1, t)))


def f12_pow(a, e: int):
    r = F12_ONE
    b = a
    while e:
        if e & 1:
            r = f12_mul(r, b)
        b = f12_sqr(b)
        e >>= 1
    return r


def f12_eq(a, b):
    return all(f2_eq(a[i][j], b[i][j]) for i in range(2) for j in range(3))


def f12_is_one(a):
    return f12_eq(a, F12_ONE)


# Frobenius: Fp12 basis over Fp2 as powers of w: coefficient of w^k, k = 0..5, lives at
# (a[k & 1][k >> 1]).  (c w^k)^p = conj(c) * w^{kp} = conj(c) * xi^{k(p-1)/6} * w^k.
_FROB_GAMMA = [f2_pow(XI, k * (P - 1) // 6) for k in range(6)]


def f12_frobenius(a):
    out = [[None] * 3, [None] * 3]
    for k in range(6):
        i, j = k & 1, k >> 1
        out[i][j] = f2_mul(f2_conj(a[i][j]), _FROB_GAMMA[k])
    return (tuple(out[0]), tuple(out[1]))


# --------------------------------------------------------------------------------------
# Generic Jacobian points over Fp (G1) and Fp2 (G2).  Infinity = None.
# --------------------------------------------------------------------------------------
class _FpOps:
    zero = 0
    one = 1

    @staticmethod
    def add(a, b):
        return (a + b) % P

    @staticmethod
    def sub(a, b):
        return (a - b) % P

    @staticmethod
    def mul(a, b):
        return a * b % P

    @staticmethod
    def sqr(a):
        return a * a % P

    @staticmethod
    def neg(a):
        return (-a) % P

    @staticmethod
    def inv(a):
        return fp_inv(a)

    @staticmethod
    def is_zero(a):
        return a % P == 0

    @staticmethod
    def eq(a, b):
        return (a - b) % P == 0


class _Fp2Ops:
    zero = F2_ZERO
    one = F2_ONE
    add = staticmethod(f2_add)
    sub = staticmethod(f2_sub)
    mul = staticmethod(f2_mul)
    sqr = staticmethod(f2_sqr)
    neg = staticmethod(f2_neg)
    inv = staticmethod(f2_inv)
    is_zero = staticmethod(f2_is_zero)
    eq = staticmethod(f2_eq)


B1 = 4
B2 = (4, 4)  # 4 (1 + u)


def _jac_double(F, pt):
    if pt is None:
        return None
    X1, Y1, Z1 = pt
    if F.is_zero(Y1):
        return None
    A = F.sqr(X1)
    B = F.sqr(Y1)
    C = F.sqr(B)
    D = F.sub(F.sqr(F.add(X1, B)), F.add(A, C))
    D = F.add(D, D)
    E = F.add(F.add(A, A), A)
    Fq = F.sqr(E)
    X3 = F.sub(Fq, F.add(D, D))
    C8 = F.add(C, C)
    C8 = F.add(C8, C8)
    C8 = F.add(C8, C8)
    Y3 = F.sub(F.mul(E, F.sub(D, X3)), C8)
    Z3 = F.mul(Y1, Z1)
    Z3 = F.add(Z3, Z3)
    return (X3, Y3, Z3)


def _jac_add(F, p1, p2):
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    X1, Y1, Z1 = p1
    X2, Y2, Z2 = p2
    Z1Z1 = F.sqr(Z1)
    Z2Z2 = F.sqr(Z2)
    U1 = F.mul(X1, Z2Z2)
    U2 = F.mul(X2, Z1Z1)
    S1 = F.mul(F.mul(Y1, Z2), Z2Z2)
    S2 = F.mul(F.mul(Y2, Z1), Z1Z1)
    if F.eq(U1, U2):
        if F.eq(S1, S2):
            return _jac_double(F, p1)
        return None
    H = F.sub(U2, U1)
    I = F.sqr(F.add(H, H))
    J = F.mul(H, I)
    rr = F.sub(S2, S1)
    rr = F.add(rr, rr)
    V = F.mul(U1, I)
    X3 = F.sub(F.sub(F.sqr(rr), J), F.add(V, V))
    S1J = F.mul(S1, J)
    Y3 = F.sub(F.mul(rr, F.sub(V, X3)), F.add(S1J, S1J))
    Z3 = F.mul(F.sub(F.sqr(F.add(Z1, Z2)), F.add(Z1Z1, Z2Z2)), H)
    return (X3, Y3, Z3)


def _jac_neg(F, pt):
    if pt is None:
        return None
    return (pt[0], F.neg(pt[1]), pt[2])


def _jac_mul(F, pt, k: int):
    if k < 0:
        return _jac_mul(F, _jac_neg(F, pt), -k)
    acc = None
    for bit in bin(k)[2:] if k else "":
        acc = _jac_double(F, acc)
        if bit == "1":
            acc = _jac_add(F, acc, pt)
    return acc


def _jac_to_affine(F, pt):
    if pt is None:
        return None
    X, Y, Z = pt
    zi = F.inv(Z)
    zi2 = F.sqr(zi)
    return (F.mul(X, zi2), F.mul(Y, F.mul(zi2, zi)))


def _jac_from_affine(F, a):
    if a is None:
        return None
    return (a[0], a[1], F.one)


def _jac_eq(F, p1, p2):
    if p1 is None or p2 is None:
        return p1 is None and p2 is None
    return _jac_to_affine(F, p1) == _jac_to_affine(F, p2)


# G1 (affine tuples (x, y) or None) -------------------------------------------------------

def g1_add(a, b):
    return _jac_to_affine(_FpOps, _jac_add(_FpOps, _jac_from_affine(_FpOps, a), _jac_from_affine(_FpOps, b)))


def g1_neg(a):
    return None if a is None else (a[0], (-a[1]) % P)


def g1_mul(a, k: int):
    return _jac_to_affine(_FpOps, _jac_mul(_FpOps, _jac_from_affine(_FpOps, a), k))


def g1_on_curve(a) -> bool:
    if a is None:
        return True
    x, y = a
    return (y * y - x * x * x - B1) % P == 0


def g1_in_subgroup(a) -> bool:
    """Definition of G1 membership: [r]P == O (blst POINTonE1_in_G1 computes the same predicate)."""
    return g1_on_curve(a) and g1_mul(a, R) is None


G1_GEN = (G1_X, G1_Y)

# G2 --------------------------------------------------------------------------------------

def g2_add(a, b):
    return _jac_to_affine(_Fp2Ops, _jac_add(_Fp2Ops, _jac_from_affine(_Fp2Ops, a), _jac_from_affine(_Fp2Ops, b)))


def g2_neg(a):
    return None if a is None else (a[0], f2_neg(a[1]))


def g2_mul(a, k: int):
    return _jac_to_affine(_Fp2Ops, _jac_mul(_Fp2Ops, _jac_from_affine(_Fp2Ops, a), k))


def g2_on_curve(a) -> bool:
    if a is None:
        return True
    x, y = a
    return f2_is_zero(f2_sub(f2_sqr(y), f2_add(f2_mul(f2_sqr(x), x), B2)))


def g2_in_subgroup(a) -> bool:
    """Definition of G2 membership: [r]Q == O (blst POINTonE2_in_G2 computes the same predicate)."""
    return g2_on_curve(a) and g2_mul(a, R) is None


G2_GEN = (G2_X, G2_Y)

# psi = untwist-Frobenius-twist endomorphism on E2: (x, y) -> (conj(x) cx, conj(y) cy)
PSI_CX = f2_inv(f2_pow(XI, (P - 1) // 3))
PSI_CY = f2_inv(f2_pow(XI, (P - 1) // 2))


def g2_psi(a):
    if a is None:
        return None
    return (f2_mul(f2_conj(a[0]), PSI_CX), f2_mul(f2_conj(a[1]), PSI_CY))


# --------------------------------------------------------------------------------------
# Serialisation (ZCash BLS12-381 format as implemented by blst)
# --------------------------------------------------------------------------------------
BLST_SUCCESS = "BLST_SUCCESS"
BLST_BAD_ENCODING = "BLST_BAD_ENCODING"
BLST_POINT_NOT_ON_CURVE = "BLST_POINT_NOT_ON_CURVE"
BLST_POINT_NOT_IN_GROUP = "BLST_POINT_NOT_IN_GROUP"
BLST_PK_IS_INFINITY = "BLST_PK_IS_INFINITY"


class BlsDecodeError(Exception):
    def __init__(self, code: str):
        super().__init__(code)
        self.code = code


def g1_compress(a) -> bytes:
    if a is None:
        return bytes([0xC0]) + bytes(47)
    x, y = a
    out = bytearray(x.to_bytes(48, "big"))
    out[0] |= 0x80 | (0x20 if fp_sgn(y) else 0)
    return bytes(out)


def g2_compress(a) -> bytes:
    if a is None:
        return bytes([0xC0]) + bytes(95)
    x, y = a
    out = bytearray(x[1].to_bytes(48, "big") + x[0].to_bytes(48, "big"))
    out[0] |= 0x80 | (0x20 if f2_sgn_zcash(y) else 0)
    return bytes(out)


def g1_uncompress(b: bytes):
    """blst POINTonE1_Uncompress_Z (48-byte compressed form).  Returns affine or None (infinity);
    raises BlsDecodeError.  No subgroup check here (that is key_validate's job)."""
    if len(b) != 48 or not (b[0] & 0x80):
        raise BlsDecodeError(BLST_BAD_ENCODING)
    if b[0] & 0x40:
        if (b[0] & 0x3F) == 0 and not any(b[1:]):
            return None
        raise BlsDecodeError(BLST_BAD_ENCODING)
    x = int.from_bytes(bytes([b[0] & 0x1F]) + b[1:], "big")
    if x >= P:
        raise BlsDecodeError(BLST_BAD_ENCODING)
    y = fp_sqrt(x * x * x + B1)
    if y is None:
        raise BlsDecodeError(BLST_POINT_NOT_ON_CURVE)
    if fp_sgn(y) != ((b[0] >> 5) & 1):
        y = (-y) % P
    if x == 0:
        # blst: "(0,±2) is not in group" — reported by the uncompress step itself
        raise BlsDecodeError(BLST_POINT_NOT_IN_GROUP)
    return (x, y)


def g2_uncompress(b: bytes):
    """blst POINTonE2_Uncompress_Z (96-byte compressed form): no subgroup check."""
    if len(b) != 96 or not (b[0] & 0x80):
        raise BlsDecodeError(BLST_BAD_ENCODING)
    if b[0] & 0x40:
        if (b[0] & 0x3F) == 0 and not any(b[1:]):
            return None
        raise BlsDecodeError(BLST_BAD_ENCODING)
    x1 = int.from_bytes(bytes([b[0] & 0x1F]) + b[1:48], "big")
    x0 = int.from_bytes(b[48:96], "big")
    if x1 >= P or x0 >= P:
        raise BlsDecodeError(BLST_BAD_ENCODING)
    x = (x0, x1)
    y = f2_sqrt(f2_add(f2_mul(f2_sqr(x), x), B2))
    if y is None:
        raise BlsDecodeError(BLST_POINT_NOT_ON_CURVE)
    if f2_sgn_zcash(y) != ((b[0] >> 5) & 1):
        y = f2_neg(y)
    return (x, y)


# --------------------------------------------------------------------------------------
# Hash to G2: BLS12381G2_XMD:SHA-256_SSWU_RO_ (RFC 9380 §8.8.2)
# --------------------------------------------------------------------------------------

def expand_message_xmd(msg: bytes, dst: bytes, len_in_bytes: int) -> bytes:
    """RFC 9380 §5.3.1 with H = SHA-256 (b_in_bytes 32, s_in_bytes 64)."""
    ell = (len_in_bytes + 31) // 32
    assert ell <= 255 and len(dst) <= 255
    dst_prime = dst + bytes([len(dst)])
    msg_prime = bytes(64) + msg + len_in_bytes.to_bytes(2, "big") + b"\x00" + dst_prime
    b0 = hashlib.sha256(msg_prime).digest()
    bi = hashlib.sha256(b0 + b"\x01" + dst_prime).digest()
    out = bi
    for i in range(2, ell + 1):
        bi = hashlib.sha256(bytes(x ^ y for x, y in zip(b0, bi)) + bytes([i]) + dst_prime).digest()
        out += bi
    return out[:len_in_bytes]


def hash_to_field_fp2(msg: bytes, dst: bytes, count: int = 2):
    L = 64
    ub = expand_message_xmd(msg, dst, count * 2 * L)
    out = []
    for i in range(count):
        e = []
        for j in range(2):
            off = L * (j + i * 2)
            e.append(int.from_bytes(ub[off:off + L], "big") % P)
        out.append((e[0], e[1]))
    return out


SSWU_A = (0, 240)
SSWU_B = (1012, 1012)
SSWU_Z = ((-2) % P, (-1) % P)


def map_to_curve_sswu_e2(u):
    """RFC 9380 §6.6.2 simplified SWU onto E2': y^2 = x^3 + A' x + B' (straight-line form)."""
    A, B, Z = SSWU_A, SSWU_B, SSWU_Z
    u2 = f2_sqr(u)
    Zu2 = f2_mul(Z, u2)
    den = f2_add(f2_sqr(Zu2), Zu2)  # Z^2 u^4 + Z u^2
    if f2_is_zero(den):
        x1 = f2_mul(B, f2_inv(f2_mul(Z, A)))
    else:
        x1 = f2_mul(f2_mul(f2_neg(B), f2_inv(A)), f2_add(F2_ONE, f2_inv(den)))
    gx1 = f2_add(f2_add(f2_mul(f2_sqr(x1), x1), f2_mul(A, x1)), B)
    x2 = f2_mul(Zu2, x1)
    gx2 = f2_add(f2_add(f2_mul(f2_sqr(x2), x2), f2_mul(A, x2)), B)
    if f2_is_square(gx1):
        x, y = x1, f2_sqrt(gx1)
    else:
        x, y = x2, f2_sqrt(gx2)
    if f2_sgn0_rfc(u) != f2_sgn0_rfc(y):
        y = f2_neg(y)
    return (x, y)


def _hx(s: str) -> int:
    return int(s, 16)


_PM = P  # shorthand in the constant table
# RFC 9380 Appendix E.3 — 3-isogeny E2' -> E2 constants (c0, c1)
ISO3_XNUM = [
    (_hx("5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6"),
     _hx("5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6")),
    (0, _hx("11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71a")),
    (_hx("11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71e"),
     _hx("8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38d")),
    (_hx("171d6541fa38ccfaed6dea691f5fb614cb14b4e7f4e810aa22d6108f142b85757098e38d0f671c7188e2aaaaaaaa5ed1"), 0),
]
ISO3_XDEN = [
    (0, _hx("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa63")),
    (0xC, _hx("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa9f")),
    (1, 0),
]
ISO3_YNUM = [
    (_hx("1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706"),
     _hx("1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706")),
    (0, _hx("5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97be")),
    (_hx("11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71c"),
     _hx("8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38f")),
    (_hx("124c9ad43b6cf79bfbf7043de3811ad0761b0f37a1e26286b0e977c69aa274524e79097a56dc4bd9e1b371c71c718b10"), 0),
]
ISO3_YDEN = [
    (_hx("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa8fb"),
     _hx("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa8fb")),
    (0, _hx("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa9d3")),
    (0x12, _hx("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa99")),
    (1, 0),
]


def _poly_eval(coeffs, x):
    acc = F2_ZERO
    for c in reversed(coeffs):
        acc = f2_add(f2_mul(acc, x), c)
    return acc


def iso3_map(pt):
    """RFC 9380 Appendix E.3 3-isogeny E2' -> E2 (affine)."""
    if pt is None:
        return None
    x, y = pt
    xd = _poly_eval(ISO3_XDEN, x)
    yd = _poly_eval(ISO3_YDEN, x)
    if f2_is_zero(xd) or f2_is_zero(yd):
        return None
    xo = f2_mul(_poly_eval(ISO3_XNUM, x), f2_inv(xd))
    yo = f2_mul(y, f2_mul(_poly_eval(ISO3_YNUM, x), f2_inv(yd)))
    return (xo, yo)


# RFC 9380 §8.8.2 h_eff for G2
H_EFF_G2 = _hx(
    "bc69f08f2ee75b3584c6a0ea91b352888e2a8e9145ad7689986ff031508ffe1329c2f178731db956d82bf015d1212b02ec0ec69d7477c1ae954cbc06689f6a359894c0adebbf6b4e8020005aaa95551"
)


def clear_cofactor_g2(pt):
    """RFC 9380 clear_cofactor(P) = h_eff * P (blst computes the same point via psi,
    Budroni–Pintore: [x^2-x-1]P + [x-1]psi(P) + psi^2(2P))."""
    return g2_mul(pt, H_EFF_G2)


def clear_cofactor_g2_psi(pt):
    """Budroni–Pintore form of the same map (used to cross-check H_EFF_G2)."""
    t1 = g2_mul(pt, X * X - X - 1)
    t2 = g2_mul(g2_psi(pt), X - 1)
    t3 = g2_psi(g2_psi(g2_add(pt, pt)))
    return g2_add(g2_add(t1, t2), t3)


def hash_to_g2(msg: bytes, dst: bytes = DST_POP):
    u0, u1 = hash_to_field_fp2(msg, dst, 2)
    q0 = iso3_map(map_to_curve_sswu_e2(u0))
    q1 = iso3_map(map_to_curve_sswu_e2(u1))
    return clear_cofactor_g2(g2_add(q0, q1))


# --------------------------------------------------------------------------------------
# Pairing
# --------------------------------------------------------------------------------------

def _line_to_f12(c0, c_v, c_w3):
    """Sparse Fp12 element c0 + c_v * w^2 + c_w3 * w^3 (w^2 = v)."""
    return ((c0, c_v, F2_ZERO), (F2_ZERO, c_w3, F2_ZERO))


def miller_loop(p1, q2):
    """f_{|x|,Q}(P), lines scaled by w^3 (an Fp4 factor killed by the final exponentiation),
    conjugated at the end because x < 0.  Affine T on the twist (oracle clarity)."""
    if p1 is None or q2 is None:
        return F12_ONE
    xp, yp = p1
    T = q2
    f = F12_ONE
    for bit in bin(X_ABS)[3:]:
        # doubling step
        xt, yt = T
        lam = f2_mul(f2_muls(f2_sqr(xt), 3), f2_inv(f2_muls(yt, 2)))
        line = _line_to_f12(f2_sub(f2_mul(lam, xt), yt), f2_neg(f2_muls(lam, xp)), (yp % P, 0))
        f = f12_mul(f12_sqr(f), line)
        x3 = f2_sub(f2_sqr(lam), f2_muls(xt, 2))
        y3 = f2_sub(f2_mul(lam, f2_sub(xt, x3)), yt)
        T = (x3, y3)
        if bit == "1":
            xt, yt = T
            xq, yq = q2
            lam = f2_mul(f2_sub(yq, yt), f2_inv(f2_sub(xq, xt)))
            line = _line_to_f12(f2_sub(f2_mul(lam, xt), yt), f2_neg(f2_muls(lam, xp)), (yp % P, 0))
            f = f12_mul(f, line)
            x3 = f2_sub(f2_sub(f2_sqr(lam), xt), xq)
            y3 = f2_sub(f2_mul(lam, f2_sub(xt, x3)), yt)
            T = (x3, y3)
    return f12_conj(f)


FINAL_EXP_HARD = (P ** 4 - P ** 2 + 1) // R


def final_exponentiation(f):
    """f^((p^12-1)/r) = ((f^(p^6-1))^(p^2+1))^((p^4-p^2+1)/r), hard part by plain pow."""
    f = f12_mul(f12_conj(f), f12_inv(f))  # f^(p^6 - 1)
    f = f12_mul(f12_frobenius(f12_frobenius(f)), f)  # ^(p^2 + 1)
    return f12_pow(f, FINAL_EXP_HARD)


def pairing(p1, q2):
    return final_exponentiation(miller_loop(p1, q2))


def multi_pairing_is_one(pairs) -> bool:
    f = F12_ONE
    for p1, q2 in pairs:
        f = f12_mul(f, miller_loop(p1, q2))
    return f12_is_one(final_exponentiation(f))


# --------------------------------------------------------------------------------------
# blst / lighthouse layer.  Results mirror the NIF: ("ok", value) or
# ("error", message) with message = format!("{:?}", bls::Error).
# --------------------------------------------------------------------------------------
INFINITY_PUBKEY = bytes([0xC0]) + bytes(47)
INFINITY_SIGNATURE = bytes([0xC0]) + bytes(95)
NONE_SIGNATURE = bytes(96)


class BlsError(Exception):
    def __init__(self, msg: str):
        super().__init__(msg)
        self.msg = msg


def _blst_err(code: str) -> BlsError:
    return BlsError(f"BlstError({code})")


def pubkey_deserialize(b: bytes):
    """lighthouse GenericPublicKey::deserialize + blst PublicKey::key_validate
    (called per key at native/bls_nif/src/lib.rs:56-57,70-75,92-96,110-114,129-134)."""
    b = bytes(b)
    if b == INFINITY_PUBKEY:
        raise BlsError("InvalidInfinityPublicKey")
    if len(b) != 48:
        raise BlsError(f"InvalidByteLength {{ got: {len(b)}, expected: 48 }}")
    try:
        pt = g1_uncompress(b)
    except BlsDecodeError as e:
        raise _blst_err(e.code)
    if pt is None:
        raise _blst_err(BLST_PK_IS_INFINITY)
    if not g1_in_subgroup(pt):
        raise _blst_err(BLST_POINT_NOT_IN_GROUP)
    return pt


class Sig:
    """lighthouse GenericSignature / GenericAggregateSignature after deserialize:
    point None for the all-zero NONE encoding, is_infinity iff bytes == INFINITY_SIGNATURE."""

    __slots__ = ("present", "point", "is_infinity")

    def __init__(self, present, point, is_infinity):
        self.present = present
        self.point = point
        self.is_infinity = is_infinity


def signature_deserialize(b: bytes) -> Sig:
    """lighthouse GenericSignature::deserialize -> blst Signature::from_bytes (no subgroup
    check at decode).  Called at native/bls_nif/src/lib.rs:38,55,68,90,108."""
    b = bytes(b)
    if b == NONE_SIGNATURE:
        return Sig(False, None, False)
    try:
        pt = g2_uncompress(b)
    except BlsDecodeError as e:
        raise _blst_err(e.code)
    return Sig(True, pt, b == INFINITY_SIGNATURE)


def _core_aggregate_verify(sig_pt, pks, msgs) -> bool:
    """blst aggregate_verify(sig_groupcheck=true, msgs, DST_POP, pks, pk_validate=false)."""
    if len(pks) == 0 or len(msgs) != len(pks):
        return False
    if sig_pt is not None and not g2_in_subgroup(sig_pt):
        return False  # BLST_POINT_NOT_IN_GROUP
    pairs = []
    for pk, m in zip(pks, msgs):
        if pk is None:
            return False  # BLST_PK_IS_INFINITY
        pairs.append((pk, hash_to_g2(m)))
    # infinite signatures are skipped by blst's PAIRING_Aggregate; e(-g1, O) = 1
    if sig_pt is not None:
        pairs.append((g1_neg(G1_GEN), sig_pt))
    return multi_pairing_is_one(pairs)


def _check_msg(m: bytes):
    # Hash256::from_slice asserts len == 32 (the reference NIF panics otherwise; we error)
    if len(m) != 32:
        raise BlsError(f"InvalidMessageLength {{ got: {len(m)}, expected: 32 }}")


def _wrap(fn):
    def inner(*a, **kw):
        try:
            return ("ok", fn(*a, **kw))
        except BlsError as e:
            return ("error", e.msg)

    inner.__name__ = fn.__name__
    inner.__doc__ = fn.__doc__
    return inner


@_wrap
def sign(private_key: bytes, message: bytes) -> bytes:
    """native/bls_nif/src/lib.rs:14-29: SecretKey::deserialize then sk.sign(Hash256)."""
    sk_b = bytes(private_key)
    if len(sk_b) != 32:
        raise BlsError(f"InvalidSecretKeyLength {{ got: {len(sk_b)}, expected: 32 }}")
    if sk_b == bytes(32):
        raise BlsError("InvalidZeroSecretKey")
    sk = int.from_bytes(sk_b, "big")
    if sk >= R:
        raise _blst_err(BLST_BAD_ENCODING)
    _check_msg(message)
    return g2_compress(g2_mul(hash_to_g2(bytes(message)), sk))


@_wrap
def aggregate(signatures) -> bytes:
    """native/bls_nif/src/lib.rs:31-51: [] -> error; first undecodable -> error; sum of the
    present points (no subgroup check) starting from infinity; compress."""
    if len(signatures) == 0:
        raise BlsError("Empty signature vector")
    sigs = [signature_deserialize(s) for s in signatures]
    acc = None
    for s in sigs:
        if s.present:
            acc = g2_add(acc, s.point)
    return g2_compress(acc)


@_wrap
def verify(public_key: bytes, message: bytes, signature: bytes) -> bool:
    """native/bls_nif/src/lib.rs:53-60: signature decoded first, then the public key."""
    sig = signature_deserialize(signature)
    pk = pubkey_deserialize(public_key)
    _check_msg(message)
    if not sig.present:
        return False
    return _core_aggregate_verify(sig.point, [pk], [bytes(message)])


@_wrap
def aggregate_verify(public_keys, messages, signature) -> bool:
    """native/bls_nif/src/lib.rs:62-82."""
    sig = signature_deserialize(signature)
    pks = [pubkey_deserialize(k) for k in public_keys]
    for m in messages:
        _check_msg(m)
    if len(messages) == 0 or len(messages) != len(pks):
        return False
    if not sig.present:
        return False
    return _core_aggregate_verify(sig.point, pks, [bytes(m) for m in messages])


def _fav(pks, message, sig) -> bool:
    if len(pks) == 0:
        return False
    if not sig.present:
        return False
    agg = None
    for pk in pks:
        agg = g1_add(agg, pk)
    if agg is None:
        return False  # BLST_PK_IS_INFINITY
    return _core_aggregate_verify(sig.point, [agg], [bytes(message)])


@_wrap
def fast_aggregate_verify(public_keys, message, signature) -> bool:
    """native/bls_nif/src/lib.rs:84-100."""
    sig = signature_deserialize(signature)
    pks = [pubkey_deserialize(k) for k in public_keys]
    _check_msg(message)
    return _fav(pks, message, sig)


@_wrap
def eth_fast_aggregate_verify(public_keys, message, signature) -> bool:
    """native/bls_nif/src/lib.rs:102-119 (+ lighthouse: true iff no keys and sig == infinity)."""
    sig = signature_deserialize(signature)
    pks = [pubkey_deserialize(k) for k in public_keys]
    _check_msg(message)
    if len(pks) == 0 and sig.is_infinity:
        return True
    return _fav(pks, message, sig)


@_wrap
def eth_aggregate_pubkeys(public_keys) -> bytes:
    """native/bls_nif/src/lib.rs:121-145."""
    if len(public_keys) == 0:
        raise BlsError("Empty public key vector")
    pks = [pubkey_deserialize(k) for k in public_keys]
    agg = None
    for pk in pks:
        agg = g1_add(agg, pk)
    return g1_compress(agg)


def sk_to_pk(sk: int) -> bytes:
    return g1_compress(g1_mul(G1_GEN, sk))
