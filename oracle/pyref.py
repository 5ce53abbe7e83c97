"""Pure-Python restatement of the ringo-snark hot path -- TEST INFRASTRUCTURE ONLY.

This module is the *checker*, never the product: only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import it.  Big-int loops; use it for small cases (N <= 2^12)
and as the independent cross-check of the C oracle (oracle/oracle.c).

Every function cites the reference file:line it restates (paths relative to the
sp301415/ringo-snark tree).

Pinning status (see DESIGN.md "Oracle"):
  * field constants (q, qInvNeg, R^2) are checked against the reference's generated code
    (tests/golden/fields.json, extracted by tests/golden/make_fields.py);
  * bigpoly transforms are restated from in-repo source (math/bigpoly/ntt.go) and checked by
    the evaluation identity NTT(a)[i] = a(psi^(2*brv(i)+1)) (independent of the loop structure);
  * Lattigo v6.1.0 conventions (prime generator, primitive root search, RNS NTT ordering,
    Montgomery 2^64 forms) are restated from the library's published algorithm; the library's
    source is absent here and Go cannot run => PARITY UNPINNED at the Lattigo boundary.
"""
import ctypes
import ctypes.util
import hashlib
import math

MASK64 = (1 << 64) - 1


# --------------------------------------------------------------------------------------------
# Field: gnark-crypto generated Montgomery field (jindo/internal/zp/element.go)
# --------------------------------------------------------------------------------------------
class Field:
    """Z_q with Montgomery form R = 2^(64*L) (jindo/internal/zp/element.go:37-72,781-789).

    Elements are Python ints holding the *Montgomery representation* (x*R mod q) unless a
    method says otherwise, exactly like gnark's `Uint [L]uint64`.
    """

    def __init__(self, q, limbs=None):
        self.q = q
        self.L = limbs if limbs is not None else (q.bit_length() + 63) // 64
        self.R = 1 << (64 * self.L)
        self.Rinv = pow(self.R, -1, q)
        self.qInvNeg = (-pow(q, -1, 1 << 64)) & MASK64  # element.go:70-72
        self.rSquare = self.R * self.R % q  # element.go:781-789

    # representation helpers -------------------------------------------------------------
    def to_mont(self, x):  # SetBigInt / toMont (element.go:794-796)
        return x % self.q * self.R % self.q

    def from_mont(self, x):  # fromMont; Slice returns these canonical limbs (element.go:1769-1773)
        return x * self.Rinv % self.q

    def limbs(self, x):
        return [(x >> (64 * i)) & MASK64 for i in range(self.L)]

    def from_limbs(self, ls):
        return sum(int(v) << (64 * i) for i, v in enumerate(ls))

    # arithmetic on Montgomery representations (all outputs fully reduced, element.go:397-466)
    def add(self, a, b):  # element.go:397-413
        return (a + b) % self.q

    def sub(self, a, b):  # element.go:437-451
        return (a - b) % self.q

    def neg(self, a):  # element.go:454-466
        return (-a) % self.q

    def mul(self, a, b):  # Montgomery CIOS, element_purego.go:46-213 => a*b*R^-1 mod q
        return a * b * self.Rinv % self.q

    def mont_cios(self, x, y):
        """Literal word-level CIOS (element_purego.go:46-213 generalised to L words) --
        used by the tests to show the value-level `mul` equals the reference's algorithm on
        the reference's static edge values (element_test.go:315-358)."""
        L, q = self.L, self.q
        ql = self.limbs(q)
        xl, yl = self.limbs(x), self.limbs(y)
        t = [0] * (L + 2)
        for i in range(L):
            c = 0
            for j in range(L):
                s = t[j] + xl[i] * yl[j] + c
                t[j], c = s & MASK64, s >> 64
            s = t[L] + c
            t[L], t[L + 1] = s & MASK64, s >> 64
            m = (t[0] * self.qInvNeg) & MASK64
            s = t[0] + m * ql[0]
            c = s >> 64
            for j in range(1, L):
                s = t[j] + m * ql[j] + c
                t[j - 1], c = s & MASK64, s >> 64
            s = t[L] + c
            t[L - 1], c = s & MASK64, s >> 64
            t[L] = t[L + 1] + c
        z = sum(t[j] << (64 * j) for j in range(L + 1))
        if z >= q:
            z -= q
        return z

    def inverse(self, a):  # Inverse on Montgomery reps: (a R^-1)^-1 R = a^-1 R^2
        v = self.from_mont(a)
        return self.to_mont(pow(v, -1, self.q))

    def from_u64(self, v):  # SetUint64 (element.go:93-97)
        return self.to_mont(v)


def bit_reverse(i, logn):
    r = 0
    for _ in range(logn):
        r = (r << 1) | (i & 1)
        i >>= 1
    return r


def bit_reverse_inplace(v):
    """math/bigpoly/vec.go:123-137 (returns a new list)."""
    n = len(v)
    logn = n.bit_length() - 1
    out = [None] * n
    for i in range(n):
        out[bit_reverse(i, logn)] = v[i]
    return out


# --------------------------------------------------------------------------------------------
# bigpoly transformers (math/bigpoly/ntt.go)
# --------------------------------------------------------------------------------------------
def _find_root(p, t1, t2):
    """Generator search shared by both constructors: first x = 2, 3, ... with
    (x^t1)^t2 != 1 (ntt.go:46-53 cyclic, :173-180 negacyclic)."""
    x = 2
    while x < p:
        g = pow(x, t1, p)
        if pow(g, t2, p) != 1:
            return g
        x += 1
    raise ValueError("no root")


def mod_switch(pbig, qbig, q):
    """CyclotomicEvaluator.ModSwitchTo (math/bigpoly/cyclotomic.go:98-124) over Python ints, the
    value SetBigInt receives per coefficient: c = p q; cRem = c mod qBig (big.Int Mod: Euclidean);
    cRem -= qBig when cRem > qBig >> 1; c = (c - cRem) / qBig (exact); c mod q."""
    half = qbig >> 1
    out = []
    for p in pbig:
        c = int(p) * q
        r = c % qbig
        if r > half:
            r -= qbig
        c = (c - r) // qbig
        out.append(c % q)
    return out


def cyclotomic_tables(F, N):
    """NewCyclotomicTransformer (ntt.go:153-203).  Returns (tw, twInv, rankInv) as Montgomery
    reps; tw[k] = psi^brv(k), twInv[k] = psi^-brv(k)."""
    if N <= 0 or N & (N - 1):
        raise ValueError("rank must be a power of two")
    p = F.q
    if (p - 1) % (2 * N):
        raise ValueError("NTT not supported")
    psi = _find_root(p, (p - 1) // (2 * N), N)
    psi_inv = pow(psi, -1, p)
    tw = [F.to_mont(pow(psi, i, p)) for i in range(N)]
    twi = [F.to_mont(pow(psi_inv, i, p)) for i in range(N)]
    return bit_reverse_inplace(tw), bit_reverse_inplace(twi), F.to_mont(pow(N, -1, p)), psi


def cyclic_tables(F, N):
    """NewCyclicTransformer (ntt.go:26-95): per-stage tables tw[m+i] = brv_{N/2}(w^j)[i]."""
    if N <= 0 or N & (N - 1):
        raise ValueError("rank must be a power of two")
    p = F.q
    if (p - 1) % (2 * N):
        raise ValueError("NTT not supported")
    w = _find_root(p, (p - 1) // N, N >> 1)
    w_inv = pow(w, -1, p)
    ref = bit_reverse_inplace([F.to_mont(pow(w, i, p)) for i in range(N // 2)]) if N >= 2 else []
    refi = bit_reverse_inplace([F.to_mont(pow(w_inv, i, p)) for i in range(N // 2)]) if N >= 2 else []
    tw = [0] * N
    twi = [0] * N
    m = 1
    while m <= N // 2:
        for i in range(m):
            tw[m + i] = ref[i]
            twi[m + i] = refi[i]
        m <<= 1
    return tw, twi, F.to_mont(pow(N, -1, p)), w


def ntt_fwd(F, a, tw):
    """nttInPlaceRef (ntt.go:261-275) with butterfly (ntt.go:254-259); natural -> bit-reversed."""
    p = list(a)
    N = len(p)
    t = N
    m = 1
    while m <= N // 2:
        t >>= 1
        for i in range(m):
            w = tw[m + i]
            j1 = 2 * i * t
            for j in range(j1, j1 + t):
                v = F.mul(p[j + t], w)
                u = p[j]
                p[j] = F.add(u, v)
                p[j + t] = F.sub(u, v)
        m <<= 1
    return p


def ntt_inv(F, a, twi, rank_inv):
    """inttInPlaceRef (ntt.go:372-386), invButterfly (:365-370), then x rankInv (:242-243)."""
    p = list(a)
    N = len(p)
    t = 1
    m = N // 2
    while m >= 1:
        for i in range(m):
            w = twi[m + i]
            j1 = 2 * i * t
            for j in range(j1, j1 + t):
                u, v = p[j], p[j + t]
                p[j] = F.add(u, v)
                p[j + t] = F.mul(F.sub(u, v), w)
        t <<= 1
        m >>= 1
    return [F.mul(x, rank_inv) for x in p]


# pointwise ops (math/bigpoly/vec.go:9-121; base_op.go:49-171)
def vec_add(F, a, b):
    return [F.add(x, y) for x, y in zip(a, b)]


def vec_sub(F, a, b):
    return [F.sub(x, y) for x, y in zip(a, b)]


def vec_neg(F, a):
    return [F.neg(x) for x in a]


def vec_mul(F, a, b):
    return [F.mul(x, y) for x, y in zip(a, b)]


def vec_smul(F, a, c):
    return [F.mul(x, c) for x in a]


# --------------------------------------------------------------------------------------------
# Lattigo v6.1.0 ring restatement (third-party, source absent: PARITY UNPINNED)
# --------------------------------------------------------------------------------------------
def is_prime(n):
    if n < 2:
        return False
    small = [2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37]
    for s in small:
        if n % s == 0:
            return n == s
    d, r = n - 1, 0
    while d % 2 == 0:
        d //= 2
        r += 1
    for a in small:
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(r - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def next_upstream_primes(bits, nth_root, k):
    """ring.NewNTTFriendlyPrimesGenerator(bits, nthRoot).NextUpstreamPrimes(k)
    (called at jindo/params.go:279-282,290-293): candidates 2^bits + 1 + j*nthRoot, j >= 1."""
    out = []
    x = (1 << bits) + 1
    while len(out) < k:
        x += nth_root
        if x.bit_length() > 61:
            raise ValueError("prime generator exhausted")
        if is_prime(x):
            out.append(x)
    return out


def _factors(n):
    fs = []
    d = 2
    while d * d <= n:
        if n % d == 0:
            fs.append(d)
            while n % d == 0:
                n //= d
        d += 1 if d == 2 else 2
        if d > 1 << 22:  # fall back to sympy for large cofactors
            import sympy
            return sorted(set(fs) | set(sympy.factorint(n).keys()))
    if n > 1:
        fs.append(n)
    return fs


def primitive_root(q):
    """ring.PrimitiveRoot: smallest g >= 3 with g^((q-1)/f) != 1 for every prime f | q-1."""
    fs = _factors(q - 1)
    g = 2
    while True:
        g += 1
        if all(pow(g, (q - 1) // f, q) != 1 for f in fs):
            return g


class SubRing:
    """One RNS limb of ring.Ring(N, q) (ring.NewRing at jindo/params.go:283,294)."""

    def __init__(self, N, q):
        if not is_prime(q) or (q - 1) % (2 * N):
            raise ValueError("invalid ring modulus")
        self.N, self.q = N, q
        g = primitive_root(q)
        self.psi = pow(g, (q - 1) // (2 * N), q)
        psi_inv = pow(self.psi, -1, q)
        logn = N.bit_length() - 1
        self.roots = [0] * N
        self.roots_inv = [0] * N
        for j in range(N):
            self.roots[bit_reverse(j, logn)] = pow(self.psi, j, q)
            self.roots_inv[bit_reverse(j, logn)] = pow(psi_inv, j, q)
        self.n_inv = pow(N, -1, q)
        self.m = 1 << 64

    # values below are plain residues in [0, q) (Lattigo stores u64 coefficients)
    def mform(self, a):
        return [x * self.m % self.q for x in a]

    def imform(self, a):
        mi = pow(self.m, -1, self.q)
        return [x * mi % self.q for x in a]

    def ntt(self, a):
        """Negacyclic NTT, natural -> bit-reversed, canonical output (ring NTT)."""
        p = list(a)
        N, q = self.N, self.q
        t, m = N, 1
        while m < N:
            t >>= 1
            for i in range(m):
                w = self.roots[m + i]
                j1 = 2 * i * t
                for j in range(j1, j1 + t):
                    u, v = p[j], p[j + t] * w % q
                    p[j], p[j + t] = (u + v) % q, (u - v) % q
            m <<= 1
        return p

    def intt(self, a):
        p = list(a)
        N, q = self.N, self.q
        t, m = 1, N // 2
        while m >= 1:
            for i in range(m):
                w = self.roots_inv[m + i]
                j1 = 2 * i * t
                for j in range(j1, j1 + t):
                    u, v = p[j], p[j + t]
                    p[j], p[j + t] = (u + v) % q, (u - v) * w % q
            t <<= 1
            m >>= 1
        return [x * self.n_inv % q for x in p]

    def mul_mont_add(self, a, b, acc):  # MulCoeffsMontgomeryThenAdd: acc += a*b*2^-64
        mi = pow(self.m, -1, self.q)
        return [(c + x * y % self.q * mi) % self.q for x, y, c in zip(a, b, acc)]


class Ring:
    def __init__(self, N, primes):
        self.N = N
        self.primes = list(primes)
        self.sub = [subring(N, q) for q in primes]
        self.Q = math.prod(primes)


# --------------------------------------------------------------------------------------------
# csprng: AES-256-CTR uniform sampler keyed by SHA-384 (math/csprng/uniform.go:38-95)
# --------------------------------------------------------------------------------------------
class _Libcrypto:
    def __init__(self):
        name = ctypes.util.find_library("crypto") or "libcrypto.so.3"
        self.lib = ctypes.CDLL(name)
        L = self.lib
        L.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
        L.EVP_aes_256_ctr.restype = ctypes.c_void_p
        L.EVP_EncryptInit_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_char_p, ctypes.c_char_p]
        L.EVP_EncryptUpdate.argtypes = [ctypes.c_void_p, ctypes.c_char_p,
                                        ctypes.POINTER(ctypes.c_int), ctypes.c_char_p, ctypes.c_int]
        L.EVP_CIPHER_CTX_free.argtypes = [ctypes.c_void_p]


_libcrypto = None


def aes256_ctr_keystream(key, iv, nbytes):
    """Raw AES-256-CTR keystream (Go cipher.NewCTR: 128-bit big-endian counter)."""
    global _libcrypto
    if _libcrypto is None:
        _libcrypto = _Libcrypto()
    L = _libcrypto.lib
    ctx = L.EVP_CIPHER_CTX_new()
    L.EVP_EncryptInit_ex(ctx, L.EVP_aes_256_ctr(), None, key, iv)
    out = ctypes.create_string_buffer(nbytes + 32)
    n = ctypes.c_int(0)
    L.EVP_EncryptUpdate(ctx, out, ctypes.byref(n), bytes(nbytes), nbytes)
    L.EVP_CIPHER_CTX_free(ctx)
    return out.raw[:nbytes]


class UniformSampler:
    """NewUniformSamplerWithSeed (uniform.go:38-54): key = SHA-384(seed)[:32], IV = [32:48].

    Sample() (uniform.go:64-82) refills its 8192-byte buffer with
    `prng.XORKeyStream(buf, buf)`: the new keystream is XORed INTO the previous buffer, so
    buffer chunk c holds KS_0 ^ KS_1 ^ ... ^ KS_c (KS_i = keystream bytes [8192 i, 8192 (i+1)));
    only the first 1024 words are plain keystream."""
    BUF = 8192

    def __init__(self, seed=None, key=None, iv=None):
        if seed is not None:
            r = hashlib.sha384(seed).digest()
            key, iv = r[:32], r[32:48]
        self.key, self.iv = key, iv
        self.ks = b""
        self.chunk = 0        # keystream chunks consumed so far
        self.buf = bytes(self.BUF)
        self.ptr = self.BUF

    def _next_chunk(self):
        need = (self.chunk + 1) * self.BUF
        if len(self.ks) < need:
            self.ks = aes256_ctr_keystream(self.key, self.iv, max(need, 2 * len(self.ks), 1 << 20))
        k = self.ks[self.chunk * self.BUF:need]
        if self.chunk:
            x = int.from_bytes(self.buf, "little") ^ int.from_bytes(k, "little")
            self.buf = x.to_bytes(self.BUF, "little")
        else:
            self.buf = k
        self.chunk += 1
        self.ptr = 0

    def read_bytes(self, n):
        out = b""
        while len(out) < n:
            if self.ptr == self.BUF:
                self._next_chunk()
            take = min(n - len(out), self.BUF - self.ptr)
            out += self.buf[self.ptr:self.ptr + take]
            self.ptr += take
        return out

    def sample(self):  # uniform.go:64-82 (little-endian u64; bufSize is a multiple of 8)
        if self.ptr == self.BUF:
            self._next_chunk()
        v = int.from_bytes(self.buf[self.ptr:self.ptr + 8], "little")
        self.ptr += 8
        return v

    def sample_n(self, n):  # uniform.go:85-93
        bound = MASK64 - MASK64 % n
        while True:
            r = self.sample()
            if r < bound:
                return r % n

    def sample_float(self):  # uniform.go:95-100: (Sample() mod 2^52) / 2^52, exactly
        return (self.sample() % (1 << 52)) / float(1 << 52)


# --------------------------------------------------------------------------------------------
# Jindo parameters (jindo/params.go)
# --------------------------------------------------------------------------------------------
def encode_parameters(q):
    """newEncodeParameters (params.go:18-40): p-1 = b^(2^e) by repeated exact square roots."""
    base = q - 1
    log_exp = 0
    while True:
        s = math.isqrt(base)
        if s * s != base:
            break
        base = s
        log_exp += 1
    if base >= 1 << 64:
        raise ValueError("modulus not jindo-friendly")
    return base, 1 << log_exp


def _find_msis_rank(d, q, beta):  # params.go:53-61
    if beta > q:
        raise ValueError("findMSISRank: beta > q")
    lb, lq, ld = math.log2(beta), math.log2(q), math.log2(1.005)
    return int(math.ceil((lb * lb) / (4 * d * lq * ld)))


class JindoParams:
    """NewParameters (params.go:126-320).  Float search restated with Python's libm; Go's
    math.Log2 may differ in the last ulp, so shapes used for parity come from committed
    fixtures (tests/golden/jindo_*.json)."""

    RLWE_RANK, MAX_LOGQ, ETA, TAIL_CUT = 1 << 13, 240, 6, 5

    def __init__(self, field_q, target_n, batch):
        if target_n < 1 or batch < 1:
            raise ValueError("NewParameters: targetN, batch must be >= 1")
        base, exp = encode_parameters(field_q)
        self.field_q = field_q
        t, b, k = float(batch), float(base), float(exp)
        d = float(max(k, 256))
        l = d / k
        nu = self.RLWE_RANK / d
        eta, tail = self.ETA, self.TAIL_CUT
        max_cols = int(math.ceil(float(target_n) / l))
        min_size = math.inf
        best = None
        nn = 1
        while nn <= max_cols:
            n = float(nn)
            m = math.ceil(float(target_n) / (n * l))
            x_one = math.sqrt(k) * b
            c_one = math.sqrt(k) * min(b, (2.0 ** (120 / k))) / 2
            ecd_sd = 2 / (b - 1) * (b + 1) * eta
            ecd_blind_sd = 2 * x_one / (b - 1) * (b + 1) * eta
            mask_sd = 2 * c_one / (b - 1) * (b + 1) * eta
            mask_blind_sd = 2 * c_one * x_one / (b - 1) * (b + 1) * eta
            mlwe_sd = 2 * math.sqrt(2) * eta
            mask_mlwe_sd = 2 * c_one * math.sqrt(2) * eta
            fij = tail * (b + 1) * ecd_sd
            f0j = tail * (b + 1) * math.sqrt(m + 1) * ecd_blind_sd
            fin = tail * (b + 1) * math.sqrt(n + 1) * mask_sd
            f0n = tail * (b + 1) * math.sqrt((m + 1) * n + 1) * mask_blind_sd
            res_i = math.sqrt(n) * c_one * fij + fin
            res_0 = math.sqrt(n) * c_one * f0j + f0n
            pr = math.sqrt(m) * x_one * fij + f0j
            if t > 1:
                res_i *= math.sqrt(t) * c_one
                res_0 *= math.sqrt(t) * c_one
                pr *= math.sqrt(t) * c_one
            res_ecd_two = math.sqrt(d * (m * res_i * res_i + res_0 * res_0))
            mlwe_inf = tail * mlwe_sd
            mask_mlwe_inf = tail * math.sqrt(n + 1) * mask_mlwe_sd
            res_mlwe_inf = math.sqrt(n) * c_one * mlwe_inf + mask_mlwe_inf
            if t > 1:
                res_mlwe_inf *= math.sqrt(t) * c_one
            mu = 1
            while True:
                res_mlwe_two = math.sqrt(d * (float(mu) + nu)) * res_mlwe_inf
                res_two = math.sqrt(res_ecd_two ** 2 + res_mlwe_two ** 2)
                in_cut_two = res_two
                if t == 1:
                    ext_beta = 2 * (res_two + in_cut_two)
                    c_ext_one = 2 * c_one
                    d_ext_one = 1.0
                else:
                    ext_beta = 2 * (2 * c_one) * (res_two + in_cut_two)
                    c_ext_one = (2 * c_one) * (2 * c_one)
                    d_ext_one = 2 * c_one
                in_beta = 2 * d_ext_one * c_ext_one * ext_beta
                logq = math.ceil(math.log2(in_beta))
                q_limbs = int(math.ceil(logq / 60.0))
                q_bits = int(math.ceil(logq / float(q_limbs)))
                q = (2.0 ** (float(q_bits * q_limbs)))
                if math.log2(q) > self.MAX_LOGQ:
                    mu += 1
                    continue
                if _find_msis_rank(d, q, in_beta) == mu:
                    in_rank = float(mu)
                    break
                mu += 1
            in_cut_inf = in_cut_two / ((1 + math.sqrt(n) * c_one) * math.sqrt(in_rank * d))
            if t > 1:
                in_cut_inf /= math.sqrt(t) * c_one
            in_dcmp_inf = q / in_cut_inf
            if t > 1:
                in_dcmp_inf *= math.sqrt(t) * c_one
            in_dcmp_two = math.sqrt((n + 1) * in_rank * d) * in_dcmp_inf
            out_cut_two = in_dcmp_two
            out_beta = 2 * d_ext_one * (2 * (in_dcmp_two + out_cut_two))
            logqq = math.ceil(math.log2(out_beta))
            qq_limbs = int(math.ceil(logqq / 60.0))
            qq_bits = int(math.ceil(logqq / float(qq_limbs)))
            qq = (2.0 ** (float(qq_bits * qq_limbs)))
            if math.log2(qq) > self.MAX_LOGQ:
                nn <<= 1
                continue
            out_rank = float(_find_msis_rank(d, qq, out_beta))
            out_cut_inf = out_cut_two / math.sqrt(out_rank * d)
            if t > 1:
                out_cut_inf /= math.sqrt(t) * c_one
            com_size = t * out_rank * d * math.log2(qq / out_cut_inf)
            pf = 0.0
            pf += n * d * math.log2(pr)
            pf += d * math.log2(q)
            pf += m * d * math.log2(res_i)
            pf += d * math.log2(res_0)
            pf += (in_rank + nu) * d * math.log2(res_mlwe_inf)
            pf += ((n + 1) * in_rank * d) * math.log2(in_dcmp_inf)
            if com_size + pf < min_size:
                min_size = com_size + pf
                ql = int(math.ceil(math.log2(q) / 60))
                qb = int(math.ceil(math.log2(q) / float(ql)))
                qql = int(math.ceil(math.log2(qq) / 60))
                qqb = int(math.ceil(math.log2(qq) / float(qql)))
                best = dict(
                    batch=batch, rank=int(n) * int(m) * int(l), rows=int(m) + 1, cols=int(n),
                    base=base, exp=exp, slots=int(d) // exp, d=int(d),
                    in_msis=int(in_rank), out_msis=int(out_rank), mlwe=int(nu),
                    log_in_cut=int(math.floor(math.log2(in_cut_inf))),
                    log_out_cut=int(math.floor(math.log2(out_cut_inf))),
                    in_com_dcmp_len=int((n + 1) * in_rank),
                    q=next_upstream_primes(qb, 2 * int(d), ql),
                    qo=next_upstream_primes(qqb, 2 * int(d), qql),
                    ecd_sd=ecd_sd / math.sqrt(2 * math.pi),
                    ecd_blind_sd=ecd_blind_sd / math.sqrt(2 * math.pi),
                    mask_sd=mask_sd / math.sqrt(2 * math.pi),
                    mask_blind_sd=mask_blind_sd / math.sqrt(2 * math.pi),
                    mlwe_sd=mlwe_sd / math.sqrt(2 * math.pi),
                    mask_mlwe_sd=mask_mlwe_sd / math.sqrt(2 * math.pi),
                    res_two_nm=res_two + in_cut_two,
                    in_com_dcmp_two_nm=in_dcmp_two + out_cut_two,
                )
            nn <<= 1
        self.__dict__.update(best)

    def as_dict(self):
        keys = ["batch", "rank", "rows", "cols", "base", "exp", "slots", "d", "in_msis",
                "out_msis", "mlwe", "log_in_cut", "log_out_cut", "in_com_dcmp_len", "q", "qo",
                "ecd_sd", "ecd_blind_sd", "mask_sd", "mask_blind_sd", "mlwe_sd", "mask_mlwe_sd",
                "res_two_nm", "in_com_dcmp_two_nm"]
        return {k: getattr(self, k) for k in keys}


# --------------------------------------------------------------------------------------------
# Commit key (jindo/entities.go:21-73)
# --------------------------------------------------------------------------------------------
def commit_key(P, crs):
    """Returns (In[inMSIS][rows][nq][d], MLWE[inMSIS][mlwe][nq][d], Out[outMSIS][dcmp][nqo][d]);
    draw order coeff-major, limb-minor (entities.go:29-33,42-46,55-59)."""
    u = UniformSampler(crs)
    d = P.d

    def poly(primes):
        c = [[0] * d for _ in primes]
        for k in range(d):
            for l, q in enumerate(primes):
                c[l][k] = u.sample_n(q)
        return c

    ck_in = [[poly(P.q) for _ in range(P.rows)] for _ in range(P.in_msis)]
    ck_mlwe = [[poly(P.q) for _ in range(P.mlwe)] for _ in range(P.in_msis)]
    ck_out = [[poly(P.qo) for _ in range(P.in_com_dcmp_len)] for _ in range(P.out_msis)]
    return ck_in, ck_mlwe, ck_out


# --------------------------------------------------------------------------------------------
# Commit with injected randomness (jindo/prover.go:45-202, encoder.go:113-201, rns.go:76-114)
# --------------------------------------------------------------------------------------------
def base_encode(P, F, v_mont):
    """baseEncodeTo (encoder.go:120-146): digits of canonical v[i] -> coeff j*slots+i
    (same integer in every RNS limb); returns one integer list of length d."""
    if len(v_mont) > P.slots:
        raise ValueError("len(v) > slots")
    out = [0] * P.d
    for i, x in enumerate(v_mont):
        c = F.from_mont(x)
        for j in range(P.exp - 1):
            c, r = divmod(c, P.base)  # divMod64 (utils.go:12-19)
            out[j * P.slots + i] = r
        out[(P.exp - 1) * P.slots + i] = c
    return out


def signed_to_residue(c, q):
    """setCoeffSigned (utils.go:49-61) / encoder.go:173-181: Go's truncated `c%q + q`."""
    return c if c >= 0 else q - ((-c) % q)


def rand_encode(P, F, ring, v_mont, noise):
    """randEncodeTo (encoder.go:149-201) with the Gaussian samples `noise` (length d) given."""
    digits = base_encode(P, F, v_mont)
    out = []
    for l, sr in enumerate(ring.sub):
        q = sr.q
        s = sr.mform([signed_to_residue(c, q) for c in noise])  # :166-184
        shift = [0] * P.d
        for i in range(P.d - P.slots):  # :186-190
            shift[i + P.slots] = s[i]
        for i in range(P.d - P.slots, P.d):  # :191-195
            shift[i - (P.d - P.slots)] = q - s[i]
        shift = [(x - y * (P.base % q)) % q for x, y in zip(shift, s)]  # MulScalarThenSub :196
        dm = sr.mform(digits)  # :198
        acc = [(x + y) % q for x, y in zip(dm, shift)]  # :199
        out.append(sr.ntt(acc))  # :200
    return out


def mlwe_poly(ring, noise):
    """prover.go:130-142: setCoeffSigned -> MForm -> NTT."""
    return [sr.ntt(sr.mform([signed_to_residue(c, sr.q) for c in noise])) for sr in ring.sub]


def _gadgets(primes):
    Q = math.prod(primes)
    return [(Q // q) * pow(Q // q, -1, q) % Q for q in primes], Q


def reconstruct(primes, residues):
    """reconstructTo (rns.go:76-105) for one coefficient: balanced fast path for a single
    limb / agreeing limbs, else centred CRT with ties (>= Q>>1) going negative."""
    bal = [r - q if r > q >> 1 else r for r, q in zip(residues, primes)]
    if all(b == bal[0] for b in bal):
        return bal[0]
    gad, Q = _gadgets(primes)
    acc = sum(r * g for r, g in zip(residues, gad)) % Q
    if acc >= Q >> 1:
        acc -= Q
    return acc


def round_to(P, src_primes, dst_ring, poly_limbs, cut):
    """IMForm -> INTT -> CRT -> Rsh(cut) (floor) -> mod q' -> MForm -> NTT (prover.go:164-176)."""
    coeffs = []
    for l, q in enumerate(src_primes):
        sr = subring(P.d, q)
        coeffs.append(sr.intt(sr.imform(poly_limbs[l])))
    vals = [reconstruct(src_primes, [coeffs[l][k] for l in range(len(src_primes))]) >> cut
            for k in range(P.d)]
    return [sr.ntt(sr.mform([v % sr.q for v in vals])) for sr in dst_ring.sub]


_SUBRING_CACHE = {}


def subring(N, q):
    if (N, q) not in _SUBRING_CACHE:
        _SUBRING_CACHE[(N, q)] = SubRing(N, q)
    return _SUBRING_CACHE[(N, q)]


def commit(P, F, ck, v_mont, rnd):
    """Prover.Commit (prover.go:45-62) with injected randomness:
       rnd['last_row']  : cols*slots field elems (Montgomery; last must be 0)   (:68-72)
       rnd['mask']      : rows x slots field elems (Montgomery)                  (:95-115)
       rnd['enc_noise'] : (cols+1) x rows x d ints   (encoder Gaussian samples)
       rnd['mlwe_noise']: (cols+1) x (inMSIS+mlwe) x d ints                      (:130-139)
    Returns (commitment[outMSIS][nq][d], opening dict)."""
    if len(v_mont) > P.rank:
        raise ValueError("len(v) > params.rank")
    ck_in, ck_mlwe, ck_out = ck
    ringQ, ringQO = Ring(P.d, P.q), Ring(P.d, P.qo)
    cs = P.cols * P.slots
    last = rnd["last_row"]
    first = [0] * cs
    first[0] = v_mont[0]
    for i in range(1, cs):
        first[i] = F.sub(v_mont[i] if i < len(v_mont) else 0, last[i - 1])
    nq, nqo = len(P.q), len(P.qo)
    zero = lambda n: [[0] * P.d for _ in range(n)]
    enc = [[zero(nq) for _ in range(P.rows)] for _ in range(P.cols + 1)]
    mlwe = [[None] * (P.in_msis + P.mlwe) for _ in range(P.cols + 1)]
    incom = [None] * P.in_com_dcmp_len
    for i in range(P.cols + 1):
        en = rnd["enc_noise"][i]
        rs, re_ = i * P.slots, (i + 1) * P.slots
        if i == P.cols:
            enc[i][0] = rand_encode(P, F, ringQ, rnd["mask"][0], en[0])
            for j in range(1, P.rows - 1):
                if j * cs > len(v_mont):
                    break
                enc[i][j] = rand_encode(P, F, ringQ, rnd["mask"][j], en[j])
            enc[i][P.rows - 1] = rand_encode(P, F, ringQ, rnd["mask"][P.rows - 1], en[P.rows - 1])
        else:
            enc[i][0] = rand_encode(P, F, ringQ, first[rs:re_], en[0])
            for j in range(1, P.rows - 1):
                s0 = j * cs + rs
                if s0 > len(v_mont):
                    break
                enc[i][j] = rand_encode(P, F, ringQ, v_mont[s0:min(j * cs + re_, len(v_mont))], en[j])
            enc[i][P.rows - 1] = rand_encode(P, F, ringQ, last[rs:re_], en[P.rows - 1])
        for j in range(P.in_msis + P.mlwe):
            mlwe[i][j] = mlwe_poly(ringQ, rnd["mlwe_noise"][i][j])
        for j in range(P.in_msis):
            com = []
            for l, sr in enumerate(ringQ.sub):
                acc = [0] * P.d
                for k in range(P.rows):
                    acc = sr.mul_mont_add(ck_in[j][k][l], enc[i][k][l], acc)
                for k in range(P.mlwe):
                    acc = sr.mul_mont_add(ck_mlwe[j][k][l], mlwe[i][k][l], acc)
                acc = [(x + y) % sr.q for x, y in zip(mlwe[i][P.mlwe + j][l], acc)]
                com.append(acc)
            incom[i * P.in_msis + j] = round_to(P, P.q, ringQO, com, P.log_in_cut)
    value = []
    for i in range(P.out_msis):
        com = []
        for l, sr in enumerate(ringQO.sub):
            acc = [0] * P.d
            for j in range(P.in_com_dcmp_len):
                acc = sr.mul_mont_add(ck_out[i][j][l], incom[j][l], acc)
            com.append(acc)
        r = round_to(P, P.qo, ringQO, com, P.log_out_cut)
        value.append(r + [[0] * P.d for _ in range(nq - nqo)])
    return value, {"InCommit": incom, "Encode": enc, "MLWE": mlwe}


# --------------------------------------------------------------------------------------------
# Encoder.deltaInv (jindo/encoder.go:50-67) with Go's big.Float semantics, exactly
# --------------------------------------------------------------------------------------------
def _bigfloat_round(num, den, prec):
    """num/den > 0 rounded to `prec` significant bits, nearest even (big.Float's default
    ToNearestEven); returns (m, e) with value m * 2^e, 2^(prec-1) <= m < 2^prec."""
    e = num.bit_length() - den.bit_length() - prec
    while True:
        D = den << e if e >= 0 else den
        N = num if e >= 0 else num << -e
        q, r = divmod(N, D)
        if q >= 1 << prec:
            e += 1
        elif q < 1 << (prec - 1):
            e -= 1
        else:
            break
    if 2 * r > D or (2 * r == D and q & 1):
        q += 1
        if q == 1 << prec:
            q >>= 1
            e += 1
    return q, e


def delta_inv(base, exp):
    """deltaInv = [-1/p, -b/p, ..., -b^(exp-1)/p], p = b^exp + 1: pFloatInv = Quo(1, pFloat) at
    prec = bitlen(p), negated, Float64() of each term, then pFloatInv.Mul(pFloatInv, bFloat) (every
    big.Float result rounded to prec bits); |term| < 2^-50 / (b exp) -> 0 (encoder.go:50-67)."""
    from fractions import Fraction
    p = base ** exp + 1
    prec = p.bit_length()
    m, e = _bigfloat_round(1, p, prec)
    thr = math.ldexp(1.0, -50) / (float(base) * float(exp))
    out = []
    for _ in range(exp):
        x = Fraction(m) * (Fraction(2) ** e)
        d = -float(x)  # Float64(): nearest even
        if abs(d) < thr:
            d = 0.0
        out.append(d)
        num = m * base
        m, e2 = _bigfloat_round(num, 1, prec)
        e += e2
    return out
