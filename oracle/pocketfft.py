"""TEST INFRASTRUCTURE ONLY (the checker, never the product): the spectrum that
fourier.find_peaks sees, restated operation for operation, for any frame shape and for
float32 and float64 images.

The reference computes `np.abs(fftshift(fft2(image - np.mean(image))))`
(/root/reference/pyfcd/fourier.py:18) with two third-party libraries that are not in
/root/reference:

* scipy.fft.fft2 = pocketfft (C++, pocketfft_hdronly.hpp as vendored by scipy 1.7.1, the
  version this container's reference interpreter runs).  For a real image scipy's `c2c`
  takes its symmetric path (`c2c_sym_internal`): a real-to-complex transform of every row
  (`pocketfft_r`: the FFTPACK `rfftp` passes radf2 / radf3 / radf4 / radf5 and the generic
  radfg, or Bluestein's algorithm `fftblue` for lengths with a large prime factor), a
  complex transform of every column of the half spectrum (`pocketfft_c`: `cfftp` pass2 /
  3 / 4 / 5 / 7 / 8 / 11 and the generic passg, or Bluestein), then the other half filled
  as the complex conjugate of its mirror bin.  The arithmetic type T is the image's
  (float32 -> complex64, float64 -> complex128); no fused multiply-adds; twiddles from
  `sincos_2pibyn` (two tables of exp(2 pi i x / n) in double, multiplied, rounded to T).
* numpy 1.26.4: `np.mean` = the add-reduction over 8192-element buffer chunks, each summed
  pairwise (8 accumulators over blocks of <= 128, halving in multiples of 8 above), the
  chunk sums accumulated in order, one division, all in T; `np.abs` of complex = its
  AVX512F loop: larger * sqrt(fma(r, r, 1)) with r = smaller / larger.

Where two carrier peaks tie in exact arithmetic (the unrotated pattern.py board, SURVEY.md
§8a parity fact 2; symmetric boards at any shape) the reference's pick is decided by the
rounding of these exact operations; restating them makes the engine's peak indices
bit-exact there too (csrc/kernels_pocketfft.hip is the device form of this file).

Pinned: tests/golden/spectrum.npz, mixed.npz and shapes.npz hold sha256 digests of scipy's
fft2, numpy's mean and the reference's find_peaks spectrum for images of many shapes in
both precisions (tests/golden/make_golden.py, run by the reference's interpreter), checked
by tests/test_oracle_golden.py.
"""
import ctypes
import ctypes.util
import math
from decimal import Decimal, getcontext
from fractions import Fraction

import numpy as np

# ================================================================ exact constants
getcontext().prec = 60


def _round_sig(x, p):
    """Fraction x rounded to p significant bits, round-half-even."""
    if x == 0:
        return Fraction(0)
    s = -1 if x < 0 else 1
    x = abs(x)
    e = x.numerator.bit_length() - x.denominator.bit_length()
    if Fraction(2) ** e > x:
        e -= 1
    if Fraction(2) ** (e + 1) <= x:
        e += 1
    scale = Fraction(2) ** (e - p + 1)
    m = x / scale
    q, r = divmod(m.numerator, m.denominator)
    if 2 * r > m.denominator or (2 * r == m.denominator and q % 2 == 1):
        q += 1
    return s * q * scale


def _to_T(fr, dtype):
    """A Fraction (already a long double) converted to float (24 bits) or double (53)."""
    return dtype(float(_round_sig(fr, 24 if dtype == np.float32 else 53)))


# pocketfft: constexpr auto pi = 3.141592653589793238462643383279502884197L (x87 long double)
_PI_LD = _round_sig(Fraction(Decimal("3.141592653589793238462643383279502884197")), 64)


def _dec_pi():
    getcontext().prec = 60
    return Decimal("3.14159265358979323846264338327950288419716939937510582097494459")


def _dec_cos_sin(num, den):
    """cos / sin(2 pi num / den) to ~55 digits (Taylor series in Decimal)."""
    x = 2 * _dec_pi() * Decimal(num) / Decimal(den)
    c, s, term, k = Decimal(0), Decimal(0), Decimal(1), 0
    while True:
        if k % 4 == 0:
            c += term
        elif k % 4 == 1:
            s += term
        elif k % 4 == 2:
            c -= term
        else:
            s -= term
        k += 1
        term = term * x / k
        if abs(term) < Decimal(10) ** -58 and k > 4:
            break
    return c, s


def _ld_const(dec):
    """T0(<long double literal>): the decimal constant as a long double."""
    return _round_sig(Fraction(dec), 64)


def pass_consts(ip, dtype):
    """cos / sin(2 pi m / ip), m = 1 .. (ip - 1) / 2, as the T0 literals of pass3 / 5 / 7 / 11
    and radf3 / radf5 (correctly rounded decimal literals -> long double -> T0)."""
    out = []
    for m in range(1, (ip - 1) // 2 + 1):
        c, s = _dec_cos_sin(m, ip)
        out.append((_to_T(_ld_const(c), dtype), _to_T(_ld_const(s), dtype)))
    return out


# ================================================================ twiddles: sincos_2pibyn
# pocketfft's calc() takes cos and sin of the same argument, which the compiler merges into
# one glibc sincos() call (the only trigonometric symbols scipy's pypocketfft imports are
# sincos / sincosl).  glibc's sincos differs from its sin / cos in the last bit for ~0.1 %
# of arguments, so the restatement calls the same sincos.
_LIBM = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
_LIBM.sincos.argtypes = [ctypes.c_double, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
_LIBM.sincos.restype = None


def _sincos(a):
    s, c = ctypes.c_double(), ctypes.c_double()
    _LIBM.sincos(a, ctypes.byref(s), ctypes.byref(c))
    return s.value, c.value


def _calc(x, n, ang):
    """exp(2 pi i x / n) by octant reduction (sincos_2pibyn::calc), double."""
    x <<= 3
    if x < 4 * n:
        if x < 2 * n:
            if x < n:
                s, c = _sincos(float(x) * ang)
                return c, s
            s, c = _sincos(float(2 * n - x) * ang)
            return s, c
        x -= 2 * n
        if x < n:
            s, c = _sincos(float(x) * ang)
            return -s, c
        s, c = _sincos(float(2 * n - x) * ang)
        return -c, s
    x = 8 * n - x
    if x < 2 * n:
        if x < n:
            s, c = _sincos(float(x) * ang)
            return c, -s
        s, c = _sincos(float(2 * n - x) * ang)
        return s, -c
    x -= 2 * n
    if x < n:
        s, c = _sincos(float(x) * ang)
        return -s, -c
    s, c = _sincos(float(2 * n - x) * ang)
    return -c, -s


_SC_CACHE = {}


def sincos_2pibyn(n):
    """(v1, v2, mask, shift) of pocketfft's sincos_2pibyn<T>(n) (Thigh = double)."""
    if n in _SC_CACHE:
        return _SC_CACHE[n]
    ang = float(_round_sig(_PI_LD / 4 / n, 64))  # Thigh(0.25L * pi / n)
    nval = (n + 2) // 2
    shift = 1
    while (1 << shift) * (1 << shift) < nval:
        shift += 1
    mask = (1 << shift) - 1
    v1 = np.array([(1.0, 0.0)] + [_calc(i, n, ang) for i in range(1, mask + 1)], np.float64)
    n2 = (nval + mask) // (mask + 1)
    v2 = np.array([(1.0, 0.0)] + [_calc(i * (mask + 1), n, ang) for i in range(1, n2)], np.float64)
    _SC_CACHE[n] = (v1, v2, mask, shift)
    return _SC_CACHE[n]


def twiddle(n, idx, dtype):
    """sincos_2pibyn<T>(n)[idx] for an int array idx: (re, im) arrays of T."""
    v1, v2, mask, shift = sincos_2pibyn(n)
    idx = np.asarray(idx, np.int64)
    upper = 2 * idx > n
    j = np.where(upper, n - idx, idx)
    x1, x2 = v1[j & mask], v2[j >> shift]
    re = (x1[..., 0] * x2[..., 0] - x1[..., 1] * x2[..., 1]).astype(dtype)
    im = (x1[..., 0] * x2[..., 1] + x1[..., 1] * x2[..., 0]).astype(dtype)
    im = np.where(upper, -im, im).astype(dtype)
    return re, im


# ================================================================ plans
def largest_prime_factor(n):
    res = 1
    while n % 2 == 0:
        res, n = 2, n // 2
    x = 3
    while x * x <= n:
        while n % x == 0:
            res, n = x, n // x
        x += 2
    return n if n > 1 else res


def cost_guess(n):
    lfp, ni, result = 1.1, n, 0.0
    while n % 2 == 0:
        result += 2
        n //= 2
    x = 3
    while x * x <= n:
        while n % x == 0:
            result += x if x <= 5 else lfp * x
            n //= x
        x += 2
    if n > 1:
        result += n if n <= 5 else lfp * n
    return result * ni


def good_size_cmplx(n):
    """Smallest 2^a 3^b 5^c 7^d 11^e >= n."""
    if n <= 12:
        return n
    m = n
    while True:
        k = m
        for p in (2, 3, 5, 7, 11):
            while k % p == 0:
                k //= p
        if k == 1:
            return m
        m += 1


def _odd_factors(f, left):
    d = 3
    while d * d <= left:
        while left % d == 0:
            f.append(d)
            left //= d
        d += 2
    if left > 1:
        f.append(left)
    return f


def rfactors(n):
    """rfftp::factorize: 4s first, a single 2 moved to the front, then odd factors."""
    f, left = [], n
    while left % 4 == 0:
        f.append(4)
        left //= 4
    if left % 2 == 0:
        left //= 2
        f.append(2)
        f[0], f[-1] = f[-1], f[0]
    return _odd_factors(f, left)


def cfactors(n):
    """cfftp::factorize: 8s, then 4s, a single 2 moved to the front, then odd factors."""
    f, left = [], n
    while left & 7 == 0:
        f.append(8)
        left >>= 3
    while left & 3 == 0:
        f.append(4)
        left >>= 2
    if left & 1 == 0:
        left >>= 1
        f.append(2)
        f[0], f[-1] = f[-1], f[0]
    return _odd_factors(f, left)


def use_bluestein(n, real):
    """pocketfft_r / pocketfft_c plan choice: Bluestein when it is guessed cheaper."""
    tmp = 0 if n < 50 else largest_prime_factor(n)
    if tmp * tmp <= n:
        return False
    comp1 = (0.5 if real else 1.0) * cost_guess(n)
    comp2 = 2 * cost_guess(good_size_cmplx(2 * n - 1)) * 1.5
    return comp2 < comp1


def rtwiddles(n, fact, dtype):
    """rfftp::comp_twiddle: per pass tw ((ip - 1) * (ido - 1) T) and, for ip > 5, tws (2 ip T)."""
    tws, l1 = [], 1
    for k, ip in enumerate(fact):
        ido = n // (l1 * ip)
        tw = np.zeros(max((ip - 1) * (ido - 1), 1), dtype)
        if k < len(fact) - 1 and ido > 2:
            j = np.arange(1, ip)[:, None]
            i = np.arange(1, (ido - 1) // 2 + 1)[None, :]
            re, im = twiddle(n, j * l1 * i, dtype)
            pos = (j - 1) * (ido - 1) + 2 * i - 2
            tw[pos.ravel()] = re.ravel()
            tw[(pos + 1).ravel()] = im.ravel()
        csarr = None
        if ip > 5:
            csarr = np.zeros(2 * ip, dtype)
            csarr[0], csarr[1] = 1, 0
            i, ic = 2, 2 * ip - 2
            while i <= ic:
                re, im = twiddle(n, [i // 2 * (n // ip)], dtype)
                csarr[i], csarr[i + 1] = re[0], im[0]
                csarr[ic], csarr[ic + 1] = re[0], -im[0]
                i += 2
                ic -= 2
        tws.append((tw, csarr))
        l1 *= ip
    return tws


def ctwiddles(n, fact, dtype):
    """cfftp::comp_twiddle: per pass tw [(ip - 1)][(ido - 1)] complex and, for ip > 11, tws [ip]."""
    tws, l1 = [], 1
    for ip in fact:
        ido = n // (l1 * ip)
        j = np.arange(1, ip)[:, None]
        i = np.arange(1, ido)[None, :]
        tr, ti = twiddle(n, j * l1 * i, dtype) if ido > 1 else (np.zeros((ip - 1, 0), dtype),) * 2
        csarr = twiddle(n, np.arange(ip) * l1 * ido, dtype) if ip > 11 else None
        tws.append(((tr, ti), csarr))
        l1 *= ip
    return tws


# ================================================================ complex helpers on (re, im)
def _add(a, b):
    return a[0] + b[0], a[1] + b[1]


def _sub(a, b):
    return a[0] - b[0], a[1] - b[1]


def _smul(v, w, fwd):
    """special_mul<fwd>: v * conj(w) forward, v * w backward."""
    if fwd:
        return v[0] * w[0] + v[1] * w[1], v[1] * w[0] - v[0] * w[1]
    return v[0] * w[0] - v[1] * w[1], v[0] * w[1] + v[1] * w[0]


def _rot90(a, fwd):
    return (a[1], -a[0]) if fwd else (-a[1], a[0])


def _rot45(a, fwd, h):
    if fwd:
        return h * (a[0] + a[1]), h * (a[1] - a[0])
    return h * (a[0] - a[1]), h * (a[1] + a[0])


def _rot135(a, fwd, h):
    if fwd:
        return h * (a[1] - a[0]), h * (-a[0] - a[1])
    return h * (-a[0] - a[1]), h * (a[0] - a[1])


def _neg(a):
    return -a[0], -a[1]


# ================================================================ cfftp passes
# Vectorised over (batch, k, i): CC(i, m, k) = cc[i + ido*(m + ip*k)] -> C[:, k, m, i];
# CH(i, k, m) = ch[i + ido*(k + l1*m)] -> result list over m of [:, k, i] planes.
def _twiddled(out, wa, fwd):
    """special_mul<fwd>(out[m], WA(m - 1, i)) for i >= 1; i = 0 untouched."""
    res = [out[0]]
    for m in range(1, len(out)):
        v = out[m]
        if v[0].shape[-1] > 1:
            w = (wa[0][m - 1][None, None, :], wa[1][m - 1][None, None, :])
            t = _smul((v[0][..., 1:], v[1][..., 1:]), w, fwd)
            v = (np.concatenate([v[0][..., :1], t[0]], -1), np.concatenate([v[1][..., :1], t[1]], -1))
        res.append(v)
    return res


def _cpass(ip, ido, l1, c, fwd, tw, csarr, dtype):
    B = c[0].shape[0]
    C = [(c[0].reshape(B, l1, ip, ido)[:, :, m, :], c[1].reshape(B, l1, ip, ido)[:, :, m, :]) for m in range(ip)]
    T = dtype
    h = T(0.707106781186547524400844362104849)
    out = [None] * ip
    if ip == 2:
        out[0] = _add(C[0], C[1])
        out[1] = _sub(C[0], C[1])
    elif ip == 4:
        t2, t1 = _add(C[0], C[2]), _sub(C[0], C[2])
        t3, t4 = _add(C[1], C[3]), _sub(C[1], C[3])
        t4 = _rot90(t4, fwd)
        out[0], out[2] = _add(t2, t3), _sub(t2, t3)
        out[1], out[3] = _add(t1, t4), _sub(t1, t4)
    elif ip == 8:
        a1, a5 = _add(C[1], C[5]), _sub(C[1], C[5])
        a3, a7 = _add(C[3], C[7]), _sub(C[3], C[7])
        a1, a3 = _add(a1, a3), _sub(a1, a3)
        a3 = _rot90(a3, fwd)
        a7 = _rot90(a7, fwd)
        a5, a7 = _add(a5, a7), _sub(a5, a7)
        a5 = _rot45(a5, fwd, h)
        a7 = _rot135(a7, fwd, h)
        a0, a4 = _add(C[0], C[4]), _sub(C[0], C[4])
        a2, a6 = _add(C[2], C[6]), _sub(C[2], C[6])
        a0, a2 = _add(a0, a2), _sub(a0, a2)
        out[0], out[4] = _add(a0, a1), _sub(a0, a1)
        out[2], out[6] = _add(a2, a3), _sub(a2, a3)
        a6 = _rot90(a6, fwd)
        a4, a6 = _add(a4, a6), _sub(a4, a6)
        out[1], out[5] = _add(a4, a5), _sub(a4, a5)
        out[3], out[7] = _add(a6, a7), _sub(a6, a7)
    elif ip in (3, 5, 7, 11):
        # PREPn / PARTSTEPna: t_first = CC(0); pairs (t_m, t_{ip-m}) = PM(CC(m), CC(ip-m));
        # out_u = ca + cb, out_{ip-u} = ca - cb with
        # ca = t0 + sum_m twr(u m) * s_m, cb = i * sum_m twi(u m) * d_m (coefficients in order m)
        sg = -1 if fwd else 1
        cs = pass_consts(ip, T)
        half = (ip - 1) // 2
        s = [_add(C[m], C[ip - m]) for m in range(1, half + 1)]
        d = [_sub(C[m], C[ip - m]) for m in range(1, half + 1)]
        t0 = C[0]
        if ip == 3:  # CH(0) = t0 + t1
            out[0] = _add(t0, s[0])
        else:  # CH(0).r = t0.r + t1.r + t2.r ... left to right
            r, i_ = t0[0], t0[1]
            for m in range(half):
                r, i_ = r + s[m][0], i_ + s[m][1]
            out[0] = (r, i_)
        for u in range(1, half + 1):
            car, cai = t0[0], t0[1]
            cbi = cbr = None
            for m in range(1, half + 1):
                q = (u * m) % ip
                sgn = 1
                if q > half:
                    q, sgn = ip - q, -1
                twr, twi = cs[q - 1][0], T(sg * sgn) * cs[q - 1][1]
                if ip == 3:  # ca = t0 + t1 * twr (complex times scalar)
                    car, cai = car + s[0][0] * twr, cai + s[0][1] * twr
                else:
                    car, cai = car + twr * s[m - 1][0], cai + twr * s[m - 1][1]
                pr, pi_ = twi * d[m - 1][0], twi * d[m - 1][1]
                if ip == 3:  # cb{-t2.i * twi, t2.r * twi}
                    pr, pi_ = d[0][0] * twi, d[0][1] * twi
                cbi = pr if cbi is None else cbi + pr
                cbr = pi_ if cbr is None else cbr + pi_
            ca, cb = (car, cai), (-cbr, cbi)
            out[u], out[ip - u] = _add(ca, cb), _sub(ca, cb)
    else:
        return _passg(ip, ido, l1, C, fwd, tw, csarr, dtype)
    out = _twiddled(out, tw, fwd)
    r = np.stack([o[0] for o in out], 1).reshape(B, -1)
    i = np.stack([o[1] for o in out], 1).reshape(B, -1)
    return r, i


def _passg(ip, ido, l1, C, fwd, tw, csarr, dtype):
    """cfftp::passg (ip > 11): output layout CX(i, k, m) = [:, m, k, i]."""
    B = C[0][0].shape[0]
    T = dtype
    wr = csarr[0].astype(T)
    wi = (-csarr[1] if fwd else csarr[1]).astype(T)
    wr[0], wi[0] = 1, 0
    ipph = (ip + 1) // 2
    CH = [None] * ip
    CH[0] = C[0]
    for j in range(1, ipph):
        jc = ip - j
        CH[j], CH[jc] = _add(C[j], C[jc]), _sub(C[j], C[jc])
    r, i_ = CH[0]
    for j in range(1, ipph):
        r, i_ = r + CH[j][0], i_ + CH[j][1]
    CX = [None] * ip
    CX[0] = (r, i_)
    for l in range(1, ipph):
        lc = ip - l
        xr = CH[0][0] + wr[l] * CH[1][0] + wr[2 * l] * CH[2][0]
        xi = CH[0][1] + wr[l] * CH[1][1] + wr[2 * l] * CH[2][1]
        yr = -(wi[l] * CH[ip - 1][1] + wi[2 * l] * CH[ip - 2][1])
        yi = wi[l] * CH[ip - 1][0] + wi[2 * l] * CH[ip - 2][0]
        iwal = 2 * l
        j, jc = 3, ip - 3
        while j < ipph - 1:
            iwal += l
            if iwal > ip:
                iwal -= ip
            a = iwal
            iwal += l
            if iwal > ip:
                iwal -= ip
            b = iwal
            xr = xr + (CH[j][0] * wr[a] + CH[j + 1][0] * wr[b])
            xi = xi + (CH[j][1] * wr[a] + CH[j + 1][1] * wr[b])
            yr = yr - (CH[jc][1] * wi[a] + CH[jc - 1][1] * wi[b])
            yi = yi + (CH[jc][0] * wi[a] + CH[jc - 1][0] * wi[b])
            j += 2
            jc -= 2
        while j < ipph:
            iwal += l
            if iwal > ip:
                iwal -= ip
            xr = xr + CH[j][0] * wr[iwal]
            xi = xi + CH[j][1] * wr[iwal]
            yr = yr - CH[jc][1] * wi[iwal]
            yi = yi + CH[jc][0] * wi[iwal]
            j += 1
            jc -= 1
        CX[l], CX[lc] = (xr, xi), (yr, yi)
    out = [CX[0]] + [None] * (ip - 1)
    for j in range(1, ipph):
        jc = ip - j
        out[j], out[jc] = _add(CX[j], CX[jc]), _sub(CX[j], CX[jc])
    out = _twiddled(out, tw, fwd)
    r = np.stack([o[0] for o in out], 1).reshape(B, -1)
    i = np.stack([o[1] for o in out], 1).reshape(B, -1)
    return r, i


class CfftPlan:
    """cfftp<T0>(n): factors and twiddles."""

    def __init__(self, n, dtype):
        self.n, self.dtype = n, dtype
        self.fact = cfactors(n)
        self.tws = ctwiddles(n, self.fact, dtype)

    def exec(self, c, fwd):
        """pass_all<fwd> on (re, im) [B, n] arrays (fct = 1)."""
        if self.n == 1:
            return c
        l1 = 1
        for k, ip in enumerate(self.fact):
            ido = self.n // (l1 * ip)
            tw, csarr = self.tws[k]
            c = _cpass(ip, ido, l1, c, fwd, tw, csarr, self.dtype)
            l1 *= ip
        return c


class Bluestein:
    """fftblue<T0>(n)."""

    def __init__(self, n, dtype):
        T = dtype
        self.n, self.dtype = n, dtype
        self.n2 = good_size_cmplx(2 * n - 1)
        self.plan = CfftPlan(self.n2, dtype)
        coeff = np.zeros(n, np.int64)
        acc = 0
        for m in range(1, n):
            acc += 2 * m - 1
            if acc >= 2 * n:
                acc -= 2 * n
            coeff[m] = acc
        bkr, bki = twiddle(2 * n, coeff, T)
        bkr[0], bki[0] = 1, 0
        self.bk = (bkr, bki)
        xn2 = T(T(1) / T(self.n2))
        tr = np.zeros(self.n2, T)
        ti = np.zeros(self.n2, T)
        tr[0], ti[0] = bkr[0] * xn2, bki[0] * xn2
        tr[1:n], ti[1:n] = bkr[1:] * xn2, bki[1:] * xn2
        tr[self.n2 - n + 1:], ti[self.n2 - n + 1:] = (bkr[1:] * xn2)[::-1], (bki[1:] * xn2)[::-1]
        fr, fi = self.plan.exec((tr[None], ti[None]), True)
        h = self.n2 // 2 + 1
        self.bkf = (fr[0, :h], fi[0, :h])

    def fft(self, c, fwd):
        """fft<fwd>(c, 1) on (re, im) [B, n]."""
        T = self.dtype
        n, n2 = self.n, self.n2
        B = c[0].shape[0]
        ar, ai = _smul(c, (self.bk[0][None], self.bk[1][None]), fwd)
        akr = np.zeros((B, n2), T)
        aki = np.zeros((B, n2), T)
        akr[:, :n], aki[:, :n] = ar, ai
        akr, aki = self.plan.exec((akr, aki), True)
        # akf[m] *= bkf[m] (m < (n2+1)/2), akf[n2-m] *= bkf[m], akf[n2/2] *= bkf[n2/2]
        idx = np.arange(n2)
        src = np.where(idx <= n2 // 2, idx, n2 - idx)
        akr, aki = _smul((akr, aki), (self.bkf[0][src][None], self.bkf[1][src][None]), not fwd)
        akr, aki = self.plan.exec((akr, aki), False)
        return _smul((akr[:, :n], aki[:, :n]), (self.bk[0][None], self.bk[1][None]), fwd)


def cfft(c, fwd=True, dtype=np.float32):
    """pocketfft_c<T>(n).exec(c, 1, fwd) along axis 1 of (re, im) [B, n] arrays."""
    n = c[0].shape[1]
    if use_bluestein(n, False):
        return Bluestein(n, dtype).fft(c, fwd)
    return CfftPlan(n, dtype).exec(c, fwd)


# ================================================================ rfftp forward
# CC(a, b, c) = cc[a + ido*(b + l1*c)] -> cc.reshape(B, ip, l1, ido)[:, c, b, a];
# CH(a, b, c) = ch[a + ido*(b + ip*c)] -> ch.reshape(B, l1, ip, ido)[:, c, b, a].
def _radf(ip, ido, l1, p1, tw, csarr, dtype):
    T = dtype
    B = p1.shape[0]
    CC = p1.reshape(B, ip, l1, ido)
    CH = np.zeros((B, l1, ip, ido), T)
    WA = lambda x, i: tw[i + x * (ido - 1)]  # noqa: E731
    ii = np.arange(2, ido, 2) if ido > 2 else np.zeros(0, np.int64)
    ic = ido - ii
    h = T(0.707106781186547524400844362104849)
    if ip == 2:
        CH[:, :, 0][..., 0] = CC[:, 0][..., 0] + CC[:, 1][..., 0]
        CH[:, :, 1][..., ido - 1] = CC[:, 0][..., 0] - CC[:, 1][..., 0]
        if ido % 2 == 0:
            CH[:, :, 1][..., 0] = -CC[:, 1][..., ido - 1]
            CH[:, :, 0][..., ido - 1] = CC[:, 0][..., ido - 1]
        if ido > 2:
            w0, w1 = WA(0, ii - 2), WA(0, ii - 1)
            tr2 = w0 * CC[:, 1][..., ii - 1] + w1 * CC[:, 1][..., ii]
            ti2 = w0 * CC[:, 1][..., ii] - w1 * CC[:, 1][..., ii - 1]
            CH[:, :, 0][..., ii - 1] = CC[:, 0][..., ii - 1] + tr2
            CH[:, :, 1][..., ic - 1] = CC[:, 0][..., ii - 1] - tr2
            CH[:, :, 0][..., ii] = ti2 + CC[:, 0][..., ii]
            CH[:, :, 1][..., ic] = ti2 - CC[:, 0][..., ii]
    elif ip == 4:
        tr1 = CC[:, 3][..., 0] + CC[:, 1][..., 0]
        CH[:, :, 2][..., 0] = CC[:, 3][..., 0] - CC[:, 1][..., 0]
        tr2 = CC[:, 0][..., 0] + CC[:, 2][..., 0]
        CH[:, :, 1][..., ido - 1] = CC[:, 0][..., 0] - CC[:, 2][..., 0]
        CH[:, :, 0][..., 0] = tr2 + tr1
        CH[:, :, 3][..., ido - 1] = tr2 - tr1
        if ido % 2 == 0:
            e = ido - 1
            ti1 = -h * (CC[:, 1][..., e] + CC[:, 3][..., e])
            tr1 = h * (CC[:, 1][..., e] - CC[:, 3][..., e])
            CH[:, :, 0][..., e] = CC[:, 0][..., e] + tr1
            CH[:, :, 2][..., e] = CC[:, 0][..., e] - tr1
            CH[:, :, 3][..., 0] = ti1 + CC[:, 2][..., e]
            CH[:, :, 1][..., 0] = ti1 - CC[:, 2][..., e]
        if ido > 2:
            cr, ci = {}, {}
            for m in (1, 2, 3):
                w0, w1 = WA(m - 1, ii - 2), WA(m - 1, ii - 1)
                cr[m] = w0 * CC[:, m][..., ii - 1] + w1 * CC[:, m][..., ii]
                ci[m] = w0 * CC[:, m][..., ii] - w1 * CC[:, m][..., ii - 1]
            tr1, tr4 = cr[3] + cr[1], cr[3] - cr[1]
            ti1, ti4 = ci[1] + ci[3], ci[1] - ci[3]
            tr2, tr3 = CC[:, 0][..., ii - 1] + cr[2], CC[:, 0][..., ii - 1] - cr[2]
            ti2, ti3 = CC[:, 0][..., ii] + ci[2], CC[:, 0][..., ii] - ci[2]
            CH[:, :, 0][..., ii - 1] = tr2 + tr1
            CH[:, :, 3][..., ic - 1] = tr2 - tr1
            CH[:, :, 0][..., ii] = ti1 + ti2
            CH[:, :, 3][..., ic] = ti1 - ti2
            CH[:, :, 2][..., ii - 1] = tr3 + ti4
            CH[:, :, 1][..., ic - 1] = tr3 - ti4
            CH[:, :, 2][..., ii] = tr4 + ti3
            CH[:, :, 1][..., ic] = tr4 - ti3
    elif ip == 3:
        (taur, taui), = pass_consts(3, T)
        cr2 = CC[:, 1][..., 0] + CC[:, 2][..., 0]
        CH[:, :, 0][..., 0] = CC[:, 0][..., 0] + cr2
        CH[:, :, 2][..., 0] = taui * (CC[:, 2][..., 0] - CC[:, 1][..., 0])
        CH[:, :, 1][..., ido - 1] = CC[:, 0][..., 0] + taur * cr2
        if ido > 1 and len(ii):
            dr, di = {}, {}
            for m in (1, 2):
                w0, w1 = WA(m - 1, ii - 2), WA(m - 1, ii - 1)
                dr[m] = w0 * CC[:, m][..., ii - 1] + w1 * CC[:, m][..., ii]
                di[m] = w0 * CC[:, m][..., ii] - w1 * CC[:, m][..., ii - 1]
            cr2, ci2 = dr[1] + dr[2], di[1] + di[2]
            CH[:, :, 0][..., ii - 1] = CC[:, 0][..., ii - 1] + cr2
            CH[:, :, 0][..., ii] = CC[:, 0][..., ii] + ci2
            tr2 = CC[:, 0][..., ii - 1] + taur * cr2
            ti2 = CC[:, 0][..., ii] + taur * ci2
            tr3 = taui * (di[1] - di[2])
            ti3 = taui * (dr[2] - dr[1])
            CH[:, :, 2][..., ii - 1] = tr2 + tr3
            CH[:, :, 1][..., ic - 1] = tr2 - tr3
            CH[:, :, 2][..., ii] = ti3 + ti2
            CH[:, :, 1][..., ic] = ti3 - ti2
    elif ip == 5:
        (tr11, ti11), (tr12, ti12) = pass_consts(5, T)
        cr2, ci5 = CC[:, 4][..., 0] + CC[:, 1][..., 0], CC[:, 4][..., 0] - CC[:, 1][..., 0]
        cr3, ci4 = CC[:, 3][..., 0] + CC[:, 2][..., 0], CC[:, 3][..., 0] - CC[:, 2][..., 0]
        c0 = CC[:, 0][..., 0]
        CH[:, :, 0][..., 0] = c0 + cr2 + cr3
        CH[:, :, 1][..., ido - 1] = c0 + tr11 * cr2 + tr12 * cr3
        CH[:, :, 2][..., 0] = ti11 * ci5 + ti12 * ci4
        CH[:, :, 3][..., ido - 1] = c0 + tr12 * cr2 + tr11 * cr3
        CH[:, :, 4][..., 0] = ti12 * ci5 - ti11 * ci4
        if ido > 1 and len(ii):
            dr, di = {}, {}
            for m in (1, 2, 3, 4):
                w0, w1 = WA(m - 1, ii - 2), WA(m - 1, ii - 1)
                dr[m] = w0 * CC[:, m][..., ii - 1] + w1 * CC[:, m][..., ii]
                di[m] = w0 * CC[:, m][..., ii] - w1 * CC[:, m][..., ii - 1]
            cr2, ci5 = dr[4] + dr[1], dr[4] - dr[1]
            ci2, cr5 = di[1] + di[4], di[1] - di[4]
            cr3, ci4 = dr[3] + dr[2], dr[3] - dr[2]
            ci3, cr4 = di[2] + di[3], di[2] - di[3]
            a, b = CC[:, 0][..., ii - 1], CC[:, 0][..., ii]
            CH[:, :, 0][..., ii - 1] = a + cr2 + cr3
            CH[:, :, 0][..., ii] = b + ci2 + ci3
            tr2 = a + tr11 * cr2 + tr12 * cr3
            ti2 = b + tr11 * ci2 + tr12 * ci3
            tr3 = a + tr12 * cr2 + tr11 * cr3
            ti3 = b + tr12 * ci2 + tr11 * ci3
            tr5, tr4 = cr5 * ti11 + cr4 * ti12, cr5 * ti12 - cr4 * ti11
            ti5, ti4 = ci5 * ti11 + ci4 * ti12, ci5 * ti12 - ci4 * ti11
            CH[:, :, 2][..., ii - 1] = tr2 + tr5
            CH[:, :, 1][..., ic - 1] = tr2 - tr5
            CH[:, :, 2][..., ii] = ti5 + ti2
            CH[:, :, 1][..., ic] = ti5 - ti2
            CH[:, :, 4][..., ii - 1] = tr3 + tr4
            CH[:, :, 3][..., ic - 1] = tr3 - tr4
            CH[:, :, 4][..., ii] = ti4 + ti3
            CH[:, :, 3][..., ic] = ti4 - ti3
    else:
        return _radfg(ip, ido, l1, p1, tw, csarr, dtype)
    return CH.reshape(B, -1)


def _radfg(ip, ido, l1, cc, wa, csarr, dtype):
    """rfftp::radfg (ip > 5, odd): works in place on cc (C1 / C2 views), result in cc."""
    T = dtype
    B = cc.shape[0]
    cc = cc.copy()
    ipph = (ip + 1) // 2
    idl1 = ido * l1
    C1 = cc.reshape(B, ip, l1, ido)     # C1(a, b, c) = cc[a + ido*(b + l1*c)] -> [:, c, b, a]
    C2 = cc.reshape(B, ip, idl1)        # C2(a, b) = cc[a + idl1*b] -> [:, b, a]
    ch = np.zeros((B, ip, idl1), T)     # CH2(a, b) = ch[a + idl1*b]; CH(a, b, c) = ch[a + ido*(b + l1*c)]
    if ido > 1:
        i = np.arange(1, ido - 1, 2)
        for j in range(1, ipph):
            jc = ip - j
            is_, is2 = (j - 1) * (ido - 1), (jc - 1) * (ido - 1)
            idij = is_ + (i - 1)
            idij2 = is2 + (i - 1)
            t1, t2 = C1[:, j][..., i].copy(), C1[:, j][..., i + 1].copy()
            t3, t4 = C1[:, jc][..., i].copy(), C1[:, jc][..., i + 1].copy()
            x1 = wa[idij] * t1 + wa[idij + 1] * t2
            x2 = wa[idij] * t2 - wa[idij + 1] * t1
            x3 = wa[idij2] * t3 + wa[idij2 + 1] * t4
            x4 = wa[idij2] * t4 - wa[idij2 + 1] * t3
            C1[:, j][..., i] = x3 + x1
            C1[:, jc][..., i + 1] = x3 - x1
            C1[:, j][..., i + 1] = x2 + x4
            C1[:, jc][..., i] = x2 - x4
    for j in range(1, ipph):
        jc = ip - j
        t1, t2 = C1[:, j][..., 0].copy(), C1[:, jc][..., 0].copy()
        C1[:, j][..., 0] = t2 + t1
        C1[:, jc][..., 0] = t2 - t1
    cs = csarr
    for l in range(1, ipph):
        lc = ip - l
        ch[:, l] = C2[:, 0] + cs[2 * l] * C2[:, 1] + cs[4 * l] * C2[:, 2]
        ch[:, lc] = cs[2 * l + 1] * C2[:, ip - 1] + cs[4 * l + 1] * C2[:, ip - 2]
        iang = 2 * l
        j, jc = 3, ip - 3
        while j < ipph - 3:
            a = []
            for _ in range(4):
                iang += l
                if iang > ip:
                    iang -= ip
                a.append(iang)
            ch[:, l] = ch[:, l] + (cs[2 * a[0]] * C2[:, j] + cs[2 * a[1]] * C2[:, j + 1]
                                   + cs[2 * a[2]] * C2[:, j + 2] + cs[2 * a[3]] * C2[:, j + 3])
            ch[:, lc] = ch[:, lc] + (cs[2 * a[0] + 1] * C2[:, jc] + cs[2 * a[1] + 1] * C2[:, jc - 1]
                                     + cs[2 * a[2] + 1] * C2[:, jc - 2] + cs[2 * a[3] + 1] * C2[:, jc - 3])
            j += 4
            jc -= 4
        while j < ipph - 1:
            a = []
            for _ in range(2):
                iang += l
                if iang > ip:
                    iang -= ip
                a.append(iang)
            ch[:, l] = ch[:, l] + (cs[2 * a[0]] * C2[:, j] + cs[2 * a[1]] * C2[:, j + 1])
            ch[:, lc] = ch[:, lc] + (cs[2 * a[0] + 1] * C2[:, jc] + cs[2 * a[1] + 1] * C2[:, jc - 1])
            j += 2
            jc -= 2
        while j < ipph:
            iang += l
            if iang > ip:
                iang -= ip
            ch[:, l] = ch[:, l] + cs[2 * iang] * C2[:, j]
            ch[:, lc] = ch[:, lc] + cs[2 * iang + 1] * C2[:, jc]
            j += 1
            jc -= 1
    acc = C2[:, 0].copy()
    for j in range(1, ipph):
        acc = acc + C2[:, j]
    ch[:, 0] = acc
    CH = ch.reshape(B, ip, l1, ido)     # CH(a, b, c) -> [:, c, b, a]
    out = np.zeros((B, l1, ip, ido), T)  # CC(a, b, c) = cc[a + ido*(b + ip*c)] -> [:, c, b, a]
    out[:, :, 0][..., :] = CH[:, 0]
    for j in range(1, ipph):
        jc = ip - j
        j2 = 2 * j - 1
        out[:, :, j2][..., ido - 1] = CH[:, j][..., 0]
        out[:, :, j2 + 1][..., 0] = CH[:, jc][..., 0]
    if ido > 1:
        i = np.arange(1, ido - 1, 2)
        ic = ido - i - 2
        for j in range(1, ipph):
            jc = ip - j
            j2 = 2 * j - 1
            out[:, :, j2 + 1][..., i] = CH[:, j][..., i] + CH[:, jc][..., i]
            out[:, :, j2][..., ic] = CH[:, j][..., i] - CH[:, jc][..., i]
            out[:, :, j2 + 1][..., i + 1] = CH[:, j][..., i + 1] + CH[:, jc][..., i + 1]
            out[:, :, j2][..., ic + 1] = CH[:, jc][..., i + 1] - CH[:, j][..., i + 1]
    return out.reshape(B, -1)


def rfft_rows(x, dtype=None):
    """pocketfft r2c (forward) of every row of [rows, n] -> (re, im) [rows, n/2+1] of T."""
    T = np.dtype(dtype or x.dtype).type
    p1 = np.array(x, T, copy=True, order="C")
    rows, n = p1.shape
    if use_bluestein(n, True):
        br = Bluestein(n, T)
        zr, zi = br.fft((p1, np.zeros_like(p1)), True)
        # exec_r: c[0] = tmp[0].r; c[1 .. n-1] = tmp[1].r, tmp[1].i, tmp[2].r, ...
        flat = np.stack([zr, zi], -1).reshape(rows, 2 * n)
        p1 = np.concatenate([zr[:, :1], flat[:, 2:n + 1]], 1)
    elif n > 1:
        fact = rfactors(n)
        tws = rtwiddles(n, fact, T)
        l1 = n
        for k in reversed(range(len(fact))):  # rfftp::exec, r2hc: factors last to first
            ip = fact[k]
            ido = n // l1
            l1 //= ip
            p1 = _radf(ip, ido, l1, p1, tws[k][0], tws[k][1], T)
    re = np.zeros((rows, n // 2 + 1), T)
    im = np.zeros((rows, n // 2 + 1), T)
    re[:, 0] = p1[:, 0]
    re[:, 1:(n + 1) // 2] = p1[:, 1:n - 1 + n % 2:2]
    im[:, 1:(n + 1) // 2] = p1[:, 2:n:2]
    if n % 2 == 0:
        re[:, n // 2] = p1[:, n - 1]
    return re, im


def spectrum_dtype(dtype):
    """The real type scipy 1.7.1's fft2 computes an image of this dtype in
    (`scipy/fft/_pocketfft/helper.py:91-92`, `_asfarray`): float32 and float16 -> float32
    (pocketfft has no half precision), float64 stays float64, and every non-float dtype
    (bool, int, uint) -> float64.  fourier.py:18's `image - np.mean(image)` gives the same
    types (an integer image minus its float64 mean is float64)."""
    dt = np.dtype(dtype)
    if dt in (np.float32, np.float16):
        return np.float32
    return np.float64


def fft2(x):
    """scipy.fft.fft2 of a real image (c2c_sym_internal): complex [H, W], complex64 for
    float32 / float16 images, complex128 for everything else (spectrum_dtype)."""
    x = np.ascontiguousarray(x)
    T = spectrum_dtype(x.dtype)
    x = x.astype(T)
    H, W = x.shape
    hr, hi = rfft_rows(x, T)                            # [H, W/2+1]
    cr, ci = cfft((hr.T.copy(), hi.T.copy()), True, T)  # columns as rows: [W/2+1, H]
    half = np.empty((H, W // 2 + 1), np.complex64 if T == np.float32 else np.complex128)
    half.real, half.imag = cr.T, ci.T
    out = np.empty((H, W), half.dtype)
    wh = W // 2 + 1
    out[:, :wh] = half
    # rev_iter over (i, j < W/2 + 1) in row-major order: out[(H - i) % H, (W - j) % W] = conj(out[i, j])
    for j in range(wh):
        jm = (W - j) % W
        if jm >= wh:
            out[(H - np.arange(H)) % H, jm] = np.conj(half[:, j])
        else:  # self-mirrored column (0, and W/2 for even W): sequential overwrite semantics
            col = half[:, j].copy()
            for i in range(H):
                col[(H - i) % H] = np.conj(col[i])
            out[:, j] = col
    return out


# ================================================================ numpy 1.26.4 reductions
def _pairwise(a, lo, n, T):
    if n < 8:
        res = T(0.0)
        for i in range(n):
            res = T(res + a[lo + i])
        return res
    if n <= 128:
        r = a[lo:lo + 8].copy()
        i = 8
        while i < n - (n % 8):
            r = (r + a[lo + i:lo + i + 8]).astype(T)
            i += 8
        res = T(T(T(r[0] + r[1]) + T(r[2] + r[3])) + T(T(r[4] + r[5]) + T(r[6] + r[7])))
        while i < n:
            res = T(res + a[lo + i])
            i += 1
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return T(_pairwise(a, lo, n2, T) + _pairwise(a, lo + n2, n - n2, T))


def sum_T(x, T):
    """np.add.reduce of a float32 / float64 array over all axes."""
    a = np.ascontiguousarray(x, T).ravel()
    acc = T(0)
    for i in range(0, a.size, 8192):
        acc = T(acc + _pairwise(a, i, min(8192, a.size - i), T))
    return acc


def mean_T(x, T):
    return T(sum_T(x, T) / T(np.asarray(x).size))


def _fma_exact(a, b, c):
    """fma(a, b, c) in float64, correctly rounded (numpy has no fma): Dekker's two-product,
    two-sum, and an exact rational fallback for the (rare) possible double roundings."""
    a, b, c = (np.asarray(v, np.float64) for v in (a, b, c))
    p = a * b
    sp = 134217729.0 * a
    ah = sp - (sp - a)
    al = a - ah
    sb = 134217729.0 * b
    bh = sb - (sb - b)
    bl = b - bh
    e = ((ah * bh - p) + ah * bl + al * bh) + al * bl  # a*b = p + e exactly
    s = p + c
    bb = s - p
    t = (p - (s - bb)) + (c - bb)  # p + c = s + t exactly
    u = t + e
    res = s + u
    # exact whenever u carries the tail exactly and res is not a tie candidate
    uu = u - t
    exact_u = (e - uu) == 0
    suspicious = ~exact_u | (np.abs(res - s) == 0.5 * np.spacing(np.abs(s)))
    if np.any(suspicious):
        res = res.copy()
        for k in zip(*np.nonzero(suspicious)):
            v = Fraction(float(a[k])) * Fraction(float(b[k])) + Fraction(float(c[k]))
            res[k] = float(v)  # Fraction -> float is correctly rounded
    return res


def abs_c(z):
    """np.abs of complex64 / complex128 (numpy 1.26.4, AVX512F): larger * sqrt(fma(r, r, 1))."""
    if z.dtype == np.complex64:
        T = np.float32
    else:
        T = np.float64
    re, im = np.abs(z.real), np.abs(z.imag)
    big = np.maximum(re, im)
    small = np.minimum(im, re)
    r = np.where(big == 0, T(0), small / np.where(big == 0, T(1), big)).astype(T)
    if T == np.float32:
        r64 = r.astype(np.float64)  # r*r + 1 is exact in f64: one rounding = fma's
        return (np.sqrt((r64 * r64 + 1.0).astype(np.float32)) * big).astype(np.float32)
    return np.sqrt(_fma_exact(r, r, np.ones_like(r))) * big


def find_peaks_spectrum(image):
    """|fftshift(fft2(image - mean(image)))| as fourier.py:18, in spectrum_dtype's precision:
    an integer image's mean is float64 and exact (every partial sum is an integer below
    2^53 for images up to 16384^2 of 16-bit samples), so converting first changes nothing."""
    T = spectrum_dtype(np.asarray(image).dtype)
    img = np.ascontiguousarray(image, T)
    return np.fft.fftshift(abs_c(fft2((img - mean_T(img, T)).astype(T))))


# ---- float32 names (fourier.py:18 for a float32 image), used by tests and tools
def mean_f32(x):
    return mean_T(x, np.float32)


def abs_c64(z):
    return abs_c(np.asarray(z, np.complex64))
