"""TEST INFRASTRUCTURE ONLY (the checker, never the product): the float32 spectrum
that fourier.find_peaks sees, restated operation for operation.

The reference computes `np.abs(fftshift(fft2(image - np.mean(image))))`
(/root/reference/pyfcd/fourier.py:18) with two third-party libraries that are not in
/root/reference:

* scipy.fft.fft2 = pocketfft (C++, pocketfft_hdronly.hpp as vendored by scipy 1.7.1,
  the version this container's reference interpreter runs).  For a real float32 image
  scipy's `c2c` takes its symmetric path (`c2c_sym_internal`): a real-to-complex
  transform of every row (`rfftp`, FFTPACK radf4 / radf2 passes), a complex transform
  of every column of the half spectrum (`cfftp`, pass8 / pass4 / pass2), then the other
  half filled as the complex conjugate of its mirror bin -- including the lower halves
  of columns 0 and W/2.  Single precision throughout, no fused multiply-adds; twiddles
  are cos / sin(2 pi m / n) rounded to float.
* numpy 1.26.4: `np.mean` of a float32 image = the add-reduction over 8192-element
  buffer chunks, each summed pairwise (8 accumulators over 128-element blocks, blocks
  combined in halves), the chunk sums accumulated in order in float32, then one float32
  division; `np.abs` of complex64 = its AVX512F loop: larger * sqrt(fma(r, r, 1)) with
  r = smaller / larger.

Why: where two carrier peaks tie in exact arithmetic (the unrotated pattern.py board,
SURVEY.md §8a parity fact 2) the reference's pick is decided by the rounding of these
exact operations; restating them makes the engine's peak indices bit-exact there too.

Pinned: tests/golden/spectrum.npz holds sha256 digests of scipy's fft2, numpy's mean
and the reference's find_peaks spectrum for several images (tests/golden/make_golden.py
`spectrum`, run by the reference's interpreter), checked by
tests/test_oracle_golden.py::test_pocketfft32_matches_scipy_digests.
"""
import math

import numpy as np

f32 = np.float32
HSQT2 = f32(0.707106781186547524400844362104849)  # pocketfft's hsqt2 as T0 = float


def twiddle(n, m):
    """sincos_2pibyn<float>(n)[m]: (cos, sin)(2 pi m / n) rounded to float."""
    a = 2 * math.pi * m / n
    return f32(math.cos(a)), f32(math.sin(a))


def _odd_factors(f, left):
    """The odd part of pocketfft's factorize: divisors 3, 5, 7, ... in turn, the rest last.
    Only 3 and 5 have passes here (5-smooth lengths); others raise."""
    d = 3
    while d * d <= left:
        while left % d == 0:
            f.append(d)
            left //= d
        d += 2
    if left > 1:
        f.append(left)
    if any(p not in (2, 3, 4, 5, 8) for p in f):
        raise ValueError("lengths with prime factors above 5 are not restated")
    return f


def rfactors(n):
    """rfftp::factorize: 4s first, a single 2 moved to the front, then 3s, 5s."""
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
    """cfftp::factorize: 8s, then 4s, a single 2 moved to the front, then 3s, 5s."""
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


def rtwiddles(n, fact):
    """rfftp::comp_twiddle: per pass (ip - 1) * (ido - 1) floats, (cos, sin) pairs."""
    tws, l1 = [], 1
    for k, ip in enumerate(fact):
        ido = n // (l1 * ip)
        tw = np.zeros(max((ip - 1) * (ido - 1), 1), np.float32)
        if k < len(fact) - 1:
            for j in range(1, ip):
                for i in range(1, (ido - 1) // 2 + 1):
                    c, s = twiddle(n, j * l1 * i)
                    tw[(j - 1) * (ido - 1) + 2 * i - 2] = c
                    tw[(j - 1) * (ido - 1) + 2 * i - 1] = s
        tws.append(tw)
        l1 *= ip
    return tws


def ctwiddles(n, fact):
    """cfftp::comp_twiddle: per pass (ip - 1) * (ido - 1) complex (cos, sin)."""
    tws, l1 = [], 1
    for ip in fact:
        ido = n // (l1 * ip)
        tr = np.zeros(max((ip - 1) * (ido - 1), 1), np.float32)
        ti = np.zeros_like(tr)
        for j in range(1, ip):
            for i in range(1, ido):
                tr[(j - 1) * (ido - 1) + i - 1], ti[(j - 1) * (ido - 1) + i - 1] = twiddle(n, j * l1 * i)
        tws.append((tr, ti))
        l1 *= ip
    return tws


# ---------------------------------------------------------------- real rows (rfftp forward)
# Arrays are [rows, n] float32, vectorised over rows; CC(a, b, c) = cc[a + ido*(b + l1*c)],
# CH(a, b, c) = ch[a + ido*(b + ip*c)], PM(a, b, c, d): a = c + d, b = c - d,
# MULPM(a, b, c, d, e, f): a = c*e + d*f, b = c*f - d*e.
def _radf2(ido, l1, cc, ch, wa):
    CC = lambda a, b, c: cc[:, a + ido * (b + l1 * c)]  # noqa: E731

    def CH(a, b, c, v):
        ch[:, a + ido * (b + 2 * c)] = v
    for k in range(l1):
        CH(0, 0, k, CC(0, k, 0) + CC(0, k, 1))
        CH(ido - 1, 1, k, CC(0, k, 0) - CC(0, k, 1))
    if ido % 2 == 0:
        for k in range(l1):
            CH(0, 1, k, -CC(ido - 1, k, 1))
            CH(ido - 1, 0, k, CC(ido - 1, k, 0))
    if ido <= 2:
        return
    for k in range(l1):
        for i in range(2, ido, 2):
            ic = ido - i
            tr2 = wa[i - 2] * CC(i - 1, k, 1) + wa[i - 1] * CC(i, k, 1)
            ti2 = wa[i - 2] * CC(i, k, 1) - wa[i - 1] * CC(i - 1, k, 1)
            CH(i - 1, 0, k, CC(i - 1, k, 0) + tr2)
            CH(ic - 1, 1, k, CC(i - 1, k, 0) - tr2)
            CH(i, 0, k, ti2 + CC(i, k, 0))
            CH(ic, 1, k, ti2 - CC(i, k, 0))


def _radf4(ido, l1, cc, ch, wa):
    CC = lambda a, b, c: cc[:, a + ido * (b + l1 * c)]  # noqa: E731
    WA = lambda x, i: wa[i + x * (ido - 1)]  # noqa: E731

    def CH(a, b, c, v):
        ch[:, a + ido * (b + 4 * c)] = v
    for k in range(l1):
        tr1 = CC(0, k, 3) + CC(0, k, 1)
        CH(0, 2, k, CC(0, k, 3) - CC(0, k, 1))
        tr2 = CC(0, k, 0) + CC(0, k, 2)
        CH(ido - 1, 1, k, CC(0, k, 0) - CC(0, k, 2))
        CH(0, 0, k, tr2 + tr1)
        CH(ido - 1, 3, k, tr2 - tr1)
    if ido % 2 == 0:
        for k in range(l1):
            ti1 = -HSQT2 * (CC(ido - 1, k, 1) + CC(ido - 1, k, 3))
            tr1 = HSQT2 * (CC(ido - 1, k, 1) - CC(ido - 1, k, 3))
            CH(ido - 1, 0, k, CC(ido - 1, k, 0) + tr1)
            CH(ido - 1, 2, k, CC(ido - 1, k, 0) - tr1)
            CH(0, 3, k, ti1 + CC(ido - 1, k, 2))
            CH(0, 1, k, ti1 - CC(ido - 1, k, 2))
    if ido <= 2:
        return
    for k in range(l1):
        for i in range(2, ido, 2):
            ic = ido - i
            cr2 = WA(0, i - 2) * CC(i - 1, k, 1) + WA(0, i - 1) * CC(i, k, 1)
            ci2 = WA(0, i - 2) * CC(i, k, 1) - WA(0, i - 1) * CC(i - 1, k, 1)
            cr3 = WA(1, i - 2) * CC(i - 1, k, 2) + WA(1, i - 1) * CC(i, k, 2)
            ci3 = WA(1, i - 2) * CC(i, k, 2) - WA(1, i - 1) * CC(i - 1, k, 2)
            cr4 = WA(2, i - 2) * CC(i - 1, k, 3) + WA(2, i - 1) * CC(i, k, 3)
            ci4 = WA(2, i - 2) * CC(i, k, 3) - WA(2, i - 1) * CC(i - 1, k, 3)
            tr1, tr4 = cr4 + cr2, cr4 - cr2
            ti1, ti4 = ci2 + ci4, ci2 - ci4
            tr2, tr3 = CC(i - 1, k, 0) + cr3, CC(i - 1, k, 0) - cr3
            ti2, ti3 = CC(i, k, 0) + ci3, CC(i, k, 0) - ci3
            CH(i - 1, 0, k, tr2 + tr1)
            CH(ic - 1, 3, k, tr2 - tr1)
            CH(i, 0, k, ti1 + ti2)
            CH(ic, 3, k, ti1 - ti2)
            CH(i - 1, 2, k, tr3 + ti4)
            CH(ic - 1, 1, k, tr3 - ti4)
            CH(i, 2, k, tr4 + ti3)
            CH(ic, 1, k, tr4 - ti3)


TAUR = f32(-0.5)
TAUI = f32(0.8660254037844386467637231707529362)
TR11 = f32(0.3090169943749474241022934171828191)
TI11 = f32(0.9510565162951535721164393333793821)
TR12 = f32(-0.8090169943749474241022934171828191)
TI12 = f32(0.5877852522924731291687059546390728)


def _radf3(ido, l1, cc, ch, wa):
    CC = lambda a, b, c: cc[:, a + ido * (b + l1 * c)]  # noqa: E731
    WA = lambda x, i: wa[i + x * (ido - 1)]  # noqa: E731

    def CH(a, b, c, v):
        ch[:, a + ido * (b + 3 * c)] = v
    for k in range(l1):
        cr2 = CC(0, k, 1) + CC(0, k, 2)
        CH(0, 0, k, CC(0, k, 0) + cr2)
        CH(0, 2, k, TAUI * (CC(0, k, 2) - CC(0, k, 1)))
        CH(ido - 1, 1, k, CC(0, k, 0) + TAUR * cr2)
    if ido == 1:
        return
    for k in range(l1):
        for i in range(2, ido, 2):
            ic = ido - i
            dr2 = WA(0, i - 2) * CC(i - 1, k, 1) + WA(0, i - 1) * CC(i, k, 1)
            di2 = WA(0, i - 2) * CC(i, k, 1) - WA(0, i - 1) * CC(i - 1, k, 1)
            dr3 = WA(1, i - 2) * CC(i - 1, k, 2) + WA(1, i - 1) * CC(i, k, 2)
            di3 = WA(1, i - 2) * CC(i, k, 2) - WA(1, i - 1) * CC(i - 1, k, 2)
            cr2 = dr2 + dr3
            ci2 = di2 + di3
            CH(i - 1, 0, k, CC(i - 1, k, 0) + cr2)
            CH(i, 0, k, CC(i, k, 0) + ci2)
            tr2 = CC(i - 1, k, 0) + TAUR * cr2
            ti2 = CC(i, k, 0) + TAUR * ci2
            tr3 = TAUI * (di2 - di3)
            ti3 = TAUI * (dr3 - dr2)
            CH(i - 1, 2, k, tr2 + tr3)
            CH(ic - 1, 1, k, tr2 - tr3)
            CH(i, 2, k, ti3 + ti2)
            CH(ic, 1, k, ti3 - ti2)


def _radf5(ido, l1, cc, ch, wa):
    CC = lambda a, b, c: cc[:, a + ido * (b + l1 * c)]  # noqa: E731
    WA = lambda x, i: wa[i + x * (ido - 1)]  # noqa: E731

    def CH(a, b, c, v):
        ch[:, a + ido * (b + 5 * c)] = v
    for k in range(l1):
        cr2, ci5 = CC(0, k, 4) + CC(0, k, 1), CC(0, k, 4) - CC(0, k, 1)
        cr3, ci4 = CC(0, k, 3) + CC(0, k, 2), CC(0, k, 3) - CC(0, k, 2)
        CH(0, 0, k, CC(0, k, 0) + cr2 + cr3)
        CH(ido - 1, 1, k, CC(0, k, 0) + TR11 * cr2 + TR12 * cr3)
        CH(0, 2, k, TI11 * ci5 + TI12 * ci4)
        CH(ido - 1, 3, k, CC(0, k, 0) + TR12 * cr2 + TR11 * cr3)
        CH(0, 4, k, TI12 * ci5 - TI11 * ci4)
    if ido == 1:
        return
    for k in range(l1):
        for i in range(2, ido, 2):
            ic = ido - i
            dr2 = WA(0, i - 2) * CC(i - 1, k, 1) + WA(0, i - 1) * CC(i, k, 1)
            di2 = WA(0, i - 2) * CC(i, k, 1) - WA(0, i - 1) * CC(i - 1, k, 1)
            dr3 = WA(1, i - 2) * CC(i - 1, k, 2) + WA(1, i - 1) * CC(i, k, 2)
            di3 = WA(1, i - 2) * CC(i, k, 2) - WA(1, i - 1) * CC(i - 1, k, 2)
            dr4 = WA(2, i - 2) * CC(i - 1, k, 3) + WA(2, i - 1) * CC(i, k, 3)
            di4 = WA(2, i - 2) * CC(i, k, 3) - WA(2, i - 1) * CC(i - 1, k, 3)
            dr5 = WA(3, i - 2) * CC(i - 1, k, 4) + WA(3, i - 1) * CC(i, k, 4)
            di5 = WA(3, i - 2) * CC(i, k, 4) - WA(3, i - 1) * CC(i - 1, k, 4)
            cr2, ci5 = dr5 + dr2, dr5 - dr2
            ci2, cr5 = di2 + di5, di2 - di5
            cr3, ci4 = dr4 + dr3, dr4 - dr3
            ci3, cr4 = di3 + di4, di3 - di4
            CH(i - 1, 0, k, CC(i - 1, k, 0) + cr2 + cr3)
            CH(i, 0, k, CC(i, k, 0) + ci2 + ci3)
            tr2 = CC(i - 1, k, 0) + TR11 * cr2 + TR12 * cr3
            ti2 = CC(i, k, 0) + TR11 * ci2 + TR12 * ci3
            tr3 = CC(i - 1, k, 0) + TR12 * cr2 + TR11 * cr3
            ti3 = CC(i, k, 0) + TR12 * ci2 + TR11 * ci3
            tr5, tr4 = cr5 * TI11 + cr4 * TI12, cr5 * TI12 - cr4 * TI11
            ti5, ti4 = ci5 * TI11 + ci4 * TI12, ci5 * TI12 - ci4 * TI11
            CH(i - 1, 2, k, tr2 + tr5)
            CH(ic - 1, 1, k, tr2 - tr5)
            CH(i, 2, k, ti5 + ti2)
            CH(ic, 1, k, ti5 - ti2)
            CH(i - 1, 4, k, tr3 + tr4)
            CH(ic - 1, 3, k, tr3 - tr4)
            CH(i, 4, k, ti4 + ti3)
            CH(ic, 3, k, ti4 - ti3)


_RADF = {2: _radf2, 3: _radf3, 4: _radf4, 5: _radf5}


def rfft_rows(x):
    """pocketfft r2c (forward) of every row of float32 [rows, n] -> complex64 [rows, n/2+1]."""
    p1 = np.array(x, np.float32, copy=True, order="C")
    rows, n = p1.shape
    fact = rfactors(n)
    tws = rtwiddles(n, fact)
    p2 = np.empty_like(p1)
    l1 = n
    for k in reversed(range(len(fact))):  # rfftp::exec, r2hc: factors last to first
        ip = fact[k]
        ido = n // l1
        l1 //= ip
        _RADF[ip](ido, l1, p1, p2, tws[k])
        p1, p2 = p2, p1
    out = np.zeros((rows, n // 2 + 1), np.complex64)  # halfcomplex r0, r1, i1, r2, i2, ... -> complex
    out.real[:, 0] = p1[:, 0]
    out.real[:, 1:(n + 1) // 2] = p1[:, 1:n - 1 + n % 2:2]
    out.imag[:, 1:(n + 1) // 2] = p1[:, 2:n:2]
    if n % 2 == 0:
        out.real[:, n // 2] = p1[:, n - 1]
    return out


# ---------------------------------------------------------------- complex columns (cfftp forward)
def _add(a, b):
    return a[0] + b[0], a[1] + b[1]


def _sub(a, b):
    return a[0] - b[0], a[1] - b[1]


def _mulc(v, w):  # special_mul<fwd = true>: v * conj(w)
    return v[0] * w[0] + v[1] * w[1], v[1] * w[0] - v[0] * w[1]


def _rot90(a):  # ROTX90<fwd>: * (-i)
    return a[1], -a[0]


def _rot45(a):
    return HSQT2 * (a[0] + a[1]), HSQT2 * (a[1] - a[0])


def _rot135(a):
    return HSQT2 * (a[1] - a[0]), HSQT2 * (-a[0] - a[1])


def _cpass(ip, ido, l1, c1, c2, tw):
    """pass2 / pass4 / pass8 <fwd = true> on [n, cols] re / im planes c1 -> c2."""
    tr, ti = tw
    (r1, i1), (r2, i2) = c1, c2

    def WA(x, i):
        return tr[i - 1 + x * (ido - 1)], ti[i - 1 + x * (ido - 1)]
    for k in range(l1):
        for i in range(ido):
            C = [(r1[i + ido * (m + ip * k)], i1[i + ido * (m + ip * k)]) for m in range(ip)]

            def put(m, v):
                o = i + ido * (k + l1 * m)
                r2[o], i2[o] = v
            if ip == 3:  # pass3
                t0 = C[0]
                t1, t2 = _add(C[1], C[2]), _sub(C[1], C[2])
                put(0, _add(t0, t1))
                ca = (t0[0] + t1[0] * TAUR, t0[1] + t1[1] * TAUR)
                cb = (-(t2[1] * -TAUI), t2[0] * -TAUI)
                if i == 0:
                    put(1, _add(ca, cb))
                    put(2, _sub(ca, cb))
                else:
                    put(1, _mulc(_add(ca, cb), WA(0, i)))
                    put(2, _mulc(_sub(ca, cb), WA(1, i)))
                continue
            if ip == 5:  # pass5
                t0 = C[0]
                t1, t4 = _add(C[1], C[4]), _sub(C[1], C[4])
                t2, t3 = _add(C[2], C[3]), _sub(C[2], C[3])
                put(0, (t0[0] + t1[0] + t2[0], t0[1] + t1[1] + t2[1]))
                for u1, u2, twar, twbr, twai, twbi in ((1, 4, TR11, TR12, -TI11, -TI12), (2, 3, TR12, TR11, -TI12, TI11)):
                    ca = (t0[0] + twar * t1[0] + twbr * t2[0], t0[1] + twar * t1[1] + twbr * t2[1])
                    cb = (-(twai * t4[1] + twbi * t3[1]), twai * t4[0] + twbi * t3[0])
                    if i == 0:
                        put(u1, _add(ca, cb))
                        put(u2, _sub(ca, cb))
                    else:
                        put(u1, _mulc(_add(ca, cb), WA(u1 - 1, i)))
                        put(u2, _mulc(_sub(ca, cb), WA(u2 - 1, i)))
                continue
            if ip == 2:
                put(0, _add(C[0], C[1]))
                d = _sub(C[0], C[1])
                put(1, d if i == 0 else _mulc(d, WA(0, i)))
            elif ip == 4:
                t2, t1 = _add(C[0], C[2]), _sub(C[0], C[2])
                t3, t4 = _add(C[1], C[3]), _sub(C[1], C[3])
                t4 = _rot90(t4)
                put(0, _add(t2, t3))
                if i == 0:
                    put(2, _sub(t2, t3))
                    put(1, _add(t1, t4))
                    put(3, _sub(t1, t4))
                else:
                    put(1, _mulc(_add(t1, t4), WA(0, i)))
                    put(2, _mulc(_sub(t2, t3), WA(1, i)))
                    put(3, _mulc(_sub(t1, t4), WA(2, i)))
            else:
                a1, a5 = _add(C[1], C[5]), _sub(C[1], C[5])
                a3, a7 = _add(C[3], C[7]), _sub(C[3], C[7])
                a1, a3 = _add(a1, a3), _sub(a1, a3)
                a3 = _rot90(a3)
                a7 = _rot90(a7)
                a5, a7 = _add(a5, a7), _sub(a5, a7)
                a5 = _rot45(a5)
                a7 = _rot135(a7)
                a0, a4 = _add(C[0], C[4]), _sub(C[0], C[4])
                a2, a6 = _add(C[2], C[6]), _sub(C[2], C[6])
                a0, a2 = _add(a0, a2), _sub(a0, a2)
                a6 = _rot90(a6)
                a4, a6 = _add(a4, a6), _sub(a4, a6)
                if i == 0:
                    put(0, _add(a0, a1))
                    put(4, _sub(a0, a1))
                    put(2, _add(a2, a3))
                    put(6, _sub(a2, a3))
                    put(1, _add(a4, a5))
                    put(5, _sub(a4, a5))
                    put(3, _add(a6, a7))
                    put(7, _sub(a6, a7))
                else:
                    put(0, _add(a0, a1))
                    put(4, _mulc(_sub(a0, a1), WA(3, i)))
                    put(2, _mulc(_add(a2, a3), WA(1, i)))
                    put(6, _mulc(_sub(a2, a3), WA(5, i)))
                    put(1, _mulc(_add(a4, a5), WA(0, i)))
                    put(5, _mulc(_sub(a4, a5), WA(4, i)))
                    put(3, _mulc(_add(a6, a7), WA(2, i)))
                    put(7, _mulc(_sub(a6, a7), WA(6, i)))


def cfft_cols(z):
    """pocketfft c2c forward along axis 0 of complex64 [n, cols] (cfftp::pass_all)."""
    n = z.shape[0]
    fact = cfactors(n)
    tws = ctwiddles(n, fact)
    c1 = (np.array(z.real, np.float32), np.array(z.imag, np.float32))
    c2 = (np.empty_like(c1[0]), np.empty_like(c1[1]))
    l1 = 1
    for k, ip in enumerate(fact):
        ido = n // (ip * l1)
        _cpass(ip, ido, l1, c1, c2, tws[k])
        c1, c2 = c2, c1
        l1 *= ip
    out = np.empty(z.shape, np.complex64)
    out.real, out.imag = c1
    return out


def fft2(x):
    """scipy.fft.fft2 of a real float32 image (c2c_sym_internal): complex64 [H, W]."""
    x = np.ascontiguousarray(x, np.float32)
    H, W = x.shape
    half = cfft_cols(rfft_rows(x))
    out = np.empty((H, W), np.complex64)
    out[:, :W // 2 + 1] = half
    i = np.arange(H)
    j = np.arange(W // 2 + 1, W)
    out[:, W // 2 + 1:] = np.conj(half[(H - i) % H][:, (W - j) % W])
    lo = np.arange(1, H // 2)
    for c in (0, W // 2):  # the rev iterator also mirrors these columns' lower halves,
        out[H - lo, c] = np.conj(half[lo, c])
        for r in (0, H // 2):  # and conjugates their self-mirrored bins in place (+0 -> -0 imag)
            out[r, c] = np.conj(half[r, c])
    return out


# ---------------------------------------------------------------- numpy 1.26.4 reductions
def _pairwise(a, lo, n):
    if n < 8:
        res = f32(0.0)
        for i in range(n):
            res = f32(res + a[lo + i])
        return res
    if n <= 128:
        r = a[lo:lo + 8].copy()
        i = 8
        while i < n - (n % 8):
            r = (r + a[lo + i:lo + i + 8]).astype(np.float32)
            i += 8
        res = f32(f32(f32(r[0] + r[1]) + f32(r[2] + r[3])) + f32(f32(r[4] + r[5]) + f32(r[6] + r[7])))
        while i < n:
            res = f32(res + a[lo + i])
            i += 1
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return f32(_pairwise(a, lo, n2) + _pairwise(a, lo + n2, n - n2))


def sum_f32(x):
    """np.add.reduce of a float32 array over all axes."""
    a = np.ascontiguousarray(x, np.float32).ravel()
    acc = f32(0)
    for i in range(0, a.size, 8192):
        acc = f32(acc + _pairwise(a, i, min(8192, a.size - i)))
    return acc


def mean_f32(x):
    return f32(sum_f32(x) / f32(np.asarray(x).size))


def abs_c64(z):
    """np.abs of complex64 (numpy 1.26.4, AVX512F): larger * sqrt(fma(r, r, 1))."""
    re, im = np.abs(z.real), np.abs(z.imag)
    big = np.maximum(re, im)
    small = np.minimum(im, re)
    r = np.where(big == 0, f32(0), small / np.where(big == 0, f32(1), big)).astype(np.float32)
    r64 = r.astype(np.float64)
    return (np.sqrt((r64 * r64 + 1.0).astype(np.float32)) * big).astype(np.float32)


def find_peaks_spectrum(image):
    """|fftshift(fft2(image - mean(image)))| of a float32 image, as fourier.py:18."""
    img = np.ascontiguousarray(image, np.float32)
    return np.fft.fftshift(abs_c64(fft2((img - mean_f32(img)).astype(np.float32))))
