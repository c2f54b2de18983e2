// The reference's peak-finding spectrum, operation for operation (fourier.py:18:
// np.abs(fftshift(scipy.fft.fft2(image - np.mean(image))))), for any frame shape and for
// float32 and float64 images: scipy 1.7.1's pocketfft (pocketfft_hdronly.hpp, not in
// /root/reference) and numpy 1.26.4's mean, restated from their published algorithms.
// The CPU restatement this mirrors, pinned bit for bit to scipy on every length
// 1..400 and the camera shapes, is oracle/pocketfft.py.
//
//  * plans: pocketfft_r / pocketfft_c choose FFTPACK passes (rfftp: radf4 / radf2 /
//    radf3 / radf5 / radfg; cfftp: pass8 / pass4 / pass2 / pass3 / pass5 / pass7 /
//    pass11 / passg) or Bluestein (fftblue, convolution length good_size_cmplx(2n - 1))
//    by the library's cost guess; twiddles from sincos_2pibyn (two tables of exp(2 pi i
//    x / n) in double through glibc's sincos, multiplied, rounded to T);
//  * every pass is the library's expression in the same order, no fused multiply-adds
//    (this header is compiled with -ffp-contract=off on the device and on the host).
//
// The passes are __host__ __device__: the kernels (kernels_pocketfft.hip) run them with
// one workgroup per row / column, (tid, nt) = (threadIdx.x, blockDim.x) and a barrier
// between phases; the host runs them with (0, 1) to build Bluestein's FFT of b_k, and
// tests/native/host_logic_test.cpp checks the host runs against the oracle.
#pragma once
#include <cmath>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#if defined(__HIPCC__)
#define PF_HD __host__ __device__
#else
#define PF_HD
#endif

namespace pf {

template <class T>
struct cx {
    T r, i;
};
template <class T>
PF_HD inline cx<T> mk(T r, T i) {
    cx<T> c;
    c.r = r;
    c.i = i;
    return c;
}
template <class T>
PF_HD inline cx<T> add(cx<T> a, cx<T> b) { return mk<T>(a.r + b.r, a.i + b.i); }
template <class T>
PF_HD inline cx<T> sub(cx<T> a, cx<T> b) { return mk<T>(a.r - b.r, a.i - b.i); }
// special_mul<fwd>: v * conj(w) forward, v * w backward
template <bool FWD, class T>
PF_HD inline cx<T> smul(cx<T> v, cx<T> w) {
    return FWD ? mk<T>(v.r * w.r + v.i * w.i, v.i * w.r - v.r * w.i) : mk<T>(v.r * w.r - v.i * w.i, v.r * w.i + v.i * w.r);
}
template <bool FWD, class T>
PF_HD inline cx<T> rot90(cx<T> a) { return FWD ? mk<T>(a.i, -a.r) : mk<T>(-a.i, a.r); }
template <bool FWD, class T>
PF_HD inline cx<T> rot45(cx<T> a, T h) {
    return FWD ? mk<T>(h * (a.r + a.i), h * (a.i - a.r)) : mk<T>(h * (a.r - a.i), h * (a.i + a.r));
}
template <bool FWD, class T>
PF_HD inline cx<T> rot135(cx<T> a, T h) {
    return FWD ? mk<T>(h * (a.i - a.r), h * (-a.r - a.i)) : mk<T>(h * (-a.r - a.i), h * (a.r - a.i));
}

// A plan (POD: passed by value to kernels).  Offsets are in units of T into the plan's
// table.  Table layout: [0] hsqt2, [1..22] the (cos, sin) literals of pass3 / 5 / 7 / 11
// (and radf3 / radf5), then the passes' twiddles.
constexpr int kMaxFact = 20;
struct Plan {
    int n;      // transform length
    int real;   // rfftp (rows: real input) unless blue
    int blue;   // Bluestein: the passes are cfftp(n2), bk / bkf its tables
    int n2;
    int nf;
    int fct[kMaxFact];
    int tw[kMaxFact];   // pass twiddles: rfftp (ip - 1)(ido - 1) T; cfftp (ip - 1)(ido - 1) complex
    int tws[kMaxFact];  // radfg: 2 ip T; passg: ip complex; -1: none
    int bk, bkf;        // Bluestein: b_k [n] complex, FFT(b_k) [n2 / 2 + 1] complex
};
constexpr int kHsqt2 = 0;
PF_HD constexpr int const_off(int ip) { return ip == 3 ? 1 : ip == 5 ? 3 : ip == 7 ? 7 : 13; }  // (cos, sin) pairs
constexpr int kConsts = 23;

// ------------------------------------------------------------------ cfftp passes
// CC(i, m, k) = cc[i + ido*(m + ip*k)], CH(i, k, m) = ch[i + ido*(k + l1*m)],
// WA(x, i) = wa[i - 1 + x*(ido - 1)]; items (k, i) over (tid, nt).
template <class T, bool FWD>
PF_HD inline void pass2(int ido, int l1, const cx<T>* cc, cx<T>* ch, const cx<T>* wa, int tid, int nt) {
    for (int it = tid; it < l1 * ido; it += nt) {
        const int k = it / ido, i = it % ido;
        const cx<T> a = cc[i + ido * (2 * k)], b = cc[i + ido * (1 + 2 * k)];
        ch[i + ido * k] = add(a, b);
        const cx<T> d = sub(a, b);
        ch[i + ido * (k + l1)] = i == 0 ? d : smul<FWD>(d, wa[i - 1]);
    }
}

template <class T, bool FWD>
PF_HD inline void pass4(int ido, int l1, const cx<T>* cc, cx<T>* ch, const cx<T>* wa, int tid, int nt) {
    for (int it = tid; it < l1 * ido; it += nt) {
        const int k = it / ido, i = it % ido;
        const cx<T>* C = cc + i + ido * 4 * k;
        const cx<T> t2 = add(C[0], C[2 * ido]), t1 = sub(C[0], C[2 * ido]);
        const cx<T> t3 = add(C[ido], C[3 * ido]);
        const cx<T> t4 = rot90<FWD>(sub(C[ido], C[3 * ido]));
        cx<T>* O = ch + i + ido * k;
        const long s = (long)ido * l1;
        O[0] = add(t2, t3);
        if (i == 0) {
            O[2 * s] = sub(t2, t3);
            O[s] = add(t1, t4);
            O[3 * s] = sub(t1, t4);
        } else {
            O[s] = smul<FWD>(add(t1, t4), wa[i - 1]);
            O[2 * s] = smul<FWD>(sub(t2, t3), wa[i - 1 + (ido - 1)]);
            O[3 * s] = smul<FWD>(sub(t1, t4), wa[i - 1 + 2 * (ido - 1)]);
        }
    }
}

template <class T, bool FWD>
PF_HD inline void pass8(int ido, int l1, const cx<T>* cc, cx<T>* ch, const cx<T>* wa, T h, int tid, int nt) {
    for (int it = tid; it < l1 * ido; it += nt) {
        const int k = it / ido, i = it % ido;
        const cx<T>* C = cc + i + ido * 8 * k;
        cx<T> a1 = add(C[ido], C[5 * ido]), a5 = sub(C[ido], C[5 * ido]);
        cx<T> a3 = add(C[3 * ido], C[7 * ido]), a7 = sub(C[3 * ido], C[7 * ido]);
        {
            const cx<T> t = a1;
            a1 = add(t, a3);
            a3 = sub(t, a3);
        }
        a3 = rot90<FWD>(a3);
        a7 = rot90<FWD>(a7);
        {
            const cx<T> t = a5;
            a5 = add(t, a7);
            a7 = sub(t, a7);
        }
        a5 = rot45<FWD>(a5, h);
        a7 = rot135<FWD>(a7, h);
        cx<T> a0 = add(C[0], C[4 * ido]), a4 = sub(C[0], C[4 * ido]);
        cx<T> a2 = add(C[2 * ido], C[6 * ido]), a6 = sub(C[2 * ido], C[6 * ido]);
        {
            const cx<T> t = a0;
            a0 = add(t, a2);
            a2 = sub(t, a2);
        }
        cx<T>* O = ch + i + ido * k;
        const long s = (long)ido * l1;
        O[0] = add(a0, a1);
        cx<T> o[8];
        o[4] = sub(a0, a1);
        o[2] = add(a2, a3);
        o[6] = sub(a2, a3);
        a6 = rot90<FWD>(a6);
        {
            const cx<T> t = a4;
            a4 = add(t, a6);
            a6 = sub(t, a6);
        }
        o[1] = add(a4, a5);
        o[5] = sub(a4, a5);
        o[3] = add(a6, a7);
        o[7] = sub(a6, a7);
        for (int m = 1; m < 8; ++m) O[m * s] = i == 0 ? o[m] : smul<FWD>(o[m], wa[i - 1 + (m - 1) * (ido - 1)]);
    }
}

// pass3 / pass5 / pass7 / pass11 (PREPn / PARTSTEPna): t0 = CC(0); pairs s_m = CC(m) +
// CC(IP - m), d_m = CC(m) - CC(IP - m); CH(0) = t0 + s_1 + s_2 + ... (left to right);
// out_u = ca + cb, out_{IP-u} = ca - cb, ca = t0 + sum_m cos(2 pi u m / IP) s_m,
// cb = i sum_m (-+)sin(2 pi u m / IP) d_m (the literals of the table, in order m).
template <class T, bool FWD, int IP>
PF_HD inline void passodd(int ido, int l1, const cx<T>* cc, cx<T>* ch, const cx<T>* wa, const T* cs, int tid, int nt) {
    constexpr int HF = (IP - 1) / 2;
    for (int it = tid; it < l1 * ido; it += nt) {
        const int k = it / ido, i = it % ido;
        const cx<T>* C = cc + i + ido * IP * k;
        cx<T> s[HF + 1], d[HF + 1];
        const cx<T> t0 = C[0];
        for (int m = 1; m <= HF; ++m) {
            s[m] = add(C[m * ido], C[(IP - m) * ido]);
            d[m] = sub(C[m * ido], C[(IP - m) * ido]);
        }
        cx<T>* O = ch + i + ido * k;
        const long st = (long)ido * l1;
        T r0 = t0.r, i0 = t0.i;
        for (int m = 1; m <= HF; ++m) {
            r0 = r0 + s[m].r;
            i0 = i0 + s[m].i;
        }
        O[0] = mk<T>(r0, i0);
        for (int u = 1; u <= HF; ++u) {
            T car = t0.r, cai = t0.i, cbr = T(0), cbi = T(0);
            for (int m = 1; m <= HF; ++m) {
                int q = (u * m) % IP;
                bool neg = FWD;
                if (q > HF) {
                    q = IP - q;
                    neg = !neg;
                }
                const T twr = cs[2 * (q - 1)], twi = neg ? -cs[2 * (q - 1) + 1] : cs[2 * (q - 1) + 1];
                car = car + twr * s[m].r;
                cai = cai + twr * s[m].i;
                const T pr = twi * d[m].r, pi = twi * d[m].i;
                cbi = m == 1 ? pr : cbi + pr;
                cbr = m == 1 ? pi : cbr + pi;
            }
            const cx<T> ca = mk<T>(car, cai), cb = mk<T>(-cbr, cbi);
            cx<T> o1 = add(ca, cb), o2 = sub(ca, cb);
            if (i > 0) {
                o1 = smul<FWD>(o1, wa[i - 1 + (u - 1) * (ido - 1)]);
                o2 = smul<FWD>(o2, wa[i - 1 + (IP - u - 1) * (ido - 1)]);
            }
            O[u * st] = o1;
            O[(IP - u) * st] = o2;
        }
    }
}

// cfftp::passg (ip > 11, odd prime): result in cc.  wal[j] = csarr[j] (conjugated forward).
template <class T, bool FWD, class Sync>
PF_HD inline void passg(int ido, int ip, int l1, cx<T>* cc, cx<T>* ch, const cx<T>* wa, const cx<T>* csarr, int tid,
                        int nt, Sync sync) {
    const int ipph = (ip + 1) / 2, idl1 = ido * l1;
    auto wal = [&](int j) { return j == 0 ? mk<T>(T(1), T(0)) : mk<T>(csarr[j].r, FWD ? -csarr[j].i : csarr[j].i); };
    // CH(i, k, 0) = CC(i, 0, k); PM(CH(i, k, j), CH(i, k, jc), CC(i, j, k), CC(i, jc, k))
    for (int it = tid; it < idl1; it += nt) {
        const int k = it / ido, i = it % ido;
        const cx<T>* C = cc + i + ido * ip * k;
        ch[it] = C[0];
        for (int j = 1; j < ipph; ++j) {
            const int jc = ip - j;
            ch[it + (long)idl1 * j] = add(C[j * ido], C[jc * ido]);
            ch[it + (long)idl1 * jc] = sub(C[j * ido], C[jc * ido]);
        }
    }
    sync();
    for (int ik = tid; ik < idl1; ik += nt) {
        auto CH2 = [&](int j) { return ch[ik + (long)idl1 * j]; };
        cx<T> tmp = CH2(0);
        for (int j = 1; j < ipph; ++j) tmp = add(tmp, CH2(j));
        cc[ik] = tmp;
        for (int l = 1; l < ipph; ++l) {
            const int lc = ip - l;
            const cx<T> w1 = wal(l), w2 = wal(2 * l);
            T xr = CH2(0).r + w1.r * CH2(1).r + w2.r * CH2(2).r;
            T xi = CH2(0).i + w1.r * CH2(1).i + w2.r * CH2(2).i;
            T yr = -(w1.i * CH2(ip - 1).i + w2.i * CH2(ip - 2).i);
            T yi = w1.i * CH2(ip - 1).r + w2.i * CH2(ip - 2).r;
            int iwal = 2 * l;
            int j = 3, jc = ip - 3;
            for (; j < ipph - 1; j += 2, jc -= 2) {
                iwal += l;
                if (iwal > ip) iwal -= ip;
                const cx<T> xw = wal(iwal);
                iwal += l;
                if (iwal > ip) iwal -= ip;
                const cx<T> xw2 = wal(iwal);
                xr = xr + (CH2(j).r * xw.r + CH2(j + 1).r * xw2.r);
                xi = xi + (CH2(j).i * xw.r + CH2(j + 1).i * xw2.r);
                yr = yr - (CH2(jc).i * xw.i + CH2(jc - 1).i * xw2.i);
                yi = yi + (CH2(jc).r * xw.i + CH2(jc - 1).r * xw2.i);
            }
            for (; j < ipph; ++j, --jc) {
                iwal += l;
                if (iwal > ip) iwal -= ip;
                const cx<T> xw = wal(iwal);
                xr = xr + CH2(j).r * xw.r;
                xi = xi + CH2(j).i * xw.r;
                yr = yr - CH2(jc).i * xw.i;
                yi = yi + CH2(jc).r * xw.i;
            }
            cc[ik + (long)idl1 * l] = mk<T>(xr, xi);
            cc[ik + (long)idl1 * lc] = mk<T>(yr, yi);
        }
    }
    sync();
    // shuffling and twiddling
    for (int it = tid; it < idl1 * (ipph - 1); it += nt) {
        const int ik = it % idl1, j = 1 + it / idl1, jc = ip - j;
        const int i = ik % ido;
        const cx<T> t1 = cc[ik + (long)idl1 * j], t2 = cc[ik + (long)idl1 * jc];
        cx<T> x1 = add(t1, t2), x2 = sub(t1, t2);
        if (i > 0) {
            x1 = smul<FWD>(x1, wa[(j - 1) * (ido - 1) + i - 1]);
            x2 = smul<FWD>(x2, wa[(jc - 1) * (ido - 1) + i - 1]);
        }
        cc[ik + (long)idl1 * j] = x1;
        cc[ik + (long)idl1 * jc] = x2;
    }
}

// cfftp::pass_all<fwd> (fct = 1) over the plan's factors (of n, or of n2 for Bluestein);
// p1 holds the input; returns the buffer holding the result (p1 or p2).
template <class T, bool FWD, class Sync>
PF_HD inline cx<T>* cfft_run(const Plan& p, const T* tab, cx<T>* p1, cx<T>* p2, int tid, int nt, Sync sync) {
    const int L = p.blue ? p.n2 : p.n;
    int l1 = 1;
    const T h = tab[kHsqt2];
    for (int k = 0; k < p.nf; ++k) {
        const int ip = p.fct[k], ido = L / (l1 * ip);
        const cx<T>* wa = reinterpret_cast<const cx<T>*>(tab + p.tw[k]);
        bool swap = true;
        switch (ip) {
            case 2: pass2<T, FWD>(ido, l1, p1, p2, wa, tid, nt); break;
            case 4: pass4<T, FWD>(ido, l1, p1, p2, wa, tid, nt); break;
            case 8: pass8<T, FWD>(ido, l1, p1, p2, wa, h, tid, nt); break;
            case 3: passodd<T, FWD, 3>(ido, l1, p1, p2, wa, tab + const_off(3), tid, nt); break;
            case 5: passodd<T, FWD, 5>(ido, l1, p1, p2, wa, tab + const_off(5), tid, nt); break;
            case 7: passodd<T, FWD, 7>(ido, l1, p1, p2, wa, tab + const_off(7), tid, nt); break;
            case 11: passodd<T, FWD, 11>(ido, l1, p1, p2, wa, tab + const_off(11), tid, nt); break;
            default:
                passg<T, FWD>(ido, ip, l1, p1, p2, wa, reinterpret_cast<const cx<T>*>(tab + p.tws[k]), tid, nt, sync);
                swap = false;
        }
        sync();
        if (swap) {
            cx<T>* t = p1;
            p1 = p2;
            p2 = t;
        }
        l1 *= ip;
    }
    return p1;
}

// ------------------------------------------------------------------ rfftp forward passes
// CC(a, b, c) = cc[a + ido*(b + l1*c)], CH(a, b, c) = ch[a + ido*(b + ip*c)]
template <class T>
PF_HD inline void radf2(int ido, int l1, const T* cc, T* ch, const T* wa, int tid, int nt) {
#define CC(a, b, c) cc[(a) + ido * ((b) + l1 * (c))]
#define CH(a, b, c) ch[(a) + ido * ((b) + 2 * (c))]
    for (int k = tid; k < l1; k += nt) {
        CH(0, 0, k) = CC(0, k, 0) + CC(0, k, 1);
        CH(ido - 1, 1, k) = CC(0, k, 0) - CC(0, k, 1);
        if ((ido & 1) == 0) {
            CH(0, 1, k) = -CC(ido - 1, k, 1);
            CH(ido - 1, 0, k) = CC(ido - 1, k, 0);
        }
    }
    if (ido <= 2) return;
    const int m = (ido - 1) / 2;
    for (int it = tid; it < l1 * m; it += nt) {
        const int k = it / m, i = 2 + 2 * (it % m), ic = ido - i;
        const T tr2 = wa[i - 2] * CC(i - 1, k, 1) + wa[i - 1] * CC(i, k, 1);
        const T ti2 = wa[i - 2] * CC(i, k, 1) - wa[i - 1] * CC(i - 1, k, 1);
        CH(i - 1, 0, k) = CC(i - 1, k, 0) + tr2;
        CH(ic - 1, 1, k) = CC(i - 1, k, 0) - tr2;
        CH(i, 0, k) = ti2 + CC(i, k, 0);
        CH(ic, 1, k) = ti2 - CC(i, k, 0);
    }
#undef CH
}

template <class T>
PF_HD inline void radf4(int ido, int l1, const T* cc, T* ch, const T* wa, T hsqt2, int tid, int nt) {
#define CH(a, b, c) ch[(a) + ido * ((b) + 4 * (c))]
#define WA(x, i) wa[(i) + (x) * (ido - 1)]
    for (int k = tid; k < l1; k += nt) {
        const T tr1 = CC(0, k, 3) + CC(0, k, 1);
        CH(0, 2, k) = CC(0, k, 3) - CC(0, k, 1);
        const T tr2 = CC(0, k, 0) + CC(0, k, 2);
        CH(ido - 1, 1, k) = CC(0, k, 0) - CC(0, k, 2);
        CH(0, 0, k) = tr2 + tr1;
        CH(ido - 1, 3, k) = tr2 - tr1;
        if ((ido & 1) == 0) {
            const T ti1 = -hsqt2 * (CC(ido - 1, k, 1) + CC(ido - 1, k, 3));
            const T tq1 = hsqt2 * (CC(ido - 1, k, 1) - CC(ido - 1, k, 3));
            CH(ido - 1, 0, k) = CC(ido - 1, k, 0) + tq1;
            CH(ido - 1, 2, k) = CC(ido - 1, k, 0) - tq1;
            CH(0, 3, k) = ti1 + CC(ido - 1, k, 2);
            CH(0, 1, k) = ti1 - CC(ido - 1, k, 2);
        }
    }
    if (ido <= 2) return;
    const int m = (ido - 1) / 2;
    for (int it = tid; it < l1 * m; it += nt) {
        const int k = it / m, i = 2 + 2 * (it % m), ic = ido - i;
        const T cr2 = WA(0, i - 2) * CC(i - 1, k, 1) + WA(0, i - 1) * CC(i, k, 1);
        const T ci2 = WA(0, i - 2) * CC(i, k, 1) - WA(0, i - 1) * CC(i - 1, k, 1);
        const T cr3 = WA(1, i - 2) * CC(i - 1, k, 2) + WA(1, i - 1) * CC(i, k, 2);
        const T ci3 = WA(1, i - 2) * CC(i, k, 2) - WA(1, i - 1) * CC(i - 1, k, 2);
        const T cr4 = WA(2, i - 2) * CC(i - 1, k, 3) + WA(2, i - 1) * CC(i, k, 3);
        const T ci4 = WA(2, i - 2) * CC(i, k, 3) - WA(2, i - 1) * CC(i - 1, k, 3);
        const T tr1 = cr4 + cr2, tr4 = cr4 - cr2;
        const T ti1 = ci2 + ci4, ti4 = ci2 - ci4;
        const T tr2 = CC(i - 1, k, 0) + cr3, tr3 = CC(i - 1, k, 0) - cr3;
        const T ti2 = CC(i, k, 0) + ci3, ti3 = CC(i, k, 0) - ci3;
        CH(i - 1, 0, k) = tr2 + tr1;
        CH(ic - 1, 3, k) = tr2 - tr1;
        CH(i, 0, k) = ti1 + ti2;
        CH(ic, 3, k) = ti1 - ti2;
        CH(i - 1, 2, k) = tr3 + ti4;
        CH(ic - 1, 1, k) = tr3 - ti4;
        CH(i, 2, k) = tr4 + ti3;
        CH(ic, 1, k) = tr4 - ti3;
    }
#undef WA
#undef CH
}

template <class T>
PF_HD inline void radf3(int ido, int l1, const T* cc, T* ch, const T* wa, const T* cs, int tid, int nt) {
#define CH(a, b, c) ch[(a) + ido * ((b) + 3 * (c))]
#define WA(x, i) wa[(i) + (x) * (ido - 1)]
    const T taur = cs[0], taui = cs[1];
    for (int k = tid; k < l1; k += nt) {
        const T cr2 = CC(0, k, 1) + CC(0, k, 2);
        CH(0, 0, k) = CC(0, k, 0) + cr2;
        CH(0, 2, k) = taui * (CC(0, k, 2) - CC(0, k, 1));
        CH(ido - 1, 1, k) = CC(0, k, 0) + taur * cr2;
    }
    if (ido == 1) return;
    const int m = (ido - 1) / 2;
    for (int it = tid; it < l1 * m; it += nt) {
        const int k = it / m, i = 2 + 2 * (it % m), ic = ido - i;
        const T dr2 = WA(0, i - 2) * CC(i - 1, k, 1) + WA(0, i - 1) * CC(i, k, 1);
        const T di2 = WA(0, i - 2) * CC(i, k, 1) - WA(0, i - 1) * CC(i - 1, k, 1);
        const T dr3 = WA(1, i - 2) * CC(i - 1, k, 2) + WA(1, i - 1) * CC(i, k, 2);
        const T di3 = WA(1, i - 2) * CC(i, k, 2) - WA(1, i - 1) * CC(i - 1, k, 2);
        const T cr2 = dr2 + dr3, ci2 = di2 + di3;
        CH(i - 1, 0, k) = CC(i - 1, k, 0) + cr2;
        CH(i, 0, k) = CC(i, k, 0) + ci2;
        const T tr2 = CC(i - 1, k, 0) + taur * cr2, ti2 = CC(i, k, 0) + taur * ci2;
        const T tr3 = taui * (di2 - di3), ti3 = taui * (dr3 - dr2);
        CH(i - 1, 2, k) = tr2 + tr3;
        CH(ic - 1, 1, k) = tr2 - tr3;
        CH(i, 2, k) = ti3 + ti2;
        CH(ic, 1, k) = ti3 - ti2;
    }
#undef WA
#undef CH
}

template <class T>
PF_HD inline void radf5(int ido, int l1, const T* cc, T* ch, const T* wa, const T* cs, int tid, int nt) {
#define CH(a, b, c) ch[(a) + ido * ((b) + 5 * (c))]
#define WA(x, i) wa[(i) + (x) * (ido - 1)]
    const T tr11 = cs[0], ti11 = cs[1], tr12 = cs[2], ti12 = cs[3];
    for (int k = tid; k < l1; k += nt) {
        const T cr2 = CC(0, k, 4) + CC(0, k, 1), ci5 = CC(0, k, 4) - CC(0, k, 1);
        const T cr3 = CC(0, k, 3) + CC(0, k, 2), ci4 = CC(0, k, 3) - CC(0, k, 2);
        CH(0, 0, k) = CC(0, k, 0) + cr2 + cr3;
        CH(ido - 1, 1, k) = CC(0, k, 0) + tr11 * cr2 + tr12 * cr3;
        CH(0, 2, k) = ti11 * ci5 + ti12 * ci4;
        CH(ido - 1, 3, k) = CC(0, k, 0) + tr12 * cr2 + tr11 * cr3;
        CH(0, 4, k) = ti12 * ci5 - ti11 * ci4;
    }
    if (ido == 1) return;
    const int m = (ido - 1) / 2;
    for (int it = tid; it < l1 * m; it += nt) {
        const int k = it / m, i = 2 + 2 * (it % m), ic = ido - i;
        const T dr2 = WA(0, i - 2) * CC(i - 1, k, 1) + WA(0, i - 1) * CC(i, k, 1);
        const T di2 = WA(0, i - 2) * CC(i, k, 1) - WA(0, i - 1) * CC(i - 1, k, 1);
        const T dr3 = WA(1, i - 2) * CC(i - 1, k, 2) + WA(1, i - 1) * CC(i, k, 2);
        const T di3 = WA(1, i - 2) * CC(i, k, 2) - WA(1, i - 1) * CC(i - 1, k, 2);
        const T dr4 = WA(2, i - 2) * CC(i - 1, k, 3) + WA(2, i - 1) * CC(i, k, 3);
        const T di4 = WA(2, i - 2) * CC(i, k, 3) - WA(2, i - 1) * CC(i - 1, k, 3);
        const T dr5 = WA(3, i - 2) * CC(i - 1, k, 4) + WA(3, i - 1) * CC(i, k, 4);
        const T di5 = WA(3, i - 2) * CC(i, k, 4) - WA(3, i - 1) * CC(i - 1, k, 4);
        const T cr2 = dr5 + dr2, ci5 = dr5 - dr2;
        const T ci2 = di2 + di5, cr5 = di2 - di5;
        const T cr3 = dr4 + dr3, ci4 = dr4 - dr3;
        const T ci3 = di3 + di4, cr4 = di3 - di4;
        CH(i - 1, 0, k) = CC(i - 1, k, 0) + cr2 + cr3;
        CH(i, 0, k) = CC(i, k, 0) + ci2 + ci3;
        const T tr2 = CC(i - 1, k, 0) + tr11 * cr2 + tr12 * cr3;
        const T ti2 = CC(i, k, 0) + tr11 * ci2 + tr12 * ci3;
        const T tr3 = CC(i - 1, k, 0) + tr12 * cr2 + tr11 * cr3;
        const T ti3 = CC(i, k, 0) + tr12 * ci2 + tr11 * ci3;
        const T tr5 = cr5 * ti11 + cr4 * ti12, tr4 = cr5 * ti12 - cr4 * ti11;
        const T ti5 = ci5 * ti11 + ci4 * ti12, ti4 = ci5 * ti12 - ci4 * ti11;
        CH(i - 1, 2, k) = tr2 + tr5;
        CH(ic - 1, 1, k) = tr2 - tr5;
        CH(i, 2, k) = ti5 + ti2;
        CH(ic, 1, k) = ti5 - ti2;
        CH(i - 1, 4, k) = tr3 + tr4;
        CH(ic - 1, 3, k) = tr3 - tr4;
        CH(i, 4, k) = ti4 + ti3;
        CH(ic, 3, k) = ti4 - ti3;
    }
#undef WA
#undef CH
#undef CC
}

// rfftp::radfg (ip > 5, odd): works in place on cc (C1 / C2 views) with ch as scratch;
// the result is in cc.  csarr: 2 ip T, csarr[2 m] = cos, [2 m + 1] = sin(2 pi m / ip).
template <class T, class Sync>
PF_HD inline void radfg(int ido, int ip, int l1, T* cc, T* ch, const T* wa, const T* csarr, int tid, int nt, Sync sync) {
    const int ipph = (ip + 1) / 2, idl1 = ido * l1;
    auto C1 = [&](int a, int b, int c) -> T& { return cc[a + ido * (b + l1 * c)]; };
    auto C2 = [&](int a, int b) -> T& { return cc[a + (long)idl1 * b]; };
    auto CH2 = [&](int a, int b) -> T& { return ch[a + (long)idl1 * b]; };
    if (ido > 1) {
        const int ni = (ido - 1) / 2;  // i = 1, 3, ..., ido - 2
        for (int it = tid; it < (ipph - 1) * l1 * ni; it += nt) {
            const int j = 1 + it / (l1 * ni), rem = it % (l1 * ni), k = rem / ni, i = 1 + 2 * (rem % ni);
            const int jc = ip - j;
            const int idij = (j - 1) * (ido - 1) + (i - 1), idij2 = (jc - 1) * (ido - 1) + (i - 1);
            const T t1 = C1(i, k, j), t2 = C1(i + 1, k, j), t3 = C1(i, k, jc), t4 = C1(i + 1, k, jc);
            const T x1 = wa[idij] * t1 + wa[idij + 1] * t2, x2 = wa[idij] * t2 - wa[idij + 1] * t1;
            const T x3 = wa[idij2] * t3 + wa[idij2 + 1] * t4, x4 = wa[idij2] * t4 - wa[idij2 + 1] * t3;
            C1(i, k, j) = x3 + x1;
            C1(i + 1, k, jc) = x3 - x1;
            C1(i + 1, k, j) = x2 + x4;
            C1(i, k, jc) = x2 - x4;
        }
        sync();
    }
    for (int it = tid; it < (ipph - 1) * l1; it += nt) {
        const int j = 1 + it / l1, k = it % l1, jc = ip - j;
        const T t1 = C1(0, k, j), t2 = C1(0, k, jc);
        C1(0, k, j) = t2 + t1;
        C1(0, k, jc) = t2 - t1;
    }
    sync();
    for (int it = tid; it < ipph * idl1; it += nt) {
        const int l = it / idl1, ik = it % idl1;
        if (l == 0) {
            T acc = C2(ik, 0);
            for (int j = 1; j < ipph; ++j) acc = acc + C2(ik, j);
            CH2(ik, 0) = acc;
            continue;
        }
        const int lc = ip - l;
        T a = C2(ik, 0) + csarr[2 * l] * C2(ik, 1) + csarr[4 * l] * C2(ik, 2);
        T b = csarr[2 * l + 1] * C2(ik, ip - 1) + csarr[4 * l + 1] * C2(ik, ip - 2);
        int iang = 2 * l;
        int j = 3, jc = ip - 3;
        for (; j < ipph - 3; j += 4, jc -= 4) {
            int ia[4];
            for (int q = 0; q < 4; ++q) {
                iang += l;
                if (iang > ip) iang -= ip;
                ia[q] = iang;
            }
            a = a + (csarr[2 * ia[0]] * C2(ik, j) + csarr[2 * ia[1]] * C2(ik, j + 1) + csarr[2 * ia[2]] * C2(ik, j + 2) +
                     csarr[2 * ia[3]] * C2(ik, j + 3));
            b = b + (csarr[2 * ia[0] + 1] * C2(ik, jc) + csarr[2 * ia[1] + 1] * C2(ik, jc - 1) +
                     csarr[2 * ia[2] + 1] * C2(ik, jc - 2) + csarr[2 * ia[3] + 1] * C2(ik, jc - 3));
        }
        for (; j < ipph - 1; j += 2, jc -= 2) {
            int ia[2];
            for (int q = 0; q < 2; ++q) {
                iang += l;
                if (iang > ip) iang -= ip;
                ia[q] = iang;
            }
            a = a + (csarr[2 * ia[0]] * C2(ik, j) + csarr[2 * ia[1]] * C2(ik, j + 1));
            b = b + (csarr[2 * ia[0] + 1] * C2(ik, jc) + csarr[2 * ia[1] + 1] * C2(ik, jc - 1));
        }
        for (; j < ipph; ++j, --jc) {
            iang += l;
            if (iang > ip) iang -= ip;
            a = a + csarr[2 * iang] * C2(ik, j);
            b = b + csarr[2 * iang + 1] * C2(ik, jc);
        }
        CH2(ik, l) = a;
        CH2(ik, lc) = b;
    }
    sync();
    // CC(a, b, c) = cc[a + ido*(b + ip*c)] from CH(a, b, c) = ch[a + ido*(b + l1*c)]
    auto CC = [&](int a, int b, int c) -> T& { return cc[a + ido * (b + ip * c)]; };
    auto CH = [&](int a, int b, int c) -> T& { return ch[a + ido * (b + l1 * c)]; };
    for (int it = tid; it < idl1; it += nt) {
        const int k = it / ido, i = it % ido;
        CC(i, 0, k) = CH(i, k, 0);
    }
    for (int it = tid; it < (ipph - 1) * l1; it += nt) {
        const int j = 1 + it / l1, k = it % l1, jc = ip - j, j2 = 2 * j - 1;
        CC(ido - 1, j2, k) = CH(0, k, j);
        CC(0, j2 + 1, k) = CH(0, k, jc);
    }
    if (ido > 1) {
        const int ni = (ido - 1) / 2;
        for (int it = tid; it < (ipph - 1) * l1 * ni; it += nt) {
            const int j = 1 + it / (l1 * ni), rem = it % (l1 * ni), k = rem / ni, q = rem % ni;
            const int i = 1 + 2 * q, ic = ido - i - 2, jc = ip - j, j2 = 2 * j - 1;
            CC(i, j2 + 1, k) = CH(i, k, j) + CH(i, k, jc);
            CC(ic, j2, k) = CH(i, k, j) - CH(i, k, jc);
            CC(i + 1, j2 + 1, k) = CH(i + 1, k, j) + CH(i + 1, k, jc);
            CC(ic + 1, j2, k) = CH(i + 1, k, jc) - CH(i + 1, k, j);
        }
    }
}

// rfftp::exec r2hc (fct = 1): p1 holds the real input; returns the buffer holding the
// halfcomplex result.
template <class T, class Sync>
PF_HD inline T* rfft_run(const Plan& p, const T* tab, T* p1, T* p2, int tid, int nt, Sync sync) {
    const int n = p.n;
    int l1 = n;
    for (int k = p.nf - 1; k >= 0; --k) {
        const int ip = p.fct[k], ido = n / l1;
        l1 /= ip;
        const T* wa = tab + p.tw[k];
        bool swap = true;
        switch (ip) {
            case 4: radf4<T>(ido, l1, p1, p2, wa, tab[kHsqt2], tid, nt); break;
            case 2: radf2<T>(ido, l1, p1, p2, wa, tid, nt); break;
            case 3: radf3<T>(ido, l1, p1, p2, wa, tab + const_off(3), tid, nt); break;
            case 5: radf5<T>(ido, l1, p1, p2, wa, tab + const_off(5), tid, nt); break;
            default:
                radfg<T>(ido, ip, l1, p1, p2, wa, tab + p.tws[k], tid, nt, sync);
                swap = false;
        }
        sync();
        if (swap) {
            T* t = p1;
            p1 = p2;
            p2 = t;
        }
    }
    return p1;
}

// fftblue::fft<fwd> (fct = 1) on A[0..n) with B as the second buffer of n2; result in A.
template <class T, bool FWD, class Sync>
PF_HD inline void blue_fft(const Plan& p, const T* tab, cx<T>* A, cx<T>* B, int tid, int nt, Sync sync) {
    const int n = p.n, n2 = p.n2;
    const cx<T>* bk = reinterpret_cast<const cx<T>*>(tab + p.bk);
    const cx<T>* bkf = reinterpret_cast<const cx<T>*>(tab + p.bkf);
    for (int m = tid; m < n; m += nt) A[m] = smul<FWD>(A[m], bk[m]);
    sync();
    const cx<T> zero = mk<T>(A[0].r * T(0), A[0].i * T(0));  // akf[0] * T0(0)
    for (int m = n + tid; m < n2; m += nt) A[m] = zero;
    sync();
    cx<T>* R = cfft_run<T, true>(p, tab, A, B, tid, nt, sync);
    for (int m = tid; m < n2; m += nt) R[m] = smul<!FWD>(R[m], bkf[m <= n2 / 2 ? m : n2 - m]);
    sync();
    cx<T>* S = cfft_run<T, false>(p, tab, R, R == A ? B : A, tid, nt, sync);
    for (int m = tid; m < n; m += nt) A[m] = smul<FWD>(S[m], bk[m]);
    sync();
}

// numpy's pairwise_sum (loops_utils.h): < 8 elements in order from 0; <= 128 with 8
// accumulators combined ((0+1)+(2+3))+((4+5)+(6+7)) and the rest in order; larger
// blocks split at n/2 rounded down to a multiple of 8.
template <class T, int D = 8>
PF_HD inline T pairwise_sum(const T* a, long n) {
    if (n < 8) {
        T res = T(0);
        for (long i = 0; i < n; ++i) res = res + a[i];
        return res;
    }
    if (n <= 128 || D == 0) {
        T r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        long i = 8;
        for (; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] = r[j] + a[i + j];
        T res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res = res + a[i];
        return res;
    }
    if constexpr (D > 0) {
        long n2 = n / 2;
        n2 -= n2 % 8;
        return pairwise_sum<T, D - 1>(a, n2) + pairwise_sum<T, D - 1>(a + n2, n - n2);
    }
    return T(0);
}

// ================================================================== host: plans
// (host functions: std::vector, glibc sincos)
// sincos_2pibyn<T>(n): two tables of exp(2 pi i x / n) (double, octant-reduced, through
// glibc's sincos like the library's compiled calc()), their product rounded to T.
struct SinCos2PiByN {
    size_t N, mask, shift;
    std::vector<double> v1, v2;  // (re, im) pairs
    static void calc(size_t x, size_t n, double ang, double* out) {
        double s, c;
        x <<= 3;
        if (x < 4 * n) {
            if (x < 2 * n) {
                if (x < n) {
                    ::sincos(double(x) * ang, &s, &c);
                    out[0] = c;
                    out[1] = s;
                    return;
                }
                ::sincos(double(2 * n - x) * ang, &s, &c);
                out[0] = s;
                out[1] = c;
                return;
            }
            x -= 2 * n;
            if (x < n) {
                ::sincos(double(x) * ang, &s, &c);
                out[0] = -s;
                out[1] = c;
                return;
            }
            ::sincos(double(2 * n - x) * ang, &s, &c);
            out[0] = -c;
            out[1] = s;
            return;
        }
        x = 8 * n - x;
        if (x < 2 * n) {
            if (x < n) {
                ::sincos(double(x) * ang, &s, &c);
                out[0] = c;
                out[1] = -s;
                return;
            }
            ::sincos(double(2 * n - x) * ang, &s, &c);
            out[0] = s;
            out[1] = -c;
            return;
        }
        x -= 2 * n;
        if (x < n) {
            ::sincos(double(x) * ang, &s, &c);
            out[0] = -s;
            out[1] = -c;
            return;
        }
        ::sincos(double(2 * n - x) * ang, &s, &c);
        out[0] = -c;
        out[1] = -s;
    }
    explicit SinCos2PiByN(size_t n) : N(n) {
        constexpr long double pi = 3.141592653589793238462643383279502884197L;
        const double ang = double(0.25L * pi / n);
        const size_t nval = (n + 2) / 2;
        shift = 1;
        while ((size_t(1) << shift) * (size_t(1) << shift) < nval) ++shift;
        mask = (size_t(1) << shift) - 1;
        v1.assign(2 * (mask + 1), 0.0);
        v1[0] = 1.0;
        for (size_t i = 1; i <= mask; ++i) calc(i, n, ang, &v1[2 * i]);
        const size_t n2 = (nval + mask) / (mask + 1);
        v2.assign(2 * n2, 0.0);
        v2[0] = 1.0;
        for (size_t i = 1; i < n2; ++i) calc(i * (mask + 1), n, ang, &v2[2 * i]);
    }
    template <class T>
    cx<T> at(size_t idx) const {
        const bool upper = 2 * idx > N;
        if (upper) idx = N - idx;
        const double* x1 = &v1[2 * (idx & mask)];
        const double* x2 = &v2[2 * (idx >> shift)];
        const T re = T(x1[0] * x2[0] - x1[1] * x2[1]);
        const T im = T(x1[0] * x2[1] + x1[1] * x2[0]);
        return mk<T>(re, upper ? -im : im);
    }
};

inline size_t largest_prime_factor(size_t n) {
    size_t res = 1;
    while ((n & 1) == 0) {
        res = 2;
        n >>= 1;
    }
    for (size_t x = 3; x * x <= n; x += 2)
        while (n % x == 0) {
            res = x;
            n /= x;
        }
    if (n > 1) res = n;
    return res;
}

inline double cost_guess(size_t n) {
    constexpr double lfp = 1.1;
    const size_t ni = n;
    double result = 0.;
    while ((n & 1) == 0) {
        result += 2;
        n >>= 1;
    }
    for (size_t x = 3; x * x <= n; x += 2)
        while (n % x == 0) {
            result += (x <= 5) ? double(x) : lfp * double(x);
            n /= x;
        }
    if (n > 1) result += (n <= 5) ? double(n) : lfp * double(n);
    return result * double(ni);
}

inline size_t good_size_cmplx(size_t n) {  // smallest 2^a 3^b 5^c 7^d 11^e >= n
    if (n <= 12) return n;
    for (size_t m = n;; ++m) {
        size_t k = m;
        for (size_t p : {2, 3, 5, 7, 11})
            while (k % p == 0) k /= p;
        if (k == 1) return m;
    }
}

inline bool use_bluestein(size_t n, bool real) {
    const size_t tmp = (n < 50) ? 0 : largest_prime_factor(n);
    if (tmp * tmp <= n) return false;
    const double comp1 = (real ? 0.5 : 1.0) * cost_guess(n);
    double comp2 = 2 * cost_guess(good_size_cmplx(2 * n - 1));
    comp2 *= 1.5;
    return comp2 < comp1;
}

inline std::vector<int> factors(int n, bool real) {
    std::vector<int> f;
    int len = n;
    if (!real)
        while ((len & 7) == 0) {
            f.push_back(8);
            len >>= 3;
        }
    while ((len & 3) == 0) {
        f.push_back(4);
        len >>= 2;
    }
    if ((len & 1) == 0) {
        len >>= 1;
        f.push_back(2);
        std::swap(f.front(), f.back());
    }
    for (int d = 3; d * d <= len; d += 2)
        while (len % d == 0) {
            f.push_back(d);
            len /= d;
        }
    if (len > 1) f.push_back(len);
    return f;
}

// the literals of pocketfft's pass3 / 5 / 7 / 11 (T0(<long double literal>)) and hsqt2
template <class T>
inline void pass_constants(std::vector<T>& tab) {
    const long double c[22] = {
        -0.5L, 0.8660254037844386467637231707529362L,                                                      // 3
        0.3090169943749474241022934171828191L, 0.9510565162951535721164393333793821L,                       // 5
        -0.8090169943749474241022934171828191L, 0.5877852522924731291687059546390728L,
        0.6234898018587335305250048840042398L, 0.7818314824680298087084445266740578L,                       // 7
        -0.2225209339563144042889025644967948L, 0.9749279121818236070181316829939312L,
        -0.9009688679024191262361023195074451L, 0.4338837391175581204757683328483587L,
        0.8412535328311811688618116489193677L, 0.5406408174555975821076359543186917L,                       // 11
        0.4154150130018864255292741492296232L, 0.9096319953545183714117153830790285L,
        -0.1423148382732851404437926686163697L, 0.9898214418809327323760920377767188L,
        -0.6548607339452850640569250724662936L, 0.7557495743542582837740358439723444L,
        -0.9594929736144973898903680570663277L, 0.2817325568414296977114179153466169L};
    tab.assign(kConsts, T(0));
    tab[kHsqt2] = T(0.707106781186547524400844362104849L);
    for (int j = 0; j < 22; ++j) tab[1 + j] = T(c[j]);
}

template <class T>
inline void append_cfftp(Plan& p, int L, std::vector<T>& tab) {
    const std::vector<int> f = factors(L, false);
    if ((int)f.size() > kMaxFact) throw std::runtime_error("pocketfft plan: too many factors");
    p.nf = (int)f.size();
    SinCos2PiByN comp(L);
    long l1 = 1;
    for (int k = 0; k < p.nf; ++k) {
        const int ip = f[k];
        const long ido = L / (l1 * ip);
        p.fct[k] = ip;
        p.tw[k] = (int)tab.size();
        tab.resize(tab.size() + 2 * (size_t)std::max<long>((ip - 1) * (ido - 1), 1), T(0));
        cx<T>* tw = reinterpret_cast<cx<T>*>(tab.data() + p.tw[k]);
        for (int j = 1; j < ip; ++j)
            for (long i = 1; i < ido; ++i) tw[(j - 1) * (ido - 1) + i - 1] = comp.at<T>((size_t)j * l1 * i);
        p.tws[k] = -1;
        if (ip > 11) {
            p.tws[k] = (int)tab.size();
            tab.resize(tab.size() + 2 * (size_t)ip, T(0));
            cx<T>* ts = reinterpret_cast<cx<T>*>(tab.data() + p.tws[k]);
            for (int j = 0; j < ip; ++j) ts[j] = comp.at<T>((size_t)j * l1 * ido);
        }
        l1 *= ip;
    }
}

template <class T>
inline void append_rfftp(Plan& p, int n, std::vector<T>& tab) {
    const std::vector<int> f = factors(n, true);
    if ((int)f.size() > kMaxFact) throw std::runtime_error("pocketfft plan: too many factors");
    p.nf = (int)f.size();
    SinCos2PiByN twid(n);
    long l1 = 1;
    for (int k = 0; k < p.nf; ++k) {
        const int ip = f[k];
        const long ido = n / (l1 * ip);
        p.fct[k] = ip;
        p.tw[k] = (int)tab.size();
        tab.resize(tab.size() + (size_t)std::max<long>((ip - 1) * (ido - 1), 1), T(0));
        if (k < p.nf - 1)
            for (int j = 1; j < ip; ++j)
                for (long i = 1; i <= (ido - 1) / 2; ++i) {
                    const cx<T> w = twid.at<T>((size_t)j * l1 * i);
                    tab[p.tw[k] + (j - 1) * (ido - 1) + 2 * i - 2] = w.r;
                    tab[p.tw[k] + (j - 1) * (ido - 1) + 2 * i - 1] = w.i;
                }
        p.tws[k] = -1;
        if (ip > 5) {
            p.tws[k] = (int)tab.size();
            tab.resize(tab.size() + 2 * (size_t)ip, T(0));
            T* cs = tab.data() + p.tws[k];
            cs[0] = T(1);
            cs[1] = T(0);
            for (int i = 2, ic = 2 * ip - 2; i <= ic; i += 2, ic -= 2) {
                const cx<T> w = twid.at<T>((size_t)(i / 2) * (n / ip));
                cs[i] = w.r;
                cs[i + 1] = w.i;
                cs[ic] = w.r;
                cs[ic + 1] = -w.i;
            }
        }
        l1 *= ip;
    }
}

struct NoSync {
    void operator()() const {}
};

// pocketfft_r (real = true: the rows' r2c) / pocketfft_c (the columns' c2c) plan of length n
// in T; tab receives the constants and every table the plan's offsets refer to.
template <class T>
inline Plan make_plan(int n, bool real, std::vector<T>& tab) {
    if (n < 1) throw std::runtime_error("pocketfft plan: bad length");
    Plan p{};
    p.n = n;
    p.real = real ? 1 : 0;
    pass_constants(tab);
    if (!use_bluestein((size_t)n, real)) {
        if (real) append_rfftp(p, n, tab);
        else append_cfftp(p, n, tab);
        for (int k = p.nf; k < kMaxFact; ++k) p.tws[k] = -1;
        return p;
    }
    // fftblue<T0>(n)
    p.blue = 1;
    p.n2 = (int)good_size_cmplx(2 * (size_t)n - 1);
    append_cfftp(p, p.n2, tab);
    SinCos2PiByN tmp(2 * (size_t)n);
    p.bk = (int)tab.size();
    tab.resize(tab.size() + 2 * (size_t)n, T(0));
    {
        cx<T>* bk = reinterpret_cast<cx<T>*>(tab.data() + p.bk);
        bk[0] = mk<T>(T(1), T(0));
        size_t coeff = 0;
        for (int m = 1; m < n; ++m) {
            coeff += 2 * (size_t)m - 1;
            if (coeff >= 2 * (size_t)n) coeff -= 2 * (size_t)n;
            bk[m] = tmp.at<T>(coeff);
        }
    }
    // FFT of the zero-padded b_k / n2 (the host runs the same passes as the device)
    std::vector<cx<T>> tb(p.n2, mk<T>(T(0), T(0))), sc(p.n2);
    {
        const cx<T>* bk = reinterpret_cast<const cx<T>*>(tab.data() + p.bk);
        const T xn2 = T(1) / T(p.n2);
        tb[0] = mk<T>(bk[0].r * xn2, bk[0].i * xn2);
        for (int m = 1; m < n; ++m) tb[m] = tb[p.n2 - m] = mk<T>(bk[m].r * xn2, bk[m].i * xn2);
    }
    const cx<T>* res = cfft_run<T, true>(p, tab.data(), tb.data(), sc.data(), 0, 1, NoSync{});
    p.bkf = (int)tab.size();
    tab.resize(tab.size() + 2 * (size_t)(p.n2 / 2 + 1), T(0));
    cx<T>* bkf = reinterpret_cast<cx<T>*>(tab.data() + p.bkf);
    for (int i = 0; i < p.n2 / 2 + 1; ++i) bkf[i] = res[i];
    for (int k = p.nf; k < kMaxFact; ++k) p.tws[k] = -1;
    return p;
}

// Host runs of the device code (tests/native/host_logic_test.cpp): r2c of one row into
// bins 0..n/2 and the forward c2c of one column (in place).
template <class T>
inline void host_r2c(const Plan& p, const std::vector<T>& tab, const T* x, cx<T>* out) {
    const int n = p.n;
    if (!p.blue) {
        std::vector<T> a(x, x + n), b(n);
        const T* r = rfft_run<T>(p, tab.data(), a.data(), b.data(), 0, 1, NoSync{});
        out[0] = mk<T>(r[0], T(0));
        for (int m = 1; m < (n + 1) / 2; ++m) out[m] = mk<T>(r[2 * m - 1], r[2 * m]);
        if (n % 2 == 0) out[n / 2] = mk<T>(r[n - 1], T(0));
        return;
    }
    std::vector<cx<T>> A(p.n2), B(p.n2);
    for (int m = 0; m < n; ++m) A[m] = mk<T>(x[m], T(0) * x[0]);
    blue_fft<T, true>(p, tab.data(), A.data(), B.data(), 0, 1, NoSync{});
    out[0] = mk<T>(A[0].r, T(0));
    for (int m = 1; m < (n + 1) / 2; ++m) out[m] = A[m];
    if (n % 2 == 0) out[n / 2] = mk<T>(A[n / 2].r, T(0));
}

template <class T>
inline void host_c2c(const Plan& p, const std::vector<T>& tab, cx<T>* c) {
    const int n = p.n;
    std::vector<cx<T>> A(p.blue ? p.n2 : n), B(p.blue ? p.n2 : n);
    for (int m = 0; m < n; ++m) A[m] = c[m];
    const cx<T>* r = A.data();
    if (p.blue) blue_fft<T, true>(p, tab.data(), A.data(), B.data(), 0, 1, NoSync{});
    else r = cfft_run<T, true>(p, tab.data(), A.data(), B.data(), 0, 1, NoSync{});
    for (int m = 0; m < n; ++m) c[m] = r[m];
}

}  // namespace pf
