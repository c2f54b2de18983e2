// Group FFT for gfx950: a B-point complex FFT held by G = B/16 lanes of ONE
// wave, 16 complex values per lane, radix-16 first pass, so B <= 256 needs at
// most one exchange (B = 128: 16 x 8, B = 256: 16 x 16).  Several groups share
// a wave (64/G of them) and exchange through their own padded LDS regions with
// wave-level synchronisation only: no workgroup barrier inside a transform.
//
// Layout ("natural strided"): lane t of the group holds element t + G*q in
// slot q, both on input and on output (Stockham autosort), which is what
// coalesced loads/stores produce when consecutive groups/lanes cover
// consecutive addresses.
//
// Per-lane twiddles of the passes after the first depend only on the lane,
// so a kernel that runs many transforms loads them once into registers.
#pragma once
#include <hip/hip_runtime.h>

#include "fft_lds.hpp"
#include "regfft.hpp"

namespace fcdk {

template <int B>
struct GSched {
    static_assert(B >= 16 && (B & (B - 1)) == 0, "group FFT length must be a power of two >= 16");
    static constexpr int E = 16;
    static constexpr int G = B / E;  // lanes per transform
    static constexpr int radix(int p) {
        int L = 1;
        for (int i = 0; i < p; ++i) L *= (B / L >= E ? E : B / L);
        return B / L >= E ? E : B / L;
    }
    static constexpr int ell(int p) {
        int L = 1;
        for (int i = 0; i < p; ++i) L *= radix(i);
        return L;
    }
    static constexpr int npass() {
        int p = 0, L = 1;
        while (L < B) {
            L *= radix(p);
            ++p;
        }
        return p;
    }
    static constexpr int NP = npass();
    // offset of pass p's twiddles in the pass-major table: sum over passes 1..p-1 of ell*(radix-1)
    static constexpr int passoff(int p) {
        int o = 0;
        for (int i = 1; i < p; ++i) o += ell(i) * (radix(i) - 1);
        return o;
    }
    static constexpr int TABLE = passoff(NP);  // table entries (complex)
    // per-lane register twiddles: sum over passes >= 1 of (E/radix)*(radix-1)
    static constexpr int nreg() {
        int o = 0;
        for (int i = 1; i < NP; ++i) o += (E / radix(i)) * (radix(i) - 1);
        return o;
    }
    static constexpr int NREG = nreg();
    static constexpr int REGOFF(int p) {
        int o = 0;
        for (int i = 1; i < p; ++i) o += (E / radix(i)) * (radix(i) - 1);
        return o;
    }
    // padded LDS region of one transform; pad() keeps the radix-16 write
    // (16t + r) and the strided read (t + G q) conflict-free
    static constexpr int REGION = padded_len(B) > 16 ? padded_len(B) : 16;
};

template <int B>
struct GroupFFT {
    using S = GSched<B>;
    static constexpr int E = S::E, G = S::G, NP = S::NP;
    float2 tw[S::NREG > 0 ? S::NREG : 1];

    // table: pass-major forward twiddles exp(-2 pi i r k / (L_p R_p)), k < L_p, r = 1..R_p-1
    __device__ __forceinline__ void load(const float2* __restrict__ table, int t) {
        load_pass<1>(table, t);
    }
    template <int P>
    __device__ __forceinline__ void load_pass(const float2* __restrict__ table, int t) {
        if constexpr (P < NP) {
            constexpr int R = S::radix(P), L = S::ell(P), BPT = E / R;
#pragma unroll
            for (int b = 0; b < BPT; ++b) {
                const int k = (t + b * G) & (L - 1);
#pragma unroll
                for (int r = 1; r < R; ++r)
                    tw[S::REGOFF(P) + b * (R - 1) + r - 1] = table[S::passoff(P) + k * (R - 1) + r - 1];
            }
            load_pass<P + 1>(table, t);
        }
    }

    // x: natural strided in and out; s: this transform's LDS region.
    template <bool INV>
    __device__ __forceinline__ void run(float2 (&x)[E], float2* s, int t) const {
        pass<0, INV>(x, s, t);
    }

    // The same with the exchange through a FLOAT region of REGION entries (real
    // parts, then imaginary parts): half the LDS per transform for two more
    // wave syncs, so more workgroups fit a CU.
    template <bool INV>
    __device__ __forceinline__ void run_half(float2 (&x)[E], float* s, int t) const {
        pass_half<0, INV>(x, s, t);
    }

    template <int P, bool INV>
    __device__ __forceinline__ void pass_half(float2 (&x)[E], float* s, int t) const {
        constexpr int R = S::radix(P), L = S::ell(P), BPT = E / R;
        float2 a[BPT][R];
#pragma unroll
        for (int b = 0; b < BPT; ++b) {
#pragma unroll
            for (int r = 0; r < R; ++r) a[b][r] = x[b + BPT * r];
            if constexpr (P > 0) {
#pragma unroll
                for (int r = 1; r < R; ++r) {
                    const float2 w = tw[S::REGOFF(P) + b * (R - 1) + r - 1];
                    a[b][r] = cmul_dir<INV>(a[b][r], w);
                }
            }
            dft_reg<R, INV>(a[b]);
        }
        if constexpr (P + 1 == NP) {
#pragma unroll
            for (int b = 0; b < BPT; ++b)
#pragma unroll
                for (int r = 0; r < R; ++r) x[b + BPT * r] = a[b][r];
        } else {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                wave_sync();
#pragma unroll
                for (int b = 0; b < BPT; ++b) {
                    const int j = t + b * G;
                    const int k = j & (L - 1);
                    const int base = (j - k) * R + k;
#pragma unroll
                    for (int r = 0; r < R; ++r) s[pad(base + r * L)] = h ? a[b][r].y : a[b][r].x;
                }
                wave_sync();
#pragma unroll
                for (int q = 0; q < E; ++q) {
                    const float v = s[pad(t + G * q)];
                    if (h) x[q].y = v; else x[q].x = v;
                }
            }
            pass_half<P + 1, INV>(x, s, t);
        }
    }

    template <int P, bool INV>
    __device__ __forceinline__ void pass(float2 (&x)[E], float2* s, int t) const {
        constexpr int R = S::radix(P), L = S::ell(P), BPT = E / R;
        float2 a[BPT][R];
#pragma unroll
        for (int b = 0; b < BPT; ++b) {
#pragma unroll
            for (int r = 0; r < R; ++r) a[b][r] = x[b + BPT * r];
            if constexpr (P > 0) {
#pragma unroll
                for (int r = 1; r < R; ++r) {
                    const float2 w = tw[S::REGOFF(P) + b * (R - 1) + r - 1];
                    a[b][r] = cmul_dir<INV>(a[b][r], w);
                }
            }
            dft_reg<R, INV>(a[b]);
        }
        if constexpr (P + 1 == NP) {
#pragma unroll
            for (int b = 0; b < BPT; ++b)
#pragma unroll
                for (int r = 0; r < R; ++r) x[b + BPT * r] = a[b][r];
        } else {
            wave_sync();  // earlier readers of s (previous transform) are done
#pragma unroll
            for (int b = 0; b < BPT; ++b) {
                const int j = t + b * G;
                const int k = j & (L - 1);
                const int base = (j - k) * R + k;
#pragma unroll
                for (int r = 0; r < R; ++r) s[pad(base + r * L)] = a[b][r];
            }
            wave_sync();
#pragma unroll
            for (int q = 0; q < E; ++q) x[q] = s[pad(t + G * q)];
            pass<P + 1, INV>(x, s, t);
        }
    }
};

// The same transform with the pass twiddles read from a table (typically in
// LDS: GSched<B>::TABLE entries, pass-major as GroupFFT::load expects) instead
// of per-lane registers: for long transforms whose register twiddles would
// cost too many VGPRs (B = 1024: 27 complex per lane).
template <int B>
struct GroupFFTTab {
    using S = GSched<B>;
    static constexpr int E = S::E, G = S::G, NP = S::NP;

    template <bool INV>
    __device__ __forceinline__ static void run(float2 (&x)[E], float2* s, int t, const float2* tab) {
        pass<0, INV>(x, s, t, tab);
    }

    template <int P, bool INV>
    __device__ __forceinline__ static void pass(float2 (&x)[E], float2* s, int t, const float2* tab) {
        constexpr int R = S::radix(P), L = S::ell(P), BPT = E / R;
        float2 a[BPT][R];
#pragma unroll
        for (int b = 0; b < BPT; ++b) {
#pragma unroll
            for (int r = 0; r < R; ++r) a[b][r] = x[b + BPT * r];
            if constexpr (P > 0) {
                const int k = (t + b * G) & (L - 1);
                const float2* tk = tab + S::passoff(P) + k * (R - 1) - 1;
#pragma unroll
                for (int r = 1; r < R; ++r) {
                    const float2 w = tk[r];
                    a[b][r] = cmul_dir<INV>(a[b][r], w);
                }
            }
            dft_reg<R, INV>(a[b]);
        }
        if constexpr (P + 1 == NP) {
#pragma unroll
            for (int b = 0; b < BPT; ++b)
#pragma unroll
                for (int r = 0; r < R; ++r) x[b + BPT * r] = a[b][r];
        } else {
            wave_sync();
#pragma unroll
            for (int b = 0; b < BPT; ++b) {
                const int j = t + b * G;
                const int k = j & (L - 1);
                const int base = (j - k) * R + k;
#pragma unroll
                for (int r = 0; r < R; ++r) s[pad(base + r * L)] = a[b][r];
            }
            wave_sync();
#pragma unroll
            for (int q = 0; q < E; ++q) x[q] = s[pad(t + G * q)];
            pass<P + 1, INV>(x, s, t, tab);
        }
    }

    // float-half exchange (GroupFFT::run_half) with the table twiddles: the folded 256-point
    // band transforms of the 4096-point fused kernel, one carrier at a time
    template <bool INV>
    __device__ __forceinline__ static void run_half(float2 (&x)[E], float* s, int t, const float2* tab) {
        pass_half<0, INV>(x, s, t, tab);
    }

    template <int P, bool INV>
    __device__ __forceinline__ static void pass_half(float2 (&x)[E], float* s, int t, const float2* tab) {
        constexpr int R = S::radix(P), L = S::ell(P), BPT = E / R;
        float2 a[BPT][R];
#pragma unroll
        for (int b = 0; b < BPT; ++b) {
#pragma unroll
            for (int r = 0; r < R; ++r) a[b][r] = x[b + BPT * r];
            if constexpr (P > 0) {
                const int k = (t + b * G) & (L - 1);
                const float2* tk = tab + S::passoff(P) + k * (R - 1) - 1;
#pragma unroll
                for (int r = 1; r < R; ++r) a[b][r] = cmul_dir<INV>(a[b][r], tk[r]);
            }
            dft_reg<R, INV>(a[b]);
        }
        if constexpr (P + 1 == NP) {
#pragma unroll
            for (int b = 0; b < BPT; ++b)
#pragma unroll
                for (int r = 0; r < R; ++r) x[b + BPT * r] = a[b][r];
        } else {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                wave_sync();
#pragma unroll
                for (int b = 0; b < BPT; ++b) {
                    const int j = t + b * G;
                    const int k = j & (L - 1);
                    const int base = (j - k) * R + k;
#pragma unroll
                    for (int r = 0; r < R; ++r) s[pad(base + r * L)] = h ? a[b][r].y : a[b][r].x;
                }
                wave_sync();
#pragma unroll
                for (int q = 0; q < E; ++q) {
                    const float v = s[pad(t + G * q)];
                    if (h) x[q].y = v; else x[q].x = v;
                }
            }
            pass_half<P + 1, INV>(x, s, t, tab);
        }
    }
};

// Two independent transforms of the same length advanced in lockstep (the two
// carriers of one row in the fused kernel): each pass's twiddles are read once
// for both, and both transforms' values cross the float-half exchange between
// the same pair of wave syncs, so one transform's LDS round trip hides behind
// the other's arithmetic.  s0 / s1: two FLOAT regions of GSched<B>::REGION.
template <int B>
struct GroupFFTTab2 {
    using S = GSched<B>;
    static constexpr int E = S::E, G = S::G, NP = S::NP;

    template <bool INV>
    __device__ __forceinline__ static void run_half(float2 (&x0)[E], float2 (&x1)[E], float* s0, float* s1, int t,
                                                    const float2* tab) {
        pass<0, INV>(x0, x1, s0, s1, t, tab);
    }

    template <int P, bool INV>
    __device__ __forceinline__ static void pass(float2 (&x0)[E], float2 (&x1)[E], float* s0, float* s1, int t,
                                                const float2* tab) {
        constexpr int R = S::radix(P), L = S::ell(P), BPT = E / R;
        float2 a0[BPT][R], a1[BPT][R];
#pragma unroll
        for (int b = 0; b < BPT; ++b) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                a0[b][r] = x0[b + BPT * r];
                a1[b][r] = x1[b + BPT * r];
            }
            if constexpr (P > 0) {
                const int k = (t + b * G) & (L - 1);
                const float2* tk = tab + S::passoff(P) + k * (R - 1) - 1;
#pragma unroll
                for (int r = 1; r < R; ++r) {
                    const float2 w = tk[r];
                    a0[b][r] = cmul_dir<INV>(a0[b][r], w);
                    a1[b][r] = cmul_dir<INV>(a1[b][r], w);
                }
            }
            dft_reg<R, INV>(a0[b]);
            dft_reg<R, INV>(a1[b]);
        }
        if constexpr (P + 1 == NP) {
#pragma unroll
            for (int b = 0; b < BPT; ++b)
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    x0[b + BPT * r] = a0[b][r];
                    x1[b + BPT * r] = a1[b][r];
                }
        } else {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                wave_sync();
#pragma unroll
                for (int b = 0; b < BPT; ++b) {
                    const int j = t + b * G;
                    const int k = j & (L - 1);
                    const int base = (j - k) * R + k;
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        s0[pad(base + r * L)] = h ? a0[b][r].y : a0[b][r].x;
                        s1[pad(base + r * L)] = h ? a1[b][r].y : a1[b][r].x;
                    }
                }
                wave_sync();
#pragma unroll
                for (int q = 0; q < E; ++q) {
                    const float v0 = s0[pad(t + G * q)], v1 = s1[pad(t + G * q)];
                    if (h) {
                        x0[q].y = v0;
                        x1[q].y = v1;
                    } else {
                        x0[q].x = v0;
                        x1[q].x = v1;
                    }
                }
            }
            pass<P + 1, INV>(x0, x1, s0, s1, t, tab);
        }
    }
};

// atan(r) = r P(r^2) on [0, 1]: minimax-fit polynomials of FCD_ATAN_TERMS terms
// (highest order first).  Max |error| evaluated in f32: 9 terms 1.0e-7 rad, 8
// terms 1.4e-7, 7 terms 3.2e-7 (tools/atan_fit.py; in f64 the fits themselves are
// 5.8e-9 / 3.7e-8 / 2.5e-7).  8 by default: one packed FMA per pixel pair less
// than 9 at the same f32 error.  7 terms (two less, band kernel 3.17 -> 3.05
// us/frame, kbench r02c8) leave the wrapped phases' tail error against the f64
// oracle unchanged (99.99th percentile 2.7e-6 rad, tools/atan_accuracy.py) but
// their systematic error integrates into the 4096^2 no-unwrap height: rel-L2
// 1.13e-5 against the 1e-5 bound (test_full_size_4096_properties, r02c9).
#ifndef FCD_ATAN_TERMS
#define FCD_ATAN_TERMS 8
#endif
constexpr int kAtanN = FCD_ATAN_TERMS;
__host__ __device__ constexpr float atan_coef(int i) {
    constexpr float C9[9] = {0.0024567286018282175f, -0.014401371590793133f, 0.03978124260902405f,
                             -0.07234858721494675f,  0.10498946160078049f,   -0.14161229133605957f,
                             0.19985906779766083f,   -0.33332598209381104f,  0.9999998807907104f};
    constexpr float C8[8] = {-0.004054554738104343f, 0.02186291478574276f,  -0.05591226741671562f,
                             0.09642193466424942f,   -0.1390862762928009f,  0.19946564733982086f,
                             -0.33329859375953674f,  0.9999993443489075f};
    constexpr float C7[7] = {0.006811772007495165f, -0.033604156225919724f, 0.07962360233068466f,
                             -0.13233338296413422f, 0.19807814061641693f,   -0.3331736922264099f,
                             0.9999961256980896f};
    return kAtanN == 9 ? C9[i] : (kAtanN == 8 ? C8[i] : C7[i]);
}
static_assert(kAtanN >= 7 && kAtanN <= 9, "FCD_ATAN_TERMS: 7, 8 or 9");

// Reduction of atan2, the quadrant form: r = (|y| - |x|) / (|y| + |x|) in [-1, 1], the
// first-quadrant angle pi/4 + r P(r^2) (the same odd polynomial: atan is odd, so the fit
// on [0, 1] holds on [-1, 1]), then pi - a where x < 0.  Against the octant form (r =
// min / max in [0, 1], then pi/2 - a where |y| > |x| and pi - a where x < 0) one compare /
// select pair less, and the zero guard is the legacy multiply (0 * rcp(0) = 0) instead of
// a clamp of the divisor.  Same f32 error (max 3.3e-7 vs 3.2e-7 rad, rms 7.8e-8 either
// way, over 4 M random angles at magnitudes e^-20 .. e^20); atan2(0, 0) = pi/4 instead of
// 0, which no phase path depends on: theta and the frame phases use the same form, so a
// frame equal to the reference still gives exactly 0.  (Fused 1024 kernel 5.87 -> 5.82
// us/frame, r03s.)
// v_mul_legacy_f32: 0 * x = 0 for every x, inf and NaN included (no clang builtin)
extern "C" __device__ float fmul_legacy(float, float) __asm("llvm.amdgcn.fmul.legacy");

// atan2(y, x) in f32 (atan_coef after the quadrant reduction, v_rcp_f32 division).
// About 20 VALU operations.
__device__ __forceinline__ float fast_atan2(float y, float x) {
    const float r = fmul_legacy(fabsf(y) - fabsf(x), __builtin_amdgcn_rcpf(fabsf(y) + fabsf(x)));
    const float s = r * r;
    float p = atan_coef(0);
#pragma unroll
    for (int c = 1; c < kAtanN; ++c) p = fmaf(p, s, atan_coef(c));
    float a = fmaf(r, p, 0.785398163397448310f);
    a = x < 0.f ? 3.14159265358979324f - a : a;
    return copysignf(a, y);
}

// fast_atan2 of two values at once: the reduction's square, polynomial and final
// product run as packed-FP32 ops (v_pk_mul / v_pk_fma: both values per instruction), the
// quadrant fix-ups per value.  Same polynomial and operation order as fast_atan2 per
// value.
__device__ __forceinline__ fv2 fast_atan2_pk(fv2 y, fv2 x) {
    const fv2 r = {fmul_legacy(fabsf(y.x) - fabsf(x.x), __builtin_amdgcn_rcpf(fabsf(y.x) + fabsf(x.x))),
                   fmul_legacy(fabsf(y.y) - fabsf(x.y), __builtin_amdgcn_rcpf(fabsf(y.y) + fabsf(x.y)))};
    const fv2 s = r * r;
    fv2 p = fv2{atan_coef(0), atan_coef(0)};
#pragma unroll
    for (int c = 1; c < kAtanN; ++c) p = p * s + atan_coef(c);
    fv2 a = r * p + 0.785398163397448310f;
    a.x = x.x < 0.f ? 3.14159265358979324f - a.x : a.x;
    a.y = x.y < 0.f ? 3.14159265358979324f - a.y : a.y;
    return fv2{copysignf(a.x, y.x), copysignf(a.y, y.y)};
}

// wrap(theta - atan2(u.y, u.x)) for two pixels (u0, u1): d - 2 pi rint(d / 2 pi),
// |d| < 2 pi, on packed ops (the phase step of fcd.py:118 with the reference
// angle theta of ccsgn).
__device__ __forceinline__ fv2 wrapped_phase_pk(fv2 theta, float2 u0, float2 u1) {
    const fv2 d = theta - fast_atan2_pk(fv2{u0.y, u1.y}, fv2{u0.x, u1.x});
    const fv2 q = d * 0.159154943091895f;
    return fv2{rintf(q.x), rintf(q.y)} * -6.28318530717959f + d;
}

// wrapped_phase_pk for NP pixel pairs at once, written stage by stage so that
// the NP independent chains interleave: back-to-back dependent packed-FP32 ops
// (the Horner steps) and a v_cndmask right behind the v_cmp that writes its mask
// each cost the issuing wave an s_nop on gfx950; NP chains side by side fill
// those slots with the other pairs' work.  Same operations, order and result per
// pixel as wrapped_phase_pk.
template <int NP>
__device__ __forceinline__ void wrapped_phase_pkn(const fv2 (&theta)[NP], const float2 (&u)[2 * NP], fv2 (&out)[NP]) {
    fv2 r[NP], s[NP], p[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        const float2 u0 = u[2 * k], u1 = u[2 * k + 1];
        r[k] = fv2{fmul_legacy(fabsf(u0.y) - fabsf(u0.x), __builtin_amdgcn_rcpf(fabsf(u0.y) + fabsf(u0.x))),
                   fmul_legacy(fabsf(u1.y) - fabsf(u1.x), __builtin_amdgcn_rcpf(fabsf(u1.y) + fabsf(u1.x)))};
    }
#pragma unroll
    for (int k = 0; k < NP; ++k) s[k] = r[k] * r[k];
#pragma unroll
    for (int k = 0; k < NP; ++k) p[k] = s[k] * atan_coef(0) + atan_coef(1);
#pragma unroll
    for (int c = 2; c < kAtanN; ++c)
#pragma unroll
        for (int k = 0; k < NP; ++k) p[k] = p[k] * s[k] + atan_coef(c);
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        const float2 u0 = u[2 * k], u1 = u[2 * k + 1];
        fv2 a = r[k] * p[k] + 0.785398163397448310f;
        a.x = u0.x < 0.f ? 3.14159265358979324f - a.x : a.x;
        a.y = u1.x < 0.f ? 3.14159265358979324f - a.y : a.y;
        const fv2 d = theta[k] - fv2{copysignf(a.x, u0.y), copysignf(a.y, u1.y)};
        const fv2 q = d * 0.159154943091895f;
        out[k] = fv2{rintf(q.x), rintf(q.y)} * -6.28318530717959f + d;
    }
}

}  // namespace fcdk
