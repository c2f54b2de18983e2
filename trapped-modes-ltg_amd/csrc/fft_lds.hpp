// Device FFT core for gfx950: LDS-staged Stockham autosort FFT with
// in-register radix-2/4/8/16 codelets and compile-time radix schedules.
//
// A "team" of TT = N / E threads computes one N-point complex FFT; each thread
// holds E complex values per pass (E = 16 for N >= 1024, so a 1024-point FFT
// is one wave64: radix 16 -> 16 -> 4).  Several teams share a workgroup; the
// workgroup barrier separates passes.  LDS rows are padded by one complex per
// 32 (pad()) so the stride-R writes of the first Stockham pass do not pile on
// one bank (MI355X_MICROARCH.md §LDS: 64 banks, ds_read_b64 in 32-lane groups).
//
// Twiddles come from a per-size global table tw[m] = exp(-2*pi*i*m/N) computed
// on the host in double precision and rounded once to float; tables are a few
// KiB and stay L1/L2-resident across the grid.
#pragma once
#include <hip/hip_runtime.h>

namespace fcdk {

// Complex arithmetic on packed-FP32 VALU ops (v_pk_add/mul/fma_f32: two lanes of work
// per op; on gfx950 a packed op issues at half the rate of a plain one, so this saves
// instructions, not issue time).
typedef float fv2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ fv2 pv(float2 a) { return fv2{a.x, a.y}; }
__device__ __forceinline__ float2 vp(fv2 v) { return make_float2(v.x, v.y); }
// The swaps and sign flips of complex products and of +-i multiplications are
// VOP3P operand modifiers (op_sel / op_sel_hi / neg_lo / neg_hi); the compiler
// does not fold a lane swap into them, so those forms are written out
// (encodings checked on the GPU by tools/pktest.hip).
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return vp(pv(a) + pv(b)); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return vp(pv(a) - pv(b)); }
// a * b
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    fv2 t, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(pv(a)), "v"(pv(b)));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
        : "=v"(r)
        : "v"(pv(a)), "v"(pv(b)), "v"(t));
    return vp(r);
}
// a * conj(b)
__device__ __forceinline__ float2 cmulc(float2 a, float2 b) {
    fv2 t, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1] neg_hi:[0,1]" : "=v"(t) : "v"(pv(a)), "v"(pv(b)));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1]" : "=v"(r) : "v"(pv(a)), "v"(pv(b)), "v"(t));
    return vp(r);
}
// a + i b, a - i b
__device__ __forceinline__ float2 caddi(float2 a, float2 b) {
    fv2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(pv(a)), "v"(pv(b)));
    return vp(r);
}
__device__ __forceinline__ float2 csubi(float2 a, float2 b) {
    fv2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(pv(a)), "v"(pv(b)));
    return vp(r);
}
// i a, -i a
__device__ __forceinline__ float2 cmuli(float2 a) {
    fv2 r;
    asm("v_pk_add_f32 %0, 0, %1 op_sel:[0,1] op_sel_hi:[0,0] neg_lo:[0,1]" : "=v"(r) : "v"(pv(a)));
    return vp(r);
}
__device__ __forceinline__ float2 cmulmi(float2 a) {
    fv2 r;
    asm("v_pk_add_f32 %0, 0, %1 op_sel:[0,1] op_sel_hi:[0,0] neg_hi:[0,1]" : "=v"(r) : "v"(pv(a)));
    return vp(r);
}
// Streaming store: the line is not kept in L2 / the Infinity Cache, so a large
// output stream does not evict the small inputs every frame re-reads.
// A load the compiler cannot move: issued where it stands (ahead of later stores, which
// a plain load's use after them would let the compiler sink it behind), NOT tracked by
// the compiler's wait insertion -- the caller waits with wait_vmcnt<N> before the first
// use, N = the vector-memory operations it issued after the load (vmcnt retires in issue
// order on gfx950, stores included).
__device__ __forceinline__ float2 load_async(const float2* p) {
    fv2 v;
    asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
    return make_float2(v.x, v.y);
}
__device__ __forceinline__ float4 load_async4(const float4* p) {
    float4 v;
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
    return v;
}
// s_waitcnt vmcnt(N), then the registers of v passed through empty volatile asm: the
// values' uses depend on those statements, and volatile asm keeps its order, so no use of
// a load_async result can be scheduled ahead of the wait (a wait with no data link to the
// registers let the compiler hoist a use above it).  N <= 63.
template <int N, int K>
__device__ __forceinline__ void wait_vmcnt_for(float2 (&v)[K]) {
    static_assert(N >= 0 && N <= 63, "vmcnt 0..63");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
#pragma unroll
    for (int i = 0; i < K; ++i) {
        fv2 t = pv(v[i]);
        asm volatile("" : "+v"(t));
        v[i] = vp(t);
    }
}
template <int N, int K>
__device__ __forceinline__ void wait_vmcnt_for(float4 (&v)[K]) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    static_assert(N >= 0 && N <= 63, "vmcnt 0..63");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
#pragma unroll
    for (int i = 0; i < K; ++i) {
        f4 t = {v[i].x, v[i].y, v[i].z, v[i].w};
        asm volatile("" : "+v"(t));
        v[i] = make_float4(t.x, t.y, t.z, t.w);
    }
}

__device__ __forceinline__ void st_stream(float* p, float v) {
    __builtin_nontemporal_store(v, p);
}
__device__ __forceinline__ void st_stream(float2* p, float2 v) {
    __builtin_nontemporal_store(pv(v), reinterpret_cast<fv2*>(p));
}

// a * w (forward) or a * conj(w) (inverse) for a forward twiddle w
template <bool INV>
__device__ __forceinline__ float2 cmul_dir(float2 a, float2 w) {
    return INV ? cmulc(a, w) : cmul(a, w);
}
__device__ __forceinline__ float2 cconj(float2 a) { return make_float2(a.x, -a.y); }
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }

__host__ __device__ constexpr int ilog2c(int n) { return n <= 1 ? 0 : 1 + ilog2c(n / 2); }

// Elements per thread for an N-point transform.
// 8 complex per thread for N >= 512 keeps a register FFT near 70 VGPRs
// (7 waves/SIMD); 16 per thread measured 130+ VGPRs (<= 2 waves/SIMD).
#ifndef FCD_ELEMS_1024
#define FCD_ELEMS_1024 8
#endif
#ifndef FCD_ELEMS_2048
#define FCD_ELEMS_2048 FCD_ELEMS_1024  // 2048- and 4096-point transforms
#endif
__host__ __device__ constexpr int fft_elems(int n) {
    return n >= 2048 ? FCD_ELEMS_2048 : (n >= 1024 ? FCD_ELEMS_1024 : (n >= 512 ? 8 : 4));
}
// Threads per team.
__host__ __device__ constexpr int fft_team(int n) { return n / fft_elems(n); }
// k_int_cols' own count at 1024 points: 16 per lane (wave-local 64-lane teams, so the
// transforms' exchanges need no workgroup barrier) at 2 waves / SIMD, 2.88 -> 2.75
// us/frame (kbench r03zb); elsewhere fft_elems.  Its pass-major twiddle table follows
// (pass_twiddles(n, int_cols_elems(n)) on the host).
#ifndef FCD_INTCOLS_ELEMS_1024
#define FCD_INTCOLS_ELEMS_1024 16
#endif
// and at 2048 / 4096 points (FCD_INTCOLS_ELEMS_WIDE, 0: fft_elems; 16: 256 / 192 VGPRs, no spills)
#ifndef FCD_INTCOLS_ELEMS_WIDE
#define FCD_INTCOLS_ELEMS_WIDE 16  // r03zk: 4096 85.4 -> 80.7, 2048 13.3 -> 12.4 us/frame
#endif
__host__ __device__ constexpr int int_cols_elems(int n) {
    return n == 1024 ? FCD_INTCOLS_ELEMS_1024 : (n >= 2048 && FCD_INTCOLS_ELEMS_WIDE ? FCD_INTCOLS_ELEMS_WIDE : fft_elems(n));
}
// k_demod_cols' count at 1024 points (FCD_DEMODCOLS_ELEMS_1024; its table likewise)
#ifndef FCD_DEMODCOLS_ELEMS_1024
#define FCD_DEMODCOLS_ELEMS_1024 8
#endif
// and at 4096 points (FCD_DEMODCOLS_ELEMS_4096, 0: fft_elems; 16: 180 VGPRs, no spills,
// 14.65 -> 13.1 us/frame; the same at 2048 measured 3.31 -> 4.03, kbench r03dc)
#ifndef FCD_DEMODCOLS_ELEMS_4096
#define FCD_DEMODCOLS_ELEMS_4096 16
#endif
__host__ __device__ constexpr int demod_cols_elems(int n) {
    return n == 1024 ? FCD_DEMODCOLS_ELEMS_1024 : (n == 4096 && FCD_DEMODCOLS_ELEMS_4096 ? FCD_DEMODCOLS_ELEMS_4096 : fft_elems(n));
}
// Padded LDS index: one spare complex per 16.  With this padding every
// exchange pattern of the register FFT (16t + r, t + 64q, base + 16r) is affine
// in the compile-time index (one address register + immediate offsets) and
// conflict-free for ds_*_b64 within each 32-lane group.
__device__ __forceinline__ int pad(int i) { return i + (i >> 4); }
__host__ __device__ constexpr int padded_len(int n) { return n + (n >> 4); }

// cos / sin of 2*pi*m/16, m = 0..15.
__device__ constexpr float kC16[16] = {
    1.0f, 0.923879532511286756f, 0.707106781186547524f, 0.382683432365089772f,
    0.0f, -0.382683432365089772f, -0.707106781186547524f, -0.923879532511286756f,
    -1.0f, -0.923879532511286756f, -0.707106781186547524f, -0.382683432365089772f,
    0.0f, 0.382683432365089772f, 0.707106781186547524f, 0.923879532511286756f};
__device__ constexpr float kS16[16] = {
    0.0f, 0.382683432365089772f, 0.707106781186547524f, 0.923879532511286756f,
    1.0f, 0.923879532511286756f, 0.707106781186547524f, 0.382683432365089772f,
    0.0f, -0.382683432365089772f, -0.707106781186547524f, -0.923879532511286756f,
    -1.0f, -0.923879532511286756f, -0.707106781186547524f, -0.382683432365089772f};

// v * W_R^K with W_R = exp(-2*pi*i/R) (forward) or its conjugate (inverse).
template <int R, int K, bool INV>
__device__ __forceinline__ float2 twc(float2 v) {
    constexpr int m = (K * (16 / R)) & 15;
    if constexpr (m == 0) {
        return v;
    } else if constexpr (m == 4) {
        return INV ? cmuli(v) : cmulmi(v);
    } else if constexpr (m == 8) {
        return make_float2(-v.x, -v.y);
    } else if constexpr (m == 12) {
        return INV ? cmulmi(v) : cmuli(v);
    } else {
        const float c = kC16[m];
        const float s = INV ? kS16[m] : -kS16[m];
        const fv2 V = pv(v);
        return vp(__builtin_elementwise_fma(V.yy, fv2{-s, c}, V.xx * fv2{c, s}));
    }
}

template <int R, int K, bool INV>
__device__ __forceinline__ void dft_combine(float2* a, const float2* e, const float2* o) {
    if constexpr (K < R / 2) {
        constexpr int m = (K * (16 / R)) & 15;
        if constexpr (m == 4 || m == 12) {  // W = -+i: the product folds into the add
            if constexpr ((m == 4) != INV) {
                a[K] = csubi(e[K], o[K]);
                a[K + R / 2] = caddi(e[K], o[K]);
            } else {
                a[K] = caddi(e[K], o[K]);
                a[K + R / 2] = csubi(e[K], o[K]);
            }
        } else if constexpr (m == 8) {
            a[K] = csub(e[K], o[K]);
            a[K + R / 2] = cadd(e[K], o[K]);
        } else {
            const float2 t = twc<R, K, INV>(o[K]);
            a[K] = cadd(e[K], t);
            a[K + R / 2] = csub(e[K], t);
        }
        dft_combine<R, K + 1, INV>(a, e, o);
    }
}

template <bool INV>
__device__ __forceinline__ void bfly4(float2& a0, float2& a1, float2& a2, float2& a3) {
    const float2 t0 = cadd(a0, a2), t1 = csub(a0, a2), t2 = cadd(a1, a3), t3 = csub(a1, a3);
    a0 = cadd(t0, t2);
    a2 = csub(t0, t2);
    // a1 = t1 + u3, a3 = t1 - u3 with u3 = (-/+i) t3
    a1 = INV ? caddi(t1, t3) : csubi(t1, t3);
    a3 = INV ? csubi(t1, t3) : caddi(t1, t3);
}

template <int R, int R1, int N1, int K2, bool INV>
__device__ __forceinline__ void dft_twiddle_step(float2* a) {
    // a[n1 + R1*k2] *= W_R^(n1*k2) for the compile-time (n1, k2) grid
    if constexpr (N1 < R1) {
        if constexpr (K2 < R / R1) {
            a[N1 + R1 * K2] = twc<R, N1 * K2, INV>(a[N1 + R1 * K2]);
            dft_twiddle_step<R, R1, N1, K2 + 1, INV>(a);
        } else {
            dft_twiddle_step<R, R1, N1 + 1, 0, INV>(a);
        }
    }
}

// In-register R-point DFT, natural order in and out (R <= 16).
// R = 16 and 8 are factored as R1 x R2 (4 x 4, 2 x 4): R2-point DFTs over
// n = n1 + R1*n2, twiddles W_R^(n1*k2), R1-point DFTs, and a compile-time
// output permutation (pure register renaming).
template <int R, bool INV>
__device__ __forceinline__ void dft_reg(float2* a) {
    if constexpr (R == 2) {
        const float2 t = a[0];
        a[0] = cadd(t, a[1]);
        a[1] = csub(t, a[1]);
    } else if constexpr (R == 4) {
        bfly4<INV>(a[0], a[1], a[2], a[3]);
    } else if constexpr (R == 8 || R == 16) {
        constexpr int R1 = R == 16 ? 4 : 2, R2 = R / R1;
#pragma unroll
        for (int n1 = 0; n1 < R1; ++n1) {
            float2 b[R2];
#pragma unroll
            for (int n2 = 0; n2 < R2; ++n2) b[n2] = a[n1 + R1 * n2];
            dft_reg<R2, INV>(b);
#pragma unroll
            for (int k2 = 0; k2 < R2; ++k2) a[n1 + R1 * k2] = b[k2];
        }
        dft_twiddle_step<R, R1, 1, 1, INV>(a);
        float2 out[R];
#pragma unroll
        for (int k2 = 0; k2 < R2; ++k2) {
            float2 c[R1];
#pragma unroll
            for (int n1 = 0; n1 < R1; ++n1) c[n1] = a[n1 + R1 * k2];
            dft_reg<R1, INV>(c);
#pragma unroll
            for (int k1 = 0; k1 < R1; ++k1) out[k2 + R2 * k1] = c[k1];
        }
#pragma unroll
        for (int k = 0; k < R; ++k) a[k] = out[k];
    } else if constexpr (R > 2) {
        float2 e[R / 2], o[R / 2];
#pragma unroll
        for (int i = 0; i < R / 2; ++i) {
            e[i] = a[2 * i];
            o[i] = a[2 * i + 1];
        }
        dft_reg<R / 2, INV>(e);
        dft_reg<R / 2, INV>(o);
        dft_combine<R, 0, INV>(a, e, o);
    }
}

// One Stockham pass over an N-point sequence held (padded) in LDS buffer s.
// L = product of the radices already applied.  Thread t of the team.
template <int N, int R, int L, bool INV>
__device__ __forceinline__ void stockham_pass(float2* s, const float2* __restrict__ tw, int t) {
    constexpr int TT = fft_team(N);
    constexpr int NB = N / R;        // butterflies in this pass
    constexpr int BPT = NB / TT;     // butterflies per thread
    static_assert(BPT >= 1 && NB % TT == 0, "bad radix schedule");
    float2 a[BPT][R];
#pragma unroll
    for (int b = 0; b < BPT; ++b) {
        const int j = t + b * TT;
        const int k = j % L;
#pragma unroll
        for (int r = 0; r < R; ++r) a[b][r] = s[pad(j + r * NB)];
        if constexpr (L > 1) {
            constexpr int step = N / (L * R);
#pragma unroll
            for (int r = 1; r < R; ++r) {
                float2 w = tw[r * k * step];
                a[b][r] = cmul_dir<INV>(a[b][r], w);
            }
        }
        dft_reg<R, INV>(a[b]);
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < BPT; ++b) {
        const int j = t + b * TT;
        const int k = j % L;
        const int base = (j - k) * R + k;
#pragma unroll
        for (int r = 0; r < R; ++r) s[pad(base + r * L)] = a[b][r];
    }
    __syncthreads();
}

template <int N, int L, bool INV>
__device__ __forceinline__ void stockham_passes(float2* s, const float2* __restrict__ tw, int t) {
    if constexpr (L < N) {
        constexpr int E = fft_elems(N);
        constexpr int R = (N / L) >= E ? E : (N / L);
        stockham_pass<N, R, L, INV>(s, tw, t);
        stockham_passes<N, L * R, INV>(s, tw, t);
    }
}

// In-place N-point FFT of the team's padded LDS row s (natural order in/out,
// unnormalised).  Must be called by every thread of the workgroup (barriers).
template <int N, bool INV>
__device__ __forceinline__ void fft_team_lds(float2* s, const float2* __restrict__ tw, int t) {
    stockham_passes<N, 1, INV>(s, tw, t);
}

}  // namespace fcdk
