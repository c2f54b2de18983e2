// Batched, band-pruned per-frame pipeline (the throughput path of fcd_process).
//
//   K1 demod_rows   frame rows -> packed-pair R2C row FFT -> only the spectrum
//                   columns the two carrier disks touch (fcd.py:28)
//   K2 demod_cols   per such column: column FFT, disk band-pass (carriers.py:17-20),
//                   inverse column FFT (fcd.py:118, first half of ifft2)
//   K3 demod_phase  per row and carrier: inverse row FFT of the band, phase
//                   -angle(A * ccsgn) = wrap(theta_ref - atan2(A)) (fcd.py:118)
//   I1 int_rows     residue census + residue-free unwrap (column-0 scan + row
//                   scan, fcd.py:119) + phi0 + i*phi1 + forward row FFT
//   I2 int_cols     per column pair (c, -c): forward column FFTs, Phi0/Phi1
//                   split, displacement solve + integration multiplier
//                   (fcd.py:122-138, fourier.py:115-137), inverse column FFT
//   I3 int_c2r      packed-pair C2R row FFT -> height (fcd.py:33)
//
// Row <-> column hand-offs use a 16-row tiled layout [row/16][col][row%16]:
// a column kernel reads/writes whole 128-byte lines (16 rows of one column),
// a row-block workgroup covers whole tiles.  All FFT data stays in registers
// (regfft.hpp); LDS carries only pass exchanges and small staging blocks.
#include <atomic>
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#include "kernels.hpp"
#include "gfft.hpp"
#include "regfft.hpp"

namespace fcdk {

#define FCD_CHECK_LAUNCH()                                                          \
    do {                                                                            \
        hipError_t e_ = hipGetLastError();                                          \
        if (e_ != hipSuccess) throw std::runtime_error(std::string("kernel launch: ") + hipGetErrorString(e_)); \
    } while (0)
#define FCD_HIPCHK(x)                                                               \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) throw std::runtime_error(std::string(#x ": ") + hipGetErrorString(e_)); \
    } while (0)

constexpr int TILE = 16;
constexpr int BLOCK = 256;
// Minimum waves per SIMD for every fast-path kernel (launch-bounds 2nd argument):
// 4 caps the allocation at 128 VGPRs, i.e. 16 waves per CU to hide HBM latency.
#ifndef FCD_MIN_WAVES
#define FCD_MIN_WAVES 4
#endif
// Minimum waves per SIMD of k_demod_cols above 1024 points (its 1024-point
// form has its own, DemodColsCfg::V); 4096 points always 2.  The register
// counts each kernel compiles to are in build/*.res (-Rpass-analysis), and
// tests/test_cpu_host.py checks the ones the occupancy statements here rely on.
#ifndef FCD_COL_WAVES
#define FCD_COL_WAVES 2
#endif
template <int N>
struct ColWaves {
    static constexpr int V = N >= 4096 ? 2 : FCD_COL_WAVES;
};
constexpr float kTwoPiF = 6.28318530717959f;

__device__ __forceinline__ long tix(int row, int col, int ncols) {
    return ((long)(row >> 4) * ncols + col) * TILE + (row & 15);
}

// Workgroup size of k_int_cols: more teams per workgroup share one twiddle table.
#ifndef FCD_INTCOLS_BLOCK
#define FCD_INTCOLS_BLOCK 256
#endif

template <int N, int B = BLOCK, int EE = fft_elems(N)>
struct KCfg {
    static constexpr int TT = Sched<N, EE>::TT;
    static constexpr int E = Sched<N, EE>::E;
    static constexpr int THREADS = TT > B ? TT : B;  // 4096-point teams span 8 waves
    static constexpr int TEAMS = THREADS / TT;
    static constexpr int ROW = padded_len(N);  // float2 per team row
    static constexpr int NLEN = N;             // twiddle table entries (float2) at the LDS base
};

// Minimum waves per SIMD of k_int_cols: both columns' transforms stay in
// registers (no LDS mirror exchange).  1024 points: 168 VGPRs, 3 waves/SIMD,
// without spills only when the mirror column is not prefetched (r01be: 3.23 vs
// 3.67 us/frame before; any spill costs more than the occupancy gains).
#ifndef FCD_INTCOLS_WAVES
#define FCD_INTCOLS_WAVES 3
#endif
// Prefetch the mirror column of the next item too (1), or load it at the top of
// the item (0: 16 fewer VGPRs live across the transforms).
#ifndef FCD_INTCOLS_WAVES_E16
#define FCD_INTCOLS_WAVES_E16 2  // at 16 elements per lane (3: 168 VGPRs, 22 spilled, 2.81 -> 3.71 us/frame, kbench r03w3)
#endif
// k_int_cols prefetches the next item's column; its mirror column is loaded at the top of
// the item (16 fewer VGPRs live across the transforms; IntColsCfg).
#ifndef FCD_INTCOLS_QUADS
#define FCD_INTCOLS_QUADS 1  // 4-row Zt tiles: sibling blocks on one XCD share each line's 4 columns
#endif
// Workgroup size of k_demod_cols up to 1024 points: 4 teams share one twiddle
// table, 78 KB of LDS -> 2 workgroups = 16 waves per CU at 1024, which needs
// <= 128 VGPRs, i.e. launch bounds of 4 waves per SIMD (compiles to 122):
// 0.84 vs 0.89 us/frame in isolation (kbench r01cd; 12 waves per CU with 256
// threads).  Larger transforms keep 256-thread workgroups.
#ifndef FCD_DEMODCOLS_BLOCK
#define FCD_DEMODCOLS_BLOCK 512
#endif
// From kDcTwGlobalMin points k_demod_cols' twiddle table stays in global memory: the
// two exchange rows alone are 70 KB at 4096, so without the 32 KB copy two workgroups
// fit per CU (16.9 -> 15.1 us/frame at 4096^2, kbench r03u).
constexpr int kDcTwGlobalMin = 4096;
#ifndef FCD_DEMODCOLS_V16
#define FCD_DEMODCOLS_V16 2
#endif
template <int N>
struct DemodColsCfg : KCfg<N, (N <= 1024 ? FCD_DEMODCOLS_BLOCK : BLOCK), demod_cols_elems(N)> {
    static constexpr int V = N <= 1024 ? (demod_cols_elems(N) == 16 ? FCD_DEMODCOLS_V16 : 4) : ColWaves<N>::V;
    static constexpr bool GTW = N >= kDcTwGlobalMin;
    static constexpr int NLEN = GTW ? 0 : N;
};

// (A lean 2048-point form without the prefetch and with the row wavenumbers from
// global memory, 128 VGPRs for 4 workgroups per CU, measured 13.1 -> 13.6 us/frame, r03v.)
template <int N>
struct IntColsCfg : KCfg<N, FCD_INTCOLS_BLOCK, int_cols_elems(N)> {
    // 16 elements per lane at 1024: 186 VGPRs, 2 waves / SIMD
    static constexpr int V = N <= 1024 ? (int_cols_elems(N) == 16 ? FCD_INTCOLS_WAVES_E16 : FCD_INTCOLS_WAVES) : ColWaves<N>::V;
    // The row wavenumber tables as LDS copies below 4096 points.  At 4096 they are read
    // from global memory (L1 / L2) and the next item's mirror column is no longer
    // prefetched (248 VGPRs, no spills): the 99 KB of LDS with the copies held the 4-wave
    // workgroup (room for two by registers) at one per CU; the twiddle table and the
    // team's exchange row (67 KB) let two run.  c5 3.13 k -> 3.36-3.38 k frames/s,
    // int_cols + c2r 124.9 -> 107.8 us/frame (r05y / r05z; the ky loads from global memory
    // WITH the mirror prefetch spill 59 VGPRs, the twiddles from global memory 62).
    static constexpr bool LKY = N < 4096;
};

// find_wrap(a, b) of the reference unwrapper with an f32 fast path:
// fl(a - b) > fl(pi) only if a - b > M_PI; equality needs the exact f64 test.
__device__ __forceinline__ int fw_fast(float a, float b) {
    const float d = a - b;
    constexpr float P = 3.14159274f;  // nearest float to M_PI (above it)
    if (d > P) return -1;
    if (d < -P) return 1;
    if (d == P || d == -P) {
        const double e = (double)a - (double)b;
        return e > 3.141592653589793 ? -1 : (e < -3.141592653589793 ? 1 : 0);
    }
    return 0;
}

// ------------------------------------------------------------------ K1
// band columns per lane that k_demod_rows keeps in registers (the rest are read
// from the table per row pair)
#ifndef FCD_DR_HCREG
#define FCD_DR_HCREG 2
#endif
constexpr int DR_HCR = FCD_DR_HCREG;
// The band values leave through a staged [NC][16] block.  (Writing each row pair's
// values straight to Xb instead, 16 bytes per column, measured 25.9 vs 26.0 us/frame at
// 4096 and 5.94 vs 5.66 at 2048 but k_demod_cols +0.24 behind it, kbench r03v.)

template <int W, int B = BLOCK>
__global__ __launch_bounds__((KCfg<W, B>::THREADS), FCD_MIN_WAVES) void k_demod_rows(const float* __restrict__ frames, int H, int nb,
                                                      DemodTables T, float2* __restrict__ Xb,
                                                      const float2* __restrict__ tw) {
    using C = KCfg<W, B>;
    constexpr int TT = C::TT, E = C::E, TEAMS = C::TEAMS;
    extern __shared__ __attribute__((aligned(16))) float2 lds_raw[];
    float2* const lds = lds_raw + C::NLEN;  // lds_raw[0, NLEN): the twiddle table
    const int team = threadIdx.x / TT, t = threadIdx.x % TT;
    float2* s = lds + team * C::ROW;
    float2* stage = lds + TEAMS * C::ROW;  // [NC][TILE + 1]
    RegFFT<W> fft;
    fft.init(tw, lds_raw, threadIdx.x, C::THREADS);
    __syncthreads();
    const int NC = T.NC;
    const int rbs = H / TILE;
    // this lane's first DR_HCR band columns, held for the whole kernel (no dependent
    // global load in front of every row pair's band extraction)
    int hcr[DR_HCR > 0 ? DR_HCR : 1];
#pragma unroll
    for (int k = 0; k < DR_HCR; ++k) hcr[k] = t + k * TT < NC ? T.hc[t + k * TT] : 0;
    // the next row pair of this team is loaded while the current one is transformed
    float2 xn[E];
    auto fetch = [&](int blk, int pr) {
        const int f = blk / rbs, rb = blk % rbs;
        const float* ra = frames + ((long)f * H + rb * TILE + 2 * pr) * W;
#pragma unroll
        for (int q = 0; q < E; ++q)
            xn[q] = make_float2(__builtin_nontemporal_load(ra + t + TT * q), __builtin_nontemporal_load(ra + W + t + TT * q));
    };
    if ((int)blockIdx.x < nb * rbs && team < TILE / 2) fetch(blockIdx.x, team);  // teams past the tile's pairs idle
    for (int blk = blockIdx.x; blk < nb * rbs; blk += gridDim.x) {
        for (int pr = team; pr < TILE / 2; pr += TEAMS) {
            float2 x[E];
#pragma unroll
            for (int q = 0; q < E; ++q) x[q] = xn[q];
            if (pr + TEAMS < TILE / 2)
                fetch(blk, pr + TEAMS);
            else if (blk + (int)gridDim.x < nb * rbs)
                fetch(blk + gridDim.x, team);
            fft.template run<false>(x, s, t);
            if constexpr (!Sched<W>::WAVE_LOCAL) __syncthreads();
#pragma unroll
            for (int q = 0; q < E; ++q) s[pad(t + TT * q)] = x[q];
            team_sync<W>();
            auto band = [&](int i, int hc) {
                const float2 zk = s[pad(hc)], zm = s[pad((W - hc) & (W - 1))];
                // X_a = (Z(k) + conj Z(-k)) / 2 ; X_b = (Z(k) - conj Z(-k)) / 2i
                const float2 xa = make_float2(0.5f * (zk.x + zm.x), 0.5f * (zk.y - zm.y));
                const float2 xb = make_float2(0.5f * (zk.y + zm.y), -0.5f * (zk.x - zm.x));
                stage[i * (TILE + 1) + 2 * pr] = xa;
                stage[i * (TILE + 1) + 2 * pr + 1] = xb;
            };
#pragma unroll
            for (int k = 0; k < DR_HCR; ++k)
                if (t + k * TT < NC) band(t + k * TT, hcr[k]);
            for (int i = t + DR_HCR * TT; i < NC; i += TT) band(i, T.hc[i]);
        }
        {
            const int f = blk / rbs, rb = blk % rbs;
            __syncthreads();
            float2* dst = Xb + (long)f * H * NC + (long)rb * NC * TILE;
            for (int idx = threadIdx.x; idx < NC * TILE; idx += C::THREADS)
                dst[idx] = stage[(idx / TILE) * (TILE + 1) + (idx % TILE)];
            __syncthreads();
        }
    }
}

// ------------------------------------------------------------------ K2
template <int H>
__global__ __launch_bounds__(DemodColsCfg<H>::THREADS, DemodColsCfg<H>::V) void k_demod_cols(const float2* __restrict__ Xb, int nb, DemodTables T,
                                                      float2* __restrict__ Ab, int NCA,
                                                      const float2* __restrict__ tw) {
    using C = DemodColsCfg<H>;
    constexpr int TT = C::TT, E = C::E, TEAMS = C::TEAMS;
    extern __shared__ __attribute__((aligned(16))) float2 lds_raw[];
    float2* const lds = lds_raw + C::NLEN;  // lds_raw[0, NLEN): the twiddle table
    const int team = threadIdx.x / TT, t = threadIdx.x % TT;
    float2* s = lds + team * C::ROW;            // holds the forward column spectrum
    float2* s2 = lds + (TEAMS + team) * C::ROW;  // exchanges of the inverse FFTs
    RegFFT<H, C::GTW, C::E> fft;
    fft.init(tw, lds_raw, threadIdx.x, C::THREADS);
    __syncthreads();
    const int NC = T.NC;
    const int items = nb * NC;
    // element q of this lane is row t + TT q (TT a multiple of the 16-row tile): its
    // tile offset is this lane's offset plus q TT NC (q TT NCA in Ab)
    static_assert(TT % TILE == 0, "row stride across whole tiles");
    const long xb_lane = (long)(t >> 4) * NC * TILE + (t & 15), xb_step = (long)TT * NC;
    const long ab_lane = (long)(t >> 4) * NCA * TILE + (t & 15), ab_step = (long)TT * NCA;
    // the next item's column is loaded while the current one is transformed (0.865 ->
    // 0.84 us/frame against a load at the top of each item, kbench r02c1)
    float2 xn[E];
    auto fetch = [&](int it) {
        const int fi = it < items ? it / NC : 0, ii = it < items ? it % NC : 0;
        const float2* src = Xb + (long)fi * H * NC + (long)ii * TILE + xb_lane;
#pragma unroll
        for (int q = 0; q < E; ++q) xn[q] = src[q * xb_step];  // tix(t + TT q, ii, NC)
    };
    fetch(blockIdx.x * TEAMS + team);
    for (int base = blockIdx.x * TEAMS; base < items; base += gridDim.x * TEAMS) {
        const int item = base + team;
        const bool valid = item < items;
        const int f = valid ? item / NC : 0, i = valid ? item % NC : 0;
        float2 x[E];
#pragma unroll
        for (int q = 0; q < E; ++q) x[q] = xn[q];
        if (base + (int)gridDim.x * TEAMS < items) fetch(item + gridDim.x * TEAMS);
        // the item's output count and first output (every column has 4 table slots),
        // read before the forward transform so that it hides their latency
        const int nout = valid ? T.nouts[i] : 0;
        int4 on = T.outs[i * 4];     // carrier, cslot, mirror, uc
        int2 rn = T.outrows[i * 4];  // shifted rows [lo, hi]
        fft.template run<false>(x, s, t);
        if constexpr (!Sched<H, C::E>::WAVE_LOCAL) __syncthreads();
#pragma unroll
        for (int q = 0; q < E; ++q) s[pad(t + TT * q)] = x[q];
        team_sync_of<Sched<H, C::E>>();
        // teams spanning waves share the workgroup barrier: every team loops to
        // the largest output count among the workgroup's items
        int nmax = nout;
        if constexpr (!Sched<H, C::E>::WAVE_LOCAL && TEAMS > 1) {
            nmax = 0;
#pragma unroll
            for (int tm = 0; tm < TEAMS; ++tm) {
                const int it = base + tm;
                nmax = max(nmax, it < items ? T.nouts[it % NC] : 0);
            }
        }
#pragma unroll 1
        for (int e = 0; e < nmax; ++e) {
            const bool live = e < nout;
            const int4 o = live ? on : make_int4(0, 0, 0, 0);
            const int2 rr = live ? rn : make_int2(1, 0);
            if (e + 1 < 4) {  // the next output's entries, during this inverse transform
                on = T.outs[i * 4 + e + 1];
                rn = T.outrows[i * 4 + e + 1];
            }
            float2 y[E];
#pragma unroll
            for (int q = 0; q < E; ++q) {
                const int u = t + TT * q;
                const int sr = (u + H / 2) & (H - 1);
                float2 v = make_float2(0.f, 0.f);
                if (sr >= rr.x && sr <= rr.y) {
                    if (o.z) {
                        v = s[pad((H - u) & (H - 1))];
                        v.y = -v.y;
                    } else {
                        v = s[pad(u)];
                    }
                }
                y[q] = v;
            }
            fft.template run<true>(y, s2, t);
            if (live) {
                float2* dst = Ab + ((long)f * 2 + o.x) * H * NCA + (long)o.y * TILE + ab_lane;
#pragma unroll
                for (int q = 0; q < E; ++q) dst[q * ab_step] = y[q];  // tix(t + TT q, o.y, NCA)
            }
        }
    }
}

// ------------------------------------------------------------------ K3
template <int W>
__global__ __launch_bounds__(KCfg<W>::THREADS, FCD_MIN_WAVES) void k_demod_phase(const float2* __restrict__ Ab, int H, int nb, int NCA,
                                                       DemodTables T, const float* __restrict__ theta,
                                                       float* __restrict__ wrapped, const float2* __restrict__ tw) {
    using C = KCfg<W>;
    constexpr int TT = C::TT, E = C::E, TEAMS = C::TEAMS;
    extern __shared__ __attribute__((aligned(16))) float2 lds_raw[];
    float2* const lds = lds_raw + C::NLEN;  // lds_raw[0, NLEN): the twiddle table
    const int team = threadIdx.x / TT, t = threadIdx.x % TT;
    float2* s = lds + team * C::ROW;
    float2* stage = lds + TEAMS * C::ROW;  // [NCc][TILE + 1]
    RegFFT<W> fft;
    fft.init(tw, lds_raw, threadIdx.x, C::THREADS);
    __syncthreads();
    const int rbs = H / TILE;
    const int items = nb * 2 * rbs;
    for (int blk = blockIdx.x; blk < items; blk += gridDim.x) {
        const int f = blk / (2 * rbs), c = (blk / rbs) % 2, rb = blk % rbs;
        const int ncc = T.NCc[c];
        const float2* src = Ab + ((long)f * 2 + c) * H * NCA + (long)rb * NCA * TILE;
        for (int idx = threadIdx.x; idx < ncc * TILE; idx += C::THREADS)
            stage[(idx / TILE) * (TILE + 1) + (idx % TILE)] = src[idx];
        int cs[E];
#pragma unroll
        for (int q = 0; q < E; ++q) cs[q] = T.colslot[c * W + t + TT * q];
        __syncthreads();
        for (int rl = team; rl < TILE; rl += TEAMS) {
            const int r = rb * TILE + rl;
            float2 x[E];
#pragma unroll
            for (int q = 0; q < E; ++q)
                x[q] = cs[q] >= 0 ? stage[cs[q] * (TILE + 1) + rl] : make_float2(0.f, 0.f);
            fft.template run<true>(x, s, t);
            const float* th = theta + ((long)c * H + r) * W;
            float* wo = wrapped + (((long)f * 2 + c) * H + r) * W;
#pragma unroll
            for (int q = 0; q < E; q += 2) {  // pixel pairs: packed atan2 + wrap (gfft.hpp)
                const int i = t + TT * q;
                const fv2 w = wrapped_phase_pk(fv2{th[i], th[i + TT]}, x[q], x[q + 1]);
                st_stream(wo + i, w.x);
                st_stream(wo + i + TT, w.y);
            }
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------ team scan
// Exclusive add-scan of v across the team; returns (exclusive, total).
template <int TT>
__device__ __forceinline__ int2 team_scan_excl(int v, int t, int* scratch) {
    if constexpr (TT <= 64) {
        const int incl = team_scan_incl_dpp<TT>(v);
        const int total = __shfl(incl, TT - 1, TT);
        return make_int2(incl - v, total);
    } else {
        constexpr int NW = TT / 64;
        const int incl = team_scan_incl_dpp<64>(v);
        const int wv = t >> 6;
        if ((t & 63) == 63) scratch[wv] = incl;
        __syncthreads();
        int before = 0, total = 0;
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            const int tk = scratch[k];
            before += k < wv ? tk : 0;
            total += tk;
        }
        __syncthreads();
        return make_int2(before + incl - v, total);
    }
}

// ------------------------------------------------------------------ I1
// The row stage of the unfused chain (phases -> unwrap -> phi0 + i phi1 -> row FFT -> Zt)
// is k_int_rows2 in int_rows.inc.

// ------------------------------------------------------------------ I2
template <int H>
__global__ __launch_bounds__(IntColsCfg<H>::THREADS, IntColsCfg<H>::V) void k_int_cols(const float2* __restrict__ Zt, int W, int nb, IntegCoef c,
                                                    float2* __restrict__ Ht, const float2* __restrict__ tw, int zts,
                                                    const int* __restrict__ colk) {
    using C = IntColsCfg<H>;
    constexpr int TT = C::TT, E = C::E, TEAMS = C::TEAMS;
    extern __shared__ __attribute__((aligned(16))) float2 lds_raw[];
    float2* const lds = lds_raw + C::NLEN;  // lds_raw[0, NLEN): the twiddle table
    const int team = threadIdx.x / TT, t = threadIdx.x % TT;
    float2* s = lds + team * C::ROW;
    RegFFT<H, false, C::E> fft;
    fft.init(tw, lds_raw, threadIdx.x, C::THREADS);
    // the row wavenumber tables (ky_eff, ky^2) of every element, read per item: LDS copies
    // (LKY) or the tables themselves
    const float* lky = c.kye;
    const float* lky2 = c.ky2;
    if constexpr (C::LKY) {
        float* const k1 = reinterpret_cast<float*>(lds + TEAMS * C::ROW);
        float* const k2 = k1 + H;
        for (int i = threadIdx.x; i < H; i += C::THREADS) {
            k1[i] = c.kye[i];
            k2[i] = c.ky2[i];
        }
        lky = k1;
        lky2 = k2;
    }
    __syncthreads();
    const int NCH = W / 2 + 1;
    const int items = nb * NCH;
    const int zmask = (1 << zts) - 1;
    // Element q of this lane is row t + TT q.  TT is a multiple of the Zt tile height,
    // so its tile offset is this lane's offset plus q TT W (and in Ht q TT NCH): the
    // addresses are one lane base and a uniform stride, computed once, instead of
    // the tile arithmetic per load (which cost ~200 VALU instructions per item).
    const long zt_lane = (((long)(t >> zts) * W) << zts) + (t & zmask);
    const long zt_step = (long)TT * W;
    const long ht_lane = (long)(t >> 4) * NCH * 16 + (t & 15);
    const long ht_step = (long)TT * NCH;
    // Both columns of the NEXT item are loaded into registers while the current
    // item is transformed (loads issued before the current item's stores).
    float2 py[E], px[E];
    auto fetch_fc = [&](int f, int col, bool mirror, float2 (&v)[E]) {
        const int cc = mirror ? (W - col) & (W - 1) : col;
        const float2* src = Zt + (long)f * H * W + ((long)cc << zts) + zt_lane;
#pragma unroll
        for (int q = 0; q < E; ++q) v[q] = src[q * zt_step];
    };
    // Items are codes: frame code / CW, column code % CW (valid below NCH).
    //
    // With 8-row Zt tiles (2048-point columns; 1024 until r04n) a column's rows fill 64
    // bytes, half a 128-byte line whose other half is the neighbouring column, and items
    // c, c + 1 always share one line (c even: their direct columns; c odd: their mirror
    // columns W - c - 1, W - c).  So adjacent items must be read while both halves sit in
    // one XCD's L2; even so the reads were 1.45x the compulsory bytes at 1024 (PMC r04e),
    // and 1024-point columns now have 16-row Zt tiles (whole lines per column: 1.00x,
    // PMC r04n, at the same step time).  XCD-AWARE
    // (dispatch deals block b to XCD b % 8): the items are cut into 8 contiguous
    // regions, one per XCD, and XCD x's blocks walk its region iteration-major -- at
    // iteration i its blocks take consecutive TEAMS-item groups of one stretch of
    // (blocks per XCD) x TEAMS items -- so neighbouring items run on the same XCD at the
    // same time (a contiguous range per block shared its edge lines with the block's
    // previous iteration, by then evicted: 1.58x the compulsory Zt reads, PMC r03zm).
    // kbench r04d: 2.63-2.69 -> 2.53 us/frame at 1024^2 x 256, 11.98 -> 11.67 at 2048^2 x 64.
    //
    // With 4-row Zt tiles (4096-point rows) a 128-byte line holds 4 columns x 4 rows,
    // and a block's next column came too late: its lines had left the XCD's L2
    // (3.9x the compulsory Zt reads, PMC r03t4096).  There the blocks work in QUADS:
    // the 4 blocks of a group sit on one XCD (dispatch deals block b to XCD b % 8)
    // and take columns 4k, 4k + 1, 4k + 2, 4k + 3 of the same quad at the same time.
    // (2-row Zt tiles: a line holds 8 columns x 2 rows, groups of 8 blocks)
    const int G = zts == 2 ? 4 : (zts == 1 ? 8 : 0);  // columns per 128-byte line
    const bool quad = G && TEAMS == 1 && gridDim.x % (8 * G) == 0 && FCD_INTCOLS_QUADS;
    const bool xcd = !quad && gridDim.x % 8 == 0;
    const int NQ = G ? (NCH + G - 1) / G : 0;
    const int CW = quad ? G * NQ : NCH;
    int c0, cstep, cend, bstride;  // first item, item step between teams, end, step between iterations
    if (quad) {
        const int q = blockIdx.x / 8, j = q % G;
        const int grp = blockIdx.x % 8 + 8 * (q / G), ngrp = gridDim.x / G;
        const int nquads = nb * NQ, perq = (nquads + ngrp - 1) / ngrp;
        const int Q0 = min(grp * perq, nquads), Q1 = min(Q0 + perq, nquads);
        c0 = G * Q0 + j;
        cstep = G;
        cend = G * Q1;
        bstride = TEAMS * cstep;
    } else if (xcd) {
        const int bpx = gridDim.x / 8;                      // blocks per XCD
        const int region = (items + 7) / 8;                 // items per XCD
        const int r0 = min((int)(blockIdx.x % 8) * region, items);
        c0 = r0 + (int)(blockIdx.x / 8) * TEAMS;
        cstep = 1;
        cend = min(r0 + region, items);
        bstride = bpx * TEAMS;
    } else {
        const int per = (items + gridDim.x - 1) / gridDim.x;
        c0 = min(blockIdx.x * per, items);
        cstep = 1;
        cend = min(c0 + per, items);
        bstride = TEAMS;
    }
    auto fetch_col = [&](int code, bool mirror, float2 (&v)[E]) {
        const bool valid = code < cend && code % CW < NCH;
        fetch_fc(valid ? code / CW : 0, valid ? code % CW : 0, mirror, v);
    };
    auto fetch = [&](int code) {
        fetch_col(code, false, px);
    };
    fetch(c0 + team * cstep);
    for (int base = c0; base < cend; base += bstride) {
        const int item = base + team * cstep;
        const bool valid = item < cend && item % CW < NCH;
        const int f = valid ? item / CW : 0, col = valid ? item % CW : 0;
        const int colm = (W - col) & (W - 1);
        // Z(-ky, -c) straight from the INVERSE-direction (unnormalised) transform of
        // column -c: sum_y z(y, -c) e^{+2 pi i ky y / H} at index ky, so both operands
        // of the Hermitian split sit in the same lane and slot (no mirror exchange).
        float2 x[E], y[E];
        fetch_col(item, true, py);
#pragma unroll
        for (int q = 0; q < E; ++q) {
            y[q] = py[q];
            x[q] = px[q];
        }
        if (colk && (colm == 0 || col == 0)) {  // column-0 unwrap offsets of the fused path: row DC bins
            const float sc = 6.28318530717959f * (float)W;
#pragma unroll
            for (int q = 0; q < E; ++q) {
                const int rr = t + TT * q;
                const float2 o = make_float2(sc * (float)colk[((long)f * 2 + 0) * H + rr],
                                             sc * (float)colk[((long)f * 2 + 1) * H + rr]);
                if (colm == 0) y[q] = make_float2(y[q].x + o.x, y[q].y + o.y);
                if (col == 0) x[q] = make_float2(x[q].x + o.x, x[q].y + o.y);
            }
        }
        // (both transforms in lockstep with a second LDS row per team measured slower:
        // 3.94 vs 3.32 us/frame, kbench r02l; the next item's loads issued between them
        // hide better.  Pairing k_demod_cols' two inverse transforms: no change, r02m)
        fft.template run<true>(y, s, t);
        if (base + bstride < cend) fetch(base + bstride + team * cstep);
        fft.template run<false>(x, s, t);
        const float kx = c.kxe[col], kx2 = c.kx2[col];
        const float hnorm = 0.5f * c.norm;
#pragma unroll
        for (int q = 0; q < E; ++q) {
            const int i = t + TT * q;
            const float2 z = x[q];
            const float2 zm = y[q];
            // 2 Phi0 and 2 Phi1 (the halves go into the multiplier's scale)
            const float2 f0 = make_float2(z.x + zm.x, z.y - zm.y);
            const float2 f1 = make_float2(z.y + zm.y, zm.x - z.x);
            const float ky = lky[i];
            float k2 = kx2 + lky2[i];
            if (i == 0 && col == 0) k2 = 1.f;
            // 1 / k^2 by the hardware reciprocal (1 ulp) instead of an IEEE division
            // (a 10-instruction sequence per element)
            const float sc = hnorm * __builtin_amdgcn_rcpf(k2);
            const float m0 = (kx * c.a0 + ky * c.b0) * sc;
            const float m1 = (kx * c.a1 + ky * c.b1) * sc;
            const float re = m0 * f0.x + m1 * f1.x;
            const float im = m0 * f0.y + m1 * f1.y;
            x[q] = make_float2(-im, re);
        }
        fft.template run<true>(x, s, t);
        if (valid) {
            float2* dst = Ht + (long)f * H * NCH + (long)col * 16 + ht_lane;
#pragma unroll
            for (int q = 0; q < E; ++q) dst[q * ht_step] = x[q];  // tix(t + TT q, col, NCH)
        }
    }
}

// ------------------------------------------------------------------ I3
// Rows per workgroup (FCD_C2R_RPW_2048 at 2048): the staged block of the half spectrum (W/2+1 columns x
// RPW rows) plus one exchange row per team stays under ~156 KiB of LDS; one
// team per row pair, so W = 1024 runs 16 waves per CU from one workgroup.
#ifndef FCD_C2R_RPW_2048
#define FCD_C2R_RPW_2048 8  // 16 waves per CU in 156 KB of LDS: 8.97 -> 7.17 us/frame (kbench r03c8; 4 before)
#endif
// 4096-point rows: 4-row blocks (two 8-wave teams, 16 waves per CU) with the twiddles
// read from the global table (C2RCfg::GTW): 152 KB of LDS instead of 116 KB for a 2-row,
// one-team block (int_cols + c2r 104.7 -> 103.1 us/frame, c5 +0.6 %, r05zh)
__host__ __device__ constexpr int c2r_rpw(int W) { return W <= 1024 ? 16 : (W == 2048 ? FCD_C2R_RPW_2048 : 4); }

template <int W>
struct C2RCfg {
    static constexpr int TT = Sched<W>::TT;
    static constexpr int E = Sched<W>::E;
    static constexpr int RPW = c2r_rpw(W);
    // staged block pitch: RPW + 1 (odd, conflict-free; the 2- and 4-row blocks of the
    // wide rows unpadded have a third / fifth less LDS but still one workgroup per CU at
    // 4096 and were slower: 42.0 -> 43.4 us/frame, kbench r03u)
    static constexpr int SP = RPW + 1;
    static constexpr int THREADS = (RPW / 2) * TT < 1024 ? ((RPW / 2) * TT > TT ? (RPW / 2) * TT : TT) : 1024;
    static constexpr int TEAMS = THREADS / TT;
    static constexpr int ROW = padded_len(W);
    static constexpr bool GTW = W >= 4096;
    static constexpr int NLEN = GTW ? 0 : W;
};

template <int W>
__global__ __launch_bounds__(C2RCfg<W>::THREADS) void k_int_c2r(const float2* __restrict__ Ht, int H, int nb, int rpw,
                                                   float* __restrict__ hout, const float2* __restrict__ tw) {
    using C = C2RCfg<W>;
    constexpr int TT = C::TT, E = C::E, TEAMS = C::TEAMS;
    extern __shared__ __attribute__((aligned(16))) float2 lds_raw[];
    float2* const lds = lds_raw + C::NLEN;  // lds_raw[0, NLEN): the twiddle table
    const int team = threadIdx.x / TT, t = threadIdx.x % TT;
    float2* s = lds + team * C::ROW;
    float2* stage = lds + TEAMS * C::ROW;  // [NCH][rpw + 1]
    RegFFT<W, C::GTW> fft;
    fft.init(tw, lds_raw, threadIdx.x, C::THREADS);
    __syncthreads();
    const int NCH = W / 2 + 1;
    // rows per staged block: the launch passes C::RPW; as a constant the block's
    // index arithmetic is shifts, and a 16-row block is one contiguous Ht tile row
    (void)rpw;
    constexpr int RPW = C::RPW;
    const int nblk = H / RPW;
    // the next item's staged block (NCH x RPW values) is prefetched into registers
    // while the current one is transformed (SPT values per thread, all in flight)
    constexpr int SPT = ((W / 2 + 1) * C::RPW + C::THREADS - 1) / C::THREADS;
    float2 pf[SPT];
    auto fetch = [&](int blk) {
        const int f = blk / nblk, r0 = (blk % nblk) * RPW;
        const float2* src = Ht + (long)f * H * NCH;
#pragma unroll
        for (int i = 0; i < SPT; ++i) {
            const int idx = threadIdx.x + i * C::THREADS;
            if constexpr (RPW == TILE) {
                pf[i] = src[(long)r0 * NCH + min(idx, NCH * TILE - 1)];  // tix(r0 + idx % 16, idx / 16, NCH)
            } else {
                const int col = min(idx / RPW, NCH - 1), rl = idx % RPW;
                pf[i] = src[tix(r0 + rl, col, NCH)];
            }
        }
    };
    // XCD-aware order: workgroups are dealt round-robin to the 8 XCDs, each with
    // its own L2.  Below W = 1024 a staged block is only rpw of a 16-row Ht tile's
    // rows, so the 16 / rpw blocks of one tile read the same 128-byte lines: give
    // them consecutive virtual ids on ONE XCD (b % 8 = XCD, b / 8 = slot) so the
    // lines are fetched into one L2 once instead of into several.
    const int G = gridDim.x;
    const int vb = (G % 8 == 0) ? (int)(blockIdx.x % 8) * (G / 8) + (int)(blockIdx.x / 8) : (int)blockIdx.x;
    if (vb < nb * nblk) fetch(vb);
    for (int blk = vb; blk < nb * nblk; blk += G) {
        const int f = blk / nblk, r0 = (blk % nblk) * RPW;
#pragma unroll
        for (int i = 0; i < SPT; ++i) {
            const int idx = threadIdx.x + i * C::THREADS;
            if (idx < NCH * RPW) stage[(idx / RPW) * C::SP + idx % RPW] = pf[i];
        }
        __syncthreads();
        if (blk + G < nb * nblk) fetch(blk + G);
        for (int pr = team; pr < RPW / 2; pr += TEAMS) {
            float2 x[E];
#pragma unroll
            for (int q = 0; q < E; ++q) {
                const int col = t + TT * q;
                float2 g1, g2;
                if (col <= W / 2) {
                    g1 = stage[col * C::SP + 2 * pr];
                    g2 = stage[col * C::SP + 2 * pr + 1];
                } else {  // row-wise Hermitian: G(y, W - c) = conj G(y, c)
                    g1 = stage[(W - col) * C::SP + 2 * pr];
                    g2 = stage[(W - col) * C::SP + 2 * pr + 1];
                    g1.y = -g1.y;
                    g2.y = -g2.y;
                }
                x[q] = make_float2(g1.x - g2.y, g1.y + g2.x);
            }
            fft.template run<true>(x, s, t);
            float* h1 = hout + ((long)f * H + r0 + 2 * pr) * W;
            // plain stores: measured faster than nt for this last stream (1.71 vs 1.77-1.82
            // us/frame at 1024^2, kbench r01ax)
#pragma unroll
            for (int q = 0; q < E; ++q) {
                h1[t + TT * q] = x[q].x;
                h1[W + t + TT * q] = x[q].y;
            }
        }
        __syncthreads();
    }
}

#include "int_rows.inc"

// ------------------------------------------------------------------ launchers
// (atomic: the exact-first chain's two halves launch from two host threads)
static std::atomic<int> g_num_cu{0};
int device_cu_count() {
    int ncu = g_num_cu.load(std::memory_order_relaxed);
    if (!ncu) {
        int dev = 0;
        hipDeviceProp_t p;
        if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&p, dev) == hipSuccess)
            ncu = p.multiProcessorCount;
        if (!ncu) ncu = 256;
        g_num_cu.store(ncu, std::memory_order_relaxed);
    }
    return ncu;
}
static int grid_for(long work_items, int per_cu) {
    const int ncu = device_cu_count();
    const long cap = (long)ncu * per_cu;
    return (int)(work_items < cap ? (work_items > 0 ? work_items : 1) : cap);
}

template <class K>
static void set_lds(K kernel, size_t bytes) {
    if (bytes > 64 * 1024)
        FCD_HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
}

#define FCD_SIZE_SWITCH(n, FN, ...)                                   \
    switch (n) {                                                      \
        case 64: FN<64>(__VA_ARGS__); break;                          \
        case 128: FN<128>(__VA_ARGS__); break;                        \
        case 256: FN<256>(__VA_ARGS__); break;                        \
        case 512: FN<512>(__VA_ARGS__); break;                        \
        case 1024: FN<1024>(__VA_ARGS__); break;                      \
        case 2048: FN<2048>(__VA_ARGS__); break;                      \
        case 4096: FN<4096>(__VA_ARGS__); break;                      \
        default: throw std::runtime_error("unsupported FFT length " + std::to_string(n)); \
    }

template <int W>
static void launch_demod_rows(const float* frames, int H, int nb, const DemodTables& T, float2* Xb, const float2* tw,
                              hipStream_t s) {
    // 4096-point rows: 1024-thread workgroups (two 8-wave teams share the twiddle table and
    // the staged band block: 16 waves per CU instead of 8) when the band block leaves room
    // for the second exchange row (c5 demod 33.6 -> 32.0 us/frame; at 2048 four 4-wave
    // teams measured 7.64 -> 7.96, r05za / r05zb)
    using C2 = KCfg<W, 1024>;
    const size_t lds2 = (size_t)C2::NLEN * 8 + (size_t)C2::TEAMS * C2::ROW * 8 + (size_t)T.NC * (TILE + 1) * 8;
    if (W >= 4096 && C2::TEAMS >= 2 && lds2 <= 160 * 1024) {
        set_lds(k_demod_rows<W, 1024>, lds2);
        const int grid = grid_for((long)nb * (H / TILE), 1);
        hipLaunchKernelGGL((k_demod_rows<W, 1024>), dim3(grid), dim3(C2::THREADS), lds2, s, frames, H, nb, T, Xb, tw);
        FCD_CHECK_LAUNCH();
        return;
    }
    using C = KCfg<W>;
    const size_t lds = (size_t)C::NLEN * 8 + (size_t)C::TEAMS * C::ROW * 8 + (size_t)T.NC * (TILE + 1) * 8;
    set_lds(k_demod_rows<W>, lds);
    const int grid = grid_for((long)nb * (H / TILE), 4);
    hipLaunchKernelGGL(k_demod_rows<W>, dim3(grid), dim3(C::THREADS), lds, s, frames, H, nb, T, Xb, tw);
    FCD_CHECK_LAUNCH();
}

template <int H>
static void launch_demod_cols(const float2* Xb, int nb, const DemodTables& T, float2* Ab, int NCA, const float2* tw,
                              hipStream_t s) {
    using C = DemodColsCfg<H>;
    const size_t lds = (size_t)C::NLEN * 8 + (size_t)2 * C::TEAMS * C::ROW * 8;
    set_lds(k_demod_cols<H>, lds);
    const int grid = grid_for(((long)nb * T.NC + C::TEAMS - 1) / C::TEAMS, 4);
    hipLaunchKernelGGL(k_demod_cols<H>, dim3(grid), dim3(C::THREADS), lds, s, Xb, nb, T, Ab, NCA, tw);
    FCD_CHECK_LAUNCH();
}

template <int W>
static void launch_demod_phase(const float2* Ab, int H, int nb, int NCA, const DemodTables& T, const float* theta,
                               float* wrapped, const float2* tw, hipStream_t s) {
    using C = KCfg<W>;
    const size_t lds = (size_t)C::NLEN * 8 + (size_t)C::TEAMS * C::ROW * 8 + (size_t)NCA * (TILE + 1) * 8;
    set_lds(k_demod_phase<W>, lds);
    const int grid = grid_for((long)nb * 2 * (H / TILE), 4);
    hipLaunchKernelGGL(k_demod_phase<W>, dim3(grid), dim3(C::THREADS), lds, s, Ab, H, nb, NCA, T, theta, wrapped, tw);
    FCD_CHECK_LAUNCH();
}

template <int W>
static int int_rows_grid(int H, int nb) {
    using C = IRCfg<W>;
    const int per_cu = (int)std::max<size_t>(1, std::min<size_t>(2048 / C::THREADS, (160 * 1024) / C::LDS_BYTES));
    return grid_for((long)nb * (H / C::ZT), per_cu);
}

template <int W>
static void launch_int_rows(int kmode, const float* w, const int* colk, const int32_t* kin, int32_t* kout,
                            int* rescount, int H, int nb, float2* Zt, const float2* tw, float2* seam, hipStream_t s,
                            const MstK* mkp) {
    MstK mk{};
    if (mkp) mk = *mkp;
    if (kmode == 3 && !mkp) throw std::runtime_error("int_rows: kmode 3 needs the MST labels");
    using C = IRCfg<W>;
    const size_t lds = C::LDS_BYTES;
    int grid = int_rows_grid<W>(H, nb);
    const long items = (long)nb * (H / C::ZT);
    const int per = (int)((items + grid - 1) / grid);  // KMODE 1: tiles per block, a contiguous range
    if (kmode == 0) {
        set_lds(k_int_rows2<W, 0>, lds);
        hipLaunchKernelGGL((k_int_rows2<W, 0>), dim3(grid), dim3(C::THREADS), lds, s, w, colk, kin, kout, rescount, H,
                           nb, Zt, tw, seam, per, mk);
    } else if (kmode == 1) {
        if (!seam) throw std::runtime_error("int_rows: the seam census needs a seam buffer");
        grid = (int)((items + per - 1) / per);
        set_lds(k_int_rows2<W, 1>, lds);
        hipLaunchKernelGGL((k_int_rows2<W, 1>), dim3(grid), dim3(C::THREADS), lds, s, w, colk, kin, kout, rescount, H,
                           nb, Zt, tw, seam, per, mk);
        if (grid > 1) {
            FCD_CHECK_LAUNCH();
            hipLaunchKernelGGL(k_ir_seam_check<W>, dim3((unsigned)((grid - 1 + 3) / 4)), dim3(256), 0, s, seam, H, nb,
                               per, grid, rescount);
        }
    } else if (kmode == 2) {
        set_lds(k_int_rows2<W, 2>, lds);
        hipLaunchKernelGGL((k_int_rows2<W, 2>), dim3(grid), dim3(C::THREADS), lds, s, w, colk, kin, kout, rescount, H,
                           nb, Zt, tw, seam, per, mk);
    } else {
        set_lds(k_int_rows2<W, 3>, lds);
        hipLaunchKernelGGL((k_int_rows2<W, 3>), dim3(grid), dim3(C::THREADS), lds, s, w, colk, kin, kout, rescount, H,
                           nb, Zt, tw, seam, per, mk);
    }
    FCD_CHECK_LAUNCH();
}

template <int W>
static void int_rows_seam_bytes_t(int H, int nb, size_t* out) {
    *out = (size_t)int_rows_grid<W>(H, nb) * 2 * W * sizeof(float2);
}

template <int H>
static void launch_int_cols(const float2* Zt, int W, int nb, const IntegCoef& c, float2* Ht, const float2* tw,
                            hipStream_t s, const int* colk) {
    using C = IntColsCfg<H>;
    const size_t lds = (size_t)C::NLEN * 8 + (size_t)C::TEAMS * C::ROW * 8 + (C::LKY ? (size_t)H * 8 : 0);
    set_lds(k_int_cols<H>, lds);
    const int grid = grid_for(((long)nb * (W / 2 + 1) + C::TEAMS - 1) / C::TEAMS, 4);
    const int zt = zt_layout(W);
    const int zts = zt == 16 ? 4 : (zt == 8 ? 3 : (zt == 4 ? 2 : 1));
    hipLaunchKernelGGL(k_int_cols<H>, dim3(grid), dim3(C::THREADS), lds, s, Zt, W, nb, c, Ht, tw, zts, colk);
    FCD_CHECK_LAUNCH();
}

int c2r_rows_per_block(int W) { return c2r_rpw(W); }

template <int W>
static void launch_int_c2r(const float2* Ht, int H, int nb, float* h, const float2* tw, hipStream_t s) {
    using C = C2RCfg<W>;
    const int rpw = C::RPW;
    const size_t lds = (size_t)C::NLEN * 8 + (size_t)C::TEAMS * C::ROW * 8 + (size_t)(W / 2 + 1) * C::SP * 8;
    set_lds(k_int_c2r<W>, lds);
    const int grid = grid_for((long)nb * (H / rpw), 2);
    hipLaunchKernelGGL(k_int_c2r<W>, dim3(grid), dim3(C::THREADS), lds, s, Ht, H, nb, rpw, h, tw);
    FCD_CHECK_LAUNCH();
}

void demod_rows(int W, const float* frames, int H, int nb, const DemodTables& T, float2* Xb, const float2* tw,
                hipStream_t s) {
    FCD_SIZE_SWITCH(W, launch_demod_rows, frames, H, nb, T, Xb, tw, s);
}
void demod_cols(int H, const float2* Xb, int nb, const DemodTables& T, float2* Ab, int NCA, const float2* tw,
                hipStream_t s) {
    FCD_SIZE_SWITCH(H, launch_demod_cols, Xb, nb, T, Ab, NCA, tw, s);
}
void demod_phase(int W, const float2* Ab, int H, int nb, int NCA, const DemodTables& T, const float* theta,
                 float* wrapped, const float2* tw, hipStream_t s) {
    FCD_SIZE_SWITCH(W, launch_demod_phase, Ab, H, nb, NCA, T, theta, wrapped, tw, s);
}
void int_rows(int W, int kmode, const float* w, const int* colk, const int32_t* kin, int32_t* kout, int* rescount,
              int H, int nb, float2* Zt, const float2* tw, float2* seam, hipStream_t s, const MstK* mk) {
    FCD_SIZE_SWITCH(W, launch_int_rows, kmode, w, colk, kin, kout, rescount, H, nb, Zt, tw, seam, s, mk);
}
size_t int_rows_seam_bytes(int W, int H, int nb) {
    size_t b = 0;
    FCD_SIZE_SWITCH(W, int_rows_seam_bytes_t, H, nb, &b);
    return b;
}
void int_cols(int H, const float2* Zt, int W, int nb, const IntegCoef& c, float2* Ht, const float2* tw,
              hipStream_t s, const int* colk) {
    FCD_SIZE_SWITCH(H, launch_int_cols, Zt, W, nb, c, Ht, tw, s, colk);
}
void int_c2r(int W, const float2* Ht, int H, int nb, float* h, const float2* tw, hipStream_t s) {
    FCD_SIZE_SWITCH(W, launch_int_c2r, Ht, H, nb, h, tw, s);
}

}  // namespace fcdk
