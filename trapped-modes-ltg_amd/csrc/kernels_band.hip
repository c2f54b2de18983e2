// K3b band_phase: band-pruned inverse row transform + phase extraction
// (the second half of ifft2(D * mask) and -angle(. * ccsgn), fcd.py:118).
//
// After the inverse column FFT (k_demod_cols) every row of carrier c holds
// non-zeros only in its disk's columns, a contiguous (mod W) run of
// NCc <= B slots starting at unshifted column lo_c.  With n = g + L*n2
// (g < L = W/B, n2 < B):
//
//   x[n] = sum_j A[j] e^{2 pi i (lo_c + j) n / W}
//        = e^{2 pi i lo_c n / W} * IDFT_B( A[j] e^{2 pi i j g / W} )[n2]
//
// so one W-point inverse becomes L pre-twiddled B-point inverses (transform
// decomposition), 16 complex per lane, one wave per 1024-point row
// (L = 8 groups of 8 lanes at B = 128), no workgroup barrier inside a
// transform.  The carrier ramp e^{2 pi i lo_c n / W} cancels in the phase:
// the reference angle theta_b is produced by this same kernel from the
// reference's band (REF = true), so
//
//   wrapped = wrap(theta_b - angle(y)) = -angle(x_frame * conj(x_ref))
//
// exactly as fcd.py:118 up to float rounding.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "gfft.hpp"
#include "kernels.hpp"

namespace fcdk {

namespace {

#ifndef FCD_BAND_WAVES
#define FCD_BAND_WAVES 3  // min waves per SIMD (launch-bounds): 3 blocks of 4 waves per CU (168 VGPRs)
#endif

// Diagnostic ablations (FCD_BAND_NOTHETA / _ABL / _NOSTORE: wrong results by design)
// exist only in builds with -DFCD_DIAGNOSTIC (tools/ablate.sh, kbench variants); the
// product build (Makefile) cannot turn them on.
#if !defined(FCD_DIAGNOSTIC) && (defined(FCD_BAND_NOTHETA) || defined(FCD_BAND_ABL) || defined(FCD_BAND_NOSTORE))
#error "FCD_BAND_* ablations are diagnostic-only: build with -DFCD_DIAGNOSTIC"
#endif

#ifndef FCD_BAND_NOTHETA
#define FCD_BAND_NOTHETA 0  // diagnostic ablation only (wrong results): no reference-angle loads
#endif

#ifndef FCD_BAND_THREADS_2048
#define FCD_BAND_THREADS_2048 512  // workgroup size of the 2048-point band kernel (256: 25.1, 512: 22.5, 768: 23.4 us/frame, kbench r01ar)
#endif

#ifndef FCD_BAND_ABL
#define FCD_BAND_ABL 0  // diagnostic ablations only (wrong results): 1 no transform, 2 no atan2, 4 no LDS stage reads
#endif

#ifndef FCD_BAND_NOSTORE
#define FCD_BAND_NOSTORE 0  // diagnostic ablation only (no output): phase stores suppressed
#endif

#ifndef FCD_ATAN_N
#define FCD_ATAN_N 2  // pixel pairs per interleaved atan2 group (wrapped_phase_pkn); 0: the per-pair form
#endif

#ifndef FCD_ATAN_GROUP
#define FCD_ATAN_GROUP 4  // atan2 chains interleaved per scheduling group (0: unbounded)
#endif

constexpr int BTILE = 16;   // rows per Ab tile (k_demod_cols layout)
constexpr int SROW = 17;    // staged tile row pitch (complex): conflict-free strided reads

template <int W, int B>
struct BPCfg {
    static constexpr int G = B / 16;        // lanes per group transform
    static constexpr int L = W / B;         // groups per row
    static constexpr int RL = W / 16;       // lanes per row
    // 2048-point rows (2 waves each): with 256 threads the 68 KB of LDS allow 2
    // workgroups = 8 waves per CU; FCD_BAND_THREADS_2048 / 128 rows in flight in one
    // workgroup share one staged tile among more waves
    static constexpr int THREADS = (16 * RL) < 256 ? 16 * RL : (W == 2048 ? FCD_BAND_THREADS_2048 : 256);
    static constexpr int RP = THREADS / RL; // rows in flight per workgroup
    static constexpr int REGION = GSched<B>::REGION;
    static constexpr bool XCH = GSched<B>::NP > 1;
    static constexpr size_t XOFF = (size_t)B * SROW + (size_t)RL * 16;  // exchange regions after stage + pre-twiddles
    // exchange in float halves (GroupFFT::run_half): 4 B per element per transform
    static constexpr size_t LDS = XOFF * 8 + (XCH ? (size_t)RP * L * REGION * 4 : 0);
};

}  // namespace

#ifdef FCD_STAMPS
// Diagnostic build only: s_memtime stamps of block 0, wave 0 (no output depends on them).
__device__ unsigned long long g_band_stamps[512];
#define STAMP(i) do { const int si_ = (i); if (blockIdx.x == 0 && threadIdx.x == 0 && si_ < 512) g_band_stamps[si_] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define STAMP(i) do { } while (0)
#endif

template <int W, int B, bool REF>
__global__ __launch_bounds__((BPCfg<W, B>::THREADS), FCD_BAND_WAVES) void k_band_phase(
    const float2* __restrict__ Ab, int H, int nb, int NCA, int ncc0, int ncc1, const float* __restrict__ theta,
    float* __restrict__ out, const float2* __restrict__ pre, const float2* __restrict__ ptw) {
    using C = BPCfg<W, B>;
    constexpr int G = C::G, L = C::L, RL = C::RL, RP = C::RP, E = 16;
    extern __shared__ __attribute__((aligned(16))) float2 lds_b[];
    float2* const stage = lds_b;  // [B][SROW]
    const int team = threadIdx.x / RL, l = threadIdx.x % RL, g = l / G, t = l % G;
    float2* const ptl = lds_b + (size_t)B * SROW;  // pre-twiddles [q][RL]
    float* const s = reinterpret_cast<float*>(lds_b + C::XOFF) + (size_t)(team * L + g) * C::REGION;
    GroupFFT<B> fft;
    fft.load(ptw, t);
    for (int i = threadIdx.x; i < RL * E; i += C::THREADS) ptl[(i % E) * RL + i / E] = pre[i];
    const int rbs = H / BTILE;
    const int items = nb * 2 * rbs;
    // item -> (frame, carrier, row tile).  Frame-fastest order: the blocks running
    // at one time work on the same (carrier, row tile) of different frames, so the
    // tile's reference angles (64 KB) are read from HBM once and then hit in L2.
    auto item_f = [&](int blk) { return blk % nb; };
    auto item_c = [&](int blk) { return (blk / nb) % 2; };
    auto item_rb = [&](int blk) { return blk / (2 * nb); };
    // Tile staging is software-pipelined: the next item's tile is loaded into
    // registers (SPT values per thread, all loads in flight at once) while
    // the current item's rows are transformed.
    constexpr int SPT_ALL = (B * BTILE + C::THREADS - 1) / C::THREADS;
    constexpr int SPT = SPT_ALL < 8 ? SPT_ALL : 8;  // prefetched per thread (VGPR budget); the rest loads at staging
    const int tile_n = NCA * BTILE;
    float2 pf[SPT];
    auto tile_src = [&](int blk) {
        const int f = item_f(blk), c = item_c(blk), rb = item_rb(blk);
        return Ab + (((long)f * 2 + c) * rbs + rb) * (long)tile_n;
    };
    auto fetch = [&](int blk) {
        const float2* src = tile_src(blk);
#pragma unroll
        for (int i = 0; i < SPT; ++i) pf[i] = src[min((int)threadIdx.x + i * C::THREADS, tile_n - 1)];
    };
    // theta of the NEXT row this wave handles is loaded before the current row's
    // stores: vmcnt counts loads and stores in issue order, so a load issued after
    // a store batch cannot be waited for without waiting for those stores too.
    // theta is the lane-contiguous copy (band_theta_lanes): 16 floats per lane
    float th[E];
    auto th_load = [&](int blk, int rl) {
        if constexpr (!REF && FCD_BAND_NOTHETA) {
#pragma unroll
            for (int q = 0; q < E; ++q) th[q] = 0.f;
        } else if constexpr (!REF) {
            const int c = item_c(blk), rb = item_rb(blk);
            const float4* tr = reinterpret_cast<const float4*>(theta + ((long)c * H + rb * BTILE + rl) * W) + l * 4;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float4 v = tr[k];
                th[4 * k] = v.x;
                th[4 * k + 1] = v.y;
                th[4 * k + 2] = v.z;
                th[4 * k + 3] = v.w;
            }
        }
    };
    if ((int)blockIdx.x < items) {
        fetch(blockIdx.x);
        th_load(blockIdx.x, team);
    }
    [[maybe_unused]] int st = 0;
    for (int blk = blockIdx.x; blk < items; blk += gridDim.x) {
        const int f = item_f(blk), c = item_c(blk), rb = item_rb(blk);
        const int ncc = c ? ncc1 : ncc0;
        STAMP(st++);
        // slots [ncc, B) are staged as zeros: the transform input needs no select
        if constexpr (SPT_ALL > SPT) {
            const float2* src = tile_src(blk);
            for (int idx = threadIdx.x + SPT * C::THREADS; idx < B * BTILE; idx += C::THREADS)
                stage[(idx >> 4) * SROW + (idx & 15)] = idx < ncc * BTILE ? src[idx] : make_float2(0.f, 0.f);
        }
#pragma unroll
        for (int i = 0; i < SPT; ++i) {
            const int idx = threadIdx.x + i * C::THREADS;
            if (idx < B * BTILE)
                stage[(idx >> 4) * SROW + (idx & 15)] = idx < ncc * BTILE ? pf[i] : make_float2(0.f, 0.f);
        }
        __syncthreads();
        STAMP(st++);
        const int nblk = blk + (int)gridDim.x;
        if (nblk < items) fetch(nblk);
        for (int rl = team; rl < BTILE; rl += RP) {
            STAMP(st++);
            const int r = rb * BTILE + rl;
            const long row = ((long)f * 2 + c) * H + r;
            float thc[E];
#pragma unroll
            for (int q = 0; q < E; ++q) thc[q] = th[q];
            if (rl + RP < BTILE)
                th_load(blk, rl + RP);
            else if (nblk < items)
                th_load(nblk, team);
            float2 x[E];
            if constexpr (FCD_BAND_ABL & 4) {  // diagnostic: no staged-tile / pre-twiddle LDS reads
#pragma unroll
                for (int q = 0; q < E; ++q) x[q] = make_float2(thc[q], (float)(q + rl));
            } else {
#pragma unroll
                for (int q = 0; q < E; ++q) x[q] = cmul(stage[(t + G * q) * SROW + rl], ptl[q * RL + l]);
            }
            STAMP(st++);
            if constexpr (!(FCD_BAND_ABL & 1)) fft.template run_half<true>(x, s, t);  // 1: no transform
            STAMP(st++);
            float* o = out + row * W;
#if FCD_ATAN_N > 0
            if constexpr (!REF && !FCD_BAND_ABL) {
                // FCD_ATAN_N pixel pairs per interleaved group (wrapped_phase_pkn)
#pragma unroll
                for (int q0 = 0; q0 < E; q0 += 2 * FCD_ATAN_N) {
                    __builtin_amdgcn_sched_barrier(0);
                    fv2 tq[FCD_ATAN_N], wq[FCD_ATAN_N];
                    float2 uq[2 * FCD_ATAN_N];
#pragma unroll
                    for (int k = 0; k < FCD_ATAN_N; ++k) {
                        tq[k] = fv2{thc[q0 + 2 * k], thc[q0 + 2 * k + 1]};
                        uq[2 * k] = x[q0 + 2 * k];
                        uq[2 * k + 1] = x[q0 + 2 * k + 1];
                    }
                    wrapped_phase_pkn<FCD_ATAN_N>(tq, uq, wq);
#pragma unroll
                    for (int k = 0; k < FCD_ATAN_N; ++k) {
                        const int n = g + L * t + RL * (q0 + 2 * k);
                        if (!FCD_BAND_NOSTORE || wq[k].x == 1234.5f) {
                            st_stream(o + n, wq[k].x);
                            st_stream(o + n + RL, wq[k].y);
                        }
                    }
                }
            } else
#endif
            {
#pragma unroll
            for (int q = 0; q < E; q += 2) {  // pixel pairs: packed atan2 / wrap
                if (FCD_ATAN_GROUP && q % FCD_ATAN_GROUP == 0) __builtin_amdgcn_sched_barrier(0);  // bound the atan2 chains in flight
                const int n = g + L * t + RL * q;
                if constexpr (REF) {
                    const fv2 a = fast_atan2_pk(fv2{x[q].y, x[q + 1].y}, fv2{x[q].x, x[q + 1].x});
                    o[n] = a.x;
                    o[n + RL] = a.y;
                } else {
                    // wrap to [-pi, pi]: d - 2 pi rint(d / 2 pi), |d| < 2 pi
                    const fv2 w = (FCD_BAND_ABL & 2) ? fv2{x[q].x - thc[q], x[q + 1].x - thc[q + 1]}  // 2: no atan2
                                                     : wrapped_phase_pk(fv2{thc[q], thc[q + 1]}, x[q], x[q + 1]);
                    // streaming store (nt): the 8 N^2-byte phase stream must not evict
                    // the reference angles from the caches every frame
                    if (!FCD_BAND_NOSTORE || w.x == 1234.5f) {
                        st_stream(o + n, w.x);
                        st_stream(o + n + RL, w.y);
                    }
                }
            }
            }
            STAMP(st++);
        }
        __syncthreads();
    }
    STAMP(st++);
}

// ------------------------------------------------------------------ theta-resident form
// The same transform and phase step with the reference angles held in registers:
// one 1024-thread workgroup per CU, one wave per row of a 16-row tile, and an item
// = (carrier, row tile, slice of the frames).  The wave loads its row of theta once
// per item and reuses it for every frame of the slice, so the per-frame reference
// reads (8 MB per 1024^2 frame through L2 in k_band_phase) disappear; the tile of
// the next frame is prefetched into registers while the current one is
// transformed, and the two staging buffers alternate so one barrier per frame
// suffices.  The 16 waves of a frame write 16 consecutive rows (64 KB) of a
// phase plane.
#ifndef FCD_BAND_RESIDENT
#define FCD_BAND_RESIDENT 1  // 0: k_band_phase for every launch
#endif
#ifndef FCD_BAND_RES_ITEMS
#define FCD_BAND_RES_ITEMS 1  // target items per CU (frame slices = items * CUs / (2 * row tiles)); 1: c2 demod group 1101-1115 -> 1081-1093 us, c3 -1.5 % (4 before, r06 it2)
#endif
// Phase stores of the theta-resident kernel: streaming (nt) or plain.  With two waves per
// row (2048) a wave's store covers 16-byte pieces of every 32-byte sector (groups 0-3 of
// each 8, the other wave groups 4-7), so streaming stores leave the HBM partial sectors;
// plain ones merge both halves in the L2 first.
#ifndef FCD_BAND_RES_STORE
#define FCD_BAND_RES_STORE 0  // 0: plain where two waves share a row, streaming otherwise; 1: always streaming; 2: always plain
#endif
#ifndef FCD_BAND_RES_ROWS
#define FCD_BAND_RES_ROWS 16  // rows per item (waves per workgroup): 16 = one Ab tile; 8 = half a tile, two workgroups per CU (same speed, kbench r02ap)
#endif

#ifndef FCD_BAND_QUAD
#define FCD_BAND_QUAD 1  // 256-bin window: the quarter-wave groups' neighbouring pixels transposed into float4 stores
#endif
#ifndef FCD_FOLD_ROWS
#define FCD_FOLD_ROWS 4  // rows per item of the folded 4096-point band kernel (4 waves each)
#endif
#ifndef FCD_FOLD_PREF
#define FCD_FOLD_PREF 0  // its pre-twiddles as factors ([RL] + [L][16]: 4 KB instead of 32 KB)
#endif

template <int W, int B, int ROWS, int FOLD = 1>
struct BRCfg {
    static_assert(FOLD == 1 || FOLD == 2, "staged band of B or 2 B bins");
    static constexpr int G = B / 16, L = W / B, RL = W / 16;
    static constexpr int SB = FOLD * B;     // staged band bins (FOLD = 2: two B-bin halves folded per group)
    static_assert(RL == 64 || RL == 128 || RL == 256, "one, two or four waves per row");
    static_assert(BTILE % ROWS == 0, "items cover whole or half Ab tiles");
    static constexpr int THREADS = ROWS * RL;
    static constexpr int SR = ROWS + 1;     // staged row pitch (complex)
    static constexpr int REGION = GSched<B>::REGION;
    static constexpr int STAGE = SB * SR;   // float2 per staging buffer
    static constexpr int TN = SB * ROWS;    // staged slots per item tile
    static constexpr int SPT = (TN + THREADS - 1) / THREADS;
    static constexpr int NBUF = 2;  // staging buffers
    // pre-twiddles exp(2 pi i (t + G q) g / W): the [16][RL] table, or at 4096-point rows its
    // factors exp(2 pi i t g / W) (per lane, in registers) and exp(2 pi i G q g / W) ([L][16]),
    // the same product k_phase_rows_wide's REF mode forms for the reference angles
    static constexpr bool PREF = W == 4096 && FCD_FOLD_PREF;
    static constexpr int PRE = PREF ? RL + L * 16 : RL * 16;
    static constexpr size_t XOFF = (size_t)(NBUF * STAGE + PRE) * 8;  // exchange regions (bytes)
    static constexpr size_t LDS = XOFF + (size_t)ROWS * L * REGION * 4;
};

template <int W, int B, int ROWS, int FOLD = 1>
__global__ __launch_bounds__((BRCfg<W, B, ROWS, FOLD>::THREADS), 1) void k_band_phase_res(
    const float2* __restrict__ Ab, int H, int nb, int NCA, int ncc0, int ncc1, const float* __restrict__ theta,
    float* __restrict__ out, const float2* __restrict__ pre, const float2* __restrict__ ptw, int slices) {
    using C = BRCfg<W, B, ROWS, FOLD>;
    constexpr int G = C::G, L = C::L, RL = C::RL, E = 16, SPT = C::SPT, TN = C::TN, SR = C::SR;
    constexpr int HALVES = BTILE / ROWS;  // item tiles per Ab tile
    extern __shared__ __attribute__((aligned(16))) float2 lds_b[];
    float2* const stage0 = lds_b;                // [NBUF][SB][SR]
    float2* const ptl = lds_b + C::NBUF * C::STAGE;  // pre-twiddles [q][RL] (PREF: [RL] + [L][16])
    const int rl = threadIdx.x / RL;             // this wave's (or wave pair's) row of the tile
    const int l = threadIdx.x % RL, g = l / G, t = l % G;
    float* const s = reinterpret_cast<float*>(lds_b) + C::XOFF / 4 + (size_t)(rl * L + g) * C::REGION;
    GroupFFT<B> fft;
    fft.load(ptw, t);
    // FOLD = 2: group g's input is A[j] + w_g A[j + B] (times the pre-twiddle of j), w_g =
    // exp(2 pi i B g / W), the 2 B-bin band folded onto one B-point transform per group
    float2 om = make_float2(1.f, 0.f);
    if constexpr (FOLD == 2) {
        double sn, cs;
        sincospi(2.0 * (double)g * B / W, &sn, &cs);
        om = make_float2((float)cs, (float)sn);
    }
    float2 pb = make_float2(1.f, 0.f);
    if constexpr (C::PREF) {  // pre[l][q]: q = 0 gives exp(2 pi i t g / W), t = 0 the G q g factor
        pb = pre[(long)l * 16];
        for (int i = threadIdx.x; i < L * 16; i += C::THREADS) ptl[RL + i] = pre[(long)(i / 16) * G * 16 + i % 16];
    } else {
        for (int i = threadIdx.x; i < RL * E; i += C::THREADS) ptl[(i % E) * RL + i / E] = pre[i];
    }
    const int rbs = H / BTILE, rts = H / ROWS;
    const int per = (nb + slices - 1) / slices;
    const int items = 2 * rts * slices;
    const int tile_n = NCA * BTILE;
    // item -> (slice fastest, carrier, row tile); frames [f0, f1) of the slice.
    // Decoded once per item (the divisions by `slices` stay off the per-frame path).
    struct Item {
        int it, c, rt, f0, f1;
    };
    auto decode = [&](int it) {
        Item d;
        const int q = it / slices;
        d.it = it;
        d.c = q % 2;
        d.rt = q / 2;
        d.f0 = (it - q * slices) * per;
        d.f1 = min(nb, d.f0 + per);
        return d;
    };
    // the block's first non-empty item at or after `it`
    auto seek = [&](int it) {
        Item d = decode(it < items ? it : 0);
        for (; it < items; it += gridDim.x) {
            d = decode(it);
            if (d.f0 < d.f1) return d;
        }
        d.it = items;
        return d;
    };
    // the item's rows of Ab tile rb: slot (j, r) at j * BTILE + hb * ROWS + r
    float2 pf[SPT];
    auto fetch = [&](const Item& d, int f) {
        const float2* src = Ab + (((long)f * 2 + d.c) * rbs + d.rt / HALVES) * (long)tile_n + (d.rt % HALVES) * ROWS;
#pragma unroll
        for (int i = 0; i < SPT; ++i) {
            const int idx = min((int)threadIdx.x + i * C::THREADS, TN - 1);
            // issued here, ahead of the frame's phase stores (the compiler would sink a plain
            // load to its use after them); awaited by the explicit wait in front of stage_in
            pf[i] = load_async(src + min(idx / ROWS, NCA - 1) * BTILE + idx % ROWS);  // past the band: zeroed at staging
        }
    };
    // one row of one (item, frame): this wave's transform, phase step and stores
    auto row_step = [&](const float2* st, const float (&th)[E], int c, int row, int f) {
        float2 x[E];
#pragma unroll
        for (int q = 0; q < E; ++q) {
            float2 a = st[(t + G * q) * SR + rl];
            if constexpr (FOLD == 2) a = cadd(a, cmul(om, st[(t + G * q + B) * SR + rl]));
            x[q] = cmul(a, C::PREF ? cmul(pb, ptl[RL + g * 16 + q]) : ptl[q * RL + l]);
        }
        fft.template run_half<true>(x, s, t);
        float* o = out + (((long)f * 2 + c) * H + row) * W;
#pragma unroll
        for (int q0 = 0; q0 < E; q0 += 2 * FCD_ATAN_N) {
            __builtin_amdgcn_sched_barrier(0);
            fv2 tq[FCD_ATAN_N], wq[FCD_ATAN_N];
            float2 uq[2 * FCD_ATAN_N];
#pragma unroll
            for (int k = 0; k < FCD_ATAN_N; ++k) {
                tq[k] = fv2{th[q0 + 2 * k], th[q0 + 2 * k + 1]};
                uq[2 * k] = x[q0 + 2 * k];
                uq[2 * k + 1] = x[q0 + 2 * k + 1];
            }
            wrapped_phase_pkn<FCD_ATAN_N>(tq, uq, wq);
            if constexpr (G == 16 && FCD_ATAN_N == 2 && FCD_BAND_QUAD) {
                // 256-bin groups are quarter waves: groups g0 .. g0 + 3 (lane rows 0-3) hold
                // the four neighbouring pixels g0 + j + L t.  A 4 x 4 transpose of slots
                // q0 .. q0 + 3 across the lane rows (permlane32 then permlane16 half
                // exchanges) gives lane row j the four pixels of slot q0 + j: float4 stores
                unsigned a0 = __float_as_uint(wq[0].x), a1 = __float_as_uint(wq[0].y);
                unsigned a2 = __float_as_uint(wq[1].x), a3 = __float_as_uint(wq[1].y);
                auto r = __builtin_amdgcn_permlane32_swap(a0, a2, false, false);
                a0 = r[0];
                a2 = r[1];
                r = __builtin_amdgcn_permlane32_swap(a1, a3, false, false);
                a1 = r[0];
                a3 = r[1];
                r = __builtin_amdgcn_permlane16_swap(a0, a1, false, false);
                a0 = r[0];
                a1 = r[1];
                r = __builtin_amdgcn_permlane16_swap(a2, a3, false, false);
                a2 = r[0];
                a3 = r[1];
                const float4 v = make_float4(__uint_as_float(a0), __uint_as_float(a1), __uint_as_float(a2), __uint_as_float(a3));
                const int j = g & 3;
                if (!FCD_BAND_NOSTORE || v.x == 1234.5f)
                    *reinterpret_cast<float4*>(o + (g - j) + L * t + RL * (q0 + j)) = v;
                continue;
            }
#pragma unroll
            for (int k = 0; k < FCD_ATAN_N; ++k) {
                const int n = g + L * t + RL * (q0 + 2 * k);
                constexpr bool NT = FCD_BAND_RES_STORE == 1 || (FCD_BAND_RES_STORE == 0 && RL == 64);
                if constexpr (FCD_BAND_NOSTORE) {
                    if (wq[k].x == 1234.5f) o[n] = wq[k].y;
                } else if constexpr (NT) {
                    st_stream(o + n, wq[k].x);
                    st_stream(o + n + RL, wq[k].y);
                } else {
                    o[n] = wq[k].x;
                    o[n + RL] = wq[k].y;
                }
            }
        }
    };
    auto load_theta = [&](float (&th)[E], int c, int row) {  // lane-contiguous copy
        const float4* tr = reinterpret_cast<const float4*>(theta + ((long)c * H + row) * W) + l * 4;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float4 v = tr[k];
            th[4 * k] = v.x;
            th[4 * k + 1] = v.y;
            th[4 * k + 2] = v.z;
            th[4 * k + 3] = v.w;
        }
    };
    auto stage_in = [&](float2* st, int ncc) {  // slots [ncc, B) staged as zeros
#pragma unroll
        for (int i = 0; i < SPT; ++i) {
            const int idx = threadIdx.x + i * C::THREADS;
            if (idx < TN) st[(idx / ROWS) * SR + idx % ROWS] = idx < ncc * ROWS ? pf[i] : make_float2(0.f, 0.f);
        }
    };
    Item cur = seek(blockIdx.x);
    if (cur.it >= items) return;
    int f = cur.f0;
    fetch(cur, f);
    float th[E];
    load_theta(th, cur.c, cur.rt * ROWS + rl);  // kept for the item's frames (the compiler waits for them)
    wait_vmcnt_for<0>(pf);                       // the tile
    int buf = 0;
    stage_in(stage0, cur.c ? ncc1 : ncc0);
    // Steady state (FCD_BAND_RES_ROTATED): the next frame's tile is loaded BEFORE this
    // frame's phase stores and staged AFTER them, on a path with no other order of memory
    // operations, so the wait for the tile (vmcnt counts stores too, in issue order) leaves
    // the stores in flight.  The loop entered at its top with the first tile staged above
    // otherwise merges the first iteration's state (only the tile outstanding) into the
    // wait: vmcnt(0), every wave waiting for its previous row's store acknowledgements
    // before each frame's barrier.  The next item's reference angles are loaded after the
    // stores (waited for at their first use, once per item).
    while (true) {
        __syncthreads();  // stage(buf) complete; stage(buf ^ 1) last read before the previous barrier
        const Item itc = cur;
        const int fcur = f;
        const bool fresh = f + 1 >= cur.f1;
        if (fresh) {
            cur = seek(cur.it + gridDim.x);
            f = cur.f0;
        } else {
            ++f;
        }
        const bool more = cur.it < items;
        // (unconditional: a conditional load would merge a path without it into the
        // compiler's count, and the waits would fall back to vmcnt(0))
        fetch(more ? cur : itc, more ? f : fcur);
        row_step(stage0 + buf * C::STAGE, th, itc.c, itc.rt * ROWS + rl, fcur);
        if (!more) break;
        if (fresh) {
            load_theta(th, cur.c, cur.rt * ROWS + rl);
            // waited for here, once per item (with the stores before it), so that no
            // per-frame wait on the non-fresh path counts a pending angle load
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        buf ^= 1;
        // the tile's SPT loads were followed by this row's E phase stores: vmcnt(E) (the
        // counter retires in issue order) leaves the stores in flight
        wait_vmcnt_for<E>(pf);
        stage_in(stage0 + buf * C::STAGE, cur.c ? ncc1 : ncc0);
    }
}

static int band_res_slices(int H, int nb, int rows) {
    const int ncu = device_cu_count();  // (atomic cache: launchers run from two host threads)
    const int tiles = 2 * (H / rows);
    const int want = (FCD_BAND_RES_ITEMS * ncu + tiles - 1) / tiles;
    return std::max(1, std::min(nb, want));
}

#ifdef FCD_STAMPS
extern "C" int fcd_debug_band_stamps(unsigned long long* out) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_band_stamps), sizeof(g_band_stamps));
}
#endif

// theta [rows][W] (natural order, the REF output) -> the lane-contiguous copy
// the phase kernels read: row element g + L t + RL q (lane l = G g + t of the
// row's RL = W / 16 lanes) at l * 16 + q.
__global__ __launch_bounds__(256) void k_theta_lanes(const float* __restrict__ theta, long n, int W, int B,
                                                     float* __restrict__ thp) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;  // destination index
    if (i >= n) return;
    const long row = i / W;
    const int e = (int)(i % W), l = e / 16, q = e % 16;
    const int G = B / 16, L = W / B, RL = W / 16;
    thp[i] = theta[row * W + (l / G) + L * (l % G) + RL * q];
}

void band_theta_lanes(int W, int B, const float* theta, int rows, float* thp, hipStream_t s) {
    const long n = (long)rows * W;
    hipLaunchKernelGGL(k_theta_lanes, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, theta, n, W, B, thp);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) throw std::runtime_error(std::string("band_theta_lanes launch: ") + hipGetErrorString(e));
}

// ------------------------------------------------------------------ launchers
static int band_grid(long items, int per_cu) {
    const int ncu = device_cu_count();  // (atomic cache: launchers run from two host threads)
    const long cap = (long)ncu * per_cu;
    return (int)(items < cap ? (items > 0 ? items : 1) : cap);
}

template <int W, int B>
static void launch_band(bool ref, const float2* Ab, int H, int nb, int NCA, int ncc0, int ncc1, const float* theta,
                        float* out, const float2* pre, const float2* ptw, hipStream_t s) {
    using C = BPCfg<W, B>;
    const size_t lds = C::LDS;
    const int per_cu = (int)std::max<size_t>(1, std::min<size_t>(8, (160 * 1024) / lds));
    const int grid = band_grid((long)nb * 2 * (H / BTILE), per_cu);
    if (ref) {
        if (lds > 64 * 1024)
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_band_phase<W, B, true>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL((k_band_phase<W, B, true>), dim3(grid), dim3(C::THREADS), lds, s, Ab, H, nb, NCA, ncc0,
                           ncc1, theta, out, pre, ptw);
    } else {
        if constexpr ((W == 1024 || W == 2048) && B <= W / 8 && FCD_BAND_RESIDENT && FCD_ATAN_N > 0 && !FCD_BAND_ABL &&
                      !FCD_BAND_NOSTORE && !FCD_BAND_NOTHETA) {
            {
                // rows per item: 1024 threads at most (2048-point rows take two waves)
                constexpr int ROWS = FCD_BAND_RES_ROWS * (W / 16) <= 1024 ? FCD_BAND_RES_ROWS : 1024 / (W / 16);
                using R = BRCfg<W, B, ROWS>;
                const int slices = band_res_slices(H, nb, ROWS);
                const int items = 2 * (H / ROWS) * slices;
                static_assert(R::LDS <= 160 * 1024, "resident band kernel LDS");
                (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_band_phase_res<W, B, ROWS>),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)R::LDS);
                hipLaunchKernelGGL((k_band_phase_res<W, B, ROWS>), dim3(band_grid(items, (int)std::max<size_t>(1, (160 * 1024) / R::LDS))),
                                   dim3(R::THREADS), R::LDS, s, Ab,
                                   H, nb, NCA, ncc0, ncc1, theta, out, pre, ptw, slices);
                const hipError_t e = hipGetLastError();
                if (e != hipSuccess) throw std::runtime_error(std::string("band_phase_res launch: ") + hipGetErrorString(e));
                return;
            }
        }
        if (lds > 64 * 1024)
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_band_phase<W, B, false>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL((k_band_phase<W, B, false>), dim3(grid), dim3(C::THREADS), lds, s, Ab, H, nb, NCA, ncc0,
                           ncc1, theta, out, pre, ptw);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) throw std::runtime_error(std::string("band_phase launch: ") + hipGetErrorString(e));
}

template <int W>
static void band_dispatch_b(int B, bool ref, const float2* Ab, int H, int nb, int NCA, int ncc0, int ncc1,
                            const float* theta, float* out, const float2* pre, const float2* ptw, hipStream_t s) {
    switch (B) {
        case 16: if constexpr (W >= 32) { launch_band<W, 16>(ref, Ab, H, nb, NCA, ncc0, ncc1, theta, out, pre, ptw, s); return; } break;
        case 32: if constexpr (W >= 64) { launch_band<W, 32>(ref, Ab, H, nb, NCA, ncc0, ncc1, theta, out, pre, ptw, s); return; } break;
        case 64: if constexpr (W >= 128) { launch_band<W, 64>(ref, Ab, H, nb, NCA, ncc0, ncc1, theta, out, pre, ptw, s); return; } break;
        case 128: if constexpr (W >= 256) { launch_band<W, 128>(ref, Ab, H, nb, NCA, ncc0, ncc1, theta, out, pre, ptw, s); return; } break;
        case 256: if constexpr (W >= 512) { launch_band<W, 256>(ref, Ab, H, nb, NCA, ncc0, ncc1, theta, out, pre, ptw, s); return; } break;
        default: break;
    }
    throw std::runtime_error("band_phase: unsupported band window " + std::to_string(B) + " for row length " +
                             std::to_string(W));
}

// 4096-point rows with a band of up to 512 bins: the theta-resident kernel at B = 256 with the
// two 256-bin halves folded per group (16 groups of 256-point transforms, one exchange each,
// float4 stores), pre / ptw the B = 256 tables, theta in the B = 256 lane order
void band_phase_fold(int W, const float2* Ab, int H, int nb, int NCA, int ncc0, int ncc1, const float* theta,
                     float* out, const float2* pre, const float2* ptw, hipStream_t s) {
    if (W != 4096 || ncc0 > 512 || ncc1 > 512 || H % BTILE != 0)
        throw std::runtime_error("band_phase_fold: 4096-point rows, bands of up to 512 bins");
    constexpr int ROWS = FCD_FOLD_ROWS;
    using R = BRCfg<4096, 256, ROWS, 2>;
    static_assert(R::LDS <= 160 * 1024, "folded band kernel LDS");
    const int slices = band_res_slices(H, nb, ROWS);
    const int items = 2 * (H / ROWS) * slices;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_band_phase_res<4096, 256, ROWS, 2>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)R::LDS);
    hipLaunchKernelGGL((k_band_phase_res<4096, 256, ROWS, 2>), dim3(band_grid(items, (int)((160 * 1024) / R::LDS))),
                       dim3(R::THREADS), R::LDS, s, Ab, H, nb, NCA, ncc0, ncc1, theta, out, pre, ptw, slices);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) throw std::runtime_error(std::string("band_phase_fold launch: ") + hipGetErrorString(e));
}

bool band_supported(int W, int B) { return B >= 16 && B <= 256 && 2 * B <= W && (B & (B - 1)) == 0; }

void band_phase(int W, int B, bool ref, const float2* Ab, int H, int nb, int NCA, int ncc0, int ncc1,
                const float* theta, float* out, const float2* pre, const float2* ptw, hipStream_t s) {
    switch (W) {
        case 64: band_dispatch_b<64>(B, ref, Ab, H, nb, NCA, ncc0, ncc1, theta, out, pre, ptw, s); break;
        case 128: band_dispatch_b<128>(B, ref, Ab, H, nb, NCA, ncc0, ncc1, theta, out, pre, ptw, s); break;
        case 256: band_dispatch_b<256>(B, ref, Ab, H, nb, NCA, ncc0, ncc1, theta, out, pre, ptw, s); break;
        case 512: band_dispatch_b<512>(B, ref, Ab, H, nb, NCA, ncc0, ncc1, theta, out, pre, ptw, s); break;
        case 1024: band_dispatch_b<1024>(B, ref, Ab, H, nb, NCA, ncc0, ncc1, theta, out, pre, ptw, s); break;
        case 2048: band_dispatch_b<2048>(B, ref, Ab, H, nb, NCA, ncc0, ncc1, theta, out, pre, ptw, s); break;
        case 4096: band_dispatch_b<4096>(B, ref, Ab, H, nb, NCA, ncc0, ncc1, theta, out, pre, ptw, s); break;
        default: throw std::runtime_error("band_phase: unsupported row length " + std::to_string(W));
    }
}

}  // namespace fcdk
