// Fused throughput kernel of the height-only path (fcd_process with no phase
// outputs, i.e. analyze.folder's use of compute_height_map, analyze.py:247-262):
//
//   band-pruned inverse row transforms of both carriers + phase   (fcd.py:118)
//   residue-free unwrap of both maps + its census                 (fcd.py:119)
//   phi0' + i*phi1' -> forward row FFT -> Zt tile                  (fourier.py:134)
//
// in ONE pass over each 8-row tile, so the wrapped phase maps (8 N^2 bytes per
// frame) never touch HBM.  One wave per row (W = 1024: 64 lanes x 16 values):
//
//   * band transform: kernels_band.hip's decomposition (8 pre-twiddled
//     128-point group FFTs per row), exchange in the row's own LDS slot;
//   * unwrap: the row's wrapped values go blocked (16 consecutive pixels per
//     lane) through the slot; h = find_wrap of horizontal neighbours (f32 with
//     the +-fl(pi) ambiguity flag), one wave-wide DPP scan gives
//     k'(r, c) = -sum_{c' < c} h(r, c'), phi' = w + 2 pi k' (k'(r, 0) = 0);
//   * the column-0 offsets colk(r) are NOT applied here: they add the constant
//     2 pi colk(r) (+ i ...) to row r, i.e. 2 pi W colk(r) to its spectrum's
//     DC bin only, which k_int_cols applies (colk from k_colk_side over the
//     column-0 values this kernel writes);
//   * census: the unwrap is the unique residue-free one iff every vertical
//     edge is consistent (int_rows.inc): |phi'(r+1,c) - phi'(r,c) + 2 pi d(r)|
//     <= pi - margin with d(r) = colk(r+1) - colk(r) = -find_wrap(w(r,0),
//     w(r+1,0)) (exact, f64).  Edges inside the tile are checked here; the
//     tile's first and last unwrapped rows go to a seam buffer and
//     k_seam_check checks the edges between tiles (no halo recompute, and
//     8 waves = exactly 2 per SIMD);
//   * z-row FFT: a 1024-point wave-local group FFT (16 x 16 x 4, twiddles from
//     an LDS table) in the slot, then the tile leaves as whole 64-byte lines.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "gfft.hpp"
#include "kernels.hpp"

namespace fcdk {

namespace {

constexpr int PR_W = 1024;            // row length of the fused kernel
constexpr int PR_B = 128;             // band window
#ifndef FCD_PR_ROWS
#define FCD_PR_ROWS 8
#endif
constexpr int PR_ROWS = FCD_PR_ROWS;  // rows per tile (one wave each)
#if !defined(FCD_DIAGNOSTIC) && defined(FCD_PR_ABL)
#error "FCD_PR_ABL ablations are diagnostic-only: build with -DFCD_DIAGNOSTIC"
#endif
#ifndef FCD_PR_ABL
#define FCD_PR_ABL 0  // diagnostic ablations only (wrong results): 1 no reference-angle loads, 2 no Zt stores,
                      // 4 no band transforms, 8 no atan2 / wrap, 16 no z-row FFT
#endif
#ifndef FCD_PR_ATAN_N
#define FCD_PR_ATAN_N 2  // pixel pairs per carrier in one interleaved atan2 group
#endif
static_assert(FCD_PR_ATAN_N > 0 && 16 % (2 * FCD_PR_ATAN_N) == 0, "atan2 groups tile the 16 values");
constexpr int PR_ZT = zt_layout(1024);  // Zt tile height (kernels.hpp zt_layout: k_int_cols / k_int_rows2 read it)
static_assert(PR_ZT == FCD_ZT_1024, "the fused 1024 kernel writes the layout zt_layout(1024) names");
static_assert(PR_ZT % PR_ROWS == 0, "a tile covers part of one Zt tile");
constexpr int PR_WAVES = PR_ROWS;     // one wave per row
constexpr int PR_THREADS = 64 * PR_WAVES;
constexpr int PR_G = PR_B / 16, PR_L = PR_W / PR_B;
constexpr int PR_SLOT = padded_len(PR_W) + 2;  // as int_rows.inc: == 2 (mod 32)
constexpr int PR_SROW = PR_ROWS + 1;           // staged band rows (odd pitch)
constexpr int PR_ZTAB = GSched<PR_W>::TABLE;   // 1008 twiddles of the 1024-point group FFT
// LDS carve (float2 units)
constexpr int OFF_STAGE = 0;                                   // [2][B][SROW]
constexpr int OFF_PRE = OFF_STAGE + 2 * PR_B * PR_SROW;        // [16][64] pre-twiddles
constexpr int OFF_ZTAB = OFF_PRE + 16 * 64;                    // z-FFT twiddles
constexpr int OFF_BTAB = OFF_ZTAB + PR_ZTAB;                   // band-FFT twiddles
constexpr int OFF_SLOT = (OFF_BTAB + GSched<PR_B>::TABLE + 1) & ~1;  // 16-byte aligned slots
constexpr int OFF_PREV = OFF_SLOT + PR_WAVES * PR_SLOT;              // last unwrapped row of the previous tile
constexpr size_t PR_LDS = (size_t)(OFF_PREV + PR_SLOT) * 8;
static_assert(PR_LDS <= 160 * 1024, "fused kernel LDS");
static_assert(PR_L * GSched<PR_B>::REGION <= PR_SLOT, "band exchange must fit the slot");
static_assert(2 * PR_L * GSched<PR_B>::REGION <= 2 * PR_SLOT, "paired float-half band exchange must fit the slot");

constexpr float kTwoPiF = 6.28318530717959f;
constexpr float kPR_VLim = 3.14159265f - 4e-3f;

__device__ __forceinline__ int fw_exact(float a, float b) {
    const double d = (double)a - (double)b;
    return d > 3.141592653589793 ? -1 : (d < -3.141592653589793 ? 1 : 0);
}

}  // namespace

#ifdef FCD_STAMPS
// diagnostic: per-phase cycle totals of block 0, per wave (tools/prstamp.cpp)
__device__ unsigned long long g_pr_stamps[PR_WAVES * 16];
#define PR_STAMP(i)                                                    \
    do {                                                               \
        const unsigned long long t_ = __builtin_readcyclecounter();   \
        ph[(i)] += t_ - tprev;                                         \
        tprev = t_;                                                    \
    } while (0)
#else
#define PR_STAMP(i) \
    do {            \
    } while (0)
#endif

#ifndef FCD_PR_ASYNC
#define FCD_PR_ASYNC 1  // counted waits for the tile / angle loads (fetch); 0: the compiler's waits
#endif
#ifndef FCD_PR_MINB
#define FCD_PR_MINB 1  // workgroups per CU the register allocation must allow (launch-bounds)
#endif
template <bool UNWRAP>
__global__ __launch_bounds__(PR_THREADS, FCD_PR_MINB) void k_phase_rows(
    const float2* __restrict__ Ab, int H, int nb, int NCA, int ncc0, int ncc1, const float* __restrict__ theta,
    const float2* __restrict__ pre, const float2* __restrict__ ptw, const float2* __restrict__ ztw,
    float* __restrict__ col0, int* __restrict__ flags, float2* __restrict__ Zt, float2* __restrict__ seam, int per) {
    extern __shared__ __attribute__((aligned(16))) float2 lds_p[];
    float2* const stage = lds_p + OFF_STAGE;
    float2* const ptl = lds_p + OFF_PRE;
    float2* const ztab = lds_p + OFF_ZTAB;
    float2* const btab = lds_p + OFF_BTAB;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int g = lane / PR_G, t = lane % PR_G;  // band group / lane in group
    // LDS slot of row w of the tile (PR_SLOT float2, padded): the last row
    // alternates between two slots, so the previous tile's last unwrapped row
    // survives for the census against this tile's first row (k = tile parity)
    auto row_slot = [&](int w, int k) {
        return lds_p + (w == PR_ROWS - 1 && k ? OFF_PREV : OFF_SLOT + w * PR_SLOT);
    };
    for (int i = threadIdx.x; i < GSched<PR_B>::TABLE; i += PR_THREADS) btab[i] = ptw[i];
    for (int i = threadIdx.x; i < 16 * 64; i += PR_THREADS) ptl[(i % 16) * 64 + i / 16] = pre[i];
    for (int i = threadIdx.x; i < PR_ZTAB; i += PR_THREADS) ztab[i] = ztw[i];
    const int rbs = H / PR_ROWS;
    const int items = nb * rbs;
    const int tiles16 = H / 16;
    // Each block takes a contiguous range of `per` consecutive tiles: consecutive tiles of a
    // frame are checked against each other here, only the range edges go to k_seam_check.
    // (A dynamic schedule -- chunks of tiles from a counter -- measured 80.0-81.6 k vs
    // 80.1-81.0 k frames/s static, r03t, and was removed.)
    const int nch = (items + per - 1) / per;
    const int ch = blockIdx.x;
    // staged band values of the next item, prefetched into registers: entry
    // e = (c, j, row) with row fastest, 8 rows = one 64-byte run of Ab's 16-row tile
    constexpr int NST = 2 * PR_B * PR_ROWS;
    constexpr int SPT = (NST + PR_THREADS - 1) / PR_THREADS;
    float2 pf[SPT];
    // (FCD_PR_ASYNC) the loads issue where they stand and are awaited by explicit counted
    // waits (fft_lds.hpp load_async): the tile of the next item before this item's Zt
    // stores, so its wait at the bottom of the loop leaves those stores in flight -- the
    // compiler's own waits merged the loop's entry path into vmcnt(0) there, and counted the
    // next tile's loads into the wait for the reference angles.  Band slots past the
    // carrier's columns load a valid in-band value and are zeroed at staging.
    auto fetch = [&](int blk) {
        const int f = blk / rbs, rb = blk % rbs;
        const int r = rb * PR_ROWS + (threadIdx.x % PR_ROWS);
#pragma unroll
        for (int i = 0; i < SPT; ++i) {
            const int e = threadIdx.x + i * PR_THREADS;
            const int c = e / (PR_B * PR_ROWS), j = (e / PR_ROWS) % PR_B;
            if constexpr (FCD_PR_ASYNC) {
                const int cc = (NST % PR_THREADS == 0 || e < NST) ? c : 0;
                const int jj = min(j, (cc ? ncc1 : ncc0) - 1);
                pf[i] = load_async(Ab + ((((long)f * 2 + cc) * tiles16 + (r >> 4)) * NCA + max(jj, 0)) * 16 + (r & 15));
            } else {
                float2 v = make_float2(0.f, 0.f);
                if ((NST % PR_THREADS == 0 || e < NST) && j < (c ? ncc1 : ncc0))
                    v = Ab[((((long)f * 2 + c) * tiles16 + (r >> 4)) * NCA + j) * 16 + (r & 15)];
                pf[i] = v;
            }
        }
    };
    // the staged tile: slots past a carrier's band as zeros (FCD_PR_ASYNC loads them)
    auto stage_tile = [&]() {
#pragma unroll
        for (int i = 0; i < SPT; ++i) {
            const int e = threadIdx.x + i * PR_THREADS;
            const int c = e / (PR_B * PR_ROWS), j = (e / PR_ROWS) % PR_B;
            const bool live = !FCD_PR_ASYNC || j < (c ? ncc1 : ncc0);
            if (NST % PR_THREADS == 0 || e < NST) stage[(e / PR_ROWS) * PR_SROW + e % PR_ROWS] = live ? pf[i] : make_float2(0.f, 0.f);
        }
    };
    if (ch < nch) fetch(ch * per);
#ifdef FCD_STAMPS
    unsigned long long ph[16] = {}, tprev = __builtin_readcyclecounter();
#endif
    if (ch < nch) {
    const int it0 = ch * per, it1 = min(it0 + per, items);
    if constexpr (FCD_PR_ASYNC) {  // the first tile, staged ahead of the loop
        wait_vmcnt_for<0>(pf);
        stage_tile();
    }
    for (int blk = it0; blk < it1; ++blk) {
        const int f = blk / rbs, rb = blk % rbs;
        const int r = rb * PR_ROWS + wave;           // this wave's row
        const int par = (blk - it0) & 1;
        float2* const slot = row_slot(wave, par);    // band exchange, unwrapped row
        PR_STAMP(0);
        if constexpr (!FCD_PR_ASYNC) stage_tile();
        __syncthreads();
        PR_STAMP(1);
        if constexpr (!FCD_PR_ASYNC) {
            if (blk + 1 < it1) fetch(blk + 1);
        }
        PR_STAMP(2);
        // ---- band transforms of both carriers -> wrapped phases (natural strided)
        float w0[16], w1[16];
        {
            // the reference angles of this lane's 16 pixels, both carriers, issued
            // before the transforms: lane-contiguous in the permuted copy
            float4 th4[2][4];
            auto load_theta = [&]() {
                if constexpr (FCD_PR_ABL & 1) {  // diagnostic: no reference-angle loads
#pragma unroll
                    for (int c = 0; c < 2; ++c)
#pragma unroll
                        for (int k = 0; k < 4; ++k) th4[c][k] = make_float4(0.f, 0.f, 0.f, 0.f);
                    return;
                }
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    const float4* tp = reinterpret_cast<const float4*>(theta + ((long)c * H + r) * PR_W) + lane * 4;
#pragma unroll
                    for (int k = 0; k < 4; ++k) th4[c][k] = FCD_PR_ASYNC ? load_async4(tp + k) : tp[k];
                }
            };
            // both carriers' transforms in lockstep (GroupFFTTab2): float-half
            // exchange regions of the two carriers side by side in the slot
            float2 x0[16], x1[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const float2 p = ptl[q * 64 + lane];
                x0[q] = cmul(stage[(t + PR_G * q) * PR_SROW + wave], p);
                x1[q] = cmul(stage[(PR_B + t + PR_G * q) * PR_SROW + wave], p);
            }
            float* const sx = reinterpret_cast<float*>(slot);
            if (!(FCD_PR_ABL & 4))  // 4: no band transforms
            GroupFFTTab2<PR_B>::template run_half<true>(x0, x1, sx + g * GSched<PR_B>::REGION,
                                                       sx + (PR_L + g) * GSched<PR_B>::REGION, t, btab);
            PR_STAMP(3);
            load_theta();  // after the transforms: register pressure
            if constexpr (FCD_PR_ASYNC) {
                // the next item's tile behind the angles: the angles' wait leaves it in flight
                fetch(blk + 1 < it1 ? blk + 1 : blk);
                wait_vmcnt_for<SPT>(th4[0]);
                wait_vmcnt_for<SPT>(th4[1]);
            }
            // FCD_PR_ATAN_N pixel pairs of each carrier per interleaved group
            // (wrapped_phase_pkn: 2 * FCD_PR_ATAN_N independent chains)
#pragma unroll
            for (int q0 = 0; q0 < 16; q0 += 2 * FCD_PR_ATAN_N) {
                __builtin_amdgcn_sched_barrier(0);
                constexpr int NPG = 2 * FCD_PR_ATAN_N;
                fv2 tq[NPG], wq[NPG];
                float2 uq[2 * NPG];
#pragma unroll
                for (int m = 0; m < FCD_PR_ATAN_N; ++m) {
                    const int q = q0 + 2 * m, k = q / 4, e = q % 4;
                    tq[2 * m] = e == 0 ? fv2{th4[0][k].x, th4[0][k].y} : fv2{th4[0][k].z, th4[0][k].w};
                    tq[2 * m + 1] = e == 0 ? fv2{th4[1][k].x, th4[1][k].y} : fv2{th4[1][k].z, th4[1][k].w};
                    uq[4 * m] = x0[q];
                    uq[4 * m + 1] = x0[q + 1];
                    uq[4 * m + 2] = x1[q];
                    uq[4 * m + 3] = x1[q + 1];
                }
                if constexpr (FCD_PR_ABL & 8) {  // 8: no atan2 / wrap
#pragma unroll
                    for (int k = 0; k < NPG; ++k) wq[k] = tq[k] - fv2{uq[2 * k].x, uq[2 * k + 1].x};
                } else {
                    wrapped_phase_pkn<NPG>(tq, uq, wq);
                }
#pragma unroll
                for (int m = 0; m < FCD_PR_ATAN_N; ++m) {
                    const int q = q0 + 2 * m;
                    w0[q] = wq[2 * m].x;
                    w0[q + 1] = wq[2 * m].y;
                    w1[q] = wq[2 * m + 1].x;
                    w1[q + 1] = wq[2 * m + 1].y;
                }
            }
            PR_STAMP(4);
        }
        // ---- natural strided -> blocked through the slot
        wave_sync();
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int n = g + PR_L * t + 64 * q;
            slot[pad(n)] = make_float2(w0[q], w1[q]);
        }
        wave_sync();
        const int j0 = lane * 16;
        // both maps at once: pixel n of map 0 / 1 is slot[pad(n)].x / .y (64-bit LDS
        // accesses, the two maps' scans interleaved)
        int bad = 0;
        {
            float2 v[17];
#pragma unroll
            for (int j = 0; j < 16; ++j) v[j] = slot[pad(j0 + j)];
            v[16] = lane < 63 ? slot[pad(j0 + 16)] : make_float2(0.f, 0.f);
            if (lane == 0) {
                col0[((long)f * 2 + 0) * H + r] = v[0].x;
                col0[((long)f * 2 + 1) * H + r] = v[0].y;
            }
            if constexpr (UNWRAP) {
                // both maps as packed pairs: dd = -find_wrap(w(j), w(j+1)) = rint((w(j) -
                // w(j+1)) / 2 pi) for every f32 difference except +-fl(pi) (exhaustively
                // checked against the comparison form; +-fl(pi) is flagged ambiguous as
                // before), so k'(c) = sum_{c' < c} dd(c') accumulates in f32 (exact
                // small integers) and phi' = w + 2 pi k' is the same fma as before.
                if (lane == 63) v[16] = v[15];  // no edge past the row end: dd = 0
                fv2 dd[16];
                fv2 run = {0.f, 0.f};
                bool amb = false;
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const fv2 d = pv(v[j]) - pv(v[j + 1]);
                    amb |= (fabsf(d.x) == 3.14159274f) || (fabsf(d.y) == 3.14159274f);
                    const fv2 q = d * 0.159154943091895f;
                    dd[j] = fv2{rintf(q.x), rintf(q.y)};
                    run += dd[j];
                }
                // one wave scan of both maps' segment sums, biased by 16 per lane into
                // 16-bit halves (|run| <= 16, prefix <= 64 * 32 < 2^16)
                const int packed = ((int)run.x + 16) | (((int)run.y + 16) << 16);
                const int incl = team_scan_incl_dpp<64>(packed);
                const int excl = incl - packed;
                fv2 acc = {(float)((excl & 0xffff) - 16 * lane), (float)((excl >> 16) - 16 * lane)};
                wave_sync();  // every lane has read its neighbour's first value
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    slot[pad(j0 + j)] = vp(acc * kTwoPiF + pv(v[j]));
                    acc += dd[j];
                }
                bad |= amb;
            }
        }
        if constexpr (UNWRAP) {  // first and last unwrapped rows of the tile -> seam buffer (k_seam_check)
            if ((wave == 0 && blk == it0 && rb > 0) || (wave == PR_ROWS - 1 && blk == it1 - 1 && rb < rbs - 1)) {
                float4* sd = reinterpret_cast<float4*>(seam + (((long)f * (H / PR_ROWS) + rb) * 2 + (wave ? 1 : 0)) * PR_W +
                                                       j0);
#pragma unroll
                for (int j = 0; j < 16; j += 2) {
                    const float2 a = slot[pad(j0 + j)], b = slot[pad(j0 + j + 1)];
                    sd[j / 2] = make_float4(a.x, a.y, b.x, b.y);
                }
            }
        }
        PR_STAMP(5);
        __syncthreads();
        PR_STAMP(6);
        // ---- vertical census against the next row of the tile (seams: k_seam_check)
        if constexpr (UNWRAP) {
            if (wave < PR_ROWS - 1 || (blk > it0 && rb > 0)) {
                // rows (wave, wave + 1); the last wave: the previous tile's last row and row 0
                const bool up = wave == PR_ROWS - 1;
                const float2* a_row = up ? row_slot(PR_ROWS - 1, par ^ 1) : slot;
                const float2* nx = up ? row_slot(0, 0) : row_slot(wave + 1, par);
                const float2 a0 = a_row[0], b0 = nx[0];  // phi'(r, 0) = w(r, 0)
                const float d0 = kTwoPiF * (float)(-fw_exact(a0.x, b0.x));
                const float d1 = kTwoPiF * (float)(-fw_exact(a0.y, b0.y));
                // largest |b - a + d| of both maps (packed differences, one max3 per pixel)
                float m = 0.f;
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const fv2 e = (pv(nx[pad(j0 + j)]) - pv(a_row[pad(j0 + j)])) + fv2{d0, d1};
                    m = fmaxf(m, fmaxf(fabsf(e.x), fabsf(e.y)));
                }
                bad |= (int)(m > kPR_VLim);
            }
            if (__any(bad) && lane == 0) atomicOr(flags + f * 2, 1);
            PR_STAMP(7);
            __syncthreads();  // every census read of the next slot precedes that row's FFT
        }
        PR_STAMP(8);
        // ---- forward row FFT of phi0' + i phi1'
        {
            __builtin_amdgcn_sched_barrier(0);
            float2 x[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) x[q] = slot[pad(lane + 64 * q)];
            // the last row transforms in its other slot (the previous tile's row,
            // no longer needed): its unwrapped row stays for the next census
            float2* const zs = row_slot(wave, par ^ 1);
            if (!(FCD_PR_ABL & 16))  // 16: no z-row FFT
            GroupFFTTab<PR_W>::template run<false>(x, zs, lane, ztab);
            wave_sync();
#pragma unroll
            for (int q = 0; q < 16; ++q) zs[pad(lane + 64 * q)] = x[q];
        }
        PR_STAMP(9);
        __syncthreads();
        PR_STAMP(10);
        // ---- whole 64-byte tile lines: Zt[f][rb][j][0..8), j the mirror-paired column order
        {  // thread i writes physical column i / ROWS + 64 k, row i % ROWS
            const int r0 = rb * PR_ROWS;
            float2* dst = Zt + (long)f * H * PR_W + (long)(r0 / PR_ZT) * PR_W * PR_ZT + (r0 % PR_ZT);
            const int c0 = threadIdx.x / PR_ROWS, rl = threadIdx.x % PR_ROWS;
            const float2* src = row_slot(rl, par ^ 1);
#pragma unroll 4
            for (int k = 0; k < PR_W / 64; ++k) {
                const float2 v = src[pad(c0 + 64 * k)];
                if (!(FCD_PR_ABL & 2) || v.x == 1234.5f) st_stream(dst + (c0 + 64 * k) * PR_ZT + rl, v);  // 2: no Zt stores
            }
        }
        PR_STAMP(11);
        __syncthreads();
        PR_STAMP(12);
        if constexpr (FCD_PR_ASYNC) {
            // the next tile: its loads were followed by at least this item's PR_W / 64 Zt
            // stores, so vmcnt(PR_W / 64) has retired them and leaves the stores in flight
            static_assert(!(FCD_PR_ABL & 2), "the counted wait needs the Zt stores");
            wait_vmcnt_for<PR_W / 64>(pf);
            stage_tile();
        }
    }
    }
#ifdef FCD_STAMPS
    if (blockIdx.x == 0 && lane == 0)
        for (int i = 0; i < 16; ++i) g_pr_stamps[wave * 16 + i] = ph[i];
#endif
}

// Census of the edges between the tile ranges of k_phase_rows' blocks (the
// edges inside a range are checked there): the last row of tile it - 1 against
// the first row of tile it, it = k * per, both unwrapped without their
// column-0 offsets.  One wave per range edge; lane L holds pixels 16L .. 16L+15.
__global__ __launch_bounds__(256) void k_seam_check(const float2* __restrict__ seam, int H, int nb, int per,
                                                    int* __restrict__ flags) {
    const int rbs = H / PR_ROWS;
    const long it = ((long)blockIdx.x * 4 + (threadIdx.x >> 6) + 1) * per;
    if (it >= (long)nb * rbs || it % rbs == 0) return;
    const int f = (int)(it / rbs), b = (int)(it % rbs) - 1;
    const int lane = threadIdx.x & 63;
    const float4* a = reinterpret_cast<const float4*>(seam + (((long)f * rbs + b) * 2 + 1) * PR_W + lane * 16);
    const float4* c = reinterpret_cast<const float4*>(seam + (((long)f * rbs + b + 1) * 2 + 0) * PR_W + lane * 16);
    float4 av[8], cv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        av[j] = a[j];
        cv[j] = c[j];
    }
    // phi'(r, 0) = w(r, 0): the column-0 jump of the true unwrap, exactly
    const float a0x = __shfl(av[0].x, 0), a0y = __shfl(av[0].y, 0);
    const float c0x = __shfl(cv[0].x, 0), c0y = __shfl(cv[0].y, 0);
    const float d0 = kTwoPiF * (float)(-fw_exact(a0x, c0x));
    const float d1 = kTwoPiF * (float)(-fw_exact(a0y, c0y));
    int bad = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        bad |= (int)(fabsf(cv[j].x - av[j].x + d0) > kPR_VLim) | (int)(fabsf(cv[j].y - av[j].y + d1) > kPR_VLim);
        bad |= (int)(fabsf(cv[j].z - av[j].z + d0) > kPR_VLim) | (int)(fabsf(cv[j].w - av[j].w + d1) > kPR_VLim);
    }
    if (__any(bad) && lane == 0) atomicOr(flags + f * 2, 1);
}

#ifdef FCD_STAMPS
extern "C" __attribute__((visibility("default"))) int fcd_debug_pr_stamps(unsigned long long* out) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pr_stamps), sizeof(g_pr_stamps));
}
#endif

bool phase_rows_supported(int W, int B, int H) {
    if (H % 16 != 0 || H < 16) return false;
    if (W == 2048 && B == 256) return true;
    if (W == 4096 && B == 512) return true;
    return W == PR_W && B == PR_B;
}

int phase_rows_tile(int W) { return W == 2048 ? 4 : (W == 4096 ? 2 : PR_ROWS); }

// Blocks of k_phase_rows at 1024-point rows: the tiles split evenly over the blocks (one
// block per CU), each a contiguous range of `per` consecutive 8-row tiles.
static void pr_layout(int H, int nb, int& grid, int& per) {
    const int ncu = device_cu_count();  // (atomic cache: launchers run from two host threads)
    const long items = (long)nb * (H / PR_ROWS);
    const int per_cu = std::max<int>(1, std::min<int>(160 * 1024 / (int)PR_LDS, 16 / PR_WAVES));
    const int slots = (int)std::min<long>(items, (long)ncu * per_cu);
    grid = per = 0;
    if (slots <= 0) return;
    per = (int)((items + slots - 1) / slots);  // tiles per block, a contiguous range
    grid = (int)((items + per - 1) / per);
}

void phase_rows(int W, bool unwrap, const float2* Ab, int H, int nb, int NCA, int ncc0, int ncc1, const float* theta,
                const float2* pre, const float2* ptw, const float2* ztw, float* col0, int* flags, float2* Zt,
                float2* seam, hipStream_t s, bool defer_seam) {
    if (W == 2048 || W == 4096) {
        phase_rows_wide(W, unwrap, Ab, H, nb, NCA, ncc0, ncc1, theta, pre, ptw, ztw, col0, flags, Zt, seam, s,
                        defer_seam);
        return;
    }
    if (W != PR_W) throw std::runtime_error("phase_rows: unsupported row length");
    int grid, per;
    pr_layout(H, nb, grid, per);
    if (grid <= 0) return;
    if (unwrap) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_phase_rows<true>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)PR_LDS);
        hipLaunchKernelGGL(k_phase_rows<true>, dim3(grid), dim3(PR_THREADS), PR_LDS, s, Ab, H, nb, NCA, ncc0, ncc1,
                           theta, pre, ptw, ztw, col0, flags, Zt, seam, per);
        if (!defer_seam) phase_rows_seam(W, H, nb, seam, flags, s);
    } else {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_phase_rows<false>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)PR_LDS);
        hipLaunchKernelGGL(k_phase_rows<false>, dim3(grid), dim3(PR_THREADS), PR_LDS, s, Ab, H, nb, NCA, ncc0, ncc1,
                           theta, pre, ptw, ztw, col0, flags, Zt, seam, per);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) throw std::runtime_error(std::string("phase_rows launch: ") + hipGetErrorString(e));
}

void phase_rows_seam(int W, int H, int nb, const float2* seam, int* flags, hipStream_t s) {
    if (W == 2048 || W == 4096) {
        phase_rows_wide_seam(W, H, nb, seam, flags, s);
        return;
    }
    int grid, per;
    pr_layout(H, nb, grid, per);
    if (grid <= 0) return;
    const long items = (long)nb * (H / PR_ROWS);
    const long edges = (items + per - 1) / per - 1;  // range edges (those at frame starts return at once)
    if (edges > 0)
        hipLaunchKernelGGL(k_seam_check, dim3((unsigned)((edges + 3) / 4)), dim3(256), 0, s, seam, H, nb, per, flags);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) throw std::runtime_error(std::string("phase_rows seam check launch: ") + hipGetErrorString(e));
}

}  // namespace fcdk
