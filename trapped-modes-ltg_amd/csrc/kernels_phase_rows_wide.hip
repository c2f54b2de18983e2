// Fused throughput kernel of the height-only path at 2048- and 4096-point rows: the
// same chain as kernels_phase_rows.hip (the 1024-wide form, which cites the
// reference lines) --
//
//   band-pruned inverse row transforms of both carriers + phase   (fcd.py:118)
//   residue-free unwrap of both maps + its census                 (fcd.py:119)
//   phi0' + i*phi1' -> forward row FFT -> Zt tile                  (fourier.py:134)
//
// -- in one pass over each tile of rows, so the wrapped phase maps (8 N^2 bytes per
// frame: 33.5 MB at 2048^2, 134 MB at 4096^2) never touch HBM.  A row is NWR = W /
// 1024 waves (16 values per lane), a tile 4 rows at 2048 and 2 at 4096 (8 waves, one
// workgroup per CU in 139-141 KB of LDS):
//
//   * band transform (B = W / 8): 8 pre-twiddled B-point group FFTs per row, B / 16
//     lanes each (so a group never spans two waves), both carriers in lockstep,
//     float-half exchange in the row's slot;
//   * unwrap: 16 consecutive pixels per lane; each wave scans its quarter / half row
//     (packed pairs of both maps, one DPP scan) and stores it WITHOUT the lower waves'
//     totals, which go through LDS and are added where the row is read (census, seam
//     rows, z-row FFT input), so the scans need no barrier between them;
//   * census: vertical edges inside the tile here, the tile range edges in
//     k_seam_check_wide (as the 1024 form);
//   * z-row FFT: W = NWR x 1024 -- wave h transforms the samples NWR m + h (the
//     wave-local 1024-point group FFT), and the Zt write-out joins the NWR outputs with
//     one radix-NWR pass, X[k + 1024 j] = sum_h W_NWR^(h j) w^(h k) Y_h[k];
//   * Zt: the tile writes its rows' parts of the Zt tiles' column runs (8-row Zt tiles
//     at 2048, FCD_ZT_4096-row at 4096, kernels.hpp zt_layout); the next tiles of the block's
//     contiguous range writes the rest right after.
//
// REF = true (4096 only, once per reference): the band transforms of the reference's
// band with angle(y) written to theta_b (the reference angle of this decomposition,
// as kernels_band.hip's REF mode at narrower rows).
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#include "gfft.hpp"
#include "kernels.hpp"

namespace fcdk {

namespace {

#ifndef FCD_WIDE_NOTHETA
#define FCD_WIDE_NOTHETA 0  // diagnostic ablation only (wrong results): no reference-angle loads
#endif
#if FCD_WIDE_NOTHETA && !defined(FCD_DIAGNOSTIC)
#error "FCD_WIDE_NOTHETA is diagnostic-only: build with -DFCD_DIAGNOSTIC"
#endif
#ifndef FCD_WIDE_ZT_NT
#define FCD_WIDE_ZT_NT 1  // streaming Zt stores at 4096 too (fused 133.6 -> 131.4 us/frame, c5 +0.6 %, r06 te; 0: plain)
#endif
#ifndef FCD_WIDE_FOLD
#define FCD_WIDE_FOLD 1  // 4096: the 512-bin band as 16 folded 256-point groups (0: 8 groups of 512)
#endif
#ifndef FCD_WIDE_LOCKSTEP
#define FCD_WIDE_LOCKSTEP 1  // 4096: both carriers' band transforms in lockstep (GroupFFTTab2, as at 2048); 0: one after the other (c5 3.70 k vs 3.76 k, r06 wl)
#endif

template <int W>
struct WideCfg {
    static_assert(W == 2048 || W == 4096, "2048- or 4096-point rows");
    static constexpr int B = W / 8;                 // band window (staged bins per carrier)
    // transform length: B, or at 4096 (FCD_WIDE_FOLD) B / 2 with the band's two halves folded
    // per group (kernels_band.hip FOLD): 16 groups of 256 points, one exchange each
    static constexpr int BF = W == 4096 && FCD_WIDE_FOLD ? B / 2 : B;
    static constexpr int FOLD = B / BF;
    static constexpr int NWR = W / 1024;            // waves per row
    static constexpr int RL = W / 16;               // lanes per row
    static constexpr int ROWS = W == 2048 ? 4 : 2;  // rows per tile
    static constexpr int THREADS = ROWS * RL;       // 512
    static constexpr int G = BF / 16, L = W / BF;
    static constexpr int ZT = zt_layout(W);         // Zt layout tile height (kernels.hpp)
    static constexpr int SLOT = padded_len(W) + 2;  // row slot (float2), 16-byte multiple
    static constexpr int HALF = padded_len(1024);   // one wave's 1024-point region; pad(k + 1024 h) = pad(k) + h HALF
    static constexpr int SROW = ROWS + 1;           // staged band rows (odd pitch)
    static constexpr int ZTAB = GSched<1024>::TABLE;
    static constexpr int NCTW = (NWR - 1) * 1024;   // join twiddles w^(h k), h = 1..NWR-1
    // band pre-twiddles: the [16][RL] table in LDS at 2048; at 4096 (32 KB) its factors,
    // exp(2 pi i (t + G q) g / W) = exp(2 pi i t g / W) exp(2 pi i G q g / W): [RL] + [L][16]
    static constexpr bool PRE_LDS = W == 2048;
    static constexpr bool CTW_LDS = W == 2048;      // join twiddles in LDS (else read from L2)
    static constexpr bool SEQ = W == 4096 && !FCD_WIDE_LOCKSTEP;  // the carriers' band transforms one after the other
    // LDS carve (float2 units)
    static constexpr int OFF_STAGE = 0;                                      // [2][B][SROW]
    static constexpr int OFF_PRE = OFF_STAGE + 2 * B * SROW;
    static constexpr int OFF_ZTAB = OFF_PRE + (PRE_LDS ? 16 * RL : RL + L * 16);
    static constexpr int OFF_CTW = OFF_ZTAB + ZTAB;
    static constexpr int OFF_BTAB = OFF_CTW + (CTW_LDS ? NCTW : 0);
    static constexpr int OFF_SLOT = (OFF_BTAB + GSched<BF>::TABLE + 1) & ~1;
    static constexpr int OFF_PREV = OFF_SLOT + ROWS * SLOT;  // the last row's second slot
    static constexpr int OFF_CARRY = OFF_PREV + SLOT;        // [ROWS + 1][NWR] wave scan totals (int)
    static constexpr size_t LDS = (size_t)OFF_CARRY * 8 + (size_t)(ROWS + 1) * NWR * 4;
    static_assert(SLOT % 2 == 0 && LDS <= 160 * 1024, "fused wide kernel LDS");
    static_assert(2 * L * GSched<BF>::REGION <= 2 * SLOT, "paired float-half band exchange fits the slot");
    static_assert(NWR * HALF <= SLOT, "NWR 1024-point exchange regions per slot");
    static_assert(ZT % ROWS == 0 && 2 * B * ROWS % THREADS == 0, "tile shapes");
};

constexpr float kTwoPiW = 6.28318530717959f;
constexpr float kW_VLim = 3.14159265f - 4e-3f;  // as the 1024 form and int_rows.inc

__device__ __forceinline__ int fw_exact_w(float a, float b) {
    const double d = (double)a - (double)b;
    return d > 3.141592653589793 ? -1 : (d < -3.141592653589793 ? 1 : 0);
}

// a wave's scan total (16-bit halves biased by 16 per lane) -> its k' sums of both maps
__device__ __forceinline__ fv2 unbias_total(int c) { return fv2{(float)((c & 0xffff) - 16 * 64), (float)((c >> 16) - 16 * 64)}; }

}  // namespace

template <int W, bool UNWRAP, bool REF>
__global__ __launch_bounds__(WideCfg<W>::THREADS, 1) void k_phase_rows_wide(
    const float2* __restrict__ Ab, int H, int nb, int NCA, int ncc0, int ncc1, const float* __restrict__ theta,
    const float2* __restrict__ pre, const float2* __restrict__ ptw, const float2* __restrict__ ztw,
    float* __restrict__ col0, int* __restrict__ flags, float2* __restrict__ Zt, float2* __restrict__ seam, int per,
    float* __restrict__ theta_out) {
    using C = WideCfg<W>;
    constexpr int B = C::B, BF = C::BF, NWR = C::NWR, RL = C::RL, ROWS = C::ROWS, G = C::G, L = C::L, SROW = C::SROW;
    extern __shared__ __attribute__((aligned(16))) float2 lds_w[];
    float2* const stage = lds_w + C::OFF_STAGE;
    float2* const ptl = lds_w + C::OFF_PRE;
    float2* const ztab = lds_w + C::OFF_ZTAB;
    float2* const ctl = lds_w + C::OFF_CTW;
    float2* const btab = lds_w + C::OFF_BTAB;
    int* const carry = reinterpret_cast<int*>(lds_w + C::OFF_CARRY);
    const int row = threadIdx.x / RL, l = threadIdx.x % RL;  // tile row; lane in the row's waves
    const int wv = l >> 6, lane = threadIdx.x & 63;          // wave of the row
    const int g = l / G, t = l % G;                          // band group / lane in group
    // FOLD: group g's input is A[j] + w_g A[j + BF], w_g = exp(2 pi i BF g / W)
    float2 om = make_float2(1.f, 0.f);
    if constexpr (C::FOLD == 2) {
        double sn, cs;
        sincospi(2.0 * (double)g * BF / W, &sn, &cs);
        om = make_float2((float)cs, (float)sn);
    }
    auto band_in = [&](int c, int q, int row_) {  // carrier c's (folded) band value t + G q of tile row row_
        float2 a = stage[(c * B + t + G * q) * SROW + row_];
        if constexpr (C::FOLD == 2) a = cadd(a, cmul(om, stage[(c * B + t + G * q + BF) * SROW + row_]));
        return a;
    };
    // the last row alternates between two slots, so the previous tile's last
    // unwrapped row survives for the census against this tile's first row
    auto slot_idx = [&](int w, int k) { return w == ROWS - 1 && k ? ROWS : w; };
    auto row_slot = [&](int w, int k) { return lds_w + (w == ROWS - 1 && k ? C::OFF_PREV : C::OFF_SLOT + w * C::SLOT); };
    // 2 pi x the k' offset of wave h of a row: the totals of its lower waves
    auto row_carry = [&](int w, int k, int h) {
        fv2 a = {0.f, 0.f};
        for (int i = 0; i < h; ++i) a += unbias_total(carry[slot_idx(w, k) * NWR + i]);
        return a * kTwoPiW;
    };
    for (int i = threadIdx.x; i < GSched<C::BF>::TABLE; i += C::THREADS) btab[i] = ptw[i];
    if constexpr (C::PRE_LDS) {
        for (int i = threadIdx.x; i < 16 * RL; i += C::THREADS) ptl[(i % 16) * RL + i / 16] = pre[i];
    } else {  // pre[l][q]: lane l = g G + t; q = 0 gives exp(2 pi i t g / W), t = 0 the G q g factor
        for (int i = threadIdx.x; i < RL; i += C::THREADS) ptl[i] = pre[(long)i * 16];
        for (int i = threadIdx.x; i < L * 16; i += C::THREADS) ptl[RL + i] = pre[(long)(i / 16) * G * 16 + i % 16];
    }
    if constexpr (!REF) {
        for (int i = threadIdx.x; i < C::ZTAB; i += C::THREADS) ztab[i] = ztw[i];
        if constexpr (C::CTW_LDS)
            for (int i = threadIdx.x; i < C::NCTW; i += C::THREADS) ctl[i] = ztw[C::ZTAB + i];
    }
    const float2* const ctw = C::CTW_LDS ? ctl : ztw + C::ZTAB;
    const int rbs = H / ROWS;
    const int items = nb * rbs;
    const int tiles16 = H / 16;
    const int it0 = blockIdx.x * per, it1 = min(it0 + per, items);  // a contiguous range of tiles
    // staged band values of the next item in registers: entry e = (c, j, row), row fastest
    constexpr int SPT = 2 * B * ROWS / C::THREADS;
    float2 pf[SPT];
    auto fetch = [&](int blk) {
        const int f = blk / rbs, rb = blk % rbs;
        const int r = rb * ROWS + (threadIdx.x % ROWS);
#pragma unroll
        for (int i = 0; i < SPT; ++i) {
            const int e = threadIdx.x + i * C::THREADS;
            const int c = e / (B * ROWS), j = (e / ROWS) % B;
            float2 v = make_float2(0.f, 0.f);
            if (j < (c ? ncc1 : ncc0)) v = Ab[((((long)f * 2 + c) * tiles16 + (r >> 4)) * NCA + j) * 16 + (r & 15)];
            pf[i] = v;
        }
    };
    if (it0 < it1) fetch(it0);
    for (int blk = it0; blk < it1; ++blk) {
        const int f = blk / rbs, rb = blk % rbs;
        const int r = rb * ROWS + row;
        const int par = (blk - it0) & 1;
        float2* const slot = row_slot(row, par);
#pragma unroll
        for (int i = 0; i < SPT; ++i) {
            const int e = threadIdx.x + i * C::THREADS;
            stage[(e / ROWS) * SROW + e % ROWS] = pf[i];
        }
        __syncthreads();
        if (blk + 1 < it1) fetch(blk + 1);
        // ---- band transforms of both carriers -> wrapped phases (natural strided:
        // this lane's value q is pixel g + L t + RL q)
        float w0[16], w1[16];
        {
            const float2 pb = C::PRE_LDS ? make_float2(1.f, 0.f) : ptl[l];
            auto pretw = [&](int q) { return C::PRE_LDS ? ptl[q * RL + l] : cmul(pb, ptl[RL + g * 16 + q]); };
            if constexpr (C::SEQ) {
                // 512-point groups: the carriers one after the other (in lockstep the
                // two transforms' registers spill), exchange in float2 regions
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    float2 x[16];
#pragma unroll
                    for (int q = 0; q < 16; ++q) x[q] = cmul(band_in(c, q, row), pretw(q));
                    if constexpr (C::FOLD == 2)
                        GroupFFTTab<BF>::template run_half<true>(x, reinterpret_cast<float*>(slot) + g * GSched<BF>::REGION,
                                                                 t, btab);
                    else
                        GroupFFTTab<BF>::template run<true>(x, slot + g * GSched<BF>::REGION, t, btab);
                    if constexpr (REF) {  // the reference's angles, natural layout
                        float* o = theta_out + ((long)c * H + r) * W;
#pragma unroll
                        for (int q = 0; q < 16; q += 2) {
                            const fv2 a = fast_atan2_pk(fv2{x[q].y, x[q + 1].y}, fv2{x[q].x, x[q + 1].x});
                            o[g + L * t + RL * q] = a.x;
                            o[g + L * t + RL * (q + 1)] = a.y;
                        }
                        continue;
                    }
                    // reference angles of this lane's 16 pixels (lane-contiguous copy, band_theta_lanes)
                    const float4* tp = reinterpret_cast<const float4*>(theta + ((long)c * H + r) * W) + l * 4;
                    float4 th4[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k) th4[k] = tp[k];
#pragma unroll
                    for (int q0 = 0; q0 < 16; q0 += 8) {  // four pixel pairs per interleaved group
                        __builtin_amdgcn_sched_barrier(0);
                        fv2 tq[4], wq[4];
                        float2 uq[8];
#pragma unroll
                        for (int m = 0; m < 4; ++m) {
                            const int q = q0 + 2 * m, k = q / 4, e = q % 4;
                            tq[m] = e == 0 ? fv2{th4[k].x, th4[k].y} : fv2{th4[k].z, th4[k].w};
                            uq[2 * m] = x[q];
                            uq[2 * m + 1] = x[q + 1];
                        }
                        wrapped_phase_pkn<4>(tq, uq, wq);
#pragma unroll
                        for (int m = 0; m < 4; ++m) {
                            const int q = q0 + 2 * m;
                            (c ? w1 : w0)[q] = wq[m].x;
                            (c ? w1 : w0)[q + 1] = wq[m].y;
                        }
                    }
                }
                if constexpr (REF) {
                    __syncthreads();  // the slots' exchange regions before the next tile
                    continue;
                }
            } else {
                float2 x0[16], x1[16];
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const float2 p = pretw(q);
                    x0[q] = cmul(band_in(0, q, row), p);
                    x1[q] = cmul(band_in(1, q, row), p);
                }
                float* const sx = reinterpret_cast<float*>(slot);
                GroupFFTTab2<BF>::template run_half<true>(x0, x1, sx + g * GSched<BF>::REGION, sx + (L + g) * GSched<BF>::REGION,
                                                         t, btab);
                if constexpr (REF) {  // the reference's angles, natural layout
#pragma unroll
                    for (int q = 0; q < 16; q += 2) {
                        const int n = g + L * t + RL * q;
                        const fv2 a0 = fast_atan2_pk(fv2{x0[q].y, x0[q + 1].y}, fv2{x0[q].x, x0[q + 1].x});
                        const fv2 a1 = fast_atan2_pk(fv2{x1[q].y, x1[q + 1].y}, fv2{x1[q].x, x1[q + 1].x});
                        float* o0 = theta_out + ((long)0 * H + r) * W;
                        float* o1 = theta_out + ((long)1 * H + r) * W;
                        o0[n] = a0.x;
                        o0[n + RL] = a0.y;
                        o1[n] = a1.x;
                        o1[n + RL] = a1.y;
                    }
                    __syncthreads();  // the slots' exchange regions before the next tile
                    continue;
                }
                // reference angles of this lane's 16 pixels (lane-contiguous copy, band_theta_lanes).
                // (Issued ahead of the band transforms with a counted wait, as the 1024 kernel
                // does: 7 VGPRs spilled at 2048 and 4096, fused 4096 133.6 -> 141 us/frame, r06 te.)
                float4 th4[2][4];
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    const float4* tp = reinterpret_cast<const float4*>(theta + ((long)c * H + r) * W) + l * 4;
#pragma unroll
                    for (int k = 0; k < 4; ++k) th4[c][k] = FCD_WIDE_NOTHETA ? make_float4(0.f, 0.f, 0.f, 0.f) : tp[k];
                }
#pragma unroll
                for (int q0 = 0; q0 < 16; q0 += 4) {  // two pixel pairs of each carrier per interleaved group
                    __builtin_amdgcn_sched_barrier(0);
                    fv2 tq[4], wq[4];
                    float2 uq[8];
#pragma unroll
                    for (int m = 0; m < 2; ++m) {
                        const int q = q0 + 2 * m, k = q / 4, e = q % 4;
                        tq[2 * m] = e == 0 ? fv2{th4[0][k].x, th4[0][k].y} : fv2{th4[0][k].z, th4[0][k].w};
                        tq[2 * m + 1] = e == 0 ? fv2{th4[1][k].x, th4[1][k].y} : fv2{th4[1][k].z, th4[1][k].w};
                        uq[4 * m] = x0[q];
                        uq[4 * m + 1] = x0[q + 1];
                        uq[4 * m + 2] = x1[q];
                        uq[4 * m + 3] = x1[q + 1];
                    }
                    wrapped_phase_pkn<4>(tq, uq, wq);
#pragma unroll
                    for (int m = 0; m < 2; ++m) {
                        const int q = q0 + 2 * m;
                        w0[q] = wq[2 * m].x;
                        w0[q + 1] = wq[2 * m].y;
                        w1[q] = wq[2 * m + 1].x;
                        w1[q + 1] = wq[2 * m + 1].y;
                    }
                }
            }
        }
        // ---- natural strided -> blocked through the slot: the row's waves' band
        // exchange regions span the whole slot, so the tile syncs before and after
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 16; ++q) slot[pad(g + L * t + RL * q)] = make_float2(w0[q], w1[q]);
        __syncthreads();
        const int j0 = l * 16;
        int bad = 0;
        {
            float2 v[17];
#pragma unroll
            for (int j = 0; j < 16; ++j) v[j] = slot[pad(j0 + j)];
            v[16] = l < RL - 1 ? slot[pad(j0 + 16)] : v[15];  // no edge past the row end: dd = 0
            if (l == 0) {
                col0[((long)f * 2 + 0) * H + r] = v[0].x;
                col0[((long)f * 2 + 1) * H + r] = v[0].y;
            }
            if constexpr (UNWRAP) {
                // dd = -find_wrap(w(j), w(j+1)) = rint((w(j) - w(j+1)) / 2 pi) except at
                // +-fl(pi) (flagged ambiguous), k' accumulated in f32 (kernels_phase_rows.hip)
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
                // both maps' segment sums in 16-bit halves biased by 16 per lane
                const int packed = ((int)run.x + 16) | (((int)run.y + 16) << 16);
                const int incl = team_scan_incl_dpp<64>(packed);
                const int excl = incl - packed;
                if (lane == 63 && wv < NWR - 1) carry[slot_idx(row, par) * NWR + wv] = incl;  // this wave's total
                fv2 acc = {(float)((excl & 0xffff) - 16 * lane), (float)((excl >> 16) - 16 * lane)};
                // every lane has read its neighbour's first value; a wave's last lane also
                // reads the next wave's first pixel, which that wave's lane 0 may already
                // have rewritten -- with its own value, as k'' = 0 there (fma(0, 2 pi, w) = w)
                wave_sync();
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    slot[pad(j0 + j)] = vp(acc * kTwoPiW + pv(v[j]));
                    acc += dd[j];
                }
                bad |= amb;
            }
        }
        __syncthreads();
        if constexpr (UNWRAP) {  // first and last unwrapped rows of the range -> seam buffer
            if ((row == 0 && blk == it0 && rb > 0) || (row == ROWS - 1 && blk == it1 - 1 && rb < rbs - 1)) {
                const fv2 cy = row_carry(row, par, wv);
                float4* sd = reinterpret_cast<float4*>(seam + (((long)f * rbs + rb) * 2 + (row ? 1 : 0)) * W + j0);
#pragma unroll
                for (int j = 0; j < 16; j += 2) {
                    const fv2 a = pv(slot[pad(j0 + j)]) + cy, b = pv(slot[pad(j0 + j + 1)]) + cy;
                    sd[j / 2] = make_float4(a.x, a.y, b.x, b.y);
                }
            }
        }
        // ---- vertical census against the next row of the tile (range edges: k_seam_check_wide)
        if constexpr (UNWRAP) {
            if (row < ROWS - 1 || (blk > it0 && rb > 0)) {
                const bool up = row == ROWS - 1;  // the previous tile's last row against row 0
                const int ar = up ? ROWS - 1 : row, ak = up ? par ^ 1 : par;
                const int nr = up ? 0 : row + 1;
                const float2* a_row = row_slot(ar, ak);
                const float2* nx = row_slot(nr, par);
                const float2 a0 = a_row[0], b0 = nx[0];  // phi'(r, 0) = w(r, 0)
                const fv2 dd = fv2{kTwoPiW * (float)(-fw_exact_w(a0.x, b0.x)), kTwoPiW * (float)(-fw_exact_w(a0.y, b0.y))} +
                               (row_carry(nr, par, wv) - row_carry(ar, ak, wv));
                float m = 0.f;
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const fv2 e = (pv(nx[pad(j0 + j)]) - pv(a_row[pad(j0 + j)])) + dd;
                    m = fmaxf(m, fmaxf(fabsf(e.x), fabsf(e.y)));
                }
                bad |= (int)(m > kW_VLim);
            }
            if (__any(bad) && lane == 0) atomicOr(flags + f * 2, 1);
            __syncthreads();  // every census read of a slot precedes that row's FFT
        }
        // ---- forward row FFT of phi0' + i phi1': NWR wave-local 1024-point transforms
        {
            fv2 cys[NWR];
#pragma unroll
            for (int h = 0; h < NWR; ++h) cys[h] = UNWRAP ? row_carry(row, par, h) : fv2{0.f, 0.f};
            float2 x[16];
#pragma unroll
            for (int q = 0; q < 16; ++q)  // sample NWR (lane + 64 q) + wv lies in wave q / (16 / NWR)
                x[q] = vp(pv(slot[pad(NWR * (lane + 64 * q) + wv)]) + cys[q / (16 / NWR)]);
            // the last row transforms in its other slot (the previous tile's row, no
            // longer needed): its unwrapped row stays for the next tile's census
            float2* const zs = row_slot(row, par ^ 1);
            __syncthreads();  // every wave's reads of the row before any exchange writes
            GroupFFTTab<1024>::template run<false>(x, zs + wv * C::HALF, lane, ztab);
            wave_sync();
#pragma unroll
            for (int q = 0; q < 16; ++q) zs[wv * C::HALF + pad(lane + 64 * q)] = x[q];
        }
        __syncthreads();
        // ---- Zt: this tile's rows of the Zt tiles' column runs; the radix-NWR join
        // X[k + 1024 j] = sum_h W_NWR^(h j) w^(h k) Y_h[k] on the way out
        {
            const int r0 = rb * ROWS;
            float2* dst = Zt + (long)f * H * W + (long)(r0 / C::ZT) * W * C::ZT + (r0 % C::ZT);
            constexpr int CPP = C::THREADS / ROWS;  // columns per pass
            const int c0 = threadIdx.x / ROWS, rl = threadIdx.x % ROWS;
            const float2* src = row_slot(rl, par ^ 1);
            constexpr int JU = NWR == 2 ? 2 : 1;  // join columns in flight (VGPRs at 4096)
            auto zst = [](float2* p, float2 v) {
                // at 4096 a tile's part of a Zt column run is 16 bytes (2 rows): streaming
                // stores write each piece on its own (PMC r04i: 279 MB written per 134 MB of
                // Zt).  With 4-row runs plain stores let the L2 join it with the next tile's
                // half (3.09k -> 3.15k frames/s, r04j); with 16-row runs (eight tiles per
                // line) plain stores cost a read of every line (r04q: reads 206 -> 279 MB),
                // so those stay streaming.  Round 6 (folded band): streaming at 4-row runs
                // too, the half lines no longer crowding the reference angles out of L2
                if constexpr (C::ROWS * 8 >= 32 || C::ZT != 2 * C::ROWS || FCD_WIDE_ZT_NT) st_stream(p, v);
                else *p = v;
            };
#pragma unroll JU
            for (int k = 0; k < 1024 / CPP; ++k) {
                const int c = c0 + CPP * k;
                if constexpr (NWR == 2) {
                    const float2 e = src[pad(c)], o = cmul(src[C::HALF + pad(c)], ctw[c]);
                    zst(dst + c * C::ZT + rl, cadd(e, o));
                    zst(dst + (c + 1024) * C::ZT + rl, csub(e, o));
                } else {
                    const float2 y0 = src[pad(c)];
                    const float2 y1 = cmul(src[C::HALF + pad(c)], ctw[c]);
                    const float2 y2 = cmul(src[2 * C::HALF + pad(c)], ctw[1024 + c]);
                    const float2 y3 = cmul(src[3 * C::HALF + pad(c)], ctw[2048 + c]);
                    const float2 a = cadd(y0, y2), b = csub(y0, y2), d = cadd(y1, y3), e = csub(y1, y3);
                    const float2 ie = make_float2(e.y, -e.x);  // -i e
                    zst(dst + c * C::ZT + rl, cadd(a, d));
                    zst(dst + (c + 1024) * C::ZT + rl, cadd(b, ie));
                    zst(dst + (c + 2048) * C::ZT + rl, csub(a, d));
                    zst(dst + (c + 3072) * C::ZT + rl, csub(b, ie));
                }
            }
        }
        __syncthreads();
    }
}

// Census of the edges between the tile ranges of k_phase_rows_wide's blocks: the last
// row of tile it - 1 against the first row of tile it, it = k * per.  One wave per
// range edge; lane L holds pixels (W / 64) L .. (W / 64) (L + 1) - 1.
template <int W>
__global__ __launch_bounds__(256) void k_seam_check_wide(const float2* __restrict__ seam, int H, int nb, int per,
                                                         int* __restrict__ flags) {
    constexpr int PL = W / 64;  // pixels per lane
    const int rbs = H / WideCfg<W>::ROWS;
    const long it = ((long)blockIdx.x * 4 + (threadIdx.x >> 6) + 1) * per;
    if (it >= (long)nb * rbs || it % rbs == 0) return;
    const int f = (int)(it / rbs), b = (int)(it % rbs) - 1;
    const int lane = threadIdx.x & 63;
    const float4* a = reinterpret_cast<const float4*>(seam + (((long)f * rbs + b) * 2 + 1) * W + lane * PL);
    const float4* c = reinterpret_cast<const float4*>(seam + (((long)f * rbs + b + 1) * 2 + 0) * W + lane * PL);
    const float4 a0v = a[0], c0v = c[0];
    const float a0x = __shfl(a0v.x, 0), a0y = __shfl(a0v.y, 0);
    const float c0x = __shfl(c0v.x, 0), c0y = __shfl(c0v.y, 0);
    const float d0 = kTwoPiW * (float)(-fw_exact_w(a0x, c0x));
    const float d1 = kTwoPiW * (float)(-fw_exact_w(a0y, c0y));
    int bad = 0;
#pragma unroll 4
    for (int j = 0; j < PL / 2; ++j) {
        const float4 av = a[j], cv = c[j];
        bad |= (int)(fabsf(cv.x - av.x + d0) > kW_VLim) | (int)(fabsf(cv.y - av.y + d1) > kW_VLim);
        bad |= (int)(fabsf(cv.z - av.z + d0) > kW_VLim) | (int)(fabsf(cv.w - av.w + d1) > kW_VLim);
    }
    if (__any(bad) && lane == 0) atomicOr(flags + f * 2, 1);
}

namespace {

int num_cus() {
    const int ncu = device_cu_count();  // (atomic cache: launchers run from two host threads)
    return ncu;
}

template <int W, bool UNWRAP, bool REF>
void launch_wide(int grid, const float2* Ab, int H, int nb, int NCA, int ncc0, int ncc1, const float* theta,
                 const float2* pre, const float2* ptw, const float2* ztw, float* col0, int* flags, float2* Zt,
                 float2* seam, int per, float* theta_out, hipStream_t s) {
    using C = WideCfg<W>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_phase_rows_wide<W, UNWRAP, REF>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)C::LDS);
    hipLaunchKernelGGL((k_phase_rows_wide<W, UNWRAP, REF>), dim3(grid), dim3(C::THREADS), C::LDS, s, Ab, H, nb, NCA,
                       ncc0, ncc1, theta, pre, ptw, ztw, col0, flags, Zt, seam, per, theta_out);
}

// blocks of k_phase_rows_wide: one per CU, each `per` consecutive tiles
template <int W>
void wide_layout(int H, int nb, int& grid, int& per) {
    const long items = (long)nb * (H / WideCfg<W>::ROWS);
    const int slots = (int)std::min<long>(items, (long)num_cus());  // one workgroup per CU
    grid = per = 0;
    if (slots <= 0) return;
    per = (int)((items + slots - 1) / slots);  // tiles per block, a contiguous range
    grid = (int)((items + per - 1) / per);
}

template <int W>
void seam_wide_t(int H, int nb, const float2* seam, int* flags, hipStream_t s) {
    int grid, per;
    wide_layout<W>(H, nb, grid, per);
    const int edges = grid - 1;  // range edges (those at frame starts return at once)
    if (edges > 0)
        hipLaunchKernelGGL(k_seam_check_wide<W>, dim3((unsigned)((edges + 3) / 4)), dim3(256), 0, s, seam, H, nb, per,
                           flags);
}

template <int W>
void phase_rows_wide_t(int mode, const float2* Ab, int H, int nb, int NCA, int ncc0, int ncc1, const float* theta,
                       const float2* pre, const float2* ptw, const float2* ztw, float* col0, int* flags, float2* Zt,
                       float2* seam, float* theta_out, hipStream_t s, bool defer_seam = false) {
    using C = WideCfg<W>;
    if (H % 16 != 0 || NCA < ncc0 || NCA < ncc1 || ncc0 > C::B || ncc1 > C::B)
        throw std::runtime_error("phase_rows_wide: unsupported geometry");
    int grid, per;
    wide_layout<W>(H, nb, grid, per);
    if (grid <= 0) return;
    if (mode == 2) {
        launch_wide<W, false, true>(grid, Ab, H, nb, NCA, ncc0, ncc1, theta, pre, ptw, ztw, col0, flags, Zt, seam, per,
                                    theta_out, s);
    } else if (mode == 1) {
        launch_wide<W, true, false>(grid, Ab, H, nb, NCA, ncc0, ncc1, theta, pre, ptw, ztw, col0, flags, Zt, seam, per,
                                    theta_out, s);
        if (!defer_seam) seam_wide_t<W>(H, nb, seam, flags, s);
    } else {
        launch_wide<W, false, false>(grid, Ab, H, nb, NCA, ncc0, ncc1, theta, pre, ptw, ztw, col0, flags, Zt, seam, per,
                                     theta_out, s);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) throw std::runtime_error(std::string("phase_rows_wide launch: ") + hipGetErrorString(e));
}

}  // namespace

void phase_rows_wide(int W, bool unwrap, const float2* Ab, int H, int nb, int NCA, int ncc0, int ncc1, const float* theta,
                     const float2* pre, const float2* ptw, const float2* ztw, float* col0, int* flags, float2* Zt,
                     float2* seam, hipStream_t s, bool defer_seam) {
    if (W == 2048)
        phase_rows_wide_t<2048>(unwrap ? 1 : 0, Ab, H, nb, NCA, ncc0, ncc1, theta, pre, ptw, ztw, col0, flags, Zt, seam,
                                nullptr, s, defer_seam);
    else if (W == 4096)
        phase_rows_wide_t<4096>(unwrap ? 1 : 0, Ab, H, nb, NCA, ncc0, ncc1, theta, pre, ptw, ztw, col0, flags, Zt, seam,
                                nullptr, s, defer_seam);
    else
        throw std::runtime_error("phase_rows_wide: 2048- or 4096-point rows");
}

void phase_rows_wide_seam(int W, int H, int nb, const float2* seam, int* flags, hipStream_t s) {
    if (W == 2048)
        seam_wide_t<2048>(H, nb, seam, flags, s);
    else if (W == 4096)
        seam_wide_t<4096>(H, nb, seam, flags, s);
    else
        throw std::runtime_error("phase_rows_wide_seam: 2048- or 4096-point rows");
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) throw std::runtime_error(std::string("phase_rows_wide seam check launch: ") + hipGetErrorString(e));
}

void phase_rows_wide_ref(int W, const float2* Ab, int H, int NCA, int ncc0, int ncc1, const float2* pre,
                         const float2* ptw, float* theta_b, hipStream_t s) {
    if (W != 4096) throw std::runtime_error("phase_rows_wide_ref: 4096-point rows only");
    phase_rows_wide_t<4096>(2, Ab, H, 1, NCA, ncc0, ncc1, nullptr, pre, ptw, nullptr, nullptr, nullptr, nullptr,
                            nullptr, theta_b, s);
}

int phase_rows_wide_bt(int W) { return W == 2048 ? WideCfg<2048>::BF : WideCfg<4096>::BF; }

size_t phase_rows_wide_lds(int W) { return W == 2048 ? WideCfg<2048>::LDS : WideCfg<4096>::LDS; }

}  // namespace fcdk
