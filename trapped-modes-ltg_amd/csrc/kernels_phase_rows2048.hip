// Fused throughput kernel of the height-only path at 2048-point rows: the same
// chain as kernels_phase_rows.hip (the 1024-wide form, which cites the reference
// lines) --
//
//   band-pruned inverse row transforms of both carriers + phase   (fcd.py:118)
//   residue-free unwrap of both maps + its census                 (fcd.py:119)
//   phi0' + i*phi1' -> forward row FFT -> Zt tile                  (fourier.py:134)
//
// -- in one pass over each 4-row tile, so the 2048^2 frame's wrapped phase maps
// (33.5 MB) never touch HBM.  A row is a wave PAIR (128 lanes x 16 values), the
// tile 4 rows = 8 waves, 139 KB of LDS (one workgroup per CU):
//
//   * band transform (B = 256): 8 pre-twiddled 256-point group FFTs per row, 16
//     lanes each, groups 0-3 in the first wave of the pair and 4-7 in the second,
//     both carriers in lockstep, float-half exchange in the row's slot;
//   * unwrap: 16 consecutive pixels per lane; each wave scans its half row (packed
//     pairs of both maps, one DPP scan); the first wave's total, through LDS, is the
//     second half's offset (the edge between pixels 1023 and 1024 belongs to the
//     first wave's last lane), added where the second half is read;
//   * census: vertical edges inside the tile here, the tile range edges in
//     k_seam_check2048 (as the 1024 form);
//   * z-row FFT: 2048 = 2 x 1024 -- wave h of the pair transforms the samples 2m + h
//     (the wave-local 1024-point group FFT), and the Zt write-out joins the halves,
//     X[k] = E[k] + w^k O[k] and X[k + 1024] = E[k] - w^k O[k];
//   * Zt: 8-row tiles at 2048 (zt_rows), so a tile writes 32-byte halves of its
//     columns' 64-byte runs; the next tile of the block's contiguous range writes the
//     other halves right after.
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#include "gfft.hpp"
#include "kernels.hpp"

namespace fcdk {

namespace {

constexpr int Q_W = 2048;                    // row length
constexpr int Q_B = 256;                     // band window
constexpr int Q_ROWS = 4;                    // rows per tile (a wave pair each)
constexpr int Q_RL = Q_W / 16;               // lanes per row
constexpr int Q_THREADS = Q_ROWS * Q_RL;     // 512
constexpr int Q_G = Q_B / 16, Q_L = Q_W / Q_B;
constexpr int Q_ZT = 8;                      // Zt tile height (int_rows.inc zt_rows(2048))
static_assert(Q_ZT % Q_ROWS == 0, "a tile covers part of one Zt tile");
constexpr int Q_SLOT = padded_len(Q_W) + 2;  // row slot (float2), 16-byte multiple
constexpr int Q_HALF = padded_len(1024);     // one wave's 1024-point exchange region; pad(k + 1024) = pad(k) + Q_HALF
constexpr int Q_SROW = Q_ROWS + 1;           // staged band rows (odd pitch)
constexpr int Q_ZTAB = GSched<1024>::TABLE;  // twiddles of the 1024-point group FFT
// LDS carve (float2 units)
constexpr int OFFQ_STAGE = 0;                               // [2][B][SROW]
constexpr int OFFQ_PRE = OFFQ_STAGE + 2 * Q_B * Q_SROW;      // [16][RL] band pre-twiddles
constexpr int OFFQ_ZTAB = OFFQ_PRE + 16 * Q_RL;              // z-FFT pass twiddles
constexpr int OFFQ_CTW = OFFQ_ZTAB + Q_ZTAB;                 // w^k = exp(-2 pi i k / 2048), k < 1024
constexpr int OFFQ_BTAB = OFFQ_CTW + 1024;                   // band-FFT pass twiddles
constexpr int OFFQ_SLOT = (OFFQ_BTAB + GSched<Q_B>::TABLE + 1) & ~1;
constexpr int OFFQ_PREV = OFFQ_SLOT + Q_ROWS * Q_SLOT;       // the last row's second slot
constexpr int OFFQ_CARRY = OFFQ_PREV + Q_SLOT;               // [ROWS + 1] first-wave scan totals (int)
constexpr size_t Q_LDS = (size_t)(OFFQ_CARRY + Q_ROWS + 1) * 8;
static_assert(Q_SLOT % 2 == 0 && Q_LDS <= 160 * 1024, "fused 2048 kernel LDS");
static_assert(2 * Q_L * GSched<Q_B>::REGION <= 2 * Q_SLOT, "paired float-half band exchange fits the slot");
static_assert(2 * Q_HALF <= Q_SLOT, "two 1024-point exchange regions per slot");

constexpr float kTwoPiQ = 6.28318530717959f;
constexpr float kQ_VLim = 3.14159265f - 4e-3f;  // as the 1024 form and int_rows.inc

__device__ __forceinline__ int fw_exact2(float a, float b) {
    const double d = (double)a - (double)b;
    return d > 3.141592653589793 ? -1 : (d < -3.141592653589793 ? 1 : 0);
}

}  // namespace

template <bool UNWRAP>
__global__ __launch_bounds__(Q_THREADS, 1) void k_phase_rows2048(
    const float2* __restrict__ Ab, int H, int nb, int NCA, int ncc0, int ncc1, const float* __restrict__ theta,
    const float2* __restrict__ pre, const float2* __restrict__ ptw, const float2* __restrict__ ztw,
    float* __restrict__ col0, int* __restrict__ flags, float2* __restrict__ Zt, float2* __restrict__ seam, int per) {
    extern __shared__ __attribute__((aligned(16))) float2 lds_q[];
    float2* const stage = lds_q + OFFQ_STAGE;
    float2* const ptl = lds_q + OFFQ_PRE;
    float2* const ztab = lds_q + OFFQ_ZTAB;
    float2* const ctw = lds_q + OFFQ_CTW;
    float2* const btab = lds_q + OFFQ_BTAB;
    int* const carry = reinterpret_cast<int*>(lds_q + OFFQ_CARRY);
    const int row = threadIdx.x / Q_RL, l = threadIdx.x % Q_RL;  // tile row; lane in the row's wave pair
    const int half = l >> 6, lane = threadIdx.x & 63;
    const int g = l / Q_G, t = l % Q_G;  // band group / lane in group
    // the last row alternates between two slots, so the previous tile's last
    // unwrapped row survives for the census against this tile's first row
    auto row_slot = [&](int w, int k) { return lds_q + (w == Q_ROWS - 1 && k ? OFFQ_PREV : OFFQ_SLOT + w * Q_SLOT); };
    // the second half row is stored WITHOUT the first half's total k' (no barrier
    // between the two waves' scans): that offset, 2 pi (carry0, carry1) of the row,
    // is added where the second half is read (census, seam rows, z-row FFT)
    auto row_carry = [&](int w, int k) {
        const int c = carry[w == Q_ROWS - 1 && k ? Q_ROWS : w];
        return fv2{kTwoPiQ * (float)((c & 0xffff) - 16 * 64), kTwoPiQ * (float)((c >> 16) - 16 * 64)};
    };
    for (int i = threadIdx.x; i < GSched<Q_B>::TABLE; i += Q_THREADS) btab[i] = ptw[i];
    for (int i = threadIdx.x; i < 16 * Q_RL; i += Q_THREADS) ptl[(i % 16) * Q_RL + i / 16] = pre[i];
    for (int i = threadIdx.x; i < Q_ZTAB; i += Q_THREADS) ztab[i] = ztw[i];
    for (int i = threadIdx.x; i < 1024; i += Q_THREADS) ctw[i] = ztw[Q_ZTAB + i];
    const int rbs = H / Q_ROWS;
    const int items = nb * rbs;
    const int tiles16 = H / 16;
    const int it0 = blockIdx.x * per, it1 = min(it0 + per, items);  // a contiguous range of tiles
    // staged band values of the next item in registers: entry e = (c, j, row), row fastest
    constexpr int NST = 2 * Q_B * Q_ROWS;
    constexpr int SPT = NST / Q_THREADS;
    static_assert(NST % Q_THREADS == 0, "whole staging rounds");
    float2 pf[SPT];
    auto fetch = [&](int blk) {
        const int f = blk / rbs, rb = blk % rbs;
        const int r = rb * Q_ROWS + (threadIdx.x % Q_ROWS);
#pragma unroll
        for (int i = 0; i < SPT; ++i) {
            const int e = threadIdx.x + i * Q_THREADS;
            const int c = e / (Q_B * Q_ROWS), j = (e / Q_ROWS) % Q_B;
            float2 v = make_float2(0.f, 0.f);
            if (j < (c ? ncc1 : ncc0)) v = Ab[((((long)f * 2 + c) * tiles16 + (r >> 4)) * NCA + j) * 16 + (r & 15)];
            pf[i] = v;
        }
    };
    if (it0 < it1) fetch(it0);
    for (int blk = it0; blk < it1; ++blk) {
        const int f = blk / rbs, rb = blk % rbs;
        const int r = rb * Q_ROWS + row;
        const int par = (blk - it0) & 1;
        float2* const slot = row_slot(row, par);
#pragma unroll
        for (int i = 0; i < SPT; ++i) {
            const int e = threadIdx.x + i * Q_THREADS;
            stage[(e / Q_ROWS) * Q_SROW + e % Q_ROWS] = pf[i];
        }
        __syncthreads();
        if (blk + 1 < it1) fetch(blk + 1);
        // ---- band transforms of both carriers -> wrapped phases (natural strided:
        // this lane's value q is pixel g + L t + RL q)
        float w0[16], w1[16];
        {
            float2 x0[16], x1[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const float2 p = ptl[q * Q_RL + l];
                x0[q] = cmul(stage[(t + Q_G * q) * Q_SROW + row], p);
                x1[q] = cmul(stage[(Q_B + t + Q_G * q) * Q_SROW + row], p);
            }
            float* const sx = reinterpret_cast<float*>(slot);
            GroupFFTTab2<Q_B>::template run_half<true>(x0, x1, sx + g * GSched<Q_B>::REGION,
                                                       sx + (Q_L + g) * GSched<Q_B>::REGION, t, btab);
            // reference angles of this lane's 16 pixels (lane-contiguous copy, band_theta_lanes)
            float4 th4[2][4];
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const float4* tp = reinterpret_cast<const float4*>(theta + ((long)c * H + r) * Q_W) + l * 4;
#pragma unroll
                for (int k = 0; k < 4; ++k) th4[c][k] = tp[k];
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
        // ---- natural strided -> blocked through the slot: both waves' band exchange
        // regions span the whole slot, so the pair syncs before and after
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 16; ++q) slot[pad(g + Q_L * t + Q_RL * q)] = make_float2(w0[q], w1[q]);
        __syncthreads();
        const int j0 = l * 16;
        int bad = 0;
        {
            float2 v[17];
#pragma unroll
            for (int j = 0; j < 16; ++j) v[j] = slot[pad(j0 + j)];
            v[16] = l < Q_RL - 1 ? slot[pad(j0 + 16)] : v[15];  // no edge past the row end: dd = 0
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
                if (half == 0 && lane == 63) carry[row == Q_ROWS - 1 && par ? Q_ROWS : row] = incl;  // first half's total
                fv2 acc = {(float)((excl & 0xffff) - 16 * lane), (float)((excl >> 16) - 16 * lane)};
                // every lane has read its neighbour's first value; the first wave's last
                // lane also reads pixel 1024, which the second wave's lane 0 may already
                // have rewritten -- with its own value, as k'' = 0 there (fma(0, 2 pi, w) = w)
                wave_sync();
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    slot[pad(j0 + j)] = vp(acc * kTwoPiQ + pv(v[j]));
                    acc += dd[j];
                }
                bad |= amb;
            }
        }
        __syncthreads();
        if constexpr (UNWRAP) {  // first and last unwrapped rows of the range -> seam buffer
            if ((row == 0 && blk == it0 && rb > 0) || (row == Q_ROWS - 1 && blk == it1 - 1 && rb < rbs - 1)) {
                const fv2 cy = half ? row_carry(row, par) : fv2{0.f, 0.f};
                float4* sd = reinterpret_cast<float4*>(seam + (((long)f * rbs + rb) * 2 + (row ? 1 : 0)) * Q_W + j0);
#pragma unroll
                for (int j = 0; j < 16; j += 2) {
                    const fv2 a = pv(slot[pad(j0 + j)]) + cy, b = pv(slot[pad(j0 + j + 1)]) + cy;
                    sd[j / 2] = make_float4(a.x, a.y, b.x, b.y);
                }
            }
        }
        // ---- vertical census against the next row of the tile (range edges: k_seam_check2048)
        if constexpr (UNWRAP) {
            if (row < Q_ROWS - 1 || (blk > it0 && rb > 0)) {
                const bool up = row == Q_ROWS - 1;  // the previous tile's last row against row 0
                const float2* a_row = up ? row_slot(Q_ROWS - 1, par ^ 1) : slot;
                const float2* nx = up ? row_slot(0, 0) : row_slot(row + 1, par);
                const float2 a0 = a_row[0], b0 = nx[0];  // phi'(r, 0) = w(r, 0)
                fv2 dd = {kTwoPiQ * (float)(-fw_exact2(a0.x, b0.x)), kTwoPiQ * (float)(-fw_exact2(a0.y, b0.y))};
                if (half) dd += (up ? row_carry(0, 0) : row_carry(row + 1, par)) - (up ? row_carry(Q_ROWS - 1, par ^ 1) : row_carry(row, par));
                float m = 0.f;
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const fv2 e = (pv(nx[pad(j0 + j)]) - pv(a_row[pad(j0 + j)])) + dd;
                    m = fmaxf(m, fmaxf(fabsf(e.x), fabsf(e.y)));
                }
                bad |= (int)(m > kQ_VLim);
            }
            if (__any(bad) && lane == 0) atomicOr(flags + f * 2, 1);
            __syncthreads();  // every census read of a slot precedes that row's FFT
        }
        // ---- forward row FFT of phi0' + i phi1': two 1024-point halves, then one radix-2 pass
        {
            float2 x[16];
            const fv2 cy = UNWRAP ? row_carry(row, par) : fv2{0.f, 0.f};
#pragma unroll
            for (int q = 0; q < 16; ++q) x[q] = q < 8 ? slot[pad(2 * (lane + 64 * q) + half)] : vp(pv(slot[pad(2 * (lane + 64 * q) + half)]) + cy);
            // the last row transforms in its other slot (the previous tile's row, no
            // longer needed): its unwrapped row stays for the next tile's census
            float2* const zs = row_slot(row, par ^ 1);
            __syncthreads();  // both waves' reads of the row before either's exchange writes
            GroupFFTTab<1024>::template run<false>(x, zs + half * Q_HALF, lane, ztab);
            wave_sync();
#pragma unroll
            for (int q = 0; q < 16; ++q) zs[half * Q_HALF + pad(lane + 64 * q)] = x[q];
        }
        __syncthreads();
        // ---- Zt: 32-byte halves of the 8-row tile's 64-byte column runs; the radix-2
        // join X[k] = E[k] + w^k O[k], X[k + 1024] = E[k] - w^k O[k] on the way out
        static_assert(!FCD_ZT_PAIRED, "the join pairs columns k and k + 1024");
        {
            const int r0 = rb * Q_ROWS;
            float2* dst = Zt + (long)f * H * Q_W + (long)(r0 / Q_ZT) * Q_W * Q_ZT + (r0 % Q_ZT);
            const int c0 = threadIdx.x / Q_ROWS, rl = threadIdx.x % Q_ROWS;
            const float2* src = row_slot(rl, par ^ 1);
#pragma unroll 4
            for (int k = 0; k < 1024 / (Q_THREADS / Q_ROWS); ++k) {
                const int c = c0 + (Q_THREADS / Q_ROWS) * k;
                const float2 e = src[pad(c)], o = cmul(src[Q_HALF + pad(c)], ctw[c]);
                st_stream(dst + c * Q_ZT + rl, cadd(e, o));
                st_stream(dst + (c + 1024) * Q_ZT + rl, csub(e, o));
            }
        }
        __syncthreads();
    }
}

// Census of the edges between the tile ranges of k_phase_rows2048's blocks: the last
// row of tile it - 1 against the first row of tile it, it = k * per.  One wave per
// range edge; lane L holds pixels 32L .. 32L+31.
__global__ __launch_bounds__(256) void k_seam_check2048(const float2* __restrict__ seam, int H, int nb, int per,
                                                        int* __restrict__ flags) {
    const int rbs = H / Q_ROWS;
    const long it = ((long)blockIdx.x * 4 + (threadIdx.x >> 6) + 1) * per;
    if (it >= (long)nb * rbs || it % rbs == 0) return;
    const int f = (int)(it / rbs), b = (int)(it % rbs) - 1;
    const int lane = threadIdx.x & 63;
    const float4* a = reinterpret_cast<const float4*>(seam + (((long)f * rbs + b) * 2 + 1) * Q_W + lane * 32);
    const float4* c = reinterpret_cast<const float4*>(seam + (((long)f * rbs + b + 1) * 2 + 0) * Q_W + lane * 32);
    const float4 a0v = a[0], c0v = c[0];
    const float a0x = __shfl(a0v.x, 0), a0y = __shfl(a0v.y, 0);
    const float c0x = __shfl(c0v.x, 0), c0y = __shfl(c0v.y, 0);
    const float d0 = kTwoPiQ * (float)(-fw_exact2(a0x, c0x));
    const float d1 = kTwoPiQ * (float)(-fw_exact2(a0y, c0y));
    int bad = 0;
#pragma unroll 4
    for (int j = 0; j < 16; ++j) {
        const float4 av = a[j], cv = c[j];
        bad |= (int)(fabsf(cv.x - av.x + d0) > kQ_VLim) | (int)(fabsf(cv.y - av.y + d1) > kQ_VLim);
        bad |= (int)(fabsf(cv.z - av.z + d0) > kQ_VLim) | (int)(fabsf(cv.w - av.w + d1) > kQ_VLim);
    }
    if (__any(bad) && lane == 0) atomicOr(flags + f * 2, 1);
}

size_t phase_rows2048_lds() { return Q_LDS; }

void phase_rows2048(bool unwrap, const float2* Ab, int H, int nb, int NCA, int ncc0, int ncc1, const float* theta,
                    const float2* pre, const float2* ptw, const float2* ztw, float* col0, int* flags, float2* Zt,
                    float2* seam, hipStream_t s) {
    static int ncu = 0;
    if (!ncu) {
        int dev = 0;
        hipDeviceProp_t p;
        if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&p, dev) == hipSuccess) ncu = p.multiProcessorCount;
        if (!ncu) ncu = 256;
    }
    if (H % 16 != 0 || NCA < ncc0 || NCA < ncc1 || ncc0 > Q_B || ncc1 > Q_B)
        throw std::runtime_error("phase_rows2048: unsupported geometry");
    const long items = (long)nb * (H / Q_ROWS);
    const int slots = (int)std::min<long>(items, (long)ncu);  // one 139 KB workgroup per CU
    if (slots <= 0) return;
    const int per = (int)((items + slots - 1) / slots);  // tiles per block, a contiguous range
    const int grid = (int)((items + per - 1) / per);
    if (unwrap) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_phase_rows2048<true>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)Q_LDS);
        hipLaunchKernelGGL(k_phase_rows2048<true>, dim3(grid), dim3(Q_THREADS), Q_LDS, s, Ab, H, nb, NCA, ncc0, ncc1,
                           theta, pre, ptw, ztw, col0, flags, Zt, seam, per);
        const int edges = grid - 1;  // range edges (those at frame starts return at once)
        if (edges > 0)
            hipLaunchKernelGGL(k_seam_check2048, dim3((unsigned)((edges + 3) / 4)), dim3(256), 0, s, seam, H, nb, per,
                               flags);
    } else {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_phase_rows2048<false>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)Q_LDS);
        hipLaunchKernelGGL(k_phase_rows2048<false>, dim3(grid), dim3(Q_THREADS), Q_LDS, s, Ab, H, nb, NCA, ncc0, ncc1,
                           theta, pre, ptw, ztw, col0, flags, Zt, seam, per);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) throw std::runtime_error(std::string("phase_rows2048 launch: ") + hipGetErrorString(e));
}

}  // namespace fcdk
