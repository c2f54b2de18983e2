// Temporal analysis of a height-map stack: per-pixel
// DFTs along time for a spatial block of a [T][rows][cols] float32 or float64
// stack (the sample type is a template parameter; arithmetic is f64 either way), as
// analyze.block_amplitude (analyze.py:543-587: np.fft.fft over time, f64) and
// analyze.spectrogram (analyze.py:419-531: scipy.signal.spectrogram per pixel).
//
// The reference loops over pixels in Python; here each lane owns pixels of
// the block and walks its time series (a coalesced row-run of every frame,
// no transpose of the stack), 2 pixels x 8 frequencies per lane accumulated
// in f64.
// The DFT is direct, not an FFT: T is any length (the number of maps), the
// work is ~T x (T/2 + 1) complex MACs per pixel (1.3e11 flop for a 128 x 128
// block of 2000 maps, ~2 ms of f64 VALU on the MI355X), and the exponentials
// come from a table exp(-2 pi i j / T) built on the host in f64 and indexed by
// (f t) mod T, kept incrementally per frequency (exact argument reduction).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "kernels.hpp"

namespace fcdk {

namespace {

constexpr int TD_THREADS = 256;  // pixels per workgroup
constexpr int TD_LDS_TAB = 8192;  // table entries held in LDS (128 KiB of double2)
constexpr int TD_BATCH = 8;       // samples per load batch
constexpr int TD_PX = 2;          // pixels per lane of k_tdft / k_spectro (4 x 4 bins: 9.7 vs 4.6 ms, r01bq)
constexpr int TD_FT_DFT = 8;      // frequencies per lane of k_tdft / k_spectro

// Pixel p of the block -> its element offset in frame 0.
__device__ __forceinline__ long pix_off(int p, int bw, long row_pitch) { return (long)(p / bw) * row_pitch + p % bw; }

}  // namespace

// X(p, f_k) = sum_t x_p(t) exp(-2 pi i f_k t / T) for the frequencies of
// blockIdx.y's tile: freqs[k] if freqs, else f = tile * 8 + k < nf.
//   REDUCE: per-workgroup sums of |X| over the pixels whose X is not NaN and
//           their count (np.nanmean's numerator / denominator) -> partial
//           [gridDim.x][nf][2]; X itself is not stored.
//   else:   X -> out [P][nf] (complex f64).
template <bool REDUCE, bool LDS, typename S>
__global__ __launch_bounds__(TD_THREADS) void k_tdft(const S* __restrict__ stack, long frame_pitch, long row_pitch,
                                                     int bw, int P, int T, const double2* __restrict__ tab,
                                                     const int* __restrict__ freqs, int nf, double2* __restrict__ out,
                                                     double* __restrict__ partial, int tchunk) {
    constexpr int FT = TD_FT_DFT, PX = TD_PX;
    // samples [t0, t1) of the series (blockIdx.z-th slice; one slice in REDUCE mode)
    const int t0 = blockIdx.z * tchunk, t1 = min(T, t0 + tchunk);
    extern __shared__ double2 tab_lds[];
    const double2* tb = tab;
    if constexpr (LDS) {
        for (int i = threadIdx.x; i < T; i += TD_THREADS) tab_lds[i] = tab[i];
        __syncthreads();
        tb = tab_lds;
    }
    // PX pixels per lane share each table read and index update (4 f64 FMAs per
    // LDS broadcast instead of 2)
    const int p0 = (blockIdx.x * TD_THREADS + threadIdx.x) * PX;
    bool live[PX];
    const S* xs[PX];
#pragma unroll
    for (int u = 0; u < PX; ++u) {
        live[u] = p0 + u < P;
        // lanes past the block read pixel 0 (loads stay unconditional, so a batch of
        // them is in flight at once); their sums are never used
        xs[u] = stack + (live[u] ? pix_off(p0 + u, bw, row_pitch) : 0);
    }
    int fk[FT], idx[FT];
    double re[PX][FT], im[PX][FT];
#pragma unroll
    for (int k = 0; k < FT; ++k) {
        const int j = blockIdx.y * FT + k;
        fk[k] = j < nf ? (freqs ? freqs[j] : j) : 0;
        idx[k] = (int)(((long)fk[k] * t0) % T);
#pragma unroll
        for (int u = 0; u < PX; ++u) re[u][k] = im[u][k] = 0.0;
    }
    auto step = [&](const S (&x)[PX]) {
#pragma unroll
        for (int k = 0; k < FT; ++k) {
            const double2 w = tb[idx[k]];  // wave-uniform index: an LDS broadcast
#pragma unroll
            for (int u = 0; u < PX; ++u) {
                re[u][k] = fma((double)x[u], w.x, re[u][k]);
                im[u][k] = fma((double)x[u], w.y, im[u][k]);
            }
            idx[k] += fk[k];
            idx[k] -= idx[k] >= T ? T : 0;
        }
    };
    // TD_BATCH samples loaded before any is used: that many loads in flight per
    // pixel and wave (few-bin calls have little arithmetic per sample to hide the latency)
    int t = t0;
    for (; t + TD_BATCH <= t1; t += TD_BATCH) {
        S xb[TD_BATCH][PX];
#pragma unroll
        for (int v = 0; v < TD_BATCH; ++v)
#pragma unroll
            for (int u = 0; u < PX; ++u) xb[v][u] = __builtin_nontemporal_load(xs[u] + (long)(t + v) * frame_pitch);
#pragma unroll
        for (int v = 0; v < TD_BATCH; ++v) step(xb[v]);
    }
    for (; t < t1; ++t) {
        S x1[PX];
#pragma unroll
        for (int u = 0; u < PX; ++u) x1[u] = __builtin_nontemporal_load(xs[u] + (long)t * frame_pitch);
        step(x1);
    }
    if constexpr (REDUCE) {
        __shared__ double red[TD_THREADS / 64][FT][2];
        const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
        for (int k = 0; k < FT; ++k) {
            double s = 0.0, c = 0.0;
#pragma unroll
            for (int u = 0; u < PX; ++u) {
                const double m = sqrt(re[u][k] * re[u][k] + im[u][k] * im[u][k]);
                const bool ok = live[u] && m == m;  // NaN samples make every bin NaN
                s += ok ? m : 0.0;
                c += ok ? 1.0 : 0.0;
            }
            for (int o = 32; o > 0; o >>= 1) {
                s += __shfl_xor(s, o, 64);
                c += __shfl_xor(c, o, 64);
            }
            if (lane == 0) {
                red[wave][k][0] = s;
                red[wave][k][1] = c;
            }
        }
        __syncthreads();
        if (threadIdx.x < FT * 2) {
            const int k = threadIdx.x >> 1, e = threadIdx.x & 1;
            const int j = blockIdx.y * FT + k;
            double acc = 0.0;
#pragma unroll
            for (int w = 0; w < TD_THREADS / 64; ++w) acc += red[w][k][e];
            if (j < nf) partial[((long)blockIdx.x * nf + j) * 2 + e] = acc;
        }
    } else {
#pragma unroll
        for (int u = 0; u < PX; ++u) {
            if (!live[u]) continue;
#pragma unroll
            for (int k = 0; k < FT; ++k) {
                const int j = blockIdx.y * FT + k;
                if (j < nf) out[((long)blockIdx.z * P + p0 + u) * nf + j] = make_double2(re[u][k], im[u][k]);
            }
        }
    }
}

// The mean-spectrum call as a GEMM on the f64 matrix cores: X[p][c] = sum_t
// x_p(t) E[t][c], E[t][2 f + e] = (cos, -sin)(2 pi f t / T)[e], with
// v_mfma_f64_16x16x4_f64 (A: lane l holds x[pixel l & 15][t + (l >> 4)], B: lane l
// holds E[t + (l >> 4)][column l & 15], C: column l & 15, row (l >> 4) + 4 r).  A
// wave owns 32 pixels x 32 bins (2 x 4 tiles of 16 x 16), so each A fragment feeds
// 4 MFMAs and each B fragment 2; B comes from the LDS table at a per-lane index
// (f t) mod T kept incrementally.  Same partial-sum output as k_tdft<true, true>.
typedef double dv4 __attribute__((ext_vector_type(4)));
#ifndef FCD_TM_WM
#define FCD_TM_WM 2  // 16-pixel tiles per wave
#endif
#ifndef FCD_TM_WN
#define FCD_TM_WN 4  // 8-bin (16-column) tiles per wave
#endif
constexpr int TM_WM = FCD_TM_WM, TM_WN = FCD_TM_WN;
constexpr int TM_PIX = 4 * 16 * TM_WM;  // pixels per workgroup (4 waves)
constexpr int TM_BINS = 8 * TM_WN;      // bins per workgroup

template <typename S>
__global__ __launch_bounds__(TD_THREADS) void k_tdft_mfma(const S* __restrict__ stack, long frame_pitch,
                                                          long row_pitch, int bw, int P, int T,
                                                          const double2* __restrict__ tab, int nf,
                                                          double* __restrict__ partial) {
    extern __shared__ double2 tm_lds[];
    for (int i = threadIdx.x; i < T; i += TD_THREADS) tm_lds[i] = tab[i];
    __syncthreads();
    const double* tl = reinterpret_cast<const double*>(tm_lds);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int kq = lane >> 4, col = lane & 15;
    const int pbase = blockIdx.x * TM_PIX + wave * 16 * TM_WM;
    const int fbase = blockIdx.y * TM_BINS;
    // A rows of this lane: pixels pbase + 16 m + col
    const S* xs[TM_WM];
    bool live[TM_WM];
#pragma unroll
    for (int m = 0; m < TM_WM; ++m) {
        const int p = pbase + 16 * m + col;
        live[m] = p < P;
        xs[m] = stack + (live[m] ? pix_off(p, bw, row_pitch) : 0);
    }
    // B columns of this lane: bin fbase + 8 n + col / 2, component col & 1
    int fq[TM_WN], idx[TM_WN], step4[TM_WN];
#pragma unroll
    for (int n = 0; n < TM_WN; ++n) {
        const int f = fbase + 8 * n + (col >> 1);
        fq[n] = f < nf ? f : 0;
        idx[n] = (int)(((long)fq[n] * kq) % T);
        step4[n] = (int)(((long)fq[n] * 4) % T);
    }
    const int comp = col & 1;
    dv4 acc[TM_WM][TM_WN];
#pragma unroll
    for (int m = 0; m < TM_WM; ++m)
#pragma unroll
        for (int n = 0; n < TM_WN; ++n) acc[m][n] = dv4{0.0, 0.0, 0.0, 0.0};
    auto kstep = [&](const S (&xa)[TM_WM], int t) {
        double a[TM_WM], b[TM_WN];
#pragma unroll
        for (int m = 0; m < TM_WM; ++m) a[m] = t + kq < T ? (double)xa[m] : 0.0;
#pragma unroll
        for (int n = 0; n < TM_WN; ++n) {
            b[n] = tl[2 * idx[n] + comp];
            idx[n] += step4[n];
            idx[n] -= idx[n] >= T ? T : 0;
        }
#pragma unroll
        for (int m = 0; m < TM_WM; ++m)
#pragma unroll
            for (int n = 0; n < TM_WN; ++n)
                acc[m][n] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[m], b[n], acc[m][n], 0, 0, 0);
    };
    // batches of TM_B K-steps: their A loads are in flight together
    constexpr int TM_B = 4;
    int t = 0;
    for (; t < T; t += 4 * TM_B) {
        S xa[TM_B][TM_WM];
#pragma unroll
        for (int q = 0; q < TM_B; ++q) {
            const int tt = min(t + 4 * q + kq, T - 1);  // clamped: samples past T are zeroed in kstep
#pragma unroll
            for (int m = 0; m < TM_WM; ++m) xa[q][m] = __builtin_nontemporal_load(xs[m] + (long)tt * frame_pitch);
        }
#pragma unroll
        for (int q = 0; q < TM_B; ++q)
            if (t + 4 * q < T) kstep(xa[q], t + 4 * q);
    }
    // |X| per (pixel, bin): re in the even column lane, im in the odd one
    __shared__ double red[TD_THREADS / 64][TM_BINS][2];
#pragma unroll
    for (int n = 0; n < TM_WN; ++n) {
        double s = 0.0, c = 0.0;
#pragma unroll
        for (int m = 0; m < TM_WM; ++m)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const double v = acc[m][n][r];
                const double w = __shfl_xor(v, 1, 64);
                const double mag = sqrt(v * v + w * w);
                const int p = pbase + 16 * m + kq + 4 * r;
                const bool ok = !comp && p < P && mag == mag;  // NaN samples make every bin NaN
                s += ok ? mag : 0.0;
                c += ok ? 1.0 : 0.0;
            }
        s += __shfl_xor(s, 16, 64);
        c += __shfl_xor(c, 16, 64);
        s += __shfl_xor(s, 32, 64);
        c += __shfl_xor(c, 32, 64);
        if (lane < 16 && !comp) {
            red[wave][8 * n + (col >> 1)][0] = s;
            red[wave][8 * n + (col >> 1)][1] = c;
        }
    }
    __syncthreads();
    if (threadIdx.x < TM_BINS * 2) {
        const int k = threadIdx.x >> 1, e = threadIdx.x & 1;
        const int j = fbase + k;
        double a = 0.0;
#pragma unroll
        for (int w = 0; w < TD_THREADS / 64; ++w) a += red[w][k][e];
        if (j < nf) partial[((long)blockIdx.x * nf + j) * 2 + e] = a;
    }
}

// Spectrogram segments on the matrix cores, as k_tdft_mfma: for segment blockIdx.y,
// X[p][2f+e] = sum_n x_p(s0 + n) w_n E[n][2f+e] (B = window x table, gathered per
// lane), the segment means from the A fragments (x_p summed over the lanes holding
// pixel p's samples), then S = |X - mean W_f|^2 scale (x2 off DC / Nyquist).
template <typename S>
__global__ __launch_bounds__(TD_THREADS) void k_spectro_mfma(const S* __restrict__ stack, long frame_pitch,
                                                             long row_pitch, int bw, int P, int nperseg, int step,
                                                             int nseg, const double* __restrict__ win,
                                                             const double2* __restrict__ tab,
                                                             const double2* __restrict__ wsum, int nf, double scale,
                                                             double* __restrict__ out) {
    extern __shared__ double2 sm_lds[];
    double2* const tb = sm_lds;                                     // [nperseg]
    double* const wl = reinterpret_cast<double*>(sm_lds + nperseg);  // [nperseg]
    for (int i = threadIdx.x; i < nperseg; i += TD_THREADS) {
        tb[i] = tab[i];
        wl[i] = win[i];
    }
    __syncthreads();
    const double* tl = reinterpret_cast<const double*>(tb);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int kq = lane >> 4, col = lane & 15, comp = col & 1;
    const int pbase = blockIdx.x * TM_PIX + wave * 16 * TM_WM;
    const int seg = blockIdx.y;
    const int fbase = blockIdx.z * TM_BINS;
    const S* xs[TM_WM];
#pragma unroll
    for (int m = 0; m < TM_WM; ++m) {
        const int p = pbase + 16 * m + col;
        xs[m] = stack + (p < P ? pix_off(p, bw, row_pitch) : 0) + (long)seg * step * frame_pitch;
    }
    int fq[TM_WN], idx[TM_WN], step4[TM_WN];
#pragma unroll
    for (int n = 0; n < TM_WN; ++n) {
        const int f = fbase + 8 * n + (col >> 1);
        fq[n] = f < nf ? f : 0;
        idx[n] = (fq[n] * kq) % nperseg;
        step4[n] = (fq[n] * 4) % nperseg;
    }
    dv4 acc[TM_WM][TM_WN];
    double sx[TM_WM];
#pragma unroll
    for (int m = 0; m < TM_WM; ++m) {
        sx[m] = 0.0;
#pragma unroll
        for (int n = 0; n < TM_WN; ++n) acc[m][n] = dv4{0.0, 0.0, 0.0, 0.0};
    }
    constexpr int TM_B = 4;
    for (int n0 = 0; n0 < nperseg; n0 += 4 * TM_B) {
        S xa[TM_B][TM_WM];
#pragma unroll
        for (int q = 0; q < TM_B; ++q) {
            const int nn = min(n0 + 4 * q + kq, nperseg - 1);  // clamped: samples past the segment are zeroed
#pragma unroll
            for (int m = 0; m < TM_WM; ++m) xa[q][m] = __builtin_nontemporal_load(xs[m] + (long)nn * frame_pitch);
        }
#pragma unroll
        for (int q = 0; q < TM_B; ++q) {
            const int nk = n0 + 4 * q;
            if (nk >= nperseg) break;
            const bool in = nk + kq < nperseg;
            const double wn = in ? wl[nk + kq] : 0.0;
            double a[TM_WM], b[TM_WN];
#pragma unroll
            for (int m = 0; m < TM_WM; ++m) {
                a[m] = in ? (double)xa[q][m] : 0.0;
                sx[m] += a[m];
            }
#pragma unroll
            for (int n = 0; n < TM_WN; ++n) {
                b[n] = wn * tl[2 * idx[n] + comp];
                idx[n] += step4[n];
                idx[n] -= idx[n] >= nperseg ? nperseg : 0;
            }
#pragma unroll
            for (int m = 0; m < TM_WM; ++m)
#pragma unroll
                for (int n = 0; n < TM_WN; ++n)
                    acc[m][n] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[m], b[n], acc[m][n], 0, 0, 0);
        }
    }
    // segment sums per pixel: lanes with the same column hold its four sample phases
#pragma unroll
    for (int m = 0; m < TM_WM; ++m) {
        sx[m] += __shfl_xor(sx[m], 16, 64);
        sx[m] += __shfl_xor(sx[m], 32, 64);
    }
    const double inv_n = 1.0 / (double)nperseg;
#pragma unroll
    for (int m = 0; m < TM_WM; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = kq + 4 * r;  // pixel pbase + 16 m + row; its sum sits in lane `row`
            const double mean = __shfl(sx[m], row, 64) * inv_n;
            const int p = pbase + 16 * m + row;
#pragma unroll
            for (int n = 0; n < TM_WN; ++n) {
                const int f = fbase + 8 * n + (col >> 1);
                const double2 W = wsum[fq[n]];
                const double v = acc[m][n][r] - mean * (comp ? W.y : W.x);
                const double o = __shfl_xor(v, 1, 64);
                if (!comp && p < P && f < nf) {
                    double sp = (v * v + o * o) * scale;
                    if (f > 0 && !(nperseg % 2 == 0 && f == nperseg / 2)) sp *= 2.0;
                    out[((long)p * nf + f) * nseg + seg] = sp;
                }
            }
        }
}

// out[i] = sum over the nz time slices of parts[z][i], in slice order (deterministic).
__global__ __launch_bounds__(TD_THREADS) void k_tdft_sum(const double2* __restrict__ parts, int nz, long n,
                                                         double2* __restrict__ out) {
    const long i = (long)blockIdx.x * TD_THREADS + threadIdx.x;
    if (i >= n) return;
    double2 a = parts[i];
    for (int z = 1; z < nz; ++z) {
        const double2 b = parts[(long)z * n + i];
        a.x += b.x;
        a.y += b.y;
    }
    out[i] = a;
}

// One-sided PSD of every segment of every pixel (scipy.signal.spectrogram with
// detrend='constant', scaling='density', mode='psd'):
//   X_f = sum_n (x_n - mean) w_n e_fn = sum_n x_n w_n e_fn - mean * W_f,
//   W_f = sum_n w_n e_fn (host, f64), so the segment is read once;
//   S_f = |X_f|^2 * scale, doubled except at DC and (even nperseg) Nyquist.
// out [P][nf][nseg]; grid (pixel tiles, segments, frequency tiles).
template <typename S>
__global__ __launch_bounds__(TD_THREADS) void k_spectro(const S* __restrict__ stack, long frame_pitch,
                                                        long row_pitch, int bw, int P, int nperseg, int step,
                                                        int nseg, const double* __restrict__ win,
                                                        const double2* __restrict__ tab,
                                                        const double2* __restrict__ wsum, int nf, double scale,
                                                        double* __restrict__ out) {
    extern __shared__ double2 sp_lds[];
    double2* const tb = sp_lds;                                     // [nperseg]
    double* const wl = reinterpret_cast<double*>(sp_lds + nperseg);  // [nperseg]
    for (int i = threadIdx.x; i < nperseg; i += TD_THREADS) {
        tb[i] = tab[i];
        wl[i] = win[i];
    }
    __syncthreads();
    constexpr int FT = TD_FT_DFT, PX = TD_PX;  // as k_tdft: 4 f64 FMAs per table read
    const int p0 = (blockIdx.x * TD_THREADS + threadIdx.x) * PX;
    const int seg = blockIdx.y;
    bool live[PX];
    const S* xs[PX];
#pragma unroll
    for (int u = 0; u < PX; ++u) {
        live[u] = p0 + u < P;
        xs[u] = stack + (live[u] ? pix_off(p0 + u, bw, row_pitch) : 0) + (long)seg * step * frame_pitch;
    }
    int fk[FT], idx[FT];
    double re[PX][FT], im[PX][FT], sum[PX];
#pragma unroll
    for (int k = 0; k < FT; ++k) {
        const int j = blockIdx.z * FT + k;
        fk[k] = j < nf ? j : 0;
        idx[k] = 0;
#pragma unroll
        for (int u = 0; u < PX; ++u) re[u][k] = im[u][k] = 0.0;
    }
#pragma unroll
    for (int u = 0; u < PX; ++u) sum[u] = 0.0;
    auto sample = [&](int n, const S (&x)[PX]) {
        const double wn = wl[n];
        double xw[PX];
#pragma unroll
        for (int u = 0; u < PX; ++u) {
            sum[u] += (double)x[u];
            xw[u] = (double)x[u] * wn;
        }
#pragma unroll
        for (int k = 0; k < FT; ++k) {
            const double2 w = tb[idx[k]];
#pragma unroll
            for (int u = 0; u < PX; ++u) {
                re[u][k] = fma(xw[u], w.x, re[u][k]);
                im[u][k] = fma(xw[u], w.y, im[u][k]);
            }
            idx[k] += fk[k];
            idx[k] -= idx[k] >= nperseg ? nperseg : 0;
        }
    };
    int n = 0;  // unconditional batched loads, as k_tdft
    for (; n + TD_BATCH <= nperseg; n += TD_BATCH) {
        S xb[TD_BATCH][PX];
#pragma unroll
        for (int v = 0; v < TD_BATCH; ++v)
#pragma unroll
            for (int u = 0; u < PX; ++u) xb[v][u] = xs[u][(long)(n + v) * frame_pitch];
#pragma unroll
        for (int v = 0; v < TD_BATCH; ++v) sample(n + v, xb[v]);
    }
    for (; n < nperseg; ++n) {
        S x1[PX];
#pragma unroll
        for (int u = 0; u < PX; ++u) x1[u] = xs[u][(long)n * frame_pitch];
        sample(n, x1);
    }
#pragma unroll
    for (int u = 0; u < PX; ++u) {
        if (!live[u]) continue;
        const double mean = sum[u] / (double)nperseg;
#pragma unroll
        for (int k = 0; k < FT; ++k) {
            const int j = blockIdx.z * FT + k;
            if (j >= nf) continue;
            const double2 W = wsum[j];
            const double xr = re[u][k] - mean * W.x, xi = im[u][k] - mean * W.y;
            double sp = (xr * xr + xi * xi) * scale;
            if (j > 0 && !(nperseg % 2 == 0 && j == nperseg / 2)) sp *= 2.0;
            out[((long)(p0 + u) * nf + j) * nseg + seg] = sp;
        }
    }
}

namespace {

void check_launch(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

// Time slices of a few-bin (REDUCE = false) call: enough workgroups to fill the chip
// (>= 1024), at least 256 samples per slice.
int temporal_bins_slices(int P, int nf, int T) {
    const long blocks = (long)temporal_dft_tiles(P) * ((nf + TD_FT_DFT - 1) / TD_FT_DFT);
    const long want = (1024 + blocks - 1) / blocks;
    return (int)std::max(1L, std::min(want, (long)T / 256));
}

// FCD_TDFT_VALU=1 selects the vector-unit kernels (read per call, so one process
// can test both families)
static bool spectrum_on_mfma(int T) {
    const char* e = std::getenv("FCD_TDFT_VALU");
    return !(e && e[0] == '1') && T <= TD_LDS_TAB;
}

int temporal_spectrum_tiles(int P, int T) {
    return spectrum_on_mfma(T) ? (P + TM_PIX - 1) / TM_PIX : temporal_dft_tiles(P);
}

namespace {

template <typename S>
void temporal_dft_t(const S* stack, long frame_pitch, long row_pitch, int bw, int P, int T, const double2* tab,
                    const int* freqs, int nf, double2* out, double* partial, double2* slices, hipStream_t s) {
    if (partial && !freqs && spectrum_on_mfma(T)) {
        const dim3 g((unsigned)((P + TM_PIX - 1) / TM_PIX), (unsigned)((nf + TM_BINS - 1) / TM_BINS));
        const size_t lb = (size_t)T * sizeof(double2);
        (void)hipFuncSetAttribute((const void*)k_tdft_mfma<S>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lb);
        hipLaunchKernelGGL(k_tdft_mfma<S>, g, dim3(TD_THREADS), lb, s, stack, frame_pitch, row_pitch, bw, P, T, tab, nf,
                           partial);
        check_launch("temporal_dft (mfma)");
        return;
    }
    const int nz = partial ? 1 : temporal_bins_slices(P, nf, T);
    const int tchunk = (T + nz - 1) / nz;
    const dim3 grid((unsigned)temporal_dft_tiles(P), (unsigned)((nf + TD_FT_DFT - 1) / TD_FT_DFT), (unsigned)nz);
    const bool lds = T <= TD_LDS_TAB;
    const size_t lb = lds ? (size_t)T * sizeof(double2) : 0;
    double2* dst = nz > 1 ? slices : out;
    if (nz > 1 && !slices) throw std::runtime_error("temporal_dft: slice workspace missing");
    if (partial) {
        if (lds) {
            (void)hipFuncSetAttribute((const void*)k_tdft<true, true, S>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)lb);
            hipLaunchKernelGGL((k_tdft<true, true, S>), grid, dim3(TD_THREADS), lb, s, stack, frame_pitch, row_pitch,
                               bw, P, T, tab, freqs, nf, dst, partial, tchunk);
        } else {
            hipLaunchKernelGGL((k_tdft<true, false, S>), grid, dim3(TD_THREADS), 0, s, stack, frame_pitch, row_pitch,
                               bw, P, T, tab, freqs, nf, dst, partial, tchunk);
        }
    } else {
        if (lds) {
            (void)hipFuncSetAttribute((const void*)k_tdft<false, true, S>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)lb);
            hipLaunchKernelGGL((k_tdft<false, true, S>), grid, dim3(TD_THREADS), lb, s, stack, frame_pitch, row_pitch,
                               bw, P, T, tab, freqs, nf, dst, partial, tchunk);
        } else {
            hipLaunchKernelGGL((k_tdft<false, false, S>), grid, dim3(TD_THREADS), 0, s, stack, frame_pitch, row_pitch,
                               bw, P, T, tab, freqs, nf, dst, partial, tchunk);
        }
        if (nz > 1) {
            const long n = (long)P * nf;
            hipLaunchKernelGGL(k_tdft_sum, dim3((unsigned)((n + TD_THREADS - 1) / TD_THREADS)), dim3(TD_THREADS), 0, s,
                               slices, nz, n, out);
        }
    }
    check_launch("temporal_dft");
}

template <typename S>
void spectrogram_t(const S* stack, long frame_pitch, long row_pitch, int bw, int P, int nperseg, int step, int nseg,
                   const double* win, const double2* tab, const double2* wsum, int nf, double scale, double* out,
                   hipStream_t s) {
    const size_t lb = (size_t)nperseg * (sizeof(double2) + sizeof(double));
    if (spectrum_on_mfma(0)) {
        const dim3 g((unsigned)((P + TM_PIX - 1) / TM_PIX), (unsigned)nseg, (unsigned)((nf + TM_BINS - 1) / TM_BINS));
        (void)hipFuncSetAttribute((const void*)k_spectro_mfma<S>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lb);
        hipLaunchKernelGGL(k_spectro_mfma<S>, g, dim3(TD_THREADS), lb, s, stack, frame_pitch, row_pitch, bw, P, nperseg,
                           step, nseg, win, tab, wsum, nf, scale, out);
        check_launch("spectrogram (mfma)");
        return;
    }
    const dim3 grid((unsigned)temporal_dft_tiles(P), (unsigned)nseg, (unsigned)((nf + TD_FT_DFT - 1) / TD_FT_DFT));
    (void)hipFuncSetAttribute((const void*)k_spectro<S>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lb);
    hipLaunchKernelGGL(k_spectro<S>, grid, dim3(TD_THREADS), lb, s, stack, frame_pitch, row_pitch, bw, P, nperseg, step,
                       nseg, win, tab, wsum, nf, scale, out);
    check_launch("spectrogram");
}

}  // namespace

void temporal_dft(Samples stack, long frame_pitch, long row_pitch, int bw, int P, int T, const double2* tab,
                  const int* freqs, int nf, double2* out, double* partial, double2* slices, hipStream_t s) {
    if (P <= 0 || T <= 0 || nf <= 0) return;
    if (stack.f64)
        temporal_dft_t(static_cast<const double*>(stack.p), frame_pitch, row_pitch, bw, P, T, tab, freqs, nf, out,
                       partial, slices, s);
    else
        temporal_dft_t(static_cast<const float*>(stack.p), frame_pitch, row_pitch, bw, P, T, tab, freqs, nf, out,
                       partial, slices, s);
}

int temporal_dft_tiles(int P) { return (P + TD_THREADS * TD_PX - 1) / (TD_THREADS * TD_PX); }

int spectro_max_nperseg() { return 160 * 1024 / 24; }

void spectrogram(Samples stack, long frame_pitch, long row_pitch, int bw, int P, int nperseg, int step, int nseg,
                 const double* win, const double2* tab, const double2* wsum, int nf, double scale, double* out,
                 hipStream_t s) {
    if (P <= 0 || nseg <= 0) return;
    if (stack.f64)
        spectrogram_t(static_cast<const double*>(stack.p), frame_pitch, row_pitch, bw, P, nperseg, step, nseg, win, tab,
                      wsum, nf, scale, out, s);
    else
        spectrogram_t(static_cast<const float*>(stack.p), frame_pitch, row_pitch, bw, P, nperseg, step, nseg, win, tab,
                      wsum, nf, scale, out, s);
}

}  // namespace fcdk
