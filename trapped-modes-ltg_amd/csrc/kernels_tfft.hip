// Mean amplitude spectrum of a long map stack by FFT (SURVEY.md §8f row 4,
// analyze.block_amplitude, analyze.py:543-587: np.nanmean(|np.fft.fft(series)|)
// over the pixels of a block, f64).
//
// The direct DFT of kernels_temporal.hip costs T x (T/2 + 1) MACs per pixel; for a
// long series this path costs O(M log M) with M = 2^ceil(log2(2T - 1)), for any T
// (the number of maps is rarely a power of two), by Bluestein's identity
//   X[k] = c[k] sum_n (x[n] c[n]) conj(c[k - n]),  c[n] = exp(-i pi n^2 / T),
// a circular convolution of length M done as FFT -> pointwise product with
// B = FFT(b) (b = conj(c) wrapped, built on the host) -> inverse FFT.  Only |X[k]| is
// wanted and |c[k]| = 1, so the last chirp multiply is skipped; 1/M is folded into B.
//
// Each length-M transform is a four-step FFT, M = M1 x M2 (both <= 1024, so
// T <= 2^19), n = M2 n1 + n2, k = k1 + M1 k2, with every sub-transform inside one
// workgroup's LDS and the data in HBM only between the steps:
//   k_tfft_cols_fwd  reads the stack (x c, zero past T), FFT over n1, twiddle
//                    W_M^(n2 k1) -> work[k1][n2]
//   k_tfft_rows      FFT over n2 -> X[k1 + M1 k2], times B, inverse FFT over k2,
//                    twiddle W_M^(-n2 k1), in place
//   k_tfft_cols_inv  inverse FFT over k1 -> conv[M2 n1 + n2]; per-bin sums of |.|
//                    over 64 pixels (NaN pixels excluded, np.nanmean)
//   k_tfft_sum       fixed-order sum of those partials (deterministic)
// so a pixel costs one read of its series plus 4 x 16 B x M of HBM traffic.
// The work array is [8-pixel group][M][8 pixels] (one 128 B segment per time slot of a
// group, a group's M slots contiguous) and the time index is the fastest block index, so
// the workgroups in flight together write / read neighbouring segments (r02u: with a
// [M][batch] layout the 16 KB row stride held every step to a third of HBM bandwidth).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include "kernels.hpp"

namespace fcdk {

namespace {

constexpr int TF_NT = 256;  // threads per workgroup
constexpr int TF_G = 8;     // pixels transformed together (8 x 16 B per time step)
constexpr int TF_GS = 64;   // pixels summed per workgroup of the last step

__device__ __forceinline__ long tf_pix_off(int p, int bw, long row_pitch) { return (long)(p / bw) * row_pitch + p % bw; }

__device__ __forceinline__ double2 zmul(double2 a, double2 b) {
    return make_double2(fma(a.x, b.x, -a.y * b.y), fma(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ double2 zmulc(double2 a, double2 b) {  // a conj(b)
    return make_double2(fma(a.x, b.x, a.y * b.y), fma(a.y, b.x, -a.x * b.y));
}

// cos(2 pi q / 16), folded to a constant once the callers' loops are unrolled
__device__ __forceinline__ constexpr double c16(int q) {
    switch (q & 15) {
        case 0: return 1.0;
        case 1: case 15: return 0.92387953251128674;
        case 2: case 14: return 0.70710678118654752;
        case 3: case 13: return 0.38268343236508977;
        case 4: case 12: return 0.0;
        case 5: case 11: return -0.38268343236508977;
        case 6: case 10: return -0.70710678118654752;
        case 7: case 9: return -0.92387953251128674;
        default: return -1.0;
    }
}

constexpr int ilog2c(int n) { return n <= 1 ? 0 : 1 + ilog2c(n >> 1); }

// In-register DFT of R <= 16 points (natural order in and out): radix-2 DIT after a
// compile-time bit reversal; forward exp(-2 pi i nk / R), INV exp(+...).
template <int R, bool INV>
__device__ __forceinline__ void dft_reg(double2 (&v)[R]) {
    constexpr int LR = ilog2c(R);
#pragma unroll
    for (int i = 0; i < R; ++i) {
        int j = 0;
#pragma unroll
        for (int b = 0; b < LR; ++b) j |= ((i >> b) & 1) << (LR - 1 - b);
        if (j > i) {
            const double2 t = v[i];
            v[i] = v[j];
            v[j] = t;
        }
    }
#pragma unroll
    for (int len = 2; len <= R; len <<= 1) {
#pragma unroll
        for (int i = 0; i < R; i += len) {
#pragma unroll
            for (int k = 0; k < len / 2; ++k) {
                const int q = k * (16 / len);
                const double2 a = v[i + k], b = v[i + k + len / 2];
                double2 t;
                if (q == 0) {
                    t = b;
                } else if (q == 4) {  // w = -i (forward) / +i (inverse)
                    t = INV ? make_double2(-b.y, b.x) : make_double2(b.y, -b.x);
                } else {
                    const double wr = c16(q), wi = INV ? c16(q - 4) : -c16(q - 4);
                    t = make_double2(fma(b.x, wr, -b.y * wi), fma(b.x, wi, b.y * wr));
                }
                v[i + k] = make_double2(a.x + t.x, a.y + t.y);
                v[i + k + len / 2] = make_double2(a.x - t.x, a.y - t.y);
            }
        }
    }
}

// LDS slot of element e of the G interleaved transforms: 8 pad slots (128 B) after
// every 128, so the two butterflies a 16-lane group writes in a radix-16 pass of
// sub-transform length 1 (2 KB apart) land on different banks.
__device__ __forceinline__ int lp(int e) { return e + ((e >> 7) << 3); }
template <int LOGL>
constexpr int lds_slots() { return (1 << LOGL) * TF_G + (((1 << LOGL) * TF_G) >> 7) * 8; }

// One radix-R Stockham pass (sub-transforms of length p merged into length pR) over
// the G interleaved transforms of length L in buf[lp(n * G + g)], in place: every
// butterfly is read into registers before the barrier, written after it.
// Twiddles W_{pR}^(r k) = twl[(r k) << (LOGL - log2(pR))], twl[j] = exp(-2 pi i j / L)
// (the workgroup's table in LDS).
template <int LOGL, int LOGP, int LOGR, bool INV>
__device__ __forceinline__ void lds_pass(double2* buf, const double2* twl) {
    constexpr int L = 1 << LOGL, R = 1 << LOGR, p = 1 << LOGP;
    constexpr int NB = (L / R) * TF_G;
    constexpr int BPT = (NB + TF_NT - 1) / TF_NT;
    constexpr int SH = LOGL - LOGP - LOGR;
    double2 v[BPT][R];
    int dst[BPT];
#pragma unroll
    for (int u = 0; u < BPT; ++u) {
        const int b = threadIdx.x + u * TF_NT;
        dst[u] = -1;
        if (NB % TF_NT == 0 || b < NB) {
            const int g = b % TF_G, i = b / TF_G, k = i & (p - 1);
#pragma unroll
            for (int r = 0; r < R; ++r) v[u][r] = buf[lp((i + r * (L / R)) * TF_G + g)];
            if constexpr (p > 1) {
#pragma unroll
                for (int r = 1; r < R; ++r) {
                    const double2 w = twl[(r * k) << SH];
                    v[u][r] = INV ? zmulc(v[u][r], w) : zmul(v[u][r], w);
                }
            }
            dft_reg<R, INV>(v[u]);
            dst[u] = ((i - k) * R + k) * TF_G + g;
        }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < BPT; ++u) {
        if (dst[u] < 0) continue;
#pragma unroll
        for (int r = 0; r < R; ++r) buf[lp(dst[u] + r * p * TF_G)] = v[u][r];
    }
    __syncthreads();
}

template <int LOGL, int LOGP, bool INV>
__device__ __forceinline__ void lds_fft_from(double2* buf, const double2* twl) {
    if constexpr (LOGP < LOGL) {
        constexpr int LOGR = LOGL - LOGP >= 4 ? 4 : LOGL - LOGP;
        lds_pass<LOGL, LOGP, LOGR, INV>(buf, twl);
        lds_fft_from<LOGL, LOGP + LOGR, INV>(buf, twl);
    }
}

// G interleaved length-2^LOGL transforms in LDS, natural order in and out; the
// caller has synchronised after filling buf and twl, and buf is synchronised on return.
template <int LOGL, bool INV>
__device__ __forceinline__ void lds_fft(double2* buf, const double2* twl) {
    lds_fft_from<LOGL, 0, INV>(buf, twl);
}

// twl[j] = exp(-2 pi i j / L) from the global exp(-2 pi i j / M) table (synchronised
// by the caller's barrier after its own fill)
template <int LOGL>
__device__ __forceinline__ void load_twl(double2* twl, const double2* __restrict__ tw, int logM) {
    for (int j = threadIdx.x; j < (1 << LOGL); j += TF_NT) twl[j] = tw[(long)j << (logM - LOGL)];
}

}  // namespace

// Step 1: column n2 = bx of group by: pixels [pbase + 8 by, +8), or with PAIR the 8
// pixel pairs (p, p + 8), p in [pbase + 16 by, +8), as x_p + i x_{p+8} (a pixel with a
// NaN sample, bad[p], enters as zeros: np.nanmean drops it anyway; a block with an
// infinity never runs paired).
template <int LOG1, typename S, bool PAIR>
__global__ __launch_bounds__(TF_NT) void k_tfft_cols_fwd(const S* __restrict__ stack, long frame_pitch,
                                                         long row_pitch, int bw, int P, int T, int pbase,
                                                         const int* __restrict__ bad,
                                                         const double2* __restrict__ chirp,
                                                         const double2* __restrict__ tw, int logM, int M2,
                                                         double2* __restrict__ work) {
    constexpr int M1 = 1 << LOG1;
    extern __shared__ double2 tf_buf[];
    double2* const twl = tf_buf + lds_slots<LOG1>();
    const int n2 = blockIdx.x, grp = blockIdx.y;
    const long M = 1L << logM;
    load_twl<LOG1>(twl, tw, logM);
    if constexpr (PAIR) {
        const int g = threadIdx.x % TF_G;  // fixed per thread (TF_NT % TF_G == 0)
        const int pa = pbase + grp * 2 * TF_G + g, pb = pa + TF_G;
        const bool oka = pa < P && !bad[pa], okb = pb < P && !bad[pb];
        const S* xa = stack + (oka ? tf_pix_off(pa, bw, row_pitch) : 0);
        const S* xb = stack + (okb ? tf_pix_off(pb, bw, row_pitch) : 0);
        for (int e = threadIdx.x; e < M1 * TF_G; e += TF_NT) {
            const long t = (long)M2 * (e / TF_G) + n2;
            double2 v = make_double2(0.0, 0.0);
            if (t < T) {
                const double a = oka ? (double)xa[t * frame_pitch] : 0.0;
                const double b = okb ? (double)xb[t * frame_pitch] : 0.0;
                const double2 c = chirp[t];
                v = make_double2(a * c.x - b * c.y, a * c.y + b * c.x);
            }
            tf_buf[lp(e)] = v;
        }
    } else {
        const int g0 = grp * TF_G;
        for (int e = threadIdx.x; e < M1 * TF_G; e += TF_NT) {
            const int n1 = e / TF_G, g = e % TF_G, p = pbase + g0 + g;
            const long t = (long)M2 * n1 + n2;
            double2 v = make_double2(0.0, 0.0);
            if (t < T && p < P) {
                const double x = (double)stack[tf_pix_off(p, bw, row_pitch) + t * frame_pitch];
                const double2 c = chirp[t];
                v = make_double2(x * c.x, x * c.y);
            }
            tf_buf[lp(e)] = v;
        }
    }
    __syncthreads();
    lds_fft<LOG1, false>(tf_buf, twl);
    for (int e = threadIdx.x; e < M1 * TF_G; e += TF_NT) {
        const int k1 = e / TF_G, g = e % TF_G;
        work[(grp * M + (long)k1 * M2 + n2) * TF_G + g] = zmul(tf_buf[lp(e)], tw[(long)n2 * k1]);
    }
}

// Step 2: row k1 = by of pixels [8 bx, +8): forward FFT, times B, inverse FFT, twiddle.
template <int LOG2>
__global__ __launch_bounds__(TF_NT) void k_tfft_rows(double2* __restrict__ work,
                                                     const double2* __restrict__ bhat,
                                                     const double2* __restrict__ tw, int logM) {
    constexpr int M2 = 1 << LOG2;
    extern __shared__ double2 tf_buf[];
    double2* const twl = tf_buf + lds_slots<LOG2>();
    const int k1 = blockIdx.x, grp = blockIdx.y;
    double2* const row = work + (((long)grp << logM) + (long)k1 * M2) * TF_G;  // M2 x 8 contiguous
    load_twl<LOG2>(twl, tw, logM);
    for (int e = threadIdx.x; e < M2 * TF_G; e += TF_NT) tf_buf[lp(e)] = row[e];
    __syncthreads();
    lds_fft<LOG2, false>(tf_buf, twl);
    for (int e = threadIdx.x; e < M2 * TF_G; e += TF_NT)
        tf_buf[lp(e)] = zmul(tf_buf[lp(e)], bhat[(long)k1 * M2 + e / TF_G]);
    __syncthreads();
    lds_fft<LOG2, true>(tf_buf, twl);
    for (int e = threadIdx.x; e < M2 * TF_G; e += TF_NT) {
        const int n2 = e / TF_G;
        row[e] = zmulc(tf_buf[lp(e)], tw[(long)n2 * k1]);
    }
}

// Step 3: column n2 = by, pixels [pbase + 64 bx, +64) in 8 groups: inverse FFT over
// k1, then per output time n = M2 n1 + n2 < nf the sum of |conv| over the pixels
// whose transform is not NaN and their count -> gpart[(pbase / 64 + bx) * nf + n].
template <int LOG1>
__global__ __launch_bounds__(TF_NT) void k_tfft_cols_inv(const double2* __restrict__ work, int M2,
                                                         const double2* __restrict__ tw, int logM, int nf,
                                                         int pbase, int P, double2* __restrict__ gpart) {
    constexpr int M1 = 1 << LOG1, PER = (M1 + TF_NT - 1) / TF_NT;
    extern __shared__ double2 tf_buf[];
    double2* const twl = tf_buf + lds_slots<LOG1>();
    const int n2 = blockIdx.x, s0 = blockIdx.y * TF_GS;
    const long M = 1L << logM;
    if (pbase + s0 >= P) return;  // whole workgroup past the block: no partial row of its own
    load_twl<LOG1>(twl, tw, logM);
    double acc_s[PER], acc_c[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) acc_s[u] = acc_c[u] = 0.0;
    for (int sub = 0; sub < TF_GS / TF_G; ++sub) {
        const int g0 = s0 + sub * TF_G;
        if (pbase + g0 >= P) break;  // uniform across the workgroup
        for (int e = threadIdx.x; e < M1 * TF_G; e += TF_NT)
            tf_buf[lp(e)] = work[((long)(g0 / TF_G) * M + (long)(e / TF_G) * M2 + n2) * TF_G + e % TF_G];
        __syncthreads();
        lds_fft<LOG1, true>(tf_buf, twl);
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int n1 = threadIdx.x + u * TF_NT;
            if (M1 % TF_NT != 0 && n1 >= M1) continue;
            // pixel (j + n1) mod 8 at step j: the 8 lanes sharing a 256 B bank window
            // read different banks
#pragma unroll
            for (int j = 0; j < TF_G; ++j) {
                const int g = (j + n1) & (TF_G - 1);
                const double2 z = tf_buf[lp(n1 * TF_G + g)];
                const double m = sqrt(z.x * z.x + z.y * z.y);
                const bool ok = pbase + g0 + g < P && m == m;
                acc_s[u] += ok ? m : 0.0;
                acc_c[u] += ok ? 1.0 : 0.0;
            }
        }
        __syncthreads();
    }
    const long grp = pbase / TF_GS + blockIdx.y;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int n1 = threadIdx.x + u * TF_NT;
        const long n = (long)M2 * n1 + n2;
        if (n1 < M1 && n < nf) gpart[grp * nf + n] = make_double2(acc_s[u], acc_c[u]);
    }
}

// Pixels of the block with a non-finite sample (any t): bad[p] |= 1 for a NaN, |= 2 for
// an infinity (zeroed beforehand).  A NaN makes every bin of the pixel's np.fft NaN, so
// np.nanmean leaves the pixel out: the paired path drops it (bad != 0).  An infinity
// (and no NaN) gives inf / NaN bins that must stay the pixel's own: such a block runs
// unpaired (temporal_inf_pixels), so it never reaches a partner series through
// z = x_p + i x_q.
template <typename S>
__global__ __launch_bounds__(TF_NT) void k_tfft_flags(const S* __restrict__ stack, long frame_pitch, long row_pitch,
                                                      int bw, int P, int T, int* __restrict__ bad) {
    const int p = blockIdx.x * TF_NT + threadIdx.x;
    if (p >= P) return;
    const S* x = stack + tf_pix_off(p, bw, row_pitch);
    const int t0 = blockIdx.y * TF_NT, t1 = min(T, t0 + TF_NT);
    int code = 0;
    int t = t0;
    auto classify = [&](double v) {
        if (v != v) code |= 1;
        else if (v - v != 0.0) code |= 2;  // +-inf
    };
    for (; t + 8 <= t1; t += 8) {  // 8 loads in flight per lane
        S v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = x[(long)(t + u) * frame_pitch];
#pragma unroll
        for (int u = 0; u < 8; ++u) classify((double)v[u]);
    }
    for (; t < t1; ++t) classify((double)x[(long)t * frame_pitch]);
    if (code) atomicOr(bad + p, code);
}

// Pixels whose series holds an infinity and no NaN (bad == 2) -> *count.
__global__ void k_tfft_inf_count(const int* __restrict__ bad, int P, int* __restrict__ count) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < P && bad[p] == 2) atomicAdd(count, 1);
}

// Step 3 of the paired path: column n2 = bx of pair group by: inverse FFT over k1, then
// Z[k] = c[k] conv[k] (the DFT of x_p + i x_{p+8}) for k = M2 n1 + n2 < T -> zo[by][k][8].
template <int LOG1>
__global__ __launch_bounds__(TF_NT) void k_tfft_cols_inv_pair(const double2* __restrict__ work, int M2,
                                                              const double2* __restrict__ tw, int logM, int T,
                                                              const double2* __restrict__ chirp,
                                                              double2* __restrict__ zo) {
    constexpr int M1 = 1 << LOG1;
    extern __shared__ double2 tf_buf[];
    double2* const twl = tf_buf + lds_slots<LOG1>();
    const int n2 = blockIdx.x, grp = blockIdx.y;
    const long M = 1L << logM;
    load_twl<LOG1>(twl, tw, logM);
    for (int e = threadIdx.x; e < M1 * TF_G; e += TF_NT)
        tf_buf[lp(e)] = work[((long)grp * M + (long)(e / TF_G) * M2 + n2) * TF_G + e % TF_G];
    __syncthreads();
    lds_fft<LOG1, true>(tf_buf, twl);
    for (int e = threadIdx.x; e < M1 * TF_G; e += TF_NT) {
        const long k = (long)M2 * (e / TF_G) + n2;
        if (k < T) zo[((long)grp * T + k) * TF_G + e % TF_G] = zmul(tf_buf[lp(e)], chirp[k]);
    }
}

// Both pixels' spectra from Z (real inputs): X_p[k] = (Z[k] + conj Z[-k]) / 2,
// X_{p+8}[k] = (Z[k] - conj Z[-k]) / 2i; per bin k < nf the sum of |X| over the
// 128 pixels of pair groups [8 by, +8) and their count -> gpart[(pbase / 128 + by) nf + k].
// A thread is (bin, slot): 8 slots of a bin in adjacent lanes, summed by shuffles.
constexpr int TF_PS = 128;  // pixels per partial row of the paired path
__global__ __launch_bounds__(TF_NT) void k_tfft_split(const double2* __restrict__ zo, int T, int nf, int pbase, int P,
                                                      const int* __restrict__ bad, double2* __restrict__ gpart) {
    const int g = threadIdx.x % TF_G;
    const int k = blockIdx.x * (TF_NT / TF_G) + threadIdx.x / TF_G;
    const int kk = min(k, nf - 1), km = kk == 0 ? 0 : T - kk;
    double s = 0.0, c = 0.0;
    for (int j = 0; j < TF_PS / (2 * TF_G); ++j) {
        const int q = blockIdx.y * (TF_PS / (2 * TF_G)) + j;
        const int pa = pbase + q * 2 * TF_G + g, pb = pa + TF_G;
        const bool oka = pa < P && !bad[pa], okb = pb < P && !bad[pb];
        const double2 z = zo[((long)q * T + kk) * TF_G + g], zm = zo[((long)q * T + km) * TF_G + g];
        const double ar = z.x + zm.x, ai = z.y - zm.y, br = z.x - zm.x, bi = z.y + zm.y;
        const double ma = 0.5 * sqrt(ar * ar + ai * ai), mb = 0.5 * sqrt(br * br + bi * bi);
        s += (oka ? ma : 0.0) + (okb ? mb : 0.0);
        c += (oka ? 1.0 : 0.0) + (okb ? 1.0 : 0.0);
    }
#pragma unroll
    for (int o = 1; o < TF_G; o <<= 1) {
        s += __shfl_xor(s, o, 64);
        c += __shfl_xor(c, o, 64);
    }
    if (g == 0 && k < nf) gpart[((long)(pbase / TF_PS) + blockIdx.y) * nf + k] = make_double2(s, c);
}

__global__ __launch_bounds__(TF_NT) void k_tfft_sum(const double2* __restrict__ gpart, int ngroups, int nf,
                                                    double* __restrict__ partial) {
    const int n = blockIdx.x * TF_NT + threadIdx.x;
    if (n >= nf) return;
    double s = 0.0, c = 0.0;
#pragma unroll 8
    for (int g = 0; g < ngroups; ++g) {
        const double2 v = gpart[(long)g * nf + n];
        s += v.x;
        c += v.y;
    }
    partial[2 * n] = s;
    partial[2 * n + 1] = c;
}

namespace {

void tf_check(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

#define FCD_TF_HIPCHK(x)                                                                         \
    do {                                                                                         \
        const hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

constexpr int TF_MAXLOG = 10;  // longest sub-transform: 1024 x 8 x 16 B (+ pads, + table) = 152 KiB of LDS

template <int L1, typename S, bool PAIR>
void launch_cols_fwd(const S* stack, long fp, long rp, int bw, int P, int T, int pbase, int ngrp, const int* bad,
                     const double2* chirp, const double2* tw, int logM, int M2, double2* work, hipStream_t s) {
    const size_t lb = (size_t)(lds_slots<L1>() + (1 << L1)) * sizeof(double2);
    (void)hipFuncSetAttribute((const void*)k_tfft_cols_fwd<L1, S, PAIR>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lb);
    hipLaunchKernelGGL((k_tfft_cols_fwd<L1, S, PAIR>), dim3((unsigned)M2, (unsigned)ngrp), dim3(TF_NT), lb, s, stack,
                       fp, rp, bw, P, T, pbase, bad, chirp, tw, logM, M2, work);
}

template <int L1>
void launch_cols_inv_pair(const double2* work, int ngrp, int M2, const double2* tw, int logM, int T,
                          const double2* chirp, double2* zo, hipStream_t s) {
    const size_t lb = (size_t)(lds_slots<L1>() + (1 << L1)) * sizeof(double2);
    (void)hipFuncSetAttribute((const void*)k_tfft_cols_inv_pair<L1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lb);
    hipLaunchKernelGGL(k_tfft_cols_inv_pair<L1>, dim3((unsigned)M2, (unsigned)ngrp), dim3(TF_NT), lb, s, work, M2, tw,
                       logM, T, chirp, zo);
}

template <int L2>
void launch_rows(double2* work, int ngrp, int M1, const double2* bhat, const double2* tw, int logM, hipStream_t s) {
    const size_t lb = (size_t)(lds_slots<L2>() + (1 << L2)) * sizeof(double2);
    (void)hipFuncSetAttribute((const void*)k_tfft_rows<L2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lb);
    hipLaunchKernelGGL(k_tfft_rows<L2>, dim3((unsigned)M1, (unsigned)ngrp), dim3(TF_NT), lb, s, work, bhat,
                       tw, logM);
}

template <int L1>
void launch_cols_inv(const double2* work, int nb, int M2, const double2* tw, int logM, int nf, int pbase, int P,
                     double2* gpart, hipStream_t s) {
    const size_t lb = (size_t)(lds_slots<L1>() + (1 << L1)) * sizeof(double2);
    (void)hipFuncSetAttribute((const void*)k_tfft_cols_inv<L1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lb);
    hipLaunchKernelGGL(k_tfft_cols_inv<L1>, dim3((unsigned)M2, (unsigned)(nb / TF_GS)), dim3(TF_NT), lb, s, work,
                       M2, tw, logM, nf, pbase, P, gpart);
}

// runtime log2 -> template instantiation (1..TF_MAXLOG)
#define TF_SWITCH(lg, CALL)                                                         \
    switch (lg) {                                                                   \
        case 1: { constexpr int LG = 1; CALL; } break;                              \
        case 2: { constexpr int LG = 2; CALL; } break;                              \
        case 3: { constexpr int LG = 3; CALL; } break;                              \
        case 4: { constexpr int LG = 4; CALL; } break;                              \
        case 5: { constexpr int LG = 5; CALL; } break;                              \
        case 6: { constexpr int LG = 6; CALL; } break;                              \
        case 7: { constexpr int LG = 7; CALL; } break;                              \
        case 8: { constexpr int LG = 8; CALL; } break;                              \
        case 9: { constexpr int LG = 9; CALL; } break;                              \
        case 10: { constexpr int LG = 10; CALL; } break;                            \
        default: throw std::runtime_error("temporal fft: sub-transform length");   \
    }

template <typename S>
void spectrum_fft_t(const S* stack, long fp, long rp, int bw, int P, int T, int nf, const TfftPlan& pl,
                    const double2* chirp, const double2* tw, const double2* bhat, const TfftWork& wk, double* partial,
                    hipStream_t s) {
    // pl.pair: wk.bad holds the block's flags (temporal_inf_pixels, no infinity among them)
    for (int pbase = 0; pbase < P; pbase += pl.Pb) {
        if (pl.pair) {
            // pixels of this batch, rounded up to whole 128-pixel partial rows; 16 per pair group
            const int nb = std::min(pl.Pb, (P - pbase + TF_PS - 1) / TF_PS * TF_PS), ngrp = nb / (2 * TF_G);
            TF_SWITCH(pl.log1, (launch_cols_fwd<LG, S, true>(stack, fp, rp, bw, P, T, pbase, ngrp, wk.bad, chirp, tw,
                                                              pl.logM, pl.M2, wk.work, s)));
            tf_check("temporal fft (columns)");
            TF_SWITCH(pl.log2, (launch_rows<LG>(wk.work, ngrp, pl.M1, bhat, tw, pl.logM, s)));
            tf_check("temporal fft (rows)");
            TF_SWITCH(pl.log1, (launch_cols_inv_pair<LG>(wk.work, ngrp, pl.M2, tw, pl.logM, T, chirp, wk.zo, s)));
            tf_check("temporal fft (inverse columns)");
            hipLaunchKernelGGL(k_tfft_split, dim3((unsigned)((nf + TF_NT / TF_G - 1) / (TF_NT / TF_G)), (unsigned)(nb / TF_PS)),
                               dim3(TF_NT), 0, s, wk.zo, T, nf, pbase, P, wk.bad, wk.gpart);
            tf_check("temporal fft (split)");
        } else {
            // pixels of this batch, rounded up to whole 64-pixel groups
            const int nb = std::min(pl.Pb, (P - pbase + TF_GS - 1) / TF_GS * TF_GS);
            TF_SWITCH(pl.log1, (launch_cols_fwd<LG, S, false>(stack, fp, rp, bw, P, T, pbase, nb / TF_G, nullptr, chirp,
                                                               tw, pl.logM, pl.M2, wk.work, s)));
            tf_check("temporal fft (columns)");
            TF_SWITCH(pl.log2, (launch_rows<LG>(wk.work, nb / TF_G, pl.M1, bhat, tw, pl.logM, s)));
            tf_check("temporal fft (rows)");
            TF_SWITCH(pl.log1, (launch_cols_inv<LG>(wk.work, nb, pl.M2, tw, pl.logM, nf, pbase, P, wk.gpart, s)));
            tf_check("temporal fft (inverse columns)");
        }
    }
    hipLaunchKernelGGL(k_tfft_sum, dim3((unsigned)((nf + TF_NT - 1) / TF_NT)), dim3(TF_NT), 0, s, wk.gpart,
                       pl.ngroups, nf, partial);
    tf_check("temporal fft (sum)");
}

}  // namespace

// FCD_TDFT_FFT=1 / =0 forces / forbids this path (read per call, so one process can
// test both).  By default the cheaper of the two by their measured rates (128 x 128
// block): the direct DFT at 4 T nf flops per series and ~40 TFLOP/s on the matrix cores
// (T <= 8192; ~27 on the vector units above), the paired FFT at 4 T + 32 M + 16 T bytes
// per series and ~2.5 TB/s (r02aj: T = 2000 3.02 vs 1.12 ms, T = 20000 475 vs 14.1).
bool temporal_spectrum_uses_fft(int T, int nf) {
    const char* e = std::getenv("FCD_TDFT_FFT");
    if (e && e[0] == '1') return true;
    if (e && e[0] == '0') return false;
    long M = 4;
    while (M < 2L * T - 1) M <<= 1;
    const double direct = 4.0 * T * (double)nf / (T <= 8192 ? 40e12 : 27e12);
    const double fft = (20.0 * T + 32.0 * (double)M) / 2.5e12;
    return fft < direct;
}

bool temporal_fft_plan(int T, int P, TfftPlan* pl, bool allow_pair) {
    int logM = 2;
    while ((1L << logM) < 2L * T - 1) ++logM;
    if (logM > 2 * TF_MAXLOG || T <= 0 || P <= 0) return false;
    pl->logM = logM;
    pl->M = 1 << logM;
    pl->log2 = (logM + 1) / 2;  // the rows (step 2, two transforms) get the longer half
    pl->log1 = logM - pl->log2;
    pl->M1 = 1 << pl->log1;
    pl->M2 = 1 << pl->log2;
    // FCD_TDFT_PAIR=0: one pixel per transform (diagnostic); default two (x_p + i x_q)
    const char* e = std::getenv("FCD_TDFT_PAIR");
    pl->pair = allow_pair && !(e && e[0] == '0');
    // pixels per batch: a work array of <= 1 GiB, a multiple of 128 pixels, <= 2^16 (grid y)
    const long cap =
        std::min(1L << 16, std::max(1L, (1L << 30) / ((long)pl->M * (long)sizeof(double2)) / TF_PS) * TF_PS);
    const long need = ((long)P + TF_PS - 1) / TF_PS * TF_PS;
    pl->Pb = (int)std::min(cap, need);
    const int per_row = pl->pair ? TF_PS : TF_GS;
    pl->ngroups = (P + per_row - 1) / per_row;
    pl->work_elems = (long)pl->Pb * pl->M / (pl->pair ? 2 : 1);
    pl->zo_elems = pl->pair ? (long)pl->Pb / 2 * T : 0;
    return true;
}

// Host tables in f64: chirp c[n] = exp(-i pi (n^2 mod 2T) / T) (exact argument
// reduction), tw[j] = exp(-2 pi i j / M), and B = FFT(b) / M in the four-step's
// [k1][k2] order (bhat[k1 M2 + k2] = B[k1 + M1 k2]), b[m] = b[M - m] = conj(c[m]).
void temporal_fft_tables(int T, const TfftPlan& pl, std::vector<double2>& chirp, std::vector<double2>& tw,
                         std::vector<double2>& bhat) {
    const double pi = 3.14159265358979323846;
    const int M = pl.M;
    chirp.resize(T);
    for (long n = 0; n < T; ++n) {
        const long r = (n * n) % (2L * T);
        const double a = -pi * (double)r / (double)T;
        chirp[n] = make_double2(std::cos(a), std::sin(a));
    }
    tw.resize(M);
    for (int j = 0; j < M; ++j) {
        const double a = -2.0 * pi * (double)j / (double)M;
        tw[j] = make_double2(std::cos(a), std::sin(a));
    }
    std::vector<std::complex<double>> b(M, 0.0);
    for (int m = 0; m < T; ++m) {
        const std::complex<double> v(chirp[m].x, -chirp[m].y);
        b[m] = v;
        if (m > 0) b[M - m] = v;
    }
    // iterative radix-2 FFT (forward), bit-reversed input order
    for (int i = 1, j = 0; i < M; ++i) {
        int bit = M >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) std::swap(b[i], b[j]);
    }
    for (int len = 2; len <= M; len <<= 1) {
        const int st = M / len;
        for (int i = 0; i < M; i += len)
            for (int k = 0; k < len / 2; ++k) {
                const std::complex<double> w(tw[(size_t)k * st].x, tw[(size_t)k * st].y);
                const std::complex<double> u = b[i + k], v = b[i + k + len / 2] * w;
                b[i + k] = u + v;
                b[i + k + len / 2] = u - v;
            }
    }
    bhat.resize(M);
    const double inv = 1.0 / (double)M;
    for (int k1 = 0; k1 < pl.M1; ++k1)
        for (int k2 = 0; k2 < pl.M2; ++k2) {
            const std::complex<double> v = b[(size_t)k1 + (size_t)pl.M1 * k2] * inv;
            bhat[(size_t)k1 * pl.M2 + k2] = make_double2(v.real(), v.imag());
        }
}

int temporal_inf_pixels(Samples stack, long frame_pitch, long row_pitch, int bw, int P, int T, int* bad, int* count,
                        hipStream_t s) {
    FCD_TF_HIPCHK(hipMemsetAsync(bad, 0, (size_t)P * sizeof(int), s));
    FCD_TF_HIPCHK(hipMemsetAsync(count, 0, sizeof(int), s));
    const dim3 g((unsigned)((P + TF_NT - 1) / TF_NT), (unsigned)((T + TF_NT - 1) / TF_NT));
    if (stack.f64)
        hipLaunchKernelGGL(k_tfft_flags<double>, g, dim3(TF_NT), 0, s, static_cast<const double*>(stack.p), frame_pitch,
                           row_pitch, bw, P, T, bad);
    else
        hipLaunchKernelGGL(k_tfft_flags<float>, g, dim3(TF_NT), 0, s, static_cast<const float*>(stack.p), frame_pitch,
                           row_pitch, bw, P, T, bad);
    tf_check("temporal fft (finite flags)");
    hipLaunchKernelGGL(k_tfft_inf_count, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, bad, P, count);
    tf_check("temporal fft (inf count)");
    int n = 0;
    FCD_TF_HIPCHK(hipMemcpyAsync(&n, count, sizeof(int), hipMemcpyDeviceToHost, s));
    FCD_TF_HIPCHK(hipStreamSynchronize(s));
    return n;
}

void temporal_spectrum_fft(Samples stack, long frame_pitch, long row_pitch, int bw, int P, int T, int nf,
                           const TfftPlan& pl, const double2* chirp, const double2* tw, const double2* bhat,
                           const TfftWork& wk, double* partial, hipStream_t s) {
    if (nf <= 0 || nf > T) throw std::runtime_error("temporal fft: bad bin count");
    if (stack.f64)
        spectrum_fft_t(static_cast<const double*>(stack.p), frame_pitch, row_pitch, bw, P, T, nf, pl, chirp, tw, bhat,
                       wk, partial, s);
    else
        spectrum_fft_t(static_cast<const float*>(stack.p), frame_pitch, row_pitch, bw, P, T, nf, pl, chirp, tw, bhat,
                       wk, partial, s);
}

}  // namespace fcdk
