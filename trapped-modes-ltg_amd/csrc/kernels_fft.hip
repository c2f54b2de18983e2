// Batched 2-D FFT building blocks and the demodulation band kernels.
//
// Replaces, on the device, the scipy.fft calls of the reference hot path:
//   fft2(displaced)                       /root/reference/pyfcd/fcd.py:28
//   ifft2(displaced_fft * carrier.mask)   /root/reference/pyfcd/fcd.py:118
//   fft2(reference), ifft2(... * mask)    /root/reference/pyfcd/carriers.py:22-24
//   fft2(image - mean) for peak finding   /root/reference/pyfcd/fourier.py:18
// and the disk band-pass of carriers.py:17-20 (skimage.draw.disk raster).
#include <atomic>
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#include "fft_lds.hpp"
#include "kernels.hpp"

namespace fcdk {

#define FCD_HIPCHK(x)                                                               \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) throw std::runtime_error(std::string(#x ": ") + hipGetErrorString(e_)); \
    } while (0)
#define FCD_CHECK_LAUNCH()                                                          \
    do {                                                                            \
        hipError_t e_ = hipGetLastError();                                          \
        if (e_ != hipSuccess) throw std::runtime_error(std::string("kernel launch: ") + hipGetErrorString(e_)); \
    } while (0)

bool fft_size_supported(int n) { return n >= 64 && n <= 4096 && (n & (n - 1)) == 0; }

constexpr float kPiF = 3.14159265358979f;
constexpr float kTwoPiF = 6.28318530717959f;

// ------------------------------------------------------------------ row FFT
// One team per row; 256-thread workgroups (a 1024-point row is one wave).
template <int N>
struct RowCfg {
    static constexpr int TT = fft_team(N);
    static constexpr int BLOCK = TT >= 256 ? TT : 256;
    static constexpr int TEAMS = BLOCK / TT;
};

template <int N, bool INV, int IN, int OUT>
__global__ __launch_bounds__(RowCfg<N>::BLOCK) void k_row_fft(const void* __restrict__ in, void* __restrict__ out,
                                                               long nrows, int H, float sub,
                                                               const float2* __restrict__ tw, PhaseOut ph) {
    using C = RowCfg<N>;
    constexpr int E = fft_elems(N);
    __shared__ __attribute__((aligned(16))) float2 lds[C::TEAMS][padded_len(N)];
    const int team = threadIdx.x / C::TT;
    const int t = threadIdx.x % C::TT;
    const long row = (long)blockIdx.x * C::TEAMS + team;
    const bool valid = row < nrows;
    float2* s = lds[team];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = t + e * C::TT;
        float2 v = make_float2(0.f, 0.f);
        if (valid) {
            if constexpr (IN == ROW_IN_REAL) {
                v.x = static_cast<const float*>(in)[row * N + i] - sub;
            } else {
                v = static_cast<const float2*>(in)[row * N + i];
            }
        }
        s[pad(i)] = v;
    }
    __syncthreads();
    fft_team_lds<N, INV>(s, tw, t);
    if (!valid) return;
    if constexpr (OUT == ROW_OUT_COMPLEX) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int i = t + e * C::TT;
            static_cast<float2*>(out)[row * N + i] = s[pad(i)];
        }
    } else if constexpr (OUT == ROW_OUT_REAL) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int i = t + e * C::TT;
            static_cast<float*>(out)[row * N + i] = s[pad(i)].x;
        }
    } else {
        // w = wrap(theta - angle(A)) == -angle(A * conj(R)) of fcd.py:118
        const long b = row / H, r = row % H;
        const float* th = ph.theta + r * N;
        float* wo = ph.wrapped + ((b * 2 + ph.carrier) * H + r) * (long)N;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int i = t + e * C::TT;
            const float2 a = s[pad(i)];
            float d = th[i] - atan2f(a.y, a.x);
            if (d > kPiF) d -= kTwoPiF;
            else if (d < -kPiF) d += kTwoPiF;
            wo[i] = d;
        }
    }
}

template <int N, bool INV, int IN, int OUT>
static void launch_row(const void* in, void* out, long nrows, int H, float sub, const float2* tw, const PhaseOut* ph,
                       hipStream_t s) {
    using C = RowCfg<N>;
    PhaseOut p{};
    if (ph) p = *ph;
    const long blocks = (nrows + C::TEAMS - 1) / C::TEAMS;
    hipLaunchKernelGGL((k_row_fft<N, INV, IN, OUT>), dim3((unsigned)blocks), dim3(C::BLOCK), 0, s, in, out, nrows, H,
                       sub, tw, p);
    FCD_CHECK_LAUNCH();
}

template <int N>
static void row_dispatch_n(bool inv, RowIn im, RowOut om, const void* in, void* out, long nrows, int H, float sub,
                           const float2* tw, const PhaseOut* ph, hipStream_t s) {
    if (!inv && im == ROW_IN_REAL && om == ROW_OUT_COMPLEX)
        launch_row<N, false, ROW_IN_REAL, ROW_OUT_COMPLEX>(in, out, nrows, H, sub, tw, ph, s);
    else if (!inv && im == ROW_IN_COMPLEX && om == ROW_OUT_COMPLEX)
        launch_row<N, false, ROW_IN_COMPLEX, ROW_OUT_COMPLEX>(in, out, nrows, H, sub, tw, ph, s);
    else if (inv && im == ROW_IN_COMPLEX && om == ROW_OUT_COMPLEX)
        launch_row<N, true, ROW_IN_COMPLEX, ROW_OUT_COMPLEX>(in, out, nrows, H, sub, tw, ph, s);
    else if (inv && im == ROW_IN_COMPLEX && om == ROW_OUT_REAL)
        launch_row<N, true, ROW_IN_COMPLEX, ROW_OUT_REAL>(in, out, nrows, H, sub, tw, ph, s);
    else if (inv && im == ROW_IN_COMPLEX && om == ROW_OUT_PHASE)
        launch_row<N, true, ROW_IN_COMPLEX, ROW_OUT_PHASE>(in, out, nrows, H, sub, tw, ph, s);
    else
        throw std::runtime_error("row_fft: unsupported mode combination");
}

void row_fft(int W, bool inverse, RowIn im, RowOut om, const void* in, void* out, long nrows, int H, float sub,
             const float2* tw, const PhaseOut* ph, hipStream_t s) {
    if (nrows <= 0) return;
    switch (W) {
        case 64: row_dispatch_n<64>(inverse, im, om, in, out, nrows, H, sub, tw, ph, s); break;
        case 128: row_dispatch_n<128>(inverse, im, om, in, out, nrows, H, sub, tw, ph, s); break;
        case 256: row_dispatch_n<256>(inverse, im, om, in, out, nrows, H, sub, tw, ph, s); break;
        case 512: row_dispatch_n<512>(inverse, im, om, in, out, nrows, H, sub, tw, ph, s); break;
        case 1024: row_dispatch_n<1024>(inverse, im, om, in, out, nrows, H, sub, tw, ph, s); break;
        case 2048: row_dispatch_n<2048>(inverse, im, om, in, out, nrows, H, sub, tw, ph, s); break;
        case 4096: row_dispatch_n<4096>(inverse, im, om, in, out, nrows, H, sub, tw, ph, s); break;
        default: throw std::runtime_error("row_fft: unsupported length " + std::to_string(W));
    }
}

// ------------------------------------------------------------------ column FFT
// A workgroup loads G adjacent columns (G*8-byte row segments), one team
// transforms each column in LDS.  Column stride padded_len(H)+1 (odd) keeps
// the transposing loads/stores bank-conflict free.
template <int N>
struct ColCfg {
    static constexpr int TT = fft_team(N);
    static constexpr int BLOCK = TT >= 512 ? TT : 512;
    static constexpr int G = BLOCK / TT;
    static constexpr int STRIDE = padded_len(N) + 1;
};

template <int N, bool INV>
__global__ __launch_bounds__(ColCfg<N>::BLOCK) void k_col_fft(float2* __restrict__ data, int W, int g_used,
                                                              const float2* __restrict__ tw) {
    using C = ColCfg<N>;
    extern __shared__ __attribute__((aligned(16))) float2 lds_dyn[];
    const int team = threadIdx.x / C::TT;
    const int t = threadIdx.x % C::TT;
    const int colblocks = W / g_used;
    const long b = blockIdx.x / colblocks;
    const int c0 = (blockIdx.x % colblocks) * g_used;
    float2* base = data + b * (long)N * W + c0;
    for (int idx = threadIdx.x; idx < N * g_used; idx += C::BLOCK) {
        const int r = idx / g_used, g = idx % g_used;
        lds_dyn[g * C::STRIDE + pad(r)] = base[(long)r * W + g];
    }
    __syncthreads();
    fft_team_lds<N, INV>(lds_dyn + team * C::STRIDE, tw, t);
    for (int idx = threadIdx.x; idx < N * g_used; idx += C::BLOCK) {
        const int r = idx / g_used, g = idx % g_used;
        base[(long)r * W + g] = lds_dyn[g * C::STRIDE + pad(r)];
    }
}

template <int N>
static void launch_col(int W, bool inv, float2* data, int nbatch, const float2* tw, hipStream_t s) {
    using C = ColCfg<N>;
    // Teams beyond the used columns transform zeros (keeps every barrier uniform).
    const int g_used = W < C::G ? W : C::G;
    const size_t lds = (size_t)C::G * C::STRIDE * sizeof(float2);
    const unsigned blocks = (unsigned)((long)nbatch * (W / g_used));
    static std::atomic<bool> attr_set{false};  // per instantiation: allow > 64 KiB dynamic LDS (gfx950 has 160 KiB)
    if (!attr_set) {
        FCD_HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_col_fft<N, true>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        FCD_HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_col_fft<N, false>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        attr_set = true;
    }
    if (inv)
        hipLaunchKernelGGL((k_col_fft<N, true>), dim3(blocks), dim3(C::BLOCK), lds, s, data, W, g_used, tw);
    else
        hipLaunchKernelGGL((k_col_fft<N, false>), dim3(blocks), dim3(C::BLOCK), lds, s, data, W, g_used, tw);
    FCD_CHECK_LAUNCH();
}

void col_fft(int H, int W, bool inverse, float2* data, int nbatch, const float2* tw, hipStream_t s) {
    if (nbatch <= 0) return;
    switch (H) {
        case 64: launch_col<64>(W, inverse, data, nbatch, tw, s); break;
        case 128: launch_col<128>(W, inverse, data, nbatch, tw, s); break;
        case 256: launch_col<256>(W, inverse, data, nbatch, tw, s); break;
        case 512: launch_col<512>(W, inverse, data, nbatch, tw, s); break;
        case 1024: launch_col<1024>(W, inverse, data, nbatch, tw, s); break;
        case 2048: launch_col<2048>(W, inverse, data, nbatch, tw, s); break;
        case 4096: launch_col<4096>(W, inverse, data, nbatch, tw, s); break;
        default: throw std::runtime_error("col_fft: unsupported length " + std::to_string(H));
    }
}

// ------------------------------------------------------------------ band-pass
// mask = ifftshift(disk(peak, R)): unshifted (i, j) is inside iff the shifted
// (i+H/2, j+W/2) lies in the skimage disk raster (carriers.py:17-20).
__global__ void k_disk_mask(const float2* __restrict__ in, float2* __restrict__ out, long n, int H, int W,
                            DiskTable t, bool tr) {
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n) return;
    const long p = idx % ((long)H * W);
    const int i = tr ? (int)(p % H) : (int)(p / W), j = tr ? (int)(p / H) : (int)(p % W);
    const int si = (i + H / 2) % H, sj = (j + W / 2) % W;  // unshifted -> shifted (any side)
    const int2 rr = reinterpret_cast<const int2*>(t.rows)[sj];
    const bool inside = si >= rr.x && si <= rr.y;
    out[idx] = inside ? in[idx] : make_float2(0.f, 0.f);
}

void disk_mask(const float2* in, float2* out, int nbatch, int H, int W, DiskTable t, hipStream_t s, bool transposed) {
    const long n = (long)nbatch * H * W;
    hipLaunchKernelGGL(k_disk_mask, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, in, out, n, H, W, t, transposed);
    FCD_CHECK_LAUNCH();
}

__global__ void k_disk_band_t(const float2* __restrict__ spec_t, float2* __restrict__ out, long n, int H, int W, int NU,
                              const int* __restrict__ cols, const int* __restrict__ uslot, int nc, DiskTable t) {
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n) return;
    const long per = (long)nc * H;
    const long b = idx / per, p = idx % per;
    const int k = (int)(p / H), i = (int)(p % H);
    const int j = cols[k];
    const int si = (i + H / 2) % H, sj = (j + W / 2) % W;
    const int2 rr = reinterpret_cast<const int2*>(t.rows)[sj];
    const bool inside = si >= rr.x && si <= rr.y;
    out[idx] = inside ? spec_t[(b * NU + uslot[k]) * H + i] : make_float2(0.f, 0.f);
}

void disk_band_t(const float2* spec_t, float2* out, int nbatch, int H, int W, int NU, const int* cols, const int* uslot,
                 int nc, DiskTable t, hipStream_t s) {
    const long n = (long)nbatch * nc * H;
    if (n <= 0) return;
    hipLaunchKernelGGL(k_disk_band_t, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, spec_t, out, n, H, W, NU, cols,
                       uslot, nc, t);
    FCD_CHECK_LAUNCH();
}

__global__ void k_angle(const float2* __restrict__ in, float* __restrict__ out, long n) {
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx < n) out[idx] = atan2f(in[idx].y, in[idx].x);
}

void angle(const float2* in, float* out, long n, hipStream_t s) {
    hipLaunchKernelGGL(k_angle, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, in, out, n);
    FCD_CHECK_LAUNCH();
}

// ------------------------------------------------------------------ batched reference setup
// fourier.find_peaks (fourier.py:7-41) for nb images at once: |F| * highpass of the
// reference's own spectrum (kernels_pocketfft.hip) with a per-image maximum, the
// above-threshold candidates per image, and the 8-connected labelling with the peak pick
// (k_label_peaks, float32 spectra).

// Correctly rounded float32 square root of a positive normal x.  v_sqrt_f32 (what
// sqrtf / __fsqrt_rn lower to here) is within 1 ulp but not correctly rounded; the
// neighbour on either side is taken when x lies beyond the midpoint towards it.  The
// midpoints have 25 significant bits, so their squares are exact in f64, and x (24
// bits) can never equal one: the comparisons decide the IEEE result exactly.
__device__ __forceinline__ float sqrt_rn(float x) {
    float s = __builtin_sqrtf(x);
    const double xd = (double)x;
    const unsigned u = __float_as_uint(s);  // s > 0: the neighbours are the adjacent encodings
    const float up = __uint_as_float(u + 1u), dn = __uint_as_float(u - 1u);
    const double mu = 0.5 * ((double)s + (double)up), md = 0.5 * ((double)dn + (double)s);
    if (mu * mu < xd) s = up;
    else if (md * md > xd) s = dn;
    return s;
}

// np.abs of a complex value as numpy 1.26.4 computes it (its AVX512F loop,
// loops_unary_complex: larger * sqrt(fma(r, r, 1)) with r = smaller / larger, inf / NaN
// cases first); this file is compiled without FMA contraction, the one FMA is explicit,
// the division is the IEEE sequence (v_div_scale / fmas / fixup).  The float64 square
// root is __dsqrt_rn (correctly rounded).
__device__ __forceinline__ float np_cabs(float2 f) {
    const float re = fabsf(f.x), im = fabsf(f.y);
    if (re == INFINITY || im == INFINITY) return INFINITY;
    if (re != re || im != im) return NAN;
    const float big = fmaxf(re, im), small = fminf(im, re);
    const float r = big == 0.f ? 0.f : __fdiv_rn(small, big);
    return __fmul_rn(sqrt_rn(__fmaf_rn(r, r, 1.0f)), big);
}
__device__ __forceinline__ double np_cabs(double2 f) {
    const double re = fabs(f.x), im = fabs(f.y);
    if (re == INFINITY || im == INFINITY) return INFINITY;
    if (re != re || im != im) return NAN;
    const double big = fmax(re, im), small = fmin(im, re);
    const double r = big == 0.0 ? 0.0 : __ddiv_rn(small, big);
    return __dmul_rn(__dsqrt_rn(__fma_rn(r, r, 1.0)), big);
}
__device__ __forceinline__ unsigned long long order_bits(float m) { return __float_as_uint(m); }
__device__ __forceinline__ unsigned long long order_bits(double m) { return (unsigned long long)__double_as_longlong(m); }
__device__ __forceinline__ float from_bits(unsigned long long u, float) { return __uint_as_float((unsigned)u); }
__device__ __forceinline__ double from_bits(unsigned long long u, double) { return __longlong_as_double((long long)u); }

template <class T, class C>
__global__ void k_spectrum_mag_b(const C* __restrict__ F, T* __restrict__ mag, unsigned long long* maxbits, int H,
                                 int W, long n, const double* __restrict__ krow_s, const double* __restrict__ kcol_s,
                                 double kmin2) {
    const long gidx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long hw = (long)H * W;
    T m = T(0);
    const long b = gidx / hw;
    if (gidx < n) {
        const long idx = gidx - b * hw;
        const int si = (int)(idx / W), sj = (int)(idx % W);
        int i = (si + H - H / 2) % H, j = (sj + W - W / 2) % W;  // fftshift: shifted (si, sj) <- unshifted (i, j)
        const int mi = (H - i) % H, mj = (W - j) % W;   // one canonical bin per Hermitian pair
        if (mi < i || (mi == i && mj < j)) {
            i = mi;
            j = mj;
        }
        m = np_cabs(F[b * hw + (long)i * W + j]);
        const double kr = krow_s[si], kc = kcol_s[sj];
        const double k2 = __dadd_rn(__dmul_rn(kr, kr), __dmul_rn(kc, kc));
        if (!(k2 > kmin2)) m = T(0);  // image_fft *= highpass_mask() (fourier.py:20-23, 34)
        mag[gidx] = m;
    }
    // the per-image maximum (a wave may span two images when H * W is not a multiple of 64)
    const unsigned long long u = order_bits(m);
    const long b0 = __shfl(b, 0, 64);
    unsigned long long uw = b == b0 ? u : 0ull;
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long v = __shfl_xor(uw, o, 64);
        uw = v > uw ? v : uw;
    }
    if ((threadIdx.x & 63) == 0 && b0 * hw < n) atomicMax(maxbits + b0, uw);
    if (b != b0 && gidx < n) atomicMax(maxbits + b, u);
}

template <class T>
__global__ void k_candidates_b(const T* __restrict__ mag, const unsigned long long* __restrict__ maxbits, int H, int W,
                               long n, int* count, int* idx_out, T* val_out, long cap) {
    const long gidx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gidx >= n) return;
    const long hw = (long)H * W, b = gidx / hw, idx = gidx - b * hw;
    const int si = (int)(idx / W), sj = (int)(idx % W);
    if (si == 0 || sj == 0 || si == H - 1 || sj == W - 1) return;  // fourier.py:154-158
    const T thr = T(0.5) * from_bits(maxbits[b], T(0));             // fourier.py:35 (exact)
    const T m = mag[gidx];
    if (m > thr) {
        const int slot = atomicAdd(count + b, 1);
        if (slot < cap) {
            idx_out[b * cap + slot] = (int)idx;
            val_out[b * cap + slot] = m;
        }
    }
}

template <class T, class C>
void candidates_t(const C* F, int nb, int H, int W, const double* krow_s, const double* kcol_s, double kmin2, T* mag,
                  unsigned long long* maxbits, int* count, int* idx, T* val, long cap, hipStream_t s) {
    const long n = (long)nb * H * W;
    FCD_HIPCHK(hipMemsetAsync(maxbits, 0, sizeof(unsigned long long) * nb, s));
    FCD_HIPCHK(hipMemsetAsync(count, 0, sizeof(int) * nb, s));
    hipLaunchKernelGGL((k_spectrum_mag_b<T, C>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, F, mag, maxbits, H,
                       W, n, krow_s, kcol_s, kmin2);
    FCD_CHECK_LAUNCH();
    hipLaunchKernelGGL((k_candidates_b<T>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, mag, maxbits, H, W, n,
                       count, idx, val, cap);
    FCD_CHECK_LAUNCH();
}

void spectrum_candidates_b(const void* F, bool f64, int nb, int H, int W, const double* krow_s, const double* kcol_s,
                           double kmin2, void* mag, unsigned long long* maxbits, int* count, int* idx, void* val,
                           long cap, hipStream_t s) {
    if (f64)
        candidates_t<double, double2>(static_cast<const double2*>(F), nb, H, W, krow_s, kcol_s, kmin2,
                                      static_cast<double*>(mag), maxbits, count, idx, static_cast<double*>(val), cap, s);
    else
        candidates_t<float, float2>(static_cast<const float2*>(F), nb, H, W, krow_s, kcol_s, kmin2,
                                    static_cast<float*>(mag), maxbits, count, idx, static_cast<float*>(val), cap, s);
}

// fourier.find_peak_locations (fourier.py:139-168) on one image's candidate list per
// workgroup: sort by raster index, 8-connected union-find (roots hook under the
// smaller root, so a component's root is its first pixel in raster order = its
// skimage label order), per blob the maximum (first pixel on ties, regionprops'
// row-major coords), then the blobs sorted by (maximum, label) and the first
// LABEL_TOP kept: the stable ascending sort's 4 dimmest blobs.
// res[b * 8]: {status (0 ok, 1: more candidates than LABEL_CAP), blobs, kept, peak raster index x 4}.
constexpr int LABEL_CAP = 4096;
constexpr int LABEL_TOP = 4;

__device__ __forceinline__ int label_find(volatile int* par, int x) {
    int p = par[x];
    while (p != x) {
        x = p;
        p = par[x];
    }
    return x;
}

template <class T>
__device__ __forceinline__ void bitonic_lds(T* key, int n2) {
    for (int k = 2; k <= n2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            __syncthreads();
            for (int i = threadIdx.x; i < n2; i += blockDim.x) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const bool asc = (i & k) == 0;
                    const T a = key[i], b = key[ixj];
                    if ((a > b) == asc) {
                        key[i] = b;
                        key[ixj] = a;
                    }
                }
            }
        }
    }
    __syncthreads();
}

__global__ __launch_bounds__(1024) void k_label_peaks(const int* __restrict__ counts, const int* __restrict__ idxs,
                                                      const float* __restrict__ vals, long cap, int H, int W,
                                                      int* __restrict__ res) {
    __shared__ unsigned long long sk[LABEL_CAP];  // (raster index, slot) for the first sort, (max, root) for the second
    __shared__ unsigned long long cm[LABEL_CAP];  // per root: (value bits, ~position) maximum
    __shared__ int key[LABEL_CAP];
    __shared__ float val[LABEL_CAP];
    __shared__ int par[LABEL_CAP];
    __shared__ int nblob;
    const int b = blockIdx.x;
    const int n = counts[b];
    int* out = res + b * 8;
    if (n > cap || n > LABEL_CAP) {  // the host labels this image from its candidate list
        if (threadIdx.x == 0) {
            out[0] = 1;
            out[1] = n;
        }
        return;
    }
    int n2 = 1;
    while (n2 < n) n2 <<= 1;
    const int* ci = idxs + (long)b * cap;
    const float* cv = vals + (long)b * cap;
    for (int i = threadIdx.x; i < n2; i += blockDim.x)
        sk[i] = i < n ? ((unsigned long long)(unsigned)ci[i] << 32) | (unsigned)i : ~0ull;
    if (threadIdx.x == 0) nblob = 0;
    bitonic_lds(sk, n2);
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int slot = (int)(sk[i] & 0xffffffffu);
        key[i] = (int)(sk[i] >> 32);
        val[i] = cv[slot];
        par[i] = i;
        cm[i] = 0;
    }
    __syncthreads();
    auto lookup = [&](int r, int c) -> int {  // position of pixel (r, c) in the sorted list, or -1
        if (r < 0 || c < 0 || r >= H || c >= W) return -1;
        const int want = r * W + c;
        int lo = 0, hi = n;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (key[mid] < want) lo = mid + 1; else hi = mid;
        }
        return lo < n && key[lo] == want ? lo : -1;
    };
    volatile int* vpar = par;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int r = key[i] / W, c = key[i] % W;
        const int nb4[4][2] = {{r - 1, c - 1}, {r - 1, c}, {r - 1, c + 1}, {r, c - 1}};
        for (int q = 0; q < 4; ++q) {
            const int j = lookup(nb4[q][0], nb4[q][1]);
            if (j < 0) continue;
            int x = i, y = j;
            for (;;) {  // unite: the larger root hooks under the smaller
                x = label_find(vpar, x);
                y = label_find(vpar, y);
                if (x == y) break;
                if (x < y) {
                    const int t = x;
                    x = y;
                    y = t;
                }
                if (atomicCAS(&par[x], x, y) == x) break;
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int rt = label_find(vpar, i);
        atomicMax(&cm[rt], ((unsigned long long)__float_as_uint(val[i]) << 32) | (0xffffffffu - (unsigned)i));
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n2; i += blockDim.x) {
        const bool root = i < n && par[i] == i;
        sk[i] = root ? ((cm[i] >> 32) << 32) | (unsigned)i : ~0ull;
        if (root) atomicAdd(&nblob, 1);
    }
    bitonic_lds(sk, n2);
    if (threadIdx.x == 0) {
        const int kept = nblob < LABEL_TOP ? nblob : LABEL_TOP;
        out[0] = 0;
        out[1] = nblob;
        out[2] = kept;
        for (int e = 0; e < LABEL_TOP; ++e) {
            int pk = -1;
            if (e < kept) {
                const int rt = (int)(sk[e] & 0xffffffffu);
                pk = key[0xffffffffu - (unsigned)(cm[rt] & 0xffffffffu)];
            }
            out[3 + e] = pk;
        }
    }
}

void label_peaks(const int* counts, const int* idx, const float* val, long cap, int nb, int H, int W, int* res,
                 hipStream_t s) {
    hipLaunchKernelGGL(k_label_peaks, dim3(nb), dim3(1024), 0, s, counts, idx, val, cap, H, W, res);
    FCD_CHECK_LAUNCH();
}

}  // namespace fcdk
