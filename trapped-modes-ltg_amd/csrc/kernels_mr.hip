// Mixed-radix transforms for frame sides that are not powers of two.
//
// The reference takes frames of any shape (scipy.fft.fft2 at fcd.py:28, fourier.py:18,
// fourier.py:134; ifft2 at fcd.py:118, carriers.py:23-24, fourier.py:137): camera sensors
// deliver 1920 x 1080, 2448 x 2048, 1280 x 1024 ... frames.  This file gives the engine's
// generic chain (fcd_engine.cpp: fft2_real / demod_phases / integrate_z /
// reference_state / process_generic) its row and column transforms at every side n:
//
//  * n whose prime factors are at most 61: one workgroup per row, the row in LDS,
//    Stockham passes of radix 8 / 4 / 2 (the power of two, in 8s then 4s), then 3s, 5s,
//    7s (register codelets) and any larger odd prime p <= 61 (a generic pass: the
//    butterfly inputs pre-twiddled in place, then each output an LDS dot product of p
//    terms), each pass reading one LDS buffer and writing the other; twiddles exp(-+2 pi
//    i m / n) from the context's table (computed in f64 on the host);
//  * n with a prime factor above 61 (1021, 2039, 4093 ...): Bluestein's identity, the
//    length-n DFT as a circular convolution of length M = 2^ceil(log2(2n - 1)): a chirp
//    c[m] = exp(-i pi (m^2 mod 2n) / n) premultiply, a radix-8/4/2 FFT of length M, a
//    multiply by the precomputed FFT of the conjugate chirp (1/M folded in), the inverse
//    FFT, the chirp postmultiply.
//
// A row's two buffers sit in LDS up to 8192 complex (128 KB); longer rows (sides above
// 8192, Bluestein's M above 8192) run the same passes in global scratch (L2 / MALL
// resident, a launch of at most kMrLongRows rows).  Sides up to kMrMaxLen = 16384.
//
// Columns: the spectral integration's column stage in place in LDS (k_mr_int_cols, no
// transposes), the demodulation's band columns and long columns through a tiled
// transpose, the row transform of length H and the transpose back.  These are the
// generic-chain transforms, not the band-pruned register FFTs of the power-of-two fast
// path.
#include <atomic>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <complex>
#include <stdexcept>
#include <string>
#include <vector>

#include "fft_lds.hpp"
#include "gfft.hpp"
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

namespace {

constexpr int MR_THREADS = 256;
constexpr int MR_LU = 8;  // row loads in flight per thread

// a / d for 0 <= a < 2^24 and the runtime divisor d (inv = 1 / d in f32): the f32 quotient
// is off by at most one, fixed by the remainder (an integer division is a ~40-instruction
// sequence on the GPU, and the passes took one per butterfly)
__device__ __forceinline__ int mr_div(int a, int d, float inv) {
    int q = (int)((float)a * inv);
    const int r = a - q * d;
    q += r >= d ? 1 : (r < 0 ? -1 : 0);
    return q;
}
constexpr float kPiF = 3.14159265358979f;
constexpr float kTwoPiF = 6.28318530717959f;
// radix-3 / radix-5 DFT constants
constexpr float kS3 = 0.866025403784438647f;                                  // sin(2 pi / 3)
constexpr float kC51 = 0.309016994374947424f, kS51 = 0.951056516295153572f;   // cos, sin(2 pi / 5)
constexpr float kC52 = -0.809016994374947424f, kS52 = 0.587785252292473129f;  // cos, sin(4 pi / 5)

template <bool INV>
__device__ __forceinline__ void dft3(float2* a) {
    const float2 t1 = cadd(a[1], a[2]), t2 = csub(a[1], a[2]);
    const float2 m = make_float2(a[0].x - 0.5f * t1.x, a[0].y - 0.5f * t1.y);
    // forward: y1 = m - i s3 t2, y2 = m + i s3 t2 (W3 = exp(-2 pi i / 3))
    const float sg = INV ? -kS3 : kS3;
    const float2 u = make_float2(sg * t2.y, -sg * t2.x);  // -i sg t2
    a[0] = cadd(a[0], t1);
    a[1] = cadd(m, u);
    a[2] = csub(m, u);
}

template <bool INV>
__device__ __forceinline__ void dft5(float2* a) {
    const float2 t1 = cadd(a[1], a[4]), t4 = csub(a[1], a[4]);
    const float2 t2 = cadd(a[2], a[3]), t3 = csub(a[2], a[3]);
    const float2 c1 = make_float2(a[0].x + kC51 * t1.x + kC52 * t2.x, a[0].y + kC51 * t1.y + kC52 * t2.y);
    const float2 c2 = make_float2(a[0].x + kC52 * t1.x + kC51 * t2.x, a[0].y + kC52 * t1.y + kC51 * t2.y);
    const float sg = INV ? -1.f : 1.f;
    // forward: y1 = c1 - i (s51 t4 + s52 t3), y2 = c2 - i (s52 t4 - s51 t3); y4, y3 the conjugate pairs
    const float2 d1 = make_float2(sg * (kS51 * t4.x + kS52 * t3.x), sg * (kS51 * t4.y + kS52 * t3.y));
    const float2 d2 = make_float2(sg * (kS52 * t4.x - kS51 * t3.x), sg * (kS52 * t4.y - kS51 * t3.y));
    a[0] = make_float2(a[0].x + t1.x + t2.x, a[0].y + t1.y + t2.y);
    a[1] = make_float2(c1.x + d1.y, c1.y - d1.x);
    a[4] = make_float2(c1.x - d1.y, c1.y + d1.x);
    a[2] = make_float2(c2.x + d2.y, c2.y - d2.x);
    a[3] = make_float2(c2.x - d2.y, c2.y + d2.x);
}

// radix 7: y_u = a0 + sum_m cos(2 pi u m / 7) s_m -+ i sum_m sin(2 pi u m / 7) d_m,
// s_m = a_m + a_{7-m}, d_m = a_m - a_{7-m}
constexpr float kC7[3] = {0.623489801858733530525f, -0.222520933956314404289f, -0.900968867902419126236f};
constexpr float kS7[3] = {0.781831482468029808708f, 0.974927912181823607018f, 0.433883739117558120475f};
template <bool INV>
__device__ __forceinline__ void dft7(float2* a) {
    float2 sm[3], dm[3];
#pragma unroll
    for (int m = 0; m < 3; ++m) {
        sm[m] = cadd(a[m + 1], a[6 - m]);
        dm[m] = csub(a[m + 1], a[6 - m]);
    }
    const float2 a0 = a[0];
    a[0] = cadd(cadd(a0, sm[0]), cadd(sm[1], sm[2]));
#pragma unroll
    for (int u = 1; u <= 3; ++u) {
        float2 ca = a0, cb = make_float2(0.f, 0.f);
#pragma unroll
        for (int m = 1; m <= 3; ++m) {
            int q = (u * m) % 7;
            const float sg = q > 3 ? -1.f : 1.f;
            q = q > 3 ? 7 - q : q;
            ca = make_float2(ca.x + kC7[q - 1] * sm[m - 1].x, ca.y + kC7[q - 1] * sm[m - 1].y);
            cb = make_float2(cb.x + sg * kS7[q - 1] * dm[m - 1].x, cb.y + sg * kS7[q - 1] * dm[m - 1].y);
        }
        // forward: y_u = ca - i cb, y_{7-u} = ca + i cb (inverse: the conjugate twiddles)
        const float2 icb = INV ? make_float2(-cb.y, cb.x) : make_float2(cb.y, -cb.x);
        a[u] = cadd(ca, icb);
        a[7 - u] = csub(ca, icb);
    }
}

template <int R, bool INV>
__device__ __forceinline__ void dft_any(float2* a) {
    if constexpr (R == 3) dft3<INV>(a);
    else if constexpr (R == 5) dft5<INV>(a);
    else if constexpr (R == 7) dft7<INV>(a);
    else dft_reg<R, INV>(a);
}

// One Stockham pass: src -> dst, L = product of the radices already applied.
template <int R, bool INV>
__device__ __forceinline__ void mr_pass(const float2* src, float2* dst, int n, int L, const float2* __restrict__ tw) {
    const int nb = n / R, step = n / (L * R);
    const float invL = 1.f / (float)L;
    for (int j = threadIdx.x; j < nb; j += MR_THREADS) {
        const int k = j - L * mr_div(j, L, invL);
        float2 a[R];
#pragma unroll
        for (int r = 0; r < R; ++r) a[r] = src[j + r * nb];
        if (L > 1) {
#pragma unroll
            for (int r = 1; r < R; ++r) a[r] = cmul_dir<INV>(a[r], tw[r * k * step]);
        }
        dft_any<R, INV>(a);
        const int base = (j - k) * R + k;
#pragma unroll
        for (int r = 0; r < R; ++r) dst[base + r * L] = a[r];
    }
}

// Generic odd radix R (a prime <= 61), two steps: the inputs of every butterfly
// pre-twiddled in place (src is consumed), then each output an R-term dot product with
// W_R^(r q) = tw[(r q mod R) n / R].
template <bool INV>
__device__ __forceinline__ void mr_pass_gen(float2* src, float2* dst, int n, int L, int R, const float2* __restrict__ tw) {
    const int nb = n / R, step = n / (L * R), wstep = n / R;
    const float invL = 1.f / (float)L, invnb = 1.f / (float)nb;
    if (L > 1) {
        for (int idx = threadIdx.x; idx < n; idx += MR_THREADS) {
            const int r = mr_div(idx, nb, invnb), j = idx - r * nb;
            if (r > 0) src[idx] = cmul_dir<INV>(src[idx], tw[r * (j - L * mr_div(j, L, invL)) * step]);
        }
        __syncthreads();
    }
    for (int idx = threadIdx.x; idx < n; idx += MR_THREADS) {
        const int q = mr_div(idx, nb, invnb), j = idx - q * nb, k = j - L * mr_div(j, L, invL);
        float2 acc = src[j];
        int m = 0;
        for (int r = 1; r < R; ++r) {
            m += q;
            if (m >= R) m -= R;
            const float2 w = tw[m * wstep];
            const float2 x = src[j + r * nb];
            acc = cadd(acc, cmul_dir<INV>(x, w));
        }
        dst[(j - k) * R + k + q * L] = acc;
    }
}

// The plan's passes over len points (b0 holds the input); returns the buffer holding the
// result.  Every pass ends with a barrier.
template <bool INV>
__device__ __forceinline__ float2* mr_run(float2* b0, float2* b1, int len, const int* fct, int nf,
                                          const float2* __restrict__ tw) {
    int L = 1;
    for (int f = 0; f < nf; ++f) {
        const int R = fct[f];
        switch (R) {
            case 8: mr_pass<8, INV>(b0, b1, len, L, tw); break;
            case 4: mr_pass<4, INV>(b0, b1, len, L, tw); break;
            case 2: mr_pass<2, INV>(b0, b1, len, L, tw); break;
            case 3: mr_pass<3, INV>(b0, b1, len, L, tw); break;
            case 5: mr_pass<5, INV>(b0, b1, len, L, tw); break;
            case 7: mr_pass<7, INV>(b0, b1, len, L, tw); break;
            default: mr_pass_gen<INV>(b0, b1, len, L, R, tw);
        }
        __syncthreads();
        float2* t = b0;
        b0 = b1;
        b1 = t;
        L *= R;
    }
    return b0;
}

// find_wrap of the reference unwrapper (exact in f64, kernels_unwrap.hip)
__device__ __forceinline__ int mr_find_wrap(float a, float b) {
    const double d = (double)a - (double)b;
    return d > 3.141592653589793 ? -1 : (d < -3.141592653589793 ? 1 : 0);
}

// ROW_IN_Z with per-map k sources (PhaseOut::kflag): the row pair staged in b1, each
// thread's contiguous run of edges summed, a block-wide exclusive scan of the two maps'
// run sums, then each run walked again: k(j) = colk(i) + sum_{j' < j} -find_wrap(w(j'),
// w(j' + 1)) -- the integers of k_colk / k_rowscan -- for a residue-free map, kin for a map
// the MST unwrapped; z(j) = (w0 + 2 pi k0) + i (w1 + 2 pi k1) (k_make_z) into b0.
template <bool INV>
__device__ __forceinline__ void mr_load_z_scan(const float* in, long row, int H, int n, const MrPlan& p,
                                            const float2* __restrict__ tw, const PhaseOut& ph, float2* b0, float2* b1) {
    __shared__ int scn[2][MR_THREADS];
    const long b = row / H, r = row % H;
    const long o0 = ((2 * b) * H + r) * n, o1 = ((2 * b + 1) * H + r) * n;
    const bool mst0 = ph.kflag[2 * b] != 0, mst1 = ph.kflag[2 * b + 1] != 0;
    for (int i = threadIdx.x; i < n; i += MR_THREADS) b1[i] = make_float2(in[o0 + i], in[o1 + i]);
    __syncthreads();
    const int per = (n + MR_THREADS - 1) / MR_THREADS;
    const int j0 = min((int)threadIdx.x * per, n), j1 = min(j0 + per, n);
    int s0 = 0, s1 = 0;
    for (int j = j0; j < j1 && j + 1 < n; ++j) {
        const float2 a = b1[j], c = b1[j + 1];
        s0 -= mr_find_wrap(a.x, c.x);
        s1 -= mr_find_wrap(a.y, c.y);
    }
    scn[0][threadIdx.x] = s0;
    scn[1][threadIdx.x] = s1;
    __syncthreads();
    for (int off = 1; off < MR_THREADS; off <<= 1) {  // inclusive Hillis-Steele scan
        const int t0 = threadIdx.x >= off ? scn[0][threadIdx.x - off] : 0;
        const int t1 = threadIdx.x >= off ? scn[1][threadIdx.x - off] : 0;
        __syncthreads();
        scn[0][threadIdx.x] += t0;
        scn[1][threadIdx.x] += t1;
        __syncthreads();
    }
    // (colk is read for the scanned maps only: with every map of a chunk unwrapped by the
    // MST the caller computes no column offsets)
    int k0 = (mst0 ? 0 : ph.colk[2 * b * H + r]) + scn[0][threadIdx.x] - s0;
    int k1 = (mst1 ? 0 : ph.colk[(2 * b + 1) * H + r]) + scn[1][threadIdx.x] - s1;
    for (int j = j0; j < j1; ++j) {
        const float2 a = b1[j];
        const int kk0 = mst0 ? ph.kin[o0 + j] : k0, kk1 = mst1 ? ph.kin[o1 + j] : k1;
        float2 v = make_float2((float)((double)a.x + 6.283185307179586 * (double)kk0),
                               (float)((double)a.y + 6.283185307179586 * (double)kk1));
        if (p.blue) v = cmul_dir<INV>(v, tw[p.tc + j]);
        b0[j] = v;
        if (j + 1 < n) {
            const float2 c = b1[j + 1];
            k0 -= mr_find_wrap(a.x, c.x);
            k1 -= mr_find_wrap(a.y, c.y);
        }
    }
    // (the caller's barrier after the zero padding orders these writes before the passes)
}

// gs (null: LDS): rows longer than the LDS holds run their passes in global scratch, the
// block's 2 len complex at gs + blockIdx.x * 2 len (the L2 / MALL-resident working set of a
// launch of at most kMrLongRows rows); blk0: the launch's first block (row batches).
// (GS a template parameter: with a runtime choice the compiler cannot tell the buffers are
// LDS and every access of the LDS rows becomes a flat one, 1.5x slower, r05)
template <bool INV, int IN, int OUT, bool GS>
__global__ __launch_bounds__(MR_THREADS) void k_mr_rows(const void* __restrict__ in, void* __restrict__ out, long nrows,
                                                        int H, float sub, MrPlan p, const float2* __restrict__ tw,
                                                        PhaseOut ph, float2* __restrict__ gs, long blk0) {
    extern __shared__ __attribute__((aligned(16))) float2 mr_lds[];
    const int n = p.n, len = p.blue ? p.M : n;
    constexpr bool PAIR = IN == ROW_IN_REAL2 || IN == ROW_IN_COMPLEX2;
    // pairs never straddle two frames (a batch gives every frame the single-frame call's
    // bits): with H odd each frame's last row transforms alone
    const long hp = (H + 1) / 2;
    const long blk = blk0 + blockIdx.x;
    const long row = PAIR ? (blk / hp) * H + 2 * (blk % hp) : blk;
    const bool second = PAIR && 2 * (blk % hp) + 1 < H;
    float2* b0 = GS ? gs + (size_t)blockIdx.x * 2 * len : mr_lds;
    float2* b1 = b0 + len;
    // the row's loads in groups of MR_LU per thread, all issued before their LDS stores
    // (a load-store pair per trip left each trip waiting for its load)
    auto load_elem = [&](int i) -> float2 {
        if constexpr (IN == ROW_IN_REAL2) {
            const float* x = static_cast<const float*>(in) + row * n + i;
            return make_float2(x[0] - sub, second ? x[n] - sub : 0.f);
        } else if constexpr (IN == ROW_IN_REAL) {
            return make_float2(static_cast<const float*>(in)[row * n + i] - sub, 0.f);
        } else if constexpr (IN == ROW_IN_Z) {  // k_make_z's arithmetic
            const long b = row / H, r = row % H;
            const long i0 = ((2 * b) * H + r) * n + i, i1 = ((2 * b + 1) * H + r) * n + i;
            float p0 = static_cast<const float*>(in)[i0], p1 = static_cast<const float*>(in)[i1];
            if (ph.kin) {
                p0 = (float)((double)p0 + 6.283185307179586 * (double)ph.kin[i0]);
                p1 = (float)((double)p1 + 6.283185307179586 * (double)ph.kin[i1]);
            }
            return make_float2(p0, p1);
        } else if constexpr (IN == ROW_IN_BAND) {
            const long b = row / H, r = row % H;
            const int sl = ph.bslot[i];
            return sl >= 0 ? static_cast<const float2*>(in)[(b * ph.bnc + sl) * H + r] : make_float2(0.f, 0.f);
        } else {
            return static_cast<const float2*>(in)[row * n + i];
        }
    };
    if constexpr (IN == ROW_IN_COMPLEX2) {  // raw rows a, b -> b0, b1 (combined below)
        for (int i0 = threadIdx.x; i0 < n; i0 += MR_LU * MR_THREADS) {
            float2 va[MR_LU], vb[MR_LU];
#pragma unroll
            for (int u = 0; u < MR_LU; ++u) {
                const int i = i0 + u * MR_THREADS;
                if (i < n) {
                    const float2* x = static_cast<const float2*>(in) + row * n + i;
                    va[u] = x[0];
                    vb[u] = second ? x[n] : make_float2(0.f, 0.f);
                }
            }
#pragma unroll
            for (int u = 0; u < MR_LU; ++u) {
                const int i = i0 + u * MR_THREADS;
                if (i < n) {
                    b0[i] = va[u];
                    b1[i] = vb[u];
                }
            }
        }
    } else if (IN != ROW_IN_Z || !ph.kflag) {  // (ROW_IN_Z with kflag: the scan form below)
        for (int i0 = threadIdx.x; i0 < n; i0 += MR_LU * MR_THREADS) {
            float2 v[MR_LU];
#pragma unroll
            for (int u = 0; u < MR_LU; ++u) {
                const int i = i0 + u * MR_THREADS;
                if (i < n) v[u] = load_elem(i);
            }
#pragma unroll
            for (int u = 0; u < MR_LU; ++u) {
                const int i = i0 + u * MR_THREADS;
                if (i < n) b0[i] = p.blue ? cmul_dir<INV>(v[u], tw[p.tc + i]) : v[u];  // Bluestein: the chirp premultiply
            }
        }
    }
    if constexpr (IN == ROW_IN_Z) {
        if (ph.kflag) mr_load_z_scan<INV>(static_cast<const float*>(in), row, H, n, p, tw, ph, b0, b1);
    }
    if constexpr (IN == ROW_IN_COMPLEX2) {
        // Re(ifft(A)) + i Re(ifft(B)) = ifft(Herm(A) + i Herm(B)), Herm(Y)(k) = (Y(k) + conj Y(-k)) / 2:
        // the thread of the pair (k, n - k) reads all four values before writing both
        __syncthreads();
        for (int i = threadIdx.x; i <= n / 2; i += MR_THREADS) {
            const int im = i ? n - i : 0;
            const float2 a = b0[i], am = b0[im], bb = b1[i], bm = b1[im];
            const float2 ha = make_float2(0.5f * (a.x + am.x), 0.5f * (a.y - am.y));
            const float2 hb = make_float2(0.5f * (bb.x + bm.x), 0.5f * (bb.y - bm.y));
            float2 v = make_float2(ha.x - hb.y, ha.y + hb.x);        // Herm(A)(k) + i Herm(B)(k)
            float2 vm = make_float2(ha.x + hb.y, -ha.y + hb.x);      // at -k: conj(Herm(A)(k)) + i conj(Herm(B)(k))
            if (p.blue) {
                v = cmul_dir<INV>(v, tw[p.tc + i]);
                vm = cmul_dir<INV>(vm, tw[p.tc + im]);
            }
            b0[i] = v;
            if (im != i) b0[im] = vm;
        }
    }
    for (int i = n + threadIdx.x; i < len; i += MR_THREADS) b0[i] = make_float2(0.f, 0.f);  // (Bluestein) zero padding
    __syncthreads();
    float2* r;
    if (!p.blue) {
        r = mr_run<INV>(b0, b1, n, p.fct, p.nf, tw);
    } else {
        // y = IFFT_M(FFT_M(a) * G) with G = FFT_M(conj chirp) / M, then the chirp postmultiply
        r = mr_run<false>(b0, b1, len, p.fct, p.nf, tw + p.tM);
        const float2* G = tw + (INV ? p.tgi : p.tgf);
        for (int i = threadIdx.x; i < len; i += MR_THREADS) r[i] = cmul(r[i], G[i]);
        __syncthreads();
        r = mr_run<true>(r, r == b0 ? b1 : b0, len, p.fct, p.nf, tw + p.tM);
        for (int i = threadIdx.x; i < n; i += MR_THREADS) r[i] = cmul_dir<INV>(r[i], tw[p.tc + i]);
        __syncthreads();
    }
    b0 = r;
    if constexpr (OUT == ROW_OUT_COMPLEX) {
        for (int i = threadIdx.x; i < n; i += MR_THREADS) static_cast<float2*>(out)[row * n + i] = b0[i];
    } else if constexpr (OUT == ROW_OUT_BAND2) {  // X_a = (Z(k) + conj Z(-k)) / 2, X_b = (Z(k) - conj Z(-k)) / 2i
        float2* o = static_cast<float2*>(out) + row * (long)ph.bnc;
        for (int i = threadIdx.x; i < n; i += MR_THREADS) {
            const int sl = ph.bslot[i];
            if (sl < 0) continue;
            const float2 z = b0[i], zm = b0[i ? n - i : 0];
            o[sl] = make_float2(0.5f * (z.x + zm.x), 0.5f * (z.y - zm.y));
            if (second) o[ph.bnc + sl] = make_float2(0.5f * (z.y + zm.y), -0.5f * (z.x - zm.x));
        }
    } else if constexpr (OUT == ROW_OUT_REAL2) {
        float* o = static_cast<float*>(out) + row * n;
        for (int i = threadIdx.x; i < n; i += MR_THREADS) {
            const float2 v = b0[i];
            o[i] = v.x;
            if (second) o[n + i] = v.y;
        }
    } else if constexpr (OUT == ROW_OUT_REAL) {
        for (int i = threadIdx.x; i < n; i += MR_THREADS) static_cast<float*>(out)[row * n + i] = b0[i].x;
    } else {
        // w = wrap(theta - angle(A)) == -angle(A * conj(R)) of fcd.py:118 (as k_row_fft)
        const long b = row / H, r = row % H;
        const float* th = ph.theta + r * n;
        float* wo = ph.wrapped + ((b * 2 + ph.carrier) * H + r) * (long)n;
        for (int i0 = threadIdx.x; i0 < n; i0 += MR_LU * MR_THREADS) {
            float t[MR_LU];  // the reference angles of the group, loaded together
#pragma unroll
            for (int u = 0; u < MR_LU; ++u) {
                const int i = i0 + u * MR_THREADS;
                if (i < n) t[u] = th[i];
            }
#pragma unroll
            for (int u = 0; u < MR_LU; ++u) {
                const int i = i0 + u * MR_THREADS;
                if (i >= n) continue;
                const float2 a = b0[i];
                float d = t[u] - fast_atan2(a.y, a.x);  // (gfft.hpp: 3.3e-7 rad, as the fast path's phase kernels)
                if (d > kPiF) d -= kTwoPiF;
                else if (d < -kPiF) d += kTwoPiF;
                wo[i] = d;
            }
        }
    }
}

// [nb][R][C] -> [nb][C][R], 32 x 32 tiles through LDS (odd pitch)
__global__ __launch_bounds__(256) void k_mr_transpose(const float2* __restrict__ in, float2* __restrict__ out, int R,
                                                      int C) {
    __shared__ float2 tile[32][33];
    const long b = blockIdx.z;
    const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
    const float2* src = in + b * (long)R * C;
    float2* dst = out + b * (long)R * C;
    const int tx = threadIdx.x % 32, ty = threadIdx.x / 32;
    for (int y = ty; y < 32; y += 8)
        if (r0 + y < R && c0 + tx < C) tile[y][tx] = src[(long)(r0 + y) * C + c0 + tx];
    __syncthreads();
    for (int y = ty; y < 32; y += 8)
        if (c0 + y < C && r0 + tx < R) dst[(long)(c0 + y) * R + r0 + tx] = tile[tx][y];
}

// ------------------------------------------------------------------ integration columns
// Column transforms of several columns at once (radices 8 / 4 / 2 / 3 / 5 / 7; a column
// length with a larger prime factor takes the transpose route), in place in one LDS buffer (column c at
// buf + c * pitch, a team of `team` threads per column, team a power of two): each pass
// first loads every butterfly input of the thread into registers (at most MC_EPL values
// per thread: len <= MC_EPL * team), then, after a barrier, writes the outputs.  One
// buffer instead of the rows' two: twice the columns per workgroup.
constexpr int MC_EPL = 16;   // values per thread, block-synchronised teams
constexpr int MC_EPL_W = 20; // values per thread, one wave per column (len <= 1280; 18 and 24 spill)

template <int R, int EPL>
constexpr int mc_nbf() { return (EPL + R - 1) / R; }  // butterflies per thread (n / R <= nbf * team)

// WAVE: the team is one wave (64 threads per column), so a pass synchronises the wave
// only; otherwise the workgroup
template <bool WAVE>
__device__ __forceinline__ void mc_sync() {
    if constexpr (WAVE) wave_sync();
    else __syncthreads();
}

template <int R, bool INV, int EPL, bool WAVE>
__device__ __forceinline__ void mc_pass(float2* buf, int pitch, int team, int n, int L, const float2* __restrict__ tw) {
    constexpr int NBF = mc_nbf<R, EPL>();
    const int nbt = n / R, step = n / (L * R);
    const float invL = 1.f / (float)L;
    const int col = WAVE ? (int)(threadIdx.x >> 6) : (int)(threadIdx.x / team);
    const int t = threadIdx.x & (team - 1);
    float2* const cb = buf + col * pitch;
    float2 a[NBF][R];
#pragma unroll
    for (int m = 0; m < NBF; ++m) {
        const int j = t + m * team;
        if (j < nbt) {
#pragma unroll
            for (int r = 0; r < R; ++r) a[m][r] = cb[j + r * nbt];
        }
    }
    mc_sync<WAVE>();
#pragma unroll
    for (int m = 0; m < NBF; ++m) {
        const int j = t + m * team;
        if (j < nbt) {
            const int k = j - L * mr_div(j, L, invL);
            if (L > 1) {
#pragma unroll
                for (int r = 1; r < R; ++r) a[m][r] = cmul_dir<INV>(a[m][r], tw[r * k * step]);
            }
            dft_any<R, INV>(a[m]);
            float2* dst = cb + (j - k) * R + k;
#pragma unroll
            for (int r = 0; r < R; ++r) dst[r * L] = a[m][r];
        }
    }
    mc_sync<WAVE>();
}

// every pass of the plan; ends with a workgroup barrier (the callers' next steps cross columns)
template <bool INV, int EPL, bool WAVE>
__device__ __forceinline__ void mc_run(float2* buf, int pitch, int team, int len, const int* fct, int nf,
                                       const float2* __restrict__ tw) {
    int L = 1;
    for (int f = 0; f < nf; ++f) {
        const int R = fct[f];
        switch (R) {
            case 8: mc_pass<8, INV, EPL, WAVE>(buf, pitch, team, len, L, tw); break;
            case 4: mc_pass<4, INV, EPL, WAVE>(buf, pitch, team, len, L, tw); break;
            case 2: mc_pass<2, INV, EPL, WAVE>(buf, pitch, team, len, L, tw); break;
            case 3: mc_pass<3, INV, EPL, WAVE>(buf, pitch, team, len, L, tw); break;
            case 5: mc_pass<5, INV, EPL, WAVE>(buf, pitch, team, len, L, tw); break;
            default: mc_pass<7, INV, EPL, WAVE>(buf, pitch, team, len, L, tw);  // (mr_int_cols_supported: no larger primes)
        }
        L *= R;
    }
    if constexpr (WAVE) __syncthreads();
}

// The length-H DFT of the workgroup's columns (Bluestein: the columns' first H values hold
// the chirp-premultiplied input, the rest zeros, on entry; the transform's H values on exit).
// tws: the passes' twiddles (LDS), tw: the plan's table (chirp, G).
template <bool INV, int NT, int EPL, bool WAVE>
__device__ __forceinline__ void mc_dft(float2* buf, int ncol, int pitch, int team, const MrPlan& p,
                                       const float2* tws, const float2* __restrict__ tw) {
    if (!p.blue) {
        mc_run<INV, EPL, WAVE>(buf, pitch, team, p.n, p.fct, p.nf, tws);
        return;
    }
    const int M = p.M, H = p.n;
    mc_run<false, EPL, WAVE>(buf, pitch, team, M, p.fct, p.nf, tws);
    const float2* G = tw + (INV ? p.tgi : p.tgf);
    for (int u = threadIdx.x; u < ncol * M; u += NT) {
        const int col = u / M, i = u - col * M;
        buf[col * pitch + i] = cmul(buf[col * pitch + i], G[i]);
    }
    __syncthreads();
    mc_run<true, EPL, WAVE>(buf, pitch, team, M, p.fct, p.nf, tws);
    for (int u = threadIdx.x; u < ncol * H; u += NT) {
        const int col = u / H, i = u - col * H;
        buf[col * pitch + i] = cmul_dir<INV>(buf[col * pitch + i], tw[p.tc + i]);
    }
    __syncthreads();
}

// The spectral integration without the Z(k) / Z(-k) pairing: with m0, m1 the real, odd
// multipliers of integ_multiply (h_hat = i (m0 Phi0 + m1 Phi1), Phi0 / Phi1 the Hermitian
// / anti-Hermitian parts of Z), h = Re(ifft2(h_hat)) = Re(ifft2((m1 + i m0) Z)) exactly
// (the conjugate-mirrored term's real part equals its unmirrored image's); the row
// inverse takes the real part (ROW_IN_COMPLEX2: each row's Hermitian part).
__device__ __forceinline__ float2 mc_mult(float2 z, int q, int r, const IntegCoef& c) {
    const float kx = c.kxe[q], ky = c.kye[r];
    float k2 = c.kx2[q] + c.ky2[r];
    if (r == 0 && q == 0) k2 = 1.f;
    const float s = c.norm / k2;
    const float m0 = (kx * c.a0 + ky * c.b0) * s;
    const float m1 = (kx * c.a1 + ky * c.b1) * s;
    return make_float2(m1 * z.x - m0 * z.y, m1 * z.y + m0 * z.x);
}

// Columns q0 .. q0 + cnt - 1 (q0 = g C) of a frame in LDS slots 0 .. cnt - 1, a team of
// NT / C threads per column, the transform's twiddles copied to LDS after the columns; reads
// and writes run over the slots fastest (C consecutive columns per row), each thread's
// loads issued together (at most MC_EPL: cnt H <= C len <= MC_EPL NT).
template <int NT, int EPL, bool WAVE>
__global__ __launch_bounds__(NT, 4) void k_mr_int_cols(float2* __restrict__ Z, int nblk, int W, int C, int ngroups,
                                                       MrPlan p, const float2* __restrict__ tw, IntegCoef ic) {
    extern __shared__ __attribute__((aligned(16))) float2 mc_lds[];
    const int H = p.n, len = p.blue ? p.M : H, pitch = len + 1;
    // XCD-aware numbering (the grid a multiple of 8; block b runs on XCD b % 8): consecutive
    // column groups on one XCD at once, so their row runs share the XCD's L2 lines
    const long wk = (long)(blockIdx.x % 8) * (gridDim.x / 8) + blockIdx.x / 8;
    if (wk >= nblk) return;
    const long b = wk / ngroups;
    const int g = (int)(wk % ngroups);
    float2* const Zb = Z + b * (long)H * W;
    const int q0 = g * C, cnt = min(C, W - q0);
    const int team = NT / C, total = cnt * H;
    const float invcnt = 1.f / (float)cnt, invH = 1.f / (float)H;
    float2* const tws = mc_lds + C * pitch;  // len twiddles (Bluestein: the M-point table)
    const float2* const twsrc = p.blue ? tw + p.tM : tw;
    for (int i = threadIdx.x; i < len; i += NT) tws[i] = twsrc[i];
    for (int m0 = 0; m0 < EPL; m0 += 8) {  // loads in groups of 8 (registers)
        float2 v[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const int u = threadIdx.x + (m0 + m) * NT;
            if (u < total) {
                const int i = mr_div(u, cnt, invcnt), sl = u - i * cnt;
                v[m] = Zb[(long)i * W + q0 + sl];
            }
        }
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const int u = threadIdx.x + (m0 + m) * NT;
            if (u < total) {
                const int i = mr_div(u, cnt, invcnt), sl = u - i * cnt;
                mc_lds[sl * pitch + i] = p.blue ? cmul_dir<false>(v[m], tw[p.tc + i]) : v[m];
            }
        }
    }
    if (p.blue)
        for (int u = threadIdx.x; u < cnt * (len - H); u += NT) {
            const int sl = u / (len - H), i = H + u - sl * (len - H);
            mc_lds[sl * pitch + i] = make_float2(0.f, 0.f);
        }
    __syncthreads();
    mc_dft<false, NT, EPL, WAVE>(mc_lds, cnt, pitch, team, p, tws, tw);
#pragma unroll 4
    for (int m = 0; m < EPL; ++m) {
        const int u = threadIdx.x + m * NT;
        if (u < total) {
            const int sl = mr_div(u, H, invH), r = u - sl * H;
            float2 v = mc_mult(mc_lds[sl * pitch + r], q0 + sl, r, ic);
            if (p.blue) v = cmul_dir<true>(v, tw[p.tc + r]);  // the inverse's chirp premultiply
            mc_lds[sl * pitch + r] = v;
        }
    }
    if (p.blue)
        for (int u = threadIdx.x; u < cnt * (len - H); u += NT) {
            const int sl = u / (len - H), i = H + u - sl * (len - H);
            mc_lds[sl * pitch + i] = make_float2(0.f, 0.f);
        }
    __syncthreads();
    mc_dft<true, NT, EPL, WAVE>(mc_lds, cnt, pitch, team, p, tws, tw);
    for (int u = threadIdx.x; u < total; u += NT) {
        const int i = mr_div(u, cnt, invcnt), sl = u - i * cnt;
        Zb[(long)i * W + q0 + sl] = mc_lds[sl * pitch + i];
    }
}

// Rows whose two buffers exceed 128 KB of LDS (len > kMrLdsLen) take global scratch,
// kMrLongRows blocks per launch.
constexpr int kMrLdsLen = 8192;
constexpr long kMrLongRows = 1024;

template <bool INV, int IN, int OUT>
void launch_mr(const MrPlan& p, const void* in, void* out, long nrows, int H, float sub, const float2* tw,
               const PhaseOut* ph, hipStream_t s, float2* gs) {
    PhaseOut q{};
    if (ph) q = *ph;
    const int len = p.blue ? p.M : p.n;
    static std::atomic<bool> attr{false};
    if (!attr) {
        // (the rows need at most 2 x 8192 complex; ROW_IN_Z's scan adds 2 KB of static LDS)
        FCD_HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_mr_rows<INV, IN, OUT, false>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024));
        attr = true;
    }
    const long grid = (IN == ROW_IN_REAL2 || IN == ROW_IN_COMPLEX2) ? nrows / H * ((H + 1) / 2) : nrows;
    if (len <= kMrLdsLen) {
        const size_t lds = 2 * (size_t)len * sizeof(float2);
        hipLaunchKernelGGL((k_mr_rows<INV, IN, OUT, false>), dim3((unsigned)grid), dim3(MR_THREADS), lds, s, in, out,
                           nrows, H, sub, p, tw, q, nullptr, 0L);
        FCD_CHECK_LAUNCH();
        return;
    }
    if (!gs) throw std::runtime_error("mr_rows: rows above 8192 points need the context's global scratch");
    for (long b0 = 0; b0 < grid; b0 += kMrLongRows) {  // (in order on the stream: the scratch is reused)
        const long nblk = std::min(kMrLongRows, grid - b0);
        hipLaunchKernelGGL((k_mr_rows<INV, IN, OUT, true>), dim3((unsigned)nblk), dim3(MR_THREADS), 0, s, in, out,
                           nrows, H, sub, p, tw, q, gs, b0);
        FCD_CHECK_LAUNCH();
    }
}

}  // namespace

// largest prime factor of n
static int mr_lpf(int n) {
    int res = 1;
    for (int d = 2; (long)d * d <= n; ++d)
        while (n % d == 0) {
            res = d;
            n /= d;
        }
    return n > 1 ? n : res;
}

// Sides up to kMrMaxLen (the MST's 32-bit vertex ids bound a frame's pixels); rows longer
// than the LDS holds (kMrLdsLen complex, Bluestein's M included) run in global scratch.
bool mr_supported(int n) { return n >= 2 && n <= kMrMaxLen; }

size_t mr_long_scratch_bytes(const MrPlan& p) {
    const int len = p.blue ? p.M : p.n;
    return len <= kMrLdsLen ? 0 : (size_t)kMrLongRows * 2 * len * sizeof(float2);
}

MrPlan mr_plan(int n) {
    if (!mr_supported(n)) throw std::runtime_error("mixed-radix plan: unsupported length " + std::to_string(n));
    MrPlan p{};
    p.n = n;
    p.blue = mr_lpf(n) > kMrMaxRadix;
    int m = n;
    if (p.blue) {
        p.M = 1;
        while (p.M < 2 * n - 1) p.M *= 2;
        m = p.M;
    }
    int two = 0;
    while (m % 2 == 0) {
        m /= 2;
        ++two;
    }
    auto add = [&](int r) {
        if (p.nf >= (int)(sizeof(p.fct) / sizeof(p.fct[0]))) throw std::runtime_error("mixed-radix plan: too many passes");
        p.fct[p.nf++] = r;
    };
    while (two >= 3 && two != 4) {  // 8s, leaving 0, 1, 2 or 4 twos for 4s / a 2
        add(8);
        two -= 3;
    }
    while (two >= 2) {
        add(4);
        two -= 2;
    }
    if (two == 1) add(2);
    for (int d = 3; d <= m; d += 2)
        while (m % d == 0) {
            add(d);
            m /= d;
        }
    // table layout (mr_tables): [n: exp(-2 pi i j / n)] then, with Bluestein, [M: exp(-2 pi i j / M)]
    // [n: chirp] [M: G forward] [M: G inverse]
    if (p.blue) {
        p.tM = n;
        p.tc = n + p.M;
        p.tgf = 2 * n + p.M;
        p.tgi = 2 * n + 2 * p.M;
    }
    return p;
}

// f64 radix-2 FFT (host; Bluestein's G tables)
static void fft_f64(std::vector<std::complex<double>>& a) {
    const size_t n = a.size();
    for (size_t i = 1, j = 0; i < n; ++i) {
        size_t bit = n >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) std::swap(a[i], a[j]);
    }
    const double pi = 3.14159265358979323846;
    for (size_t len = 2; len <= n; len <<= 1)
        for (size_t i = 0; i < n; i += len)
            for (size_t k = 0; k < len / 2; ++k) {
                const std::complex<double> w = std::polar(1.0, -2.0 * pi * (double)k / (double)len);
                const std::complex<double> u = a[i + k], v = a[i + k + len / 2] * w;
                a[i + k] = u + v;
                a[i + k + len / 2] = u - v;
            }
}

std::vector<float2> mr_tables(const MrPlan& p) {
    const double pi = 3.14159265358979323846;
    const int n = p.n;
    auto unit = [&](double a) { return make_float2((float)std::cos(a), (float)std::sin(a)); };
    std::vector<float2> t((size_t)n);
    for (int j = 0; j < n; ++j) t[j] = unit(-2.0 * pi * (double)j / (double)n);
    if (!p.blue) return t;
    const int M = p.M;
    t.resize((size_t)2 * n + 3 * (size_t)M);
    for (int j = 0; j < M; ++j) t[p.tM + j] = unit(-2.0 * pi * (double)j / (double)M);
    std::vector<std::complex<double>> c(n);
    for (int j = 0; j < n; ++j) {
        const long long q = (long long)j * j % (2LL * n);  // exact argument reduction
        c[j] = std::polar(1.0, -pi * (double)q / (double)n);
        t[p.tc + j] = make_float2((float)c[j].real(), (float)c[j].imag());
    }
    for (int dir = 0; dir < 2; ++dir) {  // G = FFT_M(g) / M, g = conj(chirp) (forward), chirp (inverse)
        std::vector<std::complex<double>> g(M, 0.0);
        for (int j = 0; j < n; ++j) {
            const std::complex<double> v = dir == 0 ? std::conj(c[j]) : c[j];
            g[j] = v;
            if (j) g[M - j] = v;
        }
        fft_f64(g);
        for (int j = 0; j < M; ++j) {
            const std::complex<double> v = g[j] / (double)M;
            t[(dir == 0 ? p.tgf : p.tgi) + j] = make_float2((float)v.real(), (float)v.imag());
        }
    }
    return t;
}

void mr_rows(const MrPlan& p, bool inverse, RowIn im, RowOut om, const void* in, void* out, long nrows, int H,
             float sub, const float2* tw, const PhaseOut* ph, hipStream_t s, float2* gs) {
    if (nrows <= 0) return;
    if (!inverse && im == ROW_IN_REAL && om == ROW_OUT_COMPLEX)
        launch_mr<false, ROW_IN_REAL, ROW_OUT_COMPLEX>(p, in, out, nrows, H, sub, tw, ph, s, gs);
    else if (!inverse && im == ROW_IN_REAL2 && om == ROW_OUT_BAND2)
        launch_mr<false, ROW_IN_REAL2, ROW_OUT_BAND2>(p, in, out, nrows, H, sub, tw, ph, s, gs);
    else if (inverse && im == ROW_IN_COMPLEX2 && om == ROW_OUT_REAL2)
        launch_mr<true, ROW_IN_COMPLEX2, ROW_OUT_REAL2>(p, in, out, nrows, H, sub, tw, ph, s, gs);
    else if (!inverse && im == ROW_IN_COMPLEX && om == ROW_OUT_COMPLEX)
        launch_mr<false, ROW_IN_COMPLEX, ROW_OUT_COMPLEX>(p, in, out, nrows, H, sub, tw, ph, s, gs);
    else if (!inverse && im == ROW_IN_Z && om == ROW_OUT_COMPLEX)
        launch_mr<false, ROW_IN_Z, ROW_OUT_COMPLEX>(p, in, out, nrows, H, sub, tw, ph, s, gs);
    else if (inverse && im == ROW_IN_COMPLEX && om == ROW_OUT_COMPLEX)
        launch_mr<true, ROW_IN_COMPLEX, ROW_OUT_COMPLEX>(p, in, out, nrows, H, sub, tw, ph, s, gs);
    else if (inverse && im == ROW_IN_COMPLEX && om == ROW_OUT_REAL)
        launch_mr<true, ROW_IN_COMPLEX, ROW_OUT_REAL>(p, in, out, nrows, H, sub, tw, ph, s, gs);
    else if (inverse && im == ROW_IN_COMPLEX && om == ROW_OUT_PHASE)
        launch_mr<true, ROW_IN_COMPLEX, ROW_OUT_PHASE>(p, in, out, nrows, H, sub, tw, ph, s, gs);
    else if (inverse && im == ROW_IN_BAND && om == ROW_OUT_PHASE)
        launch_mr<true, ROW_IN_BAND, ROW_OUT_PHASE>(p, in, out, nrows, H, sub, tw, ph, s, gs);
    else
        throw std::runtime_error("mr_rows: unsupported mode combination");
}

bool mr_int_cols_supported(const MrPlan& p) {  // (also Bluestein: M is a power of two)
    if ((p.blue ? p.M : p.n) > kMrLdsLen) return false;  // long columns: the transpose route (global-scratch rows)
    for (int f = 0; f < p.nf; ++f)
        if (p.fct[f] > 8 || p.fct[f] == 6) return false;  // the generic odd-prime passes: the transpose route
    return true;
}

// Columns per group C (a power of two <= 16: up to 128-byte row runs).  Columns up to 1280
// points: one wave per column (EPL 20 values per thread, passes synchronised per wave, the
// workgroup 64 C threads); longer ones: a team of 512 / C threads per column (EPL 16;
// 1024 threads for the 8192-point columns).  LDS: the C columns and the len twiddles, at
// most 80 KB (two workgroups per CU).
template <int NT, int EPL, bool WAVE>
static void launch_int_cols(const MrPlan& p, float2* Z, long blocks, int W, int C, int ngroups, size_t lds,
                            const float2* tw, const IntegCoef& c, hipStream_t s) {
    static std::atomic<bool> attr{false};
    if (!attr) {
        FCD_HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_mr_int_cols<NT, EPL, WAVE>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        attr = true;
    }
    const unsigned grid = (unsigned)((blocks + 7) / 8 * 8);
    hipLaunchKernelGGL((k_mr_int_cols<NT, EPL, WAVE>), dim3(grid), dim3(NT), lds, s, Z, (int)blocks, W, C, ngroups, p,
                       tw, c);
    FCD_CHECK_LAUNCH();
}

void mr_int_cols(const MrPlan& p, float2* Z, int nb, int W, const float2* tw, const IntegCoef& c, hipStream_t s) {
    if (nb <= 0) return;
    if (!mr_int_cols_supported(p)) throw std::runtime_error("mr_int_cols: a radix above 8");
    const int len = p.blue ? p.M : p.n;
    auto lds_of = [&](int C) { return (size_t)(C * (len + 1) + len) * sizeof(float2); };
    if (len <= MC_EPL_W * 64) {  // wave teams (bit-identical to the block teams: same passes and order)
        int C = 16;
        while (C > 1 && lds_of(C) > 80 * 1024) C /= 2;
        const int ngroups = (W + C - 1) / C;
        const long blocks = (long)nb * ngroups;
        switch (C) {
            case 16: launch_int_cols<1024, MC_EPL_W, true>(p, Z, blocks, W, C, ngroups, lds_of(C), tw, c, s); break;
            case 8: launch_int_cols<512, MC_EPL_W, true>(p, Z, blocks, W, C, ngroups, lds_of(C), tw, c, s); break;
            case 4: launch_int_cols<256, MC_EPL_W, true>(p, Z, blocks, W, C, ngroups, lds_of(C), tw, c, s); break;
            case 2: launch_int_cols<128, MC_EPL_W, true>(p, Z, blocks, W, C, ngroups, lds_of(C), tw, c, s); break;
            default: launch_int_cols<64, MC_EPL_W, true>(p, Z, blocks, W, C, ngroups, lds_of(C), tw, c, s);
        }
        return;
    }
    auto fits = [&](int C, int nt) { return len <= MC_EPL * (nt / C) && lds_of(C) <= (nt == 512 ? 80 : 160) * 1024; };
    int nt = 512, C = 1;
    while (C < 16 && fits(2 * C, 512)) C *= 2;
    if (!fits(C, 512)) {  // (1024 threads with twice the columns measured 2-3 % slower at 1080 x 1920, r05)
        nt = 1024;
        C = 1;
        while (C < 16 && fits(2 * C, 1024)) C *= 2;
        if (!fits(C, 1024)) throw std::runtime_error("mr_int_cols: column length " + std::to_string(len) + " exceeds the workgroup");
    }
    const int ngroups = (W + C - 1) / C;
    const long blocks = (long)nb * ngroups;
    if (nt == 512) launch_int_cols<512, MC_EPL, false>(p, Z, blocks, W, C, ngroups, lds_of(C), tw, c, s);
    else launch_int_cols<1024, MC_EPL, false>(p, Z, blocks, W, C, ngroups, lds_of(C), tw, c, s);
}

void mr_transpose(const float2* in, float2* out, int nb, int R, int C, hipStream_t s) {
    if (nb <= 0) return;
    hipLaunchKernelGGL(k_mr_transpose, dim3((unsigned)((C + 31) / 32), (unsigned)((R + 31) / 32), (unsigned)nb),
                       dim3(256), 0, s, in, out, R, C);
    FCD_CHECK_LAUNCH();
}

// Column subset (the generic chain's band-pruned column passes): gather [nb][R][C] ->
// [nb][NS][R] for the columns cols[0..NS), 32 x 32 tiles through LDS.
__global__ __launch_bounds__(256) void k_mr_gather_cols(const float2* __restrict__ in, float2* __restrict__ out, int R,
                                                        int C, const int* __restrict__ cols, int NS) {
    __shared__ float2 tile[32][33];
    const long b = blockIdx.z;
    const int r0 = blockIdx.y * 32, s0 = blockIdx.x * 32;
    const float2* src = in + b * (long)R * C;
    float2* dst = out + b * (long)NS * R;
    const int tx = threadIdx.x % 32, ty = threadIdx.x / 32;
    const int col = s0 + tx < NS ? cols[s0 + tx] : 0;
    for (int y = ty; y < 32; y += 8)
        if (r0 + y < R && s0 + tx < NS) tile[y][tx] = src[(long)(r0 + y) * C + col];
    __syncthreads();
    for (int y = ty; y < 32; y += 8)
        if (s0 + y < NS && r0 + tx < R) dst[(long)(s0 + y) * R + r0 + tx] = tile[tx][y];
}

void mr_gather_cols(const float2* in, float2* out, int nb, int R, int C, const int* cols, int NS, hipStream_t s) {
    if (nb <= 0 || NS <= 0) return;
    hipLaunchKernelGGL(k_mr_gather_cols, dim3((unsigned)((NS + 31) / 32), (unsigned)((R + 31) / 32), (unsigned)nb),
                       dim3(256), 0, s, in, out, R, C, cols, NS);
    FCD_CHECK_LAUNCH();
}

void mr_cols(const MrPlan& p, int W, bool inverse, float2* data, int nb, const float2* tw, float2* scratch,
             hipStream_t s, float2* gs) {
    const int H = p.n;
    mr_transpose(data, scratch, nb, H, W, s);
    mr_rows(p, inverse, ROW_IN_COMPLEX, ROW_OUT_COMPLEX, scratch, scratch, (long)nb * W, W, 0.f, tw, nullptr, s, gs);
    mr_transpose(scratch, data, nb, W, H, s);
}

}  // namespace fcdk
