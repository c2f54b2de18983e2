// The reference's peak-finding spectrum, bit for bit (fourier.py:18):
//   |fftshift(scipy.fft.fft2(image - np.mean(image)))|
// for images of any shape in float32 or float64, with the operations of the libraries
// the reference runs on (scipy 1.7.1's pocketfft, numpy 1.26.4; restated in
// csrc/pocketfft.hpp, the device and host code of the passes, and in oracle/pocketfft.py,
// the CPU restatement pinned to scipy):
//
//  * np.mean: 8192-element chunks, each summed pairwise (numpy's pairwise_sum), chunk
//    sums accumulated in order, one division, in the image's type (k_pf_chunk_sums,
//    k_pf_center);
//  * scipy.fft.fft2 of a real image (c2c_sym_internal): pocketfft_r over every row
//    (rfftp or Bluestein), pocketfft_c over every column of the half spectrum (cfftp or
//    Bluestein), the rest filled as conjugate mirrors in the library's iteration order
//    (k_pf_rows, k_pf_cols, k_pf_mirror);
//  * np.abs of complex64 / complex128 (kernels_fft.hip).
//
// Every butterfly is the library's expression evaluated in the same order with IEEE
// operations: this file is compiled with -ffp-contract=off.  The parallel schedule
// differs (one workgroup per row or column, one thread per butterfly of a pass, a barrier
// between passes), the arithmetic graph of every output does not.  Rows / columns whose
// two working buffers fit 64 KB stay in LDS; longer ones (Bluestein's convolution
// length, float64) work in a global scratch slot per workgroup.  Only the reference
// setup uses these transforms (once per reference); the per-frame pipeline keeps its
// register FFTs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <stdexcept>
#include <string>

#include "kernels.hpp"
#include "pocketfft.hpp"

#define FCD_CHECK_LAUNCH()                                                          \
    do {                                                                            \
        hipError_t e_ = hipGetLastError();                                          \
        if (e_ != hipSuccess) throw std::runtime_error(std::string("kernel launch: ") + hipGetErrorString(e_)); \
    } while (0)

namespace fcdk {

namespace {

constexpr int PF_THREADS = 256;
constexpr size_t PF_LDS_MAX = 64 * 1024;  // per workgroup
constexpr int PF_GLOBAL_BLOCKS = 512;     // workgroups (= scratch slots) when the buffers go to HBM

struct BarrierSync {
    __device__ void operator()() const { __syncthreads(); }
};

__device__ __forceinline__ float div_rn(float a, float b) { return __fdiv_rn(a, b); }
__device__ __forceinline__ double div_rn(double a, double b) { return __ddiv_rn(a, b); }

// ------------------------------------------------------------------ np.mean
// One workgroup per (8192-element chunk, image).  A chunk of 128 * 2^k elements is numpy's
// pairwise tree with leaves of 128: thread t sums block t with the 8 accumulators, then
// the blocks combine pairwise (left + right) up the tree; any other chunk length (the
// last chunk of an image whose size is not a multiple of 8192) is summed by one thread
// with the same recursion (pf::pairwise_sum).
template <class T>
__global__ __launch_bounds__(64) void k_pf_chunk_sums(const T* __restrict__ img, long hw, int nchunks,
                                                      T* __restrict__ sums) {
    __shared__ T blk[64];
    const int c = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
    const long lo = (long)c * 8192;
    const int csize = (int)((hw - lo) < 8192 ? (hw - lo) : 8192);
    const T* a = img + (long)b * hw + lo;
    const int nblk = csize / 128;
    const bool tree = csize % 128 == 0 && (nblk & (nblk - 1)) == 0;
    if (tree) {
        if (t < nblk) {
            const T* q = a + (long)t * 128;
            T r[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) r[j] = q[j];
            for (int i = 8; i < 128; i += 8) {
#pragma unroll
                for (int j = 0; j < 8; ++j) r[j] = r[j] + q[i + j];
            }
            blk[t] = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        }
        __syncthreads();
        for (int w = 2; w <= nblk; w <<= 1) {
            if (t < nblk / w) blk[t * w] = blk[t * w] + blk[t * w + w / 2];
            __syncthreads();
        }
    } else if (t == 0) {
        blk[0] = pf::pairwise_sum<T>(a, csize);
    }
    if (t == 0) sums[(long)b * nchunks + c] = blk[0];
}

// mean = (chunk sums accumulated in order) / n; out = img - mean
template <class T>
__global__ void k_pf_center(const T* __restrict__ img, long hw, int nchunks, const T* __restrict__ sums,
                            T* __restrict__ out) {
    __shared__ T mean_s;
    const long b = blockIdx.y;
    if (threadIdx.x == 0) {
        T acc = T(0);
        for (int c = 0; c < nchunks; ++c) acc = acc + sums[b * nchunks + c];
        mean_s = div_rn(acc, (T)hw);
    }
    __syncthreads();
    const T m = mean_s;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < hw; i += (long)gridDim.x * blockDim.x)
        out[b * hw + i] = img[b * hw + i] - m;
}

// ------------------------------------------------------------------ rows (pocketfft_r, forward)
// One workgroup per row (grid-stride over rows with a scratch slot in HBM when the
// buffers do not fit LDS); bins 0 .. W/2 of the row of F from the halfcomplex result.
template <class T, bool LDS>
__global__ __launch_bounds__(PF_THREADS) void k_pf_rows(const T* __restrict__ in, pf::cx<T>* __restrict__ F, long nrows,
                                                        int W, pf::Plan p, const T* __restrict__ tab, pf::cx<T>* gscr,
                                                        long slot) {
    extern __shared__ __attribute__((aligned(16))) unsigned char pf_smem[];
    pf::cx<T>* A = LDS ? reinterpret_cast<pf::cx<T>*>(pf_smem) : gscr + (long)blockIdx.x * slot;
    const int tid = threadIdx.x, nt = blockDim.x;
    const BarrierSync sync;
    for (long row = blockIdx.x; row < nrows; row += gridDim.x) {
        const T* x = in + row * W;
        pf::cx<T>* out = F + row * W;
        if (!p.blue) {
            T* p1 = reinterpret_cast<T*>(A);
            T* p2 = p1 + W;
            for (int i = tid; i < W; i += nt) p1[i] = x[i];
            sync();
            const T* r = pf::rfft_run<T>(p, tab, p1, p2, tid, nt, sync);
            for (int m = tid; m <= W / 2; m += nt) {
                pf::cx<T> v;
                if (m == 0) v = pf::mk<T>(r[0], T(0));
                else if (2 * m == W) v = pf::mk<T>(r[W - 1], T(0));
                else v = pf::mk<T>(r[2 * m - 1], r[2 * m]);
                out[m] = v;
            }
        } else {  // fftblue::exec_r: tmp[m] = (c[m], T0(0) * c[0]), fft<true>, halfcomplex of tmp
            pf::cx<T>* B = A + p.n2;
            const T x0 = x[0];
            for (int i = tid; i < W; i += nt) A[i] = pf::mk<T>(x[i], T(0) * x0);
            sync();
            pf::blue_fft<T, true>(p, tab, A, B, tid, nt, sync);
            for (int m = tid; m <= W / 2; m += nt)
                out[m] = (m == 0 || 2 * m == W) ? pf::mk<T>(A[m].r, T(0)) : A[m];
        }
        sync();
    }
}

// ------------------------------------------------------------------ columns (pocketfft_c, forward)
template <class T, bool LDS>
__global__ __launch_bounds__(PF_THREADS) void k_pf_cols(pf::cx<T>* __restrict__ F, int H, int W, long items,
                                                        pf::Plan p, const T* __restrict__ tab, pf::cx<T>* gscr,
                                                        long slot) {
    extern __shared__ __attribute__((aligned(16))) unsigned char pf_smem[];
    pf::cx<T>* A = LDS ? reinterpret_cast<pf::cx<T>*>(pf_smem) : gscr + (long)blockIdx.x * slot;
    const int tid = threadIdx.x, nt = blockDim.x, hc = W / 2 + 1;
    const BarrierSync sync;
    for (long item = blockIdx.x; item < items; item += gridDim.x) {
        const long b = item / hc;
        const int j = (int)(item % hc);
        pf::cx<T>* col = F + b * H * W + j;
        for (int i = tid; i < H; i += nt) A[i] = col[(long)i * W];
        sync();
        const pf::cx<T>* r = A;
        if (!p.blue) r = pf::cfft_run<T, true>(p, tab, A, A + H, tid, nt, sync);
        else pf::blue_fft<T, true>(p, tab, A, A + p.n2, tid, nt, sync);
        for (int i = tid; i < H; i += nt) col[(long)i * W] = r[i];
        sync();
    }
}

// The other half as conjugate mirrors (c2c_sym_internal's rev_iter over (i, j <= W/2) in
// row-major order, out[(H - i) % H][(W - j) % W] = conj(out[i][j])): columns past W/2
// from their mirrors; a self-mirrored column (0, and W/2 for even W) keeps its upper
// half, its lower half becomes the conjugate of the upper, and its self-mirrored bins
// (rows i with 2 i = 0 mod H) are conjugated in place.
template <class T>
__global__ void k_pf_mirror(pf::cx<T>* __restrict__ F, int H, int W, long n) {
    const long g = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n) return;
    const long hw = (long)H * W, b = g / hw, idx = g - b * hw;
    const int i = (int)(idx / W), j = (int)(idx % W);
    pf::cx<T>* f = F + b * hw;
    const int ih = (H - i) % H;
    if (j > W / 2) {
        const pf::cx<T> v = f[(long)ih * W + (W - j)];
        f[idx] = pf::mk<T>(v.r, -v.i);
    } else if ((2 * j) % W == 0) {
        if (ih < i) {
            const pf::cx<T> v = f[(long)ih * W + j];
            f[idx] = pf::mk<T>(v.r, -v.i);
        } else if (ih == i) {
            const pf::cx<T> v = f[idx];
            f[idx] = pf::mk<T>(v.r, -v.i);
        }
    }
}

template <class T>
size_t row_bytes(const pf::Plan& p) {
    return p.blue ? 2 * (size_t)p.n2 * sizeof(pf::cx<T>) : 2 * (size_t)p.n * sizeof(T);
}
template <class T>
size_t col_bytes(const pf::Plan& p) {
    return 2 * (size_t)(p.blue ? p.n2 : p.n) * sizeof(pf::cx<T>);
}

template <class T>
void fft2_t(const T* in, int nb, int H, int W, const pf::Plan& rows, const T* rtab, const pf::Plan& cols,
            const T* ctab, pf::cx<T>* F, pf::cx<T>* scratch, hipStream_t s) {
    const long nrows = (long)nb * H;
    const size_t rb = row_bytes<T>(rows), cb = col_bytes<T>(cols);
    if (rb <= PF_LDS_MAX) {
        hipLaunchKernelGGL((k_pf_rows<T, true>), dim3((unsigned)nrows), dim3(PF_THREADS), rb, s, in, F, nrows, W, rows,
                           rtab, nullptr, 0L);
    } else {
        const long slot = (long)(rb / sizeof(pf::cx<T>));
        hipLaunchKernelGGL((k_pf_rows<T, false>), dim3((unsigned)std::min<long>(nrows, PF_GLOBAL_BLOCKS)),
                           dim3(PF_THREADS), 0, s, in, F, nrows, W, rows, rtab, scratch, slot);
    }
    FCD_CHECK_LAUNCH();
    const long items = (long)nb * (W / 2 + 1);
    if (cb <= PF_LDS_MAX) {
        hipLaunchKernelGGL((k_pf_cols<T, true>), dim3((unsigned)items), dim3(PF_THREADS), cb, s, F, H, W, items, cols,
                           ctab, nullptr, 0L);
    } else {
        const long slot = (long)(cb / sizeof(pf::cx<T>));
        hipLaunchKernelGGL((k_pf_cols<T, false>), dim3((unsigned)std::min<long>(items, PF_GLOBAL_BLOCKS)),
                           dim3(PF_THREADS), 0, s, F, H, W, items, cols, ctab, scratch, slot);
    }
    FCD_CHECK_LAUNCH();
    const long n = (long)nb * H * W;
    hipLaunchKernelGGL((k_pf_mirror<T>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, F, H, W, n);
    FCD_CHECK_LAUNCH();
}

template <class T>
void center_t(const T* img, int nb, long hw, T* sums, T* out, hipStream_t s) {
    const int nchunks = pf_chunk_count(hw);
    hipLaunchKernelGGL((k_pf_chunk_sums<T>), dim3(nchunks, nb), dim3(64), 0, s, img, hw, nchunks, sums);
    FCD_CHECK_LAUNCH();
    const unsigned gx = (unsigned)std::min<long>(256, (hw + 255) / 256);
    hipLaunchKernelGGL((k_pf_center<T>), dim3(gx, nb), dim3(256), 0, s, img, hw, nchunks, sums, out);
    FCD_CHECK_LAUNCH();
}

}  // namespace

int pf_chunk_count(long hw) { return (int)((hw + 8191) / 8192); }

size_t pf_scratch_bytes(const pf::Plan& rows, const pf::Plan& cols, bool f64) {
    auto need = [&](size_t rb, size_t cb) {
        size_t b = 0;
        if (rb > PF_LDS_MAX) b = std::max(b, rb * PF_GLOBAL_BLOCKS);
        if (cb > PF_LDS_MAX) b = std::max(b, cb * PF_GLOBAL_BLOCKS);
        return b;
    };
    return f64 ? need(row_bytes<double>(rows), col_bytes<double>(cols))
               : need(row_bytes<float>(rows), col_bytes<float>(cols));
}

void pf_center(const void* img, bool f64, int nb, long hw, void* sums, void* out, hipStream_t s) {
    if (f64)
        center_t<double>(static_cast<const double*>(img), nb, hw, static_cast<double*>(sums), static_cast<double*>(out), s);
    else
        center_t<float>(static_cast<const float*>(img), nb, hw, static_cast<float*>(sums), static_cast<float*>(out), s);
}

void pf_fft2(const void* in, bool f64, int nb, int H, int W, const pf::Plan& rows, const void* rtab, const pf::Plan& cols,
             const void* ctab, void* F, void* scratch, hipStream_t s) {
    if (f64)
        fft2_t<double>(static_cast<const double*>(in), nb, H, W, rows, static_cast<const double*>(rtab), cols,
                       static_cast<const double*>(ctab), static_cast<pf::cx<double>*>(F),
                       static_cast<pf::cx<double>*>(scratch), s);
    else
        fft2_t<float>(static_cast<const float*>(in), nb, H, W, rows, static_cast<const float*>(rtab), cols,
                      static_cast<const float*>(ctab), static_cast<pf::cx<float>*>(F), static_cast<pf::cx<float>*>(scratch),
                      s);
}

}  // namespace fcdk
