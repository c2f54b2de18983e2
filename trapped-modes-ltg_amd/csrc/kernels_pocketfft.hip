// The reference's float32 peak-finding spectrum, bit for bit (fourier.py:18):
//   |fftshift(scipy.fft.fft2(image - np.mean(image)))|
// with the operations of the libraries the reference runs on (scipy 1.7.1's pocketfft,
// numpy 1.26.4; the CPU restatement and its pins: oracle/pocketfft32.py):
//
//  * np.mean of float32: 8192-element chunks, each summed pairwise (8 accumulators over
//    128-element blocks, blocks combined in halves), chunk sums accumulated in order,
//    one float32 division (k_pf_chunk_sums, k_pf_center);
//  * scipy.fft.fft2 of a real float32 image: FFTPACK radf4 / radf2 / radf3 / radf5
//    passes over every row (rfftp, factors 4... with a single 2 first, then 3s, 5s),
//    cfftp pass8 / pass4 / pass2 / pass3 / pass5 forward over every column of the half
//    spectrum, the rest filled as conjugate mirrors (k_pf_rows, k_pf_cols, k_pf_mirror);
//    even lengths whose odd part is 5-smooth (longer prime factors take pocketfft's
//    generic / Bluestein passes, not restated);
//  * np.abs of complex64: larger * sqrt(fma(r, r, 1)), r = smaller / larger (its
//    AVX512F loop; pf_cabs, used by the candidate kernel in kernels_fft.hip).
//
// Every butterfly is the library's expression evaluated in the same order with IEEE
// single-precision operations: this file is compiled with -ffp-contract=off (no fused
// multiply-adds except the one np.abs itself fuses).  The parallel schedule differs
// (one thread per butterfly of a pass, the row or column staged in LDS), the arithmetic
// graph of every output does not.  Only the reference setup uses these transforms
// (once per reference); the per-frame pipeline keeps its register FFTs.
#include <hip/hip_runtime.h>

#include <cmath>
#include <stdexcept>
#include <string>

#include "kernels.hpp"

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

namespace fcdk {

namespace {

constexpr float kHsqt2 = 0.707106781186547524400844362104849f;  // pocketfft's hsqt2 (T0 = float)
// radf3 / pass3 and radf5 / pass5 constants (T0 = float)
constexpr float kTaur = -0.5f, kTaui = 0.8660254037844386467637231707529362f;
constexpr float kTr11 = 0.3090169943749474241022934171828191f, kTi11 = 0.9510565162951535721164393333793821f;
constexpr float kTr12 = -0.8090169943749474241022934171828191f, kTi12 = 0.5877852522924731291687059546390728f;
constexpr int PF_THREADS = 256;

// ------------------------------------------------------------------ np.mean (float32)
// One workgroup per (8192-element chunk, image): thread t sums 128-element block t with
// numpy's 8 accumulators, then the blocks combine pairwise (left + right) up the tree.
// Frame sides are multiples of 64, so every chunk is 8192 elements except a last one of
// 4096: both 2^k blocks of 128, where numpy's recursive halving is exactly this tree.
__global__ __launch_bounds__(64) void k_pf_chunk_sums(const float* __restrict__ img, long hw, int nchunks,
                                                       float* __restrict__ sums) {
    __shared__ float blk[64];
    const int c = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
    const long lo = (long)c * 8192;
    const int csize = (int)((hw - lo) < 8192 ? (hw - lo) : 8192);  // 8192, or 4096 for a 64 x 64 image
    const int nblk = csize / 128;
    if (t < nblk) {
        const float* a = img + (long)b * hw + lo + (long)t * 128;
        float r[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        for (int i = 8; i < 128; i += 8) {
#pragma unroll
            for (int j = 0; j < 8; ++j) r[j] = r[j] + a[i + j];
        }
        blk[t] = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    }
    __syncthreads();
    for (int w = 2; w <= nblk; w <<= 1) {  // pairwise: rec(n) = rec(n/2) + rec(n/2)
        if (t < nblk / w) blk[t * w] = blk[t * w] + blk[t * w + w / 2];
        __syncthreads();
    }
    if (t == 0) sums[(long)b * nchunks + c] = blk[0];
}

// mean = (chunk sums accumulated in order) / n in float32; out = img - mean
__global__ void k_pf_center(const float* __restrict__ img, long hw, int nchunks, const float* __restrict__ sums,
                            float* __restrict__ out, long n) {
    __shared__ float mean_s;
    const long b = blockIdx.y;
    if (threadIdx.x == 0) {
        float acc = 0.f;
        for (int c = 0; c < nchunks; ++c) acc = acc + sums[b * nchunks + c];
        mean_s = __fdiv_rn(acc, (float)hw);
    }
    __syncthreads();
    const float m = mean_s;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < hw; i += (long)gridDim.x * blockDim.x)
        out[b * hw + i] = img[b * hw + i] - m;
}

// ------------------------------------------------------------------ rows: rfftp forward
// CC(a, b, c) = cc[a + ido*(b + l1*c)], CH(a, b, c) = ch[a + ido*(b + ip*c)]
__device__ void radf2(int ido, int l1, const float* cc, float* ch, const float* wa) {
#define CC(a, b, c) cc[(a) + ido * ((b) + l1 * (c))]
#define CH(a, b, c) ch[(a) + ido * ((b) + 2 * (c))]
    for (int k = threadIdx.x; k < l1; k += blockDim.x) {
        CH(0, 0, k) = CC(0, k, 0) + CC(0, k, 1);
        CH(ido - 1, 1, k) = CC(0, k, 0) - CC(0, k, 1);
        if ((ido & 1) == 0) {
            CH(0, 1, k) = -CC(ido - 1, k, 1);
            CH(ido - 1, 0, k) = CC(ido - 1, k, 0);
        }
    }
    if (ido <= 2) return;
    const int m = (ido - 1) / 2;
    for (int it = threadIdx.x; it < l1 * m; it += blockDim.x) {
        const int k = it / m, i = 2 + 2 * (it % m), ic = ido - i;
        const float tr2 = wa[i - 2] * CC(i - 1, k, 1) + wa[i - 1] * CC(i, k, 1);
        const float ti2 = wa[i - 2] * CC(i, k, 1) - wa[i - 1] * CC(i - 1, k, 1);
        CH(i - 1, 0, k) = CC(i - 1, k, 0) + tr2;
        CH(ic - 1, 1, k) = CC(i - 1, k, 0) - tr2;
        CH(i, 0, k) = ti2 + CC(i, k, 0);
        CH(ic, 1, k) = ti2 - CC(i, k, 0);
    }
#undef CH
}

__device__ void radf4(int ido, int l1, const float* cc, float* ch, const float* wa) {
#define CH(a, b, c) ch[(a) + ido * ((b) + 4 * (c))]
#define WA(x, i) wa[(i) + (x) * (ido - 1)]
    for (int k = threadIdx.x; k < l1; k += blockDim.x) {
        const float tr1 = CC(0, k, 3) + CC(0, k, 1);
        CH(0, 2, k) = CC(0, k, 3) - CC(0, k, 1);
        const float tr2 = CC(0, k, 0) + CC(0, k, 2);
        CH(ido - 1, 1, k) = CC(0, k, 0) - CC(0, k, 2);
        CH(0, 0, k) = tr2 + tr1;
        CH(ido - 1, 3, k) = tr2 - tr1;
        if ((ido & 1) == 0) {
            const float ti1 = -kHsqt2 * (CC(ido - 1, k, 1) + CC(ido - 1, k, 3));
            const float tq1 = kHsqt2 * (CC(ido - 1, k, 1) - CC(ido - 1, k, 3));
            CH(ido - 1, 0, k) = CC(ido - 1, k, 0) + tq1;
            CH(ido - 1, 2, k) = CC(ido - 1, k, 0) - tq1;
            CH(0, 3, k) = ti1 + CC(ido - 1, k, 2);
            CH(0, 1, k) = ti1 - CC(ido - 1, k, 2);
        }
    }
    if (ido <= 2) return;
    const int m = (ido - 1) / 2;
    for (int it = threadIdx.x; it < l1 * m; it += blockDim.x) {
        const int k = it / m, i = 2 + 2 * (it % m), ic = ido - i;
        const float cr2 = WA(0, i - 2) * CC(i - 1, k, 1) + WA(0, i - 1) * CC(i, k, 1);
        const float ci2 = WA(0, i - 2) * CC(i, k, 1) - WA(0, i - 1) * CC(i - 1, k, 1);
        const float cr3 = WA(1, i - 2) * CC(i - 1, k, 2) + WA(1, i - 1) * CC(i, k, 2);
        const float ci3 = WA(1, i - 2) * CC(i, k, 2) - WA(1, i - 1) * CC(i - 1, k, 2);
        const float cr4 = WA(2, i - 2) * CC(i - 1, k, 3) + WA(2, i - 1) * CC(i, k, 3);
        const float ci4 = WA(2, i - 2) * CC(i, k, 3) - WA(2, i - 1) * CC(i - 1, k, 3);
        const float tr1 = cr4 + cr2, tr4 = cr4 - cr2;
        const float ti1 = ci2 + ci4, ti4 = ci2 - ci4;
        const float tr2 = CC(i - 1, k, 0) + cr3, tr3 = CC(i - 1, k, 0) - cr3;
        const float ti2 = CC(i, k, 0) + ci3, ti3 = CC(i, k, 0) - ci3;
        CH(i - 1, 0, k) = tr2 + tr1;
        CH(ic - 1, 3, k) = tr2 - tr1;
        CH(i, 0, k) = ti1 + ti2;
        CH(ic, 3, k) = ti1 - ti2;
        CH(i - 1, 2, k) = tr3 + ti4;
        CH(ic - 1, 1, k) = tr3 - ti4;
        CH(i, 2, k) = tr4 + ti3;
        CH(ic, 1, k) = tr4 - ti3;
    }
#undef WA
#undef CH
}

__device__ void radf3(int ido, int l1, const float* cc, float* ch, const float* wa) {
#define CH(a, b, c) ch[(a) + ido * ((b) + 3 * (c))]
#define WA(x, i) wa[(i) + (x) * (ido - 1)]
    for (int k = threadIdx.x; k < l1; k += blockDim.x) {
        const float cr2 = CC(0, k, 1) + CC(0, k, 2);
        CH(0, 0, k) = CC(0, k, 0) + cr2;
        CH(0, 2, k) = kTaui * (CC(0, k, 2) - CC(0, k, 1));
        CH(ido - 1, 1, k) = CC(0, k, 0) + kTaur * cr2;
    }
    if (ido == 1) return;
    const int m = (ido - 1) / 2;
    for (int it = threadIdx.x; it < l1 * m; it += blockDim.x) {
        const int k = it / m, i = 2 + 2 * (it % m), ic = ido - i;
        const float dr2 = WA(0, i - 2) * CC(i - 1, k, 1) + WA(0, i - 1) * CC(i, k, 1);
        const float di2 = WA(0, i - 2) * CC(i, k, 1) - WA(0, i - 1) * CC(i - 1, k, 1);
        const float dr3 = WA(1, i - 2) * CC(i - 1, k, 2) + WA(1, i - 1) * CC(i, k, 2);
        const float di3 = WA(1, i - 2) * CC(i, k, 2) - WA(1, i - 1) * CC(i - 1, k, 2);
        const float cr2 = dr2 + dr3, ci2 = di2 + di3;
        CH(i - 1, 0, k) = CC(i - 1, k, 0) + cr2;
        CH(i, 0, k) = CC(i, k, 0) + ci2;
        const float tr2 = CC(i - 1, k, 0) + kTaur * cr2, ti2 = CC(i, k, 0) + kTaur * ci2;
        const float tr3 = kTaui * (di2 - di3), ti3 = kTaui * (dr3 - dr2);
        CH(i - 1, 2, k) = tr2 + tr3;
        CH(ic - 1, 1, k) = tr2 - tr3;
        CH(i, 2, k) = ti3 + ti2;
        CH(ic, 1, k) = ti3 - ti2;
    }
#undef WA
#undef CH
}

__device__ void radf5(int ido, int l1, const float* cc, float* ch, const float* wa) {
#define CH(a, b, c) ch[(a) + ido * ((b) + 5 * (c))]
#define WA(x, i) wa[(i) + (x) * (ido - 1)]
    for (int k = threadIdx.x; k < l1; k += blockDim.x) {
        const float cr2 = CC(0, k, 4) + CC(0, k, 1), ci5 = CC(0, k, 4) - CC(0, k, 1);
        const float cr3 = CC(0, k, 3) + CC(0, k, 2), ci4 = CC(0, k, 3) - CC(0, k, 2);
        CH(0, 0, k) = CC(0, k, 0) + cr2 + cr3;
        CH(ido - 1, 1, k) = CC(0, k, 0) + kTr11 * cr2 + kTr12 * cr3;
        CH(0, 2, k) = kTi11 * ci5 + kTi12 * ci4;
        CH(ido - 1, 3, k) = CC(0, k, 0) + kTr12 * cr2 + kTr11 * cr3;
        CH(0, 4, k) = kTi12 * ci5 - kTi11 * ci4;
    }
    if (ido == 1) return;
    const int m = (ido - 1) / 2;
    for (int it = threadIdx.x; it < l1 * m; it += blockDim.x) {
        const int k = it / m, i = 2 + 2 * (it % m), ic = ido - i;
        const float dr2 = WA(0, i - 2) * CC(i - 1, k, 1) + WA(0, i - 1) * CC(i, k, 1);
        const float di2 = WA(0, i - 2) * CC(i, k, 1) - WA(0, i - 1) * CC(i - 1, k, 1);
        const float dr3 = WA(1, i - 2) * CC(i - 1, k, 2) + WA(1, i - 1) * CC(i, k, 2);
        const float di3 = WA(1, i - 2) * CC(i, k, 2) - WA(1, i - 1) * CC(i - 1, k, 2);
        const float dr4 = WA(2, i - 2) * CC(i - 1, k, 3) + WA(2, i - 1) * CC(i, k, 3);
        const float di4 = WA(2, i - 2) * CC(i, k, 3) - WA(2, i - 1) * CC(i - 1, k, 3);
        const float dr5 = WA(3, i - 2) * CC(i - 1, k, 4) + WA(3, i - 1) * CC(i, k, 4);
        const float di5 = WA(3, i - 2) * CC(i, k, 4) - WA(3, i - 1) * CC(i - 1, k, 4);
        const float cr2 = dr5 + dr2, ci5 = dr5 - dr2;
        const float ci2 = di2 + di5, cr5 = di2 - di5;
        const float cr3 = dr4 + dr3, ci4 = dr4 - dr3;
        const float ci3 = di3 + di4, cr4 = di3 - di4;
        CH(i - 1, 0, k) = CC(i - 1, k, 0) + cr2 + cr3;
        CH(i, 0, k) = CC(i, k, 0) + ci2 + ci3;
        const float tr2 = CC(i - 1, k, 0) + kTr11 * cr2 + kTr12 * cr3;
        const float ti2 = CC(i, k, 0) + kTr11 * ci2 + kTr12 * ci3;
        const float tr3 = CC(i - 1, k, 0) + kTr12 * cr2 + kTr11 * cr3;
        const float ti3 = CC(i, k, 0) + kTr12 * ci2 + kTr11 * ci3;
        const float tr5 = cr5 * kTi11 + cr4 * kTi12, tr4 = cr5 * kTi12 - cr4 * kTi11;
        const float ti5 = ci5 * kTi11 + ci4 * kTi12, ti4 = ci5 * kTi12 - ci4 * kTi11;
        CH(i - 1, 2, k) = tr2 + tr5;
        CH(ic - 1, 1, k) = tr2 - tr5;
        CH(i, 2, k) = ti5 + ti2;
        CH(ic, 1, k) = ti5 - ti2;
        CH(i - 1, 4, k) = tr3 + tr4;
        CH(ic - 1, 3, k) = tr3 - tr4;
        CH(i, 4, k) = ti4 + ti3;
        CH(ic, 3, k) = ti4 - ti3;
    }
#undef WA
#undef CH
#undef CC
}

// One workgroup per row: the row in LDS, the rfftp passes (factors last to first),
// then the halfcomplex result r0, (r1, i1), ... as complex bins 0..W/2 of the row of F.
__global__ __launch_bounds__(PF_THREADS) void k_pf_rows(const float* __restrict__ in, float2* __restrict__ F, int W,
                                                        PfPlan plan, const float* __restrict__ tw) {
    extern __shared__ float pf_lds[];
    float* p1 = pf_lds;
    float* p2 = pf_lds + W;
    const long row = blockIdx.x;
    for (int i = threadIdx.x; i < W; i += blockDim.x) p1[i] = in[row * W + i];
    __syncthreads();
    int l1 = W;
    for (int k = plan.nf - 1; k >= 0; --k) {
        const int ip = plan.fct[k], ido = W / l1;
        l1 /= ip;
        if (ip == 4)
            radf4(ido, l1, p1, p2, tw + plan.tw[k]);
        else if (ip == 2)
            radf2(ido, l1, p1, p2, tw + plan.tw[k]);
        else if (ip == 3)
            radf3(ido, l1, p1, p2, tw + plan.tw[k]);
        else
            radf5(ido, l1, p1, p2, tw + plan.tw[k]);
        __syncthreads();
        float* t = p1;
        p1 = p2;
        p2 = t;
    }
    float2* out = F + row * W;
    for (int m = threadIdx.x; m <= W / 2; m += blockDim.x) {
        float2 v;
        if (m == 0)
            v = make_float2(p1[0], 0.f);
        else if (m == W / 2)
            v = make_float2(p1[W - 1], 0.f);
        else
            v = make_float2(p1[2 * m - 1], p1[2 * m]);
        out[m] = v;
    }
}

// ------------------------------------------------------------------ columns: cfftp forward
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
// special_mul<fwd>: v * conj(w)
__device__ __forceinline__ float2 cmulc(float2 v, float2 w) {
    return make_float2(v.x * w.x + v.y * w.y, v.y * w.x - v.x * w.y);
}
__device__ __forceinline__ float2 rot90(float2 a) { return make_float2(a.y, -a.x); }  // ROTX90<fwd>
__device__ __forceinline__ float2 rot45(float2 a) { return make_float2(kHsqt2 * (a.x + a.y), kHsqt2 * (a.y - a.x)); }
__device__ __forceinline__ float2 rot135(float2 a) {
    return make_float2(kHsqt2 * (a.y - a.x), kHsqt2 * (-a.x - a.y));
}

// CC(a, b, c) = cc[a + ido*(b + ip*c)], CH(a, b, c) = ch[a + ido*(b + l1*c)],
// WA(x, i) = wa[i - 1 + x*(ido - 1)]; items (k, i), one per thread.
__device__ void cpass(int ip, int ido, int l1, const float2* cc, float2* ch, const float2* wa) {
#define CC(a, b, c) cc[(a) + ido * ((b) + ip * (c))]
#define CH(a, b, c) ch[(a) + ido * ((b) + l1 * (c))]
#define WA(x, i) wa[(i) - 1 + (x) * (ido - 1)]
    for (int it = threadIdx.x; it < l1 * ido; it += blockDim.x) {
        const int k = it / ido, i = it % ido;
        if (ip == 3) {  // pass3<fwd>: tw1r = -1/2, tw1i = -sqrt(3)/2
            const float2 t0 = CC(i, 0, k), t1 = cadd(CC(i, 1, k), CC(i, 2, k)), t2 = csub(CC(i, 1, k), CC(i, 2, k));
            CH(i, k, 0) = cadd(t0, t1);
            const float tw1i = -kTaui;
            const float2 ca = make_float2(t0.x + t1.x * kTaur, t0.y + t1.y * kTaur);
            const float2 cb = make_float2(-(t2.y * tw1i), t2.x * tw1i);
            if (i == 0) {
                CH(i, k, 1) = cadd(ca, cb);
                CH(i, k, 2) = csub(ca, cb);
            } else {
                CH(i, k, 1) = cmulc(cadd(ca, cb), WA(0, i));
                CH(i, k, 2) = cmulc(csub(ca, cb), WA(1, i));
            }
        } else if (ip == 5) {  // pass5<fwd>: tw1i = -sin(2 pi / 5), tw2i = -sin(4 pi / 5)
            const float2 t0 = CC(i, 0, k);
            const float2 t1 = cadd(CC(i, 1, k), CC(i, 4, k)), t4 = csub(CC(i, 1, k), CC(i, 4, k));
            const float2 t2 = cadd(CC(i, 2, k), CC(i, 3, k)), t3 = csub(CC(i, 2, k), CC(i, 3, k));
            CH(i, k, 0) = make_float2(t0.x + t1.x + t2.x, t0.y + t1.y + t2.y);
#pragma unroll
            for (int h = 0; h < 2; ++h) {  // (u1, u2) = (1, 4), then (2, 3)
                const int u1 = h ? 2 : 1, u2 = h ? 3 : 4;
                const float twar = h ? kTr12 : kTr11, twbr = h ? kTr11 : kTr12;
                const float twai = h ? -kTi12 : -kTi11, twbi = h ? kTi11 : -kTi12;
                const float2 ca = make_float2(t0.x + twar * t1.x + twbr * t2.x, t0.y + twar * t1.y + twbr * t2.y);
                const float2 cb = make_float2(-(twai * t4.y + twbi * t3.y), twai * t4.x + twbi * t3.x);
                if (i == 0) {
                    CH(i, k, u1) = cadd(ca, cb);
                    CH(i, k, u2) = csub(ca, cb);
                } else {
                    CH(i, k, u1) = cmulc(cadd(ca, cb), WA(u1 - 1, i));
                    CH(i, k, u2) = cmulc(csub(ca, cb), WA(u2 - 1, i));
                }
            }
        } else if (ip == 2) {
            CH(i, k, 0) = cadd(CC(i, 0, k), CC(i, 1, k));
            const float2 d = csub(CC(i, 0, k), CC(i, 1, k));
            CH(i, k, 1) = i == 0 ? d : cmulc(d, WA(0, i));
        } else if (ip == 4) {
            const float2 t2 = cadd(CC(i, 0, k), CC(i, 2, k)), t1 = csub(CC(i, 0, k), CC(i, 2, k));
            const float2 t3 = cadd(CC(i, 1, k), CC(i, 3, k));
            const float2 t4 = rot90(csub(CC(i, 1, k), CC(i, 3, k)));
            CH(i, k, 0) = cadd(t2, t3);
            if (i == 0) {
                CH(i, k, 2) = csub(t2, t3);
                CH(i, k, 1) = cadd(t1, t4);
                CH(i, k, 3) = csub(t1, t4);
            } else {
                CH(i, k, 1) = cmulc(cadd(t1, t4), WA(0, i));
                CH(i, k, 2) = cmulc(csub(t2, t3), WA(1, i));
                CH(i, k, 3) = cmulc(csub(t1, t4), WA(2, i));
            }
        } else {  // ip == 8
            float2 a1 = cadd(CC(i, 1, k), CC(i, 5, k)), a5 = csub(CC(i, 1, k), CC(i, 5, k));
            float2 a3 = cadd(CC(i, 3, k), CC(i, 7, k)), a7 = csub(CC(i, 3, k), CC(i, 7, k));
            {
                const float2 t = a1;
                a1 = cadd(t, a3);
                a3 = csub(t, a3);
            }
            a3 = rot90(a3);
            a7 = rot90(a7);
            {
                const float2 t = a5;
                a5 = cadd(t, a7);
                a7 = csub(t, a7);
            }
            a5 = rot45(a5);
            a7 = rot135(a7);
            float2 a0 = cadd(CC(i, 0, k), CC(i, 4, k)), a4 = csub(CC(i, 0, k), CC(i, 4, k));
            float2 a2 = cadd(CC(i, 2, k), CC(i, 6, k)), a6 = csub(CC(i, 2, k), CC(i, 6, k));
            {
                const float2 t = a0;
                a0 = cadd(t, a2);
                a2 = csub(t, a2);
            }
            a6 = rot90(a6);
            {
                const float2 t = a4;
                a4 = cadd(t, a6);
                a6 = csub(t, a6);
            }
            CH(i, k, 0) = cadd(a0, a1);
            if (i == 0) {
                CH(i, k, 4) = csub(a0, a1);
                CH(i, k, 2) = cadd(a2, a3);
                CH(i, k, 6) = csub(a2, a3);
                CH(i, k, 1) = cadd(a4, a5);
                CH(i, k, 5) = csub(a4, a5);
                CH(i, k, 3) = cadd(a6, a7);
                CH(i, k, 7) = csub(a6, a7);
            } else {
                CH(i, k, 4) = cmulc(csub(a0, a1), WA(3, i));
                CH(i, k, 2) = cmulc(cadd(a2, a3), WA(1, i));
                CH(i, k, 6) = cmulc(csub(a2, a3), WA(5, i));
                CH(i, k, 1) = cmulc(cadd(a4, a5), WA(0, i));
                CH(i, k, 5) = cmulc(csub(a4, a5), WA(4, i));
                CH(i, k, 3) = cmulc(cadd(a6, a7), WA(2, i));
                CH(i, k, 7) = cmulc(csub(a6, a7), WA(6, i));
            }
        }
    }
#undef WA
#undef CH
#undef CC
}

// One workgroup per (half-spectrum column, image): the column in LDS, the cfftp passes
// (factors first to last), written back in place.
__global__ __launch_bounds__(PF_THREADS) void k_pf_cols(float2* __restrict__ F, int H, int W, PfPlan plan,
                                                        const float2* __restrict__ tw) {
    extern __shared__ float2 pfc_lds[];
    float2* p1 = pfc_lds;
    float2* p2 = pfc_lds + H;
    const int j = blockIdx.x;
    float2* col = F + (long)blockIdx.y * H * W + j;
    for (int i = threadIdx.x; i < H; i += blockDim.x) p1[i] = col[(long)i * W];
    __syncthreads();
    int l1 = 1;
    for (int k = 0; k < plan.nf; ++k) {
        const int ip = plan.fct[k], ido = H / (ip * l1);
        cpass(ip, ido, l1, p1, p2, tw + plan.tw[k]);
        __syncthreads();
        float2* t = p1;
        p1 = p2;
        p2 = t;
        l1 *= ip;
    }
    for (int i = threadIdx.x; i < H; i += blockDim.x) col[(long)i * W] = p1[i];
}

// The other half as conjugate mirrors (c2c_sym_internal's reverse iterator): columns
// W/2+1.. from (H - i, W - j); the lower halves of columns 0 and W/2 from their upper
// halves, and their self-mirrored bins (rows 0, H/2) conjugated in place.
__global__ void k_pf_mirror(float2* __restrict__ F, int H, int W, long n) {
    const long g = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n) return;
    const long hw = (long)H * W, b = g / hw, idx = g - b * hw;
    const int i = (int)(idx / W), j = (int)(idx % W);
    float2* f = F + b * hw;
    if (j > W / 2) {
        const float2 v = f[(long)((H - i) % H) * W + (W - j)];
        f[idx] = make_float2(v.x, -v.y);
    } else if (j == 0 || j == W / 2) {
        if (i > H / 2) {
            const float2 v = f[(long)(H - i) * W + j];
            f[idx] = make_float2(v.x, -v.y);
        } else if (i == 0 || i == H / 2) {
            const float2 v = f[idx];
            f[idx] = make_float2(v.x, -v.y);
        }
    }
}

}  // namespace

void pf_center(const float* img, int nb, long hw, float* sums, float* out, hipStream_t s) {
    const int nchunks = (int)((hw + 8191) / 8192);
    hipLaunchKernelGGL(k_pf_chunk_sums, dim3(nchunks, nb), dim3(64), 0, s, img, hw, nchunks, sums);
    FCD_CHECK_LAUNCH();
    const unsigned gx = (unsigned)std::min<long>(256, (hw + 255) / 256);
    hipLaunchKernelGGL(k_pf_center, dim3(gx, nb), dim3(256), 0, s, img, hw, nchunks, sums, out, (long)nb * hw);
    FCD_CHECK_LAUNCH();
}

void pf_fft2(const float* in, int nb, int H, int W, const PfPlan& rows, const float* rtw, const PfPlan& cols,
             const float2* ctw, float2* F, hipStream_t s) {
    hipLaunchKernelGGL(k_pf_rows, dim3((unsigned)((long)nb * H)), dim3(PF_THREADS), 2 * W * sizeof(float), s, in, F,
                       W, rows, rtw);
    FCD_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_pf_cols, dim3(W / 2 + 1, nb), dim3(PF_THREADS), 2 * H * sizeof(float2), s, F, H, W, cols,
                       ctw);
    FCD_CHECK_LAUNCH();
    const long n = (long)nb * H * W;
    hipLaunchKernelGGL(k_pf_mirror, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, F, H, W, n);
    FCD_CHECK_LAUNCH();
}

int pf_chunk_count(long hw) { return (int)((hw + 8191) / 8192); }

}  // namespace fcdk
