// Displacement solve + spectral height integration on the device:
//   compute_displacement_field   /root/reference/pyfcd/fcd.py:122-138
//   height_gradient = -u / h     /root/reference/pyfcd/fcd.py:32
//   integrate_in_fourier         /root/reference/pyfcd/fourier.py:115-137
//   remove_degeneracy            /root/reference/pyfcd/fourier.py:75-92 (index N/2+1, kept literally)
//
// Everything between the two unwrapped phase maps and the height is linear,
// so it folds into one per-frequency multiplier on their spectra:
//   h_hat = i/k^2 * [(kx*a0 + ky*b0) Phi0 + (kx*a1 + ky*b1) Phi1]
// with (a0, b0, a1, b1) from the carrier frequencies and the effective height
// (host side).  Both maps travel as one complex field
// z = phi0 + i*phi1; Phi0/Phi1 are split from Z(k) and Z(-k).  kx, ky are the
// reference's tables after remove_degeneracy, odd-symmetrised
// (kxe[j] = (kx[j] - kx[-j]) / 2): taking the real part of the reference's
// ifft2 is exactly the inverse of that Hermitian part.
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

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

constexpr double kTwoPi = 6.283185307179586;

static inline unsigned nblk(long n) { return (unsigned)((n + 255) / 256); }

__global__ void k_make_z(const float* __restrict__ w, const int32_t* __restrict__ k, float2* __restrict__ z,
                         long hw, long n) {
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n) return;
    const long b = idx / hw, p = idx % hw;
    const long i0 = (2 * b) * hw + p, i1 = (2 * b + 1) * hw + p;
    float p0 = w[i0], p1 = w[i1];
    if (k) {
        p0 = (float)((double)p0 + kTwoPi * (double)k[i0]);
        p1 = (float)((double)p1 + kTwoPi * (double)k[i1]);
    }
    z[idx] = make_float2(p0, p1);
}

void make_z(const float* w, const int32_t* k, float2* z, int nbatch, int H, int W, hipStream_t s) {
    const long hw = (long)H * W, n = nbatch * hw;
    hipLaunchKernelGGL(k_make_z, dim3(nblk(n)), dim3(256), 0, s, w, k, z, hw, n);
    FCD_CHECK_LAUNCH();
}

__global__ void k_pack_z(const float* __restrict__ gx, const float* __restrict__ gy, float2* __restrict__ z, long n) {
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx < n) z[idx] = make_float2(gx[idx], gy[idx]);
}

void pack_z(const float* gx, const float* gy, float2* z, long n, hipStream_t s) {
    hipLaunchKernelGGL(k_pack_z, dim3(nblk(n)), dim3(256), 0, s, gx, gy, z, n);
    FCD_CHECK_LAUNCH();
}

// tr: Z and Hh column-major per image ([b][q][r], the generic chain's transposed spectra)
__global__ void k_integ_multiply(const float2* __restrict__ Z, float2* __restrict__ Hh, int H, int W, long n,
                                 IntegCoef c, bool tr) {
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n) return;
    const long hw = (long)H * W;
    const long b = idx / hw, p = idx % hw;
    const int r = tr ? (int)(p % H) : (int)(p / W), q = tr ? (int)(p / H) : (int)(p % W);
    const int rm = (H - r) % H, qm = (W - q) % W;
    const float2 z = Z[idx];
    const float2 zm = Z[b * hw + (tr ? (long)qm * H + rm : (long)rm * W + qm)];
    // Phi0 = (Z(k) + conj Z(-k)) / 2 ; Phi1 = (Z(k) - conj Z(-k)) / (2i)
    const float2 f0 = make_float2(0.5f * (z.x + zm.x), 0.5f * (z.y - zm.y));
    const float2 dd = make_float2(z.x - zm.x, z.y + zm.y);
    const float2 f1 = make_float2(0.5f * dd.y, -0.5f * dd.x);
    const float kx = c.kxe[q], ky = c.kye[r];
    float k2 = c.kx2[q] + c.ky2[r];
    if (r == 0 && q == 0) k2 = 1.f;
    const float s = c.norm / k2;
    const float m0 = (kx * c.a0 + ky * c.b0) * s;
    const float m1 = (kx * c.a1 + ky * c.b1) * s;
    // i * (m0*f0 + m1*f1)
    const float re = m0 * f0.x + m1 * f1.x;
    const float im = m0 * f0.y + m1 * f1.y;
    Hh[idx] = make_float2(-im, re);
}

void integ_multiply(const float2* Z, float2* Hh, int nbatch, int H, int W, IntegCoef c, hipStream_t s, bool transposed) {
    const long n = (long)nbatch * H * W;
    hipLaunchKernelGGL(k_integ_multiply, dim3(nblk(n)), dim3(256), 0, s, Z, Hh, H, W, n, c, transposed);
    FCD_CHECK_LAUNCH();
}

__global__ void k_compose_phase(const float* __restrict__ w, const int32_t* __restrict__ k, float* __restrict__ out,
                                long n) {
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx < n) out[idx] = k ? (float)((double)w[idx] + kTwoPi * (double)k[idx]) : w[idx];
}

void compose_phase(const float* w, const int32_t* k, float* out, long n, hipStream_t s) {
    hipLaunchKernelGGL(k_compose_phase, dim3(nblk(n)), dim3(256), 0, s, w, k, out, n);
    FCD_CHECK_LAUNCH();
}

}  // namespace fcdk
