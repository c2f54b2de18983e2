// Frame ingest on the device: raw camera samples -> float32 frames.
//
// The reference decodes every frame on the host (analyze.load_image,
// analyze.py:25-40: skimage.io.imread(as_gray=True).astype(float32)) and the
// pipeline then reads float32.  Here the raw samples cross PCIe as they are
// stored (1 B/px for 8-bit PNG/BMP, 1.25 B/px for the 10-bit packed TIFFs of
// the high-speed camera, 2 B/px for 16-bit) and are widened to float32 in HBM
// by this kernel, so the host link carries 1/4 .. 1/2 of the float32 bytes.
// Conversion is exact: every sample value is an integer < 2^24.
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#include "../../include/fcd.h"
#include "kernels.hpp"

namespace fcdk {

namespace {

// 8 / 16-bit samples (and float64, rounded to nearest like numpy's astype(float32)): 4
// consecutive samples per thread group of the grid-stride loop (vector stores), the
// n % 4 tail by the first threads.
template <class T>
__global__ __launch_bounds__(256) void k_ingest_int(const T* __restrict__ raw, long n, float* __restrict__ out) {
    const long n4 = n / 4;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
        const T* p = raw + 4 * i;
        float4 v;
        v.x = (float)p[0];
        v.y = (float)p[1];
        v.z = (float)p[2];
        v.w = (float)p[3];
        reinterpret_cast<float4*>(out)[i] = v;
    }
    const long t = (long)blockIdx.x * 256 + threadIdx.x;
    if (t < n - 4 * n4) out[4 * n4 + t] = (float)raw[4 * n4 + t];
}

// 10-bit packed rows whose width is not a multiple of 4: one sample per thread (a sample
// always spans two bytes of its row)
__global__ __launch_bounds__(256) void k_ingest_p10_any(const unsigned char* __restrict__ raw, long n, int W, long pitch,
                                                        float* __restrict__ out) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        const long row = i / W;
        const long bit = 10L * (i - row * W);
        const unsigned char* p = raw + row * pitch + (bit >> 3);
        const unsigned v = ((unsigned)p[0] << 8 | p[1]) >> (6 - (bit & 7));
        out[i] = (float)(v & 1023u);
    }
}

// 10-bit samples packed MSB-first (TIFF BitsPerSample = 10, FillOrder = 1),
// every row starting on a byte boundary: 5 bytes hold 4 samples
//   s0 = b0 << 2 | b1 >> 6,  s1 = (b1 & 63) << 4 | b2 >> 4,
//   s2 = (b2 & 15) << 6 | b3 >> 2,  s3 = (b3 & 3) << 8 | b4.
// Rows of a multiple of 4 samples are W / 4 whole groups (k_ingest_p10_any otherwise).
__global__ __launch_bounds__(256) void k_ingest_p10(const unsigned char* __restrict__ raw, long ngroups, int gpr,
                                                    long pitch, float* __restrict__ out) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < ngroups; i += (long)gridDim.x * 256) {
        const long row = i / gpr;
        const int g = (int)(i - row * gpr);
        const unsigned char* p = raw + row * pitch + 5L * g;
        const unsigned b0 = p[0], b1 = p[1], b2 = p[2], b3 = p[3], b4 = p[4];
        float4 v;
        v.x = (float)((b0 << 2) | (b1 >> 6));
        v.y = (float)(((b1 & 63u) << 4) | (b2 >> 4));
        v.z = (float)(((b2 & 15u) << 6) | (b3 >> 2));
        v.w = (float)(((b3 & 3u) << 8) | b4);
        reinterpret_cast<float4*>(out)[i] = v;
    }
}

unsigned ingest_grid(long items) {
    const long blocks = (items + 255) / 256;
    return (unsigned)(blocks < 8192 ? (blocks > 0 ? blocks : 1) : 8192);
}

}  // namespace

size_t raw_frame_bytes(int format, int H, int W) {
    switch (format) {
        case FCD_FMT_F32: return (size_t)H * W * 4;
        case FCD_FMT_U8: return (size_t)H * W;
        case FCD_FMT_U16: return (size_t)H * W * 2;
        case FCD_FMT_P10: return (size_t)H * (((size_t)W * 10 + 7) / 8);
        default: return 0;
    }
}

void ingest(int format, const void* raw, int nframes, int H, int W, float* out, hipStream_t s) {
    const long px = (long)nframes * H * W;
    if (px == 0) return;
    switch (format) {
        case FCD_FMT_U8:
            hipLaunchKernelGGL(k_ingest_int<unsigned char>, dim3(ingest_grid(px / 4 + 1)), dim3(256), 0, s,
                               static_cast<const unsigned char*>(raw), px, out);
            break;
        case FCD_FMT_U16:
            hipLaunchKernelGGL(k_ingest_int<unsigned short>, dim3(ingest_grid(px / 4 + 1)), dim3(256), 0, s,
                               static_cast<const unsigned short*>(raw), px, out);
            break;
        case FCD_FMT_P10: {
            if (W % 4 != 0) {
                hipLaunchKernelGGL(k_ingest_p10_any, dim3(ingest_grid(px)), dim3(256), 0, s,
                                   static_cast<const unsigned char*>(raw), px, W, ((long)W * 10 + 7) / 8, out);
                break;
            }
            const int gpr = W / 4;
            const long ngroups = (long)nframes * H * gpr;
            hipLaunchKernelGGL(k_ingest_p10, dim3(ingest_grid(ngroups)), dim3(256), 0, s,
                               static_cast<const unsigned char*>(raw), ngroups, gpr, ((long)W * 10 + 7) / 8, out);
            break;
        }
        default: throw std::runtime_error("ingest: unsupported format " + std::to_string(format));
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) throw std::runtime_error(std::string("ingest launch: ") + hipGetErrorString(e));
}

void convert_f64(const double* in, long n, float* out, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_ingest_int<double>, dim3(ingest_grid(n / 4 + 1)), dim3(256), 0, s, in, n, out);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) throw std::runtime_error(std::string("convert launch: ") + hipGetErrorString(e));
}

}  // namespace fcdk
