// Memory-access calibration (tuning tool): streaming copy of 512 MiB with
// 4 / 8 / 16 bytes per lane, and a strided-4B pattern like the FFT kernels'
// natural layouts.  hipcc --offload-arch=gfx950 -O3 membench.hip -o membench
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)
template <class T>
__global__ void copyk(const T* __restrict__ a, T* __restrict__ b, long n) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) b[i] = a[i];
}
// each thread: 8 floats at stride TT (=128) inside a 1024-float row (like RegFFT natural layout)
__global__ void strided(const float* __restrict__ a, float* __restrict__ b, long rows) {
    const int t = threadIdx.x & 127, team = threadIdx.x >> 7;
    for (long r = blockIdx.x * 2L + team; r < rows; r += gridDim.x * 2L) {
        float x[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) x[q] = a[r * 1024 + t + 128 * q];
#pragma unroll
        for (int q = 0; q < 8; ++q) b[r * 1024 + t + 128 * q] = x[q];
    }
}
// write-only streams (the phase kernels' output pattern): plain or non-temporal
template <class T, bool NT>
__global__ void fillk(T* __restrict__ b, long n, T v) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        if constexpr (NT) __builtin_nontemporal_store(v, b + i); else b[i] = v;
    }
}
// the band kernel's store pattern: one wave per 4 KB row, 16 stores of 256 B each
// (lanes permuted inside the 256 B as n = g + 8 t), rows grid-strided over waves
__global__ void rowfill(float* __restrict__ b, long rows) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int n0 = (lane >> 3) + 8 * (lane & 7);
    for (long r = blockIdx.x * 4L + w; r < rows; r += gridDim.x * 4L) {
        float* o = b + r * 1024;
#pragma unroll
        for (int q = 0; q < 16; ++q) __builtin_nontemporal_store(1.f, o + n0 + 64 * q);
    }
}
// IL: the block's 4 waves write 4 consecutive rows (16 KB) interleaved at 256 B
// (store q of wave w -> 256-byte piece 4 q + w); PERM: the kernel's lane permutation
template <bool IL, bool PERM>
__global__ void rowfill2(float* __restrict__ b, long rows) {
    extern __shared__ float lds_pad[];  // dynamic LDS only limits the resident blocks
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int n0 = PERM ? (lane >> 3) + 8 * (lane & 7) : lane;
    if (rows < 0) lds_pad[threadIdx.x] = 0.f;
    for (long r0 = blockIdx.x * 4L; r0 < rows; r0 += gridDim.x * 4L) {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const long o = IL ? r0 * 1024 + (4 * q + w) * 64 : (r0 + w) * 1024 + 64 * q;
            __builtin_nontemporal_store(1.f, b + o + n0);
        }
    }
}
typedef float fv4m __attribute__((ext_vector_type(4)));
int main(int argc, char** argv) {
    if (argc > 1 && argv[1][0] == 'w') {  // write-only bandwidth over 2 GiB (past the 256 MiB MALL)
        const long wb = 2048L << 20;
        float* w;
        CK(hipMalloc(&w, wb));
        hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
        auto runw = [&](const char* name, auto fn) {
            for (int i = 0; i < 2; ++i) fn();
            hipEventRecord(e0); for (int i = 0; i < 5; ++i) fn(); hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            printf("%-28s %8.1f GB/s (write only)\n", name, 1.0 * wb * 5 / (ms * 1e-3) / 1e9);
        };
        for (int g : {2048, 8192}) {
            printf("grid %d x 256\n", g);
            runw("fill 4B plain", [&] { fillk<float, false><<<g, 256>>>(w, wb / 4, 1.f); });
            runw("fill 4B nt", [&] { fillk<float, true><<<g, 256>>>(w, wb / 4, 1.f); });
            runw("fill 16B plain", [&] { fillk<fv4m, false><<<g, 256>>>((fv4m*)w, wb / 16, fv4m{1, 1, 1, 1}); });
            runw("fill 16B nt", [&] { fillk<fv4m, true><<<g, 256>>>((fv4m*)w, wb / 16, fv4m{1, 1, 1, 1}); });
            runw("row pattern 4B nt", [&] { rowfill<<<g, 256>>>(w, wb / 4096); });
            runw("row pattern, no perm", [&] { rowfill2<false, false><<<g, 256>>>(w, wb / 4096); });
            runw("rows interleaved 256B", [&] { rowfill2<true, true><<<g, 256>>>(w, wb / 4096); });
            runw("row pattern, 12 waves/CU", [&] { rowfill2<false, true><<<g, 256, 48 << 10>>>(w, wb / 4096); });
            runw("interleaved, 12 waves/CU", [&] { rowfill2<true, true><<<g, 256, 48 << 10>>>(w, wb / 4096); });
            runw("fill 4B nt, 12 waves/CU", [&] { rowfill2<true, false><<<g, 256, 48 << 10>>>(w, wb / 4096); });
        }
        return 0;
    }
    const long bytes = 512L << 20;
    float *a, *b;
    CK(hipMalloc(&a, bytes)); CK(hipMalloc(&b, bytes));
    CK(hipMemset(a, 0, bytes)); CK(hipMemset(b, 0, bytes));
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    auto run = [&](const char* name, auto fn) {
        for (int i = 0; i < 3; ++i) fn();
        hipEventRecord(e0); for (int i = 0; i < 10; ++i) fn(); hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        printf("%-28s %8.1f GB/s (read+write)\n", name, 2.0 * bytes * 10 / (ms * 1e-3) / 1e9);
    };
    if (argc > 1) {  // PMC calibration (argument "cal"): one launch of each width over 512 MiB (known bytes)
        copyk<float><<<2048, 256>>>(a, b, bytes / 4);
        copyk<float2><<<2048, 256>>>((float2*)a, (float2*)b, bytes / 8);
        copyk<float4><<<2048, 256>>>((float4*)a, (float4*)b, bytes / 16);
        strided<<<2048, 256>>>(a, b, bytes / 4096);
        CK(hipDeviceSynchronize());
        printf("calibration launches done: %ld bytes read and written per launch\n", bytes);
        return 0;
    }
    for (int g : {2048, 8192}) {
        printf("grid %d x 256\n", g);
        run("copy 4B/lane", [&] { copyk<float><<<g, 256>>>(a, b, bytes / 4); });
        run("copy 8B/lane", [&] { copyk<float2><<<g, 256>>>((float2*)a, (float2*)b, bytes / 8); });
        run("copy 16B/lane", [&] { copyk<float4><<<g, 256>>>((float4*)a, (float4*)b, bytes / 16); });
        run("strided 4B (fft layout)", [&] { strided<<<g, 256>>>(a, b, bytes / 4096); });
    }
    return 0;
}
