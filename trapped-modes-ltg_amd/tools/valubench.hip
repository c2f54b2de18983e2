// VALU throughput calibration (tuning tool): wave64 v_fma_f32 vs v_pk_fma_f32
// streams, 8 independent chains per lane, at 1..8 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v2f __attribute__((ext_vector_type(2)));
__global__ void k_fma(float* out, int iters, float a) {
    float x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = __builtin_fmaf(x[i], a, 0.5f);
    float s = 0; for (int i = 0; i < 8; ++i) s += x[i];
    if (s == 1.2345f) out[threadIdx.x] = s;
}
__global__ void k_pk(float* out, int iters, float a) {
    v2f x[8];
    for (int i = 0; i < 8; ++i) x[i] = v2f{threadIdx.x * 0.001f + i, (float)i};
    const v2f av = v2f{a, a}, bv = v2f{0.5f, 0.25f};
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = __builtin_elementwise_fma(x[i], av, bv);
    float s = 0; for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
    if (s == 1.2345f) out[threadIdx.x] = s;
}
int main() {
    float* o; (void)hipMalloc(&o, 4096);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    const int iters = 20000;
    for (int wps : {1, 2, 4, 8}) {
        const int blocks = 256 * wps;  // one 256-thread block = 1 wave per SIMD
        for (int pk = 0; pk < 2; ++pk) {
            for (int w = 0; w < 2; ++w) { if (pk) k_pk<<<blocks, 256>>>(o, 100, 1.0001f); else k_fma<<<blocks, 256>>>(o, 100, 1.0001f); }
            (void)hipEventRecord(e0);
            if (pk) k_pk<<<blocks, 256>>>(o, iters, 1.0001f); else k_fma<<<blocks, 256>>>(o, iters, 1.0001f);
            (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
            float ms; (void)hipEventElapsedTime(&ms, e0, e1);
            const double instr_per_simd = (double)iters * 8 * wps;  // per SIMD
            const double flops = (double)blocks * 256 * iters * 8 * 2 * (pk ? 2 : 1);
            printf("waves/SIMD %d %s: %.2f ns per wave-instr per SIMD, %.1f TFLOP/s\n", wps, pk ? "v_pk_fma" : "v_fma   ",
                   ms * 1e6 / instr_per_simd, flops / (ms * 1e-3) / 1e12);
        }
    }
    return 0;
}
