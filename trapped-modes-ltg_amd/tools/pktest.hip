// Checks the packed-FP32 op_sel/neg encodings used by fft_lds.hpp's complex helpers.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
typedef float fv2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ fv2 cm(fv2 a, fv2 b) {
    fv2 t, r;
    asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(a), "v"(b));
    asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]" : "=v"(r) : "v"(a), "v"(b), "v"(t));
    return r;
}
__device__ __forceinline__ fv2 cmc(fv2 a, fv2 b) {
    fv2 t, r;
    asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1] neg_hi:[0,1]" : "=v"(t) : "v"(a), "v"(b));
    asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1]" : "=v"(r) : "v"(a), "v"(b), "v"(t));
    return r;
}
__device__ __forceinline__ fv2 addi(fv2 a, fv2 b) {  // a + i b
    fv2 r;
    asm volatile("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ fv2 subi(fv2 a, fv2 b) {  // a - i b
    fv2 r;
    asm volatile("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__global__ void k(const fv2* a, const fv2* b, fv2* o, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fv2 x = a[i], y = b[i];
    o[4 * i] = cm(x, y); o[4 * i + 1] = cmc(x, y); o[4 * i + 2] = addi(x, y); o[4 * i + 3] = subi(x, y);
}
int main() {
    const int n = 4096;
    fv2 *ha = new fv2[n], *hb = new fv2[n], *ho = new fv2[4 * n];
    for (int i = 0; i < n; ++i) { ha[i] = fv2{sinf(i * 1.3f), cosf(i * 0.7f) * 2}; hb[i] = fv2{cosf(i * 0.11f) - 0.3f, sinf(i * 2.9f)}; }
    fv2 *da, *db, *dout;
    hipMalloc(&da, n * 8); hipMalloc(&db, n * 8); hipMalloc(&dout, 4 * n * 8);
    hipMemcpy(da, ha, n * 8, hipMemcpyHostToDevice); hipMemcpy(db, hb, n * 8, hipMemcpyHostToDevice);
    k<<<n / 256, 256>>>(da, db, dout, n);
    hipMemcpy(ho, dout, 4 * n * 8, hipMemcpyDeviceToHost);
    double e[4] = {0, 0, 0, 0};
    for (int i = 0; i < n; ++i) {
        double ax = ha[i].x, ay = ha[i].y, bx = hb[i].x, by = hb[i].y;
        double r[4][2] = {{ax * bx - ay * by, ax * by + ay * bx}, {ax * bx + ay * by, ay * bx - ax * by}, {ax - by, ay + bx}, {ax + by, ay - bx}};
        for (int j = 0; j < 4; ++j) e[j] = fmax(e[j], fmax(fabs(ho[4 * i + j].x - r[j][0]), fabs(ho[4 * i + j].y - r[j][1])));
    }
    printf("cmul %.3g cmulc %.3g addi %.3g subi %.3g\n", e[0], e[1], e[2], e[3]);
    return (e[0] < 1e-5 && e[1] < 1e-5 && e[2] < 1e-6 && e[3] < 1e-6) ? 0 : 1;
}
