// Diagnostic: per-phase s_memtime stamps of band_phase (block 0, wave 0), built
// with -DFCD_STAMPS.  stampbench [nb=32]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../csrc/kernels.hpp"
extern "C" int fcd_debug_band_stamps(unsigned long long* out);
template <class T> static T* dalloc(size_t n) { T* p; (void)hipMalloc(&p, n * sizeof(T)); (void)hipMemset(p, 0, n * sizeof(T)); return p; }
int main(int argc, char** argv) {
    const int N = 1024, nb = argc > 1 ? atoi(argv[1]) : 32, NCA = 103, B = 128;
    const long hw = (long)N * N;
    float2* Ab = dalloc<float2>((size_t)nb * 2 * N * NCA);
    float* theta = dalloc<float>(2 * hw);
    float* out = dalloc<float>((size_t)nb * 2 * hw);
    std::vector<float2> ones(N, make_float2(1.f, 0.f));
    float2* pre = dalloc<float2>(N); float2* ptw = dalloc<float2>(N);
    (void)hipMemcpy(pre, ones.data(), N * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(ptw, ones.data(), N * 8, hipMemcpyHostToDevice);
    for (int i = 0; i < 3; ++i) fcdk::band_phase(N, B, false, Ab, N, nb, NCA, NCA, NCA, theta, out, pre, ptw, 0);
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> st(512);
    fcd_debug_band_stamps(st.data());
    for (int i = 1; i < 64 && st[i]; ++i) printf("%d +%llu\n", i, st[i] - st[i - 1]);
    return 0;
}
