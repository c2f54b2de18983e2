// Kernel micro-benchmark for the band-pruned fast path (tuning tool, not part
// of the product ABI).  Times each stage kernel with HIP events on synthetic
// data shaped like the 1024^2 bench workload: nb frames per launch, a carrier
// pair of radius 51 (the pattern.py board's disks), 103 half-spectrum columns.
//
//   kbench [N=1024] [nb=8] [iters=20]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../csrc/kernels.hpp"
#ifdef FCD_STAMPS
extern "C" int fcd_debug_pr_stamps(unsigned long long* out);
extern "C" int fcd_debug_band_stamps(unsigned long long* out);
#endif

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e = (x);                                                   \
        if (e != hipSuccess) {                                                \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));      \
            std::exit(1);                                                     \
        }                                                                     \
    } while (0)

template <class T>
static T* dalloc(size_t n) {
    T* p = nullptr;
    CK(hipMalloc(&p, n * sizeof(T)));
    CK(hipMemset(p, 0, n * sizeof(T)));
    return p;
}

int main(int argc, char** argv) {
    const int N = argc > 1 ? std::atoi(argv[1]) : 1024;
    const int nb = argc > 2 ? std::atoi(argv[2]) : 8;
    const int iters = argc > 3 ? std::atoi(argv[3]) : 20;
    const int H = N, W = N;
    const long hw = (long)H * W;
    const int R = N / 20;  // disk radius ~ |p0 - p1| / 2 of the 10-px board
    hipStream_t s;
    CK(hipStreamCreate(&s));

    // tables: carrier 0 disk centred at unshifted column R, carrier 1 at W - R (mirror of hc)
    std::vector<int> hc, nouts, colslot(2 * (size_t)W, -1);
    std::vector<int4> outs;
    std::vector<int2> outrows;
    const int NCc = 2 * R + 1;
    for (int j = 0; j < NCc; ++j) {
        colslot[j] = j;                              // carrier 0: uc = j
        colslot[(size_t)W + (W - j) % W] = j;       // carrier 1: uc = -j
    }
    for (int h = 0; h < NCc; ++h) {
        hc.push_back(h);
        nouts.push_back(2);
        outs.push_back(make_int4(0, h, 0, h));
        outs.push_back(make_int4(1, h, h ? 1 : 0, (W - h) % W));
        outs.push_back(make_int4(0, 0, 0, 0));
        outs.push_back(make_int4(0, 0, 0, 0));
        for (int e = 0; e < 2; ++e) outrows.push_back(make_int2(H / 2 - R, H / 2 + R));
        outrows.push_back(make_int2(1, 0));
        outrows.push_back(make_int2(1, 0));
    }
    fcdk::DemodTables T;
    int* d_hc = dalloc<int>(hc.size());
    int* d_nouts = dalloc<int>(nouts.size());
    int4* d_outs = dalloc<int4>(outs.size());
    int2* d_outrows = dalloc<int2>(outrows.size());
    int* d_colslot = dalloc<int>(colslot.size());
    CK(hipMemcpy(d_hc, hc.data(), hc.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_nouts, nouts.data(), nouts.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_outs, outs.data(), outs.size() * 16, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_outrows, outrows.data(), outrows.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_colslot, colslot.data(), colslot.size() * 4, hipMemcpyHostToDevice));
    T.hc = d_hc;
    T.nouts = d_nouts;
    T.outs = d_outs;
    T.outrows = d_outrows;
    T.colslot = d_colslot;
    T.NC = NCc;
    T.NCc[0] = T.NCc[1] = NCc;
    const int NCA = NCc;

    std::vector<float2> twh(N);
    for (int i = 0; i < N; ++i) twh[i] = make_float2(1.f, 0.f);
    float2* tw = dalloc<float2>(N);
    CK(hipMemcpy(tw, twh.data(), N * 8, hipMemcpyHostToDevice));

    std::vector<float> fr(nb * hw);
    for (size_t i = 0; i < fr.size(); ++i) fr[i] = (float)((i * 2654435761u) % 1000) * 0.001f;
    float* frames = dalloc<float>(nb * hw);
    CK(hipMemcpy(frames, fr.data(), fr.size() * 4, hipMemcpyHostToDevice));
    float2* Xb = dalloc<float2>((size_t)nb * H * T.NC);
    float2* Ab = dalloc<float2>((size_t)nb * 2 * H * NCA);
    float* theta = dalloc<float>(2 * hw);
    float* wrapped = dalloc<float>((size_t)nb * 2 * hw);
    CK(hipMemcpy(wrapped, fr.data(), fr.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(wrapped + nb * hw, fr.data(), fr.size() * 4, hipMemcpyHostToDevice));
    int* colk = dalloc<int>((size_t)nb * 2 * H);
    int* res = dalloc<int>((size_t)nb * 2);
    float2* Zt = dalloc<float2>((size_t)nb * hw);
    float2* Ht = dalloc<float2>((size_t)nb * H * (W / 2 + 1));
    const size_t irseam_bytes = fcdk::int_rows_seam_bytes(W, H, nb);  // one region per chain stream (<= 4)
    float2* irseam = dalloc<float2>(4 * irseam_bytes / sizeof(float2));
    float* hout = dalloc<float>((size_t)nb * hw);
    float* ktab = dalloc<float>(2 * (W + H));
    fcdk::IntegCoef coef{ktab, ktab + W, ktab + W + H, ktab + 2 * W + H, 1.f, 0.5f, -0.5f, 1.f, 1e-6f};

    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, double bytes_per_frame, auto fn) {
        for (int i = 0; i < 3; ++i) fn();
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < iters; ++i) fn();
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / iters;
        std::printf("%-22s %9.1f us/launch %8.2f us/frame %8.1f GB/s\n", name, us, us / nb,
                    bytes_per_frame * nb / (us * 1e-6) / 1e9);
    };
    const double f = 4.0 * hw;
    timeit("demod_rows", f + 8.0 * H * T.NC, [&] { fcdk::demod_rows(W, frames, H, nb, T, Xb, tw, s); });
    timeit("demod_cols", 8.0 * H * T.NC + 16.0 * H * NCA, [&] { fcdk::demod_cols(H, Xb, nb, T, Ab, NCA, tw, s); });
    timeit("demod_phase", 16.0 * H * NCA + 8 * f, [&] {
        fcdk::demod_phase(W, Ab, H, nb, NCA, T, theta, wrapped, tw, s);
    });
    {
        int Bw = 16;
        while (Bw < NCc) Bw *= 2;
        std::vector<float2> ones(N, make_float2(1.f, 0.f));
        float2* pre = dalloc<float2>(N);
        float2* ptw = dalloc<float2>(N);
        CK(hipMemcpy(pre, ones.data(), N * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(ptw, ones.data(), N * 8, hipMemcpyHostToDevice));
        if (fcdk::band_supported(W, Bw))
            timeit("band_phase", 16.0 * H * NCA + 8 * f, [&] {
                fcdk::band_phase(W, Bw, false, Ab, H, nb, NCA, NCc, NCc, theta, wrapped, pre, ptw, s);
            });
#ifdef FCD_STAMPS
        if (fcdk::band_supported(W, Bw)) {  // block 0, wave 0 of the last band_phase launch: cycle split
            std::vector<unsigned long long> st(512);
            CK(hipDeviceSynchronize());
            fcd_debug_band_stamps(st.data());
            const int RPW = 4;  // rows per wave per 16-row tile at W = 1024 (4 waves per block)
            const int per_item = 2 + 4 * RPW;
            double stage = 0, cm = 0, ff = 0, ph = 0, gap = 0;
            int n = 0;
            for (int it = 0; (it + 1) * per_item + 1 < 512; ++it, ++n) {
                const unsigned long long* a = st.data() + it * per_item;
                stage += a[1] - a[0];
                for (int r = 0; r < RPW; ++r) {
                    const unsigned long long* b = a + 2 + 4 * r;
                    gap += b[0] - (r ? b[-1] : a[1]);
                    cm += b[1] - b[0];
                    ff += b[2] - b[1];
                    ph += b[3] - b[2];
                }
            }
            std::printf("band stamps (memtime ticks per item, %d items): stage+bar %.0f  row-gap %.0f  cmul %.0f  fft %.0f  phase+store %.0f\n",
                        n, stage / n, gap / n, cm / n, ff / n, ph / n);
        }
#endif
        if (fcdk::phase_rows_supported(W, Bw, H)) {
            float2* ztw = dalloc<float2>(N);
            CK(hipMemcpy(ztw, ones.data(), N * 8, hipMemcpyHostToDevice));
            float* col0 = dalloc<float>((size_t)nb * 2 * H);
            float2* seam = dalloc<float2>((size_t)nb * (H / fcdk::phase_rows_tile(W)) * 2 * W);
            timeit("phase_rows (fused)", 16.0 * H * NCA + 2 * f, [&] {
                fcdk::phase_rows(W, true, Ab, H, nb, NCA, NCc, NCc, theta, pre, ptw, ztw, col0, res, Zt, seam, s);
            });
#ifdef FCD_STAMPS
            {
                std::vector<unsigned long long> st(8 * 16);
                CK(hipDeviceSynchronize());
                fcd_debug_pr_stamps(st.data());
                const char* names[13] = {"loop", "stage+bar", "fetch", "band0", "band1", "unwrap", "bar1",
                                         "census", "bar2", "zfft", "bar3", "writeout", "bar4"};
                for (int w = 0; w < 8; ++w) {
                    printf("wave %d:", w);
                    for (int i = 0; i < 13; ++i) printf(" %s=%llu", names[i], st[w * 16 + i]);
                    printf("\n");
                }
            }
#endif
        }
    }
    timeit("colk", 8.0 * H, [&] { fcdk::unwrap_colk(wrapped, 2 * nb, H, W, colk, s); });
    timeit("int_rows k0", 2 * f + 2 * f, [&] {
        fcdk::int_rows(W, 0, wrapped, colk, nullptr, nullptr, nullptr, H, nb, Zt, tw, nullptr, s);
    });
    timeit("int_rows k1", 2 * f + 2 * f, [&] {
        fcdk::int_rows(W, 1, wrapped, colk, nullptr, nullptr, res, H, nb, Zt, tw, irseam, s);
    });
    timeit("int_cols", 2 * f + 8.0 * H * (W / 2 + 1),
           [&] { fcdk::int_cols(H, Zt, W, nb, coef, Ht, tw, s); });
    timeit("int_c2r", 8.0 * H * (W / 2 + 1) + f, [&] { fcdk::int_c2r(W, Ht, H, nb, hout, tw, s); });

    // whole chain (band demod + unwrap + integration) over nb frames, split into
    // S slices on S streams: how much do kernel boundaries / ramps cost?
    {
        int Bw = 16;
        while (Bw < NCc) Bw *= 2;
        if (!fcdk::band_supported(W, Bw)) return 0;  // 4096: full-length demod only
        std::vector<float2> ones(N, make_float2(1.f, 0.f));
        float2* pre = dalloc<float2>(N);
        float2* ptw = dalloc<float2>(N);
        CK(hipMemcpy(pre, ones.data(), N * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(ptw, ones.data(), N * 8, hipMemcpyHostToDevice));
        hipStream_t ss[4];
        for (auto& x : ss) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
        hipEvent_t fork, join[4];
        CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
        for (auto& x : join) CK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
        for (int S : {1, 2, 4}) {
            if (nb % S) continue;
            const int m = nb / S;
            auto chain = [&](int k, hipStream_t st) {
                const long o = (long)k * m;
                fcdk::demod_rows(W, frames + o * hw, H, m, T, Xb + o * H * T.NC, tw, st);
                fcdk::demod_cols(H, Xb + o * H * T.NC, m, T, Ab + o * 2 * H * NCA, NCA, tw, st);
                fcdk::band_phase(W, Bw, false, Ab + o * 2 * H * NCA, H, m, NCA, NCc, NCc, theta, wrapped + o * 2 * hw,
                                 pre, ptw, st);
                fcdk::unwrap_colk(wrapped + o * 2 * hw, 2 * m, H, W, colk + o * 2 * H, st);
                fcdk::int_rows(W, 1, wrapped + o * 2 * hw, colk + o * 2 * H, nullptr, nullptr, res + 2 * o, H, m,
                               Zt + o * hw, tw, irseam + k * (irseam_bytes / sizeof(float2)), st);
                fcdk::int_cols(H, Zt + o * hw, W, m, coef, Ht + o * H * (W / 2 + 1), tw, st);
                fcdk::int_c2r(W, Ht + o * H * (W / 2 + 1), H, m, hout + o * hw, tw, st);
            };
            char name[64];
            std::snprintf(name, sizeof name, "chain x%d streams", S);
            timeit(name, 0.0, [&] {
                CK(hipEventRecord(fork, s));
                for (int k = 0; k < S; ++k) {
                    CK(hipStreamWaitEvent(ss[k], fork, 0));
                    chain(k, ss[k]);
                    CK(hipEventRecord(join[k], ss[k]));
                }
                for (int k = 0; k < S; ++k) CK(hipStreamWaitEvent(s, join[k], 0));
            });
        }
    }
    return 0;
}
