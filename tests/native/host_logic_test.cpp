// Driver for the host-side engine logic (trapped-modes-ltg_amd/csrc/host_logic.hpp),
// built with g++ under AddressSanitizer + UBSan by tests/test_host_native.py, which
// feeds it inputs and checks its outputs against the oracle.  Commands (stdin -> stdout):
//   labels    H W n, then n lines "raster_index value"  -> the <= 4 kept blobs' peaks
//   setup     H W square_size nblobs, then nblobs raster indices -> peaks, cf, radius,
//             frequencies, mask counts, per-column disk row ranges of both carriers
//   geometry  H W cf r0 c0 r1 c1 R0 R1 -> mask counts, disk row ranges
//   pfrun     n real f64 rows, then the inputs as %a -> pocketfft.hpp's r2c / forward c2c
//             (the device passes, run on the host) as %a pairs
//   parcopy   bytes -> "ok" when a par_copy of that many bytes is exact
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../trapped-modes-ltg_amd/csrc/host_logic.hpp"

static void print_rows(const std::vector<int>& rows) {
    for (size_t i = 0; i < rows.size(); ++i) std::printf("%d%c", rows[i], i + 1 == rows.size() ? '\n' : ' ');
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    const std::string cmd = argv[1];
    try {
        if (cmd == "labels") {
            int H, W, n;
            if (std::scanf("%d %d %d", &H, &W, &n) != 3) return 3;
            std::vector<int> idx(n);
            std::vector<double> val(n);
            for (int i = 0; i < n; ++i)
                if (std::scanf("%d %lf", &idx[i], &val[i]) != 2) return 3;
            for (const auto& b : fcdh::label_candidates_host(H, W, idx, val)) std::printf("%d %d\n", b.peak / W, b.peak % W);
        } else if (cmd == "setup") {
            int H, W, nb;
            double sq;
            if (std::scanf("%d %d %lf %d", &H, &W, &sq, &nb) != 4) return 3;
            std::vector<fcdh::Blob> blobs(nb);
            for (auto& b : blobs) {
                if (std::scanf("%d", &b.peak) != 1) return 3;
                b.first = b.peak;
                b.value = 0.0;
            }
            fcd_ref_info info;
            std::vector<int> rows;
            fcdh::carriers_from_blobs(H, W, info, rows, blobs, 1.0, sq);
            std::printf("%lld %lld %lld %lld\n%.17g %.17g\n", (long long)info.peaks[0][0], (long long)info.peaks[0][1],
                        (long long)info.peaks[1][0], (long long)info.peaks[1][1], info.calibration_factor, info.radius);
            std::printf("%.17g %.17g %.17g %.17g\n%d %d\n", info.frequencies[0][0], info.frequencies[0][1],
                        info.frequencies[1][0], info.frequencies[1][1], info.mask_count[0], info.mask_count[1]);
            print_rows(rows);
        } else if (cmd == "geometry") {
            int H, W;
            double cf, R[2];
            long pr[2], pc[2];
            if (std::scanf("%d %d %lf %ld %ld %ld %ld %lf %lf", &H, &W, &cf, &pr[0], &pc[0], &pr[1], &pc[1], &R[0], &R[1]) != 9)
                return 3;
            fcd_ref_info info;
            std::memset(&info, 0, sizeof(info));
            std::vector<int> rows;
            fcdh::carrier_geometry(H, W, info, rows, pr, pc, cf, R);
            std::printf("%d %d\n", info.mask_count[0], info.mask_count[1]);
            print_rows(rows);
        } else if (cmd == "pfrun") {
            // n real(1: r2c of rows | 0: forward c2c) f64(0|1) rows, then the input values as %a
            // (real: rows * n; complex: rows * n (re, im) pairs) -> the output (re, im) pairs as %a
            int n, real, f64, rows;
            if (std::scanf("%d %d %d %d", &n, &real, &f64, &rows) != 4) return 3;
            auto run = [&](auto zero) {
                using T = decltype(zero);
                std::vector<T> tab;
                const pf::Plan p = pf::make_plan<T>(n, real != 0, tab);
                std::printf("plan %d %d %d\n", p.blue, p.n2, p.nf);
                const int nin = real ? n : 2 * n, nout = real ? n / 2 + 1 : n;
                std::vector<T> in((size_t)nin);
                std::vector<pf::cx<T>> out((size_t)n);
                char buf[64];
                for (int r = 0; r < rows; ++r) {
                    for (int i = 0; i < nin; ++i) {
                        if (std::scanf("%63s", buf) != 1) throw std::runtime_error("input");
                        in[i] = (T)std::strtod(buf, nullptr);
                    }
                    if (real) {
                        pf::host_r2c<T>(p, tab, in.data(), out.data());
                    } else {
                        for (int i = 0; i < n; ++i) out[i] = pf::mk<T>(in[2 * i], in[2 * i + 1]);
                        pf::host_c2c<T>(p, tab, out.data());
                    }
                    for (int i = 0; i < nout; ++i) std::printf("%a %a\n", (double)out[i].r, (double)out[i].i);
                }
            };
            if (f64) run(0.0);
            else run(0.0f);
        } else if (cmd == "parcopy") {
            long long bytes;
            if (std::scanf("%lld", &bytes) != 1) return 3;
            std::vector<unsigned char> src((size_t)bytes), dst((size_t)bytes + 64, 0xAB);
            std::mt19937 rng(7);
            for (auto& b : src) b = (unsigned char)rng();
            fcdh::par_copy(dst.data(), src.data(), (size_t)bytes);
            const bool ok = (bytes == 0 || std::memcmp(dst.data(), src.data(), (size_t)bytes) == 0) &&
                            dst[(size_t)bytes] == 0xAB;
            std::printf("%s\n", ok ? "ok" : "mismatch");
        } else {
            return 2;
        }
    } catch (const fcdh::FcdError& e) {
        std::printf("error %d %s\n", e.code, e.what());
    }
    return 0;
}
