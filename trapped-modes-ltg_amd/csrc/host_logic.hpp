// Host-side logic of the FCD engine that needs no GPU: the reference's scalar tables
// (wavenumbers, calibration factor, carrier picks, disk raster), the labelling of the
// above-threshold spectrum pixels (fourier.find_peak_locations), the pocketfft plans of
// the exact reference spectrum, and the multi-threaded host copy of the pinned
// pipeline.  Header-only and HIP-free, so tests/native/host_logic_test.cpp builds it
// with g++ under AddressSanitizer / UBSan and checks it against the
// oracle; fcd_engine.cpp includes the same code.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/fcd.h"
#include "pocketfft.hpp"


namespace fcdh {

struct FcdError : std::runtime_error {
    int code;
    FcdError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

constexpr double kPi = 3.141592653589793;  // numpy.pi

// fourier.wavenumber (fourier.py:43-56): fftfreq(n, cf / (2 pi)), optionally fftshifted.
inline std::vector<double> wavenumber(int n, double cf, bool shifted) {
    const double d = cf / (2 * kPi);
    const double val = 1.0 / (n * d);
    std::vector<double> k(n);
    const int npos = (n - 1) / 2 + 1;
    for (int i = 0; i < n; ++i) {
        const long m = i < npos ? i : (long)i - n;
        k[i] = (double)m * val;
    }
    if (shifted) std::rotate(k.begin(), k.begin() + (n - n / 2), k.end());  // fftshift
    return k;
}

struct Blob {
    int first;     // raster index of its first pixel (skimage label order)
    int peak;      // raster index of its max pixel (first in row-major on ties)
    double value;  // |F| at the peak (float32 or float64 spectrum, exact in double)
};


// fourier.find_peak_locations (fourier.py:139-168) on the host, from an image's
// candidate list: the images whose above-threshold set exceeds the device labelling
// kernel's capacity (fcdk::label_peaks).  Returns the 4 dimmest blobs in order.
inline std::vector<Blob> label_candidates_host(int H, int W, const std::vector<int>& idx_in,
                                               const std::vector<double>& val_in) {
    const size_t n = idx_in.size();
    std::vector<size_t> order(n);
    std::iota(order.begin(), order.end(), 0);
    std::sort(order.begin(), order.end(), [&](size_t a, size_t b) { return idx_in[a] < idx_in[b]; });
    std::vector<int> idx(n);
    std::vector<double> val(n);
    for (size_t i = 0; i < n; ++i) {
        idx[i] = idx_in[order[i]];
        val[i] = val_in[order[i]];
    }
    // 8-connected labelling of the sparse set (skimage.measure.label, connectivity 2)
    std::vector<int> parent(n);
    std::iota(parent.begin(), parent.end(), 0);
    auto find = [&](int x) {
        while (parent[x] != x) {
            parent[x] = parent[parent[x]];
            x = parent[x];
        }
        return x;
    };
    auto lookup = [&](int r, int col) -> int {
        if (r < 0 || col < 0 || r >= H || col >= W) return -1;
        const int key = r * W + col;
        auto it = std::lower_bound(idx.begin(), idx.end(), key);
        return (it != idx.end() && *it == key) ? (int)(it - idx.begin()) : -1;
    };
    for (size_t i = 0; i < n; ++i) {
        const int r = idx[i] / W, col = idx[i] % W;
        const int nb[4][2] = {{r - 1, col - 1}, {r - 1, col}, {r - 1, col + 1}, {r, col - 1}};
        for (auto& q : nb) {
            const int j = lookup(q[0], q[1]);
            if (j >= 0) {
                const int a = find((int)i), b = find(j);
                if (a != b) parent[std::max(a, b)] = std::min(a, b);
            }
        }
    }
    // blobs in raster order of their first pixel; per blob the max (first on ties)
    std::vector<Blob> blobs;
    std::vector<int> blob_of(n, -1);
    for (size_t i = 0; i < n; ++i) {
        const int root = find((int)i);
        if (blob_of[root] < 0) {
            blob_of[root] = (int)blobs.size();
            blobs.push_back(Blob{idx[i], idx[i], val[i]});
        } else {
            Blob& b = blobs[blob_of[root]];
            if (val[i] > b.value) {
                b.value = val[i];
                b.peak = idx[i];
            }
        }
    }
    std::stable_sort(blobs.begin(), blobs.end(), [](const Blob& a, const Blob& b) { return a.value < b.value; });
    if (blobs.size() > 4) blobs.resize(4);
    return blobs;
}

// Carrier geometry of both carriers (Carrier.__init__, carriers.py:10-20): peak
// pixels (fftshifted row, col), calibration factor, physical wavenumbers
// (pixel_to_wavenumber, carriers.py:12) and the disk band-pass raster per carrier
// with its own radius (skimage.draw.disk: strict < 1 in f64, clipped to the image,
// carriers.py:17-20).  Sets info's geometry fields and disk_rows_host.
inline void carrier_geometry(int H, int W, fcd_ref_info& info, std::vector<int>& disk_rows_host, const long prow[2],
                             const long pcol[2], double cf, const double R[2]) {
    for (int q = 0; q < 2; ++q) {
        info.peaks[q][0] = prow[q];
        info.peaks[q][1] = pcol[q];
    }
    info.calibration_factor = cf;
    info.radius = R[0];
    const std::vector<double> krc = wavenumber(H, cf, true), kcc = wavenumber(W, cf, true);
    for (int q = 0; q < 2; ++q) {
        info.frequencies[q][0] = krc[info.peaks[q][0]];
        info.frequencies[q][1] = kcc[info.peaks[q][1]];
    }
    // disk raster (skimage.draw.disk -> ellipse, rotation 0), per shifted column the row range
    disk_rows_host.assign((size_t)4 * W, 0);
    for (int q = 0; q < 2; ++q) {
        const double Rq = R[q];
        int* rows = disk_rows_host.data() + (size_t)q * 2 * W;
        for (int j = 0; j < W; ++j) {
            rows[2 * j] = 1;
            rows[2 * j + 1] = 0;
        }
        const long pr = info.peaks[q][0], pc = info.peaks[q][1];
        const long lo_r = std::max<long>((long)std::ceil((double)pr - Rq), 0);
        const long hi_r = std::min<long>((long)std::floor((double)pr + Rq), H - 1);
        const long lo_c = std::max<long>((long)std::ceil((double)pc - Rq), 0);
        const long hi_c = std::min<long>((long)std::floor((double)pc + Rq), W - 1);
        int count = 0;
        for (long sc = lo_c; sc <= hi_c; ++sc) {
            const double cc = (double)(sc - lo_c) - (double)(pc - lo_c);
            const double cq = cc / Rq;
            const double c2 = cq * cq;
            int first = -1, last = -2;
            for (long sr = lo_r; sr <= hi_r; ++sr) {
                const double rr = (double)(sr - lo_r) - (double)(pr - lo_r);
                const double rq = rr / Rq;
                const double d = rq * rq + c2;
                if (d < 1.0) {
                    if (first < 0) first = (int)sr;
                    last = (int)sr;
                    ++count;
                }
            }
            if (first >= 0) {
                rows[2 * sc] = first;
                rows[2 * sc + 1] = last;
            }
        }
        info.mask_count[q] = count;
    }
}

// The rest of fourier.find_peaks + compute_calibration_factor + the carrier disks
// from the 4 dimmest blobs (fourier.py:38-39, fcd.py:53-101): sets info and
// disk_rows_host.
inline void carriers_from_blobs(int H, int W, fcd_ref_info& info, std::vector<int>& disk_rows_host,
                                const std::vector<Blob>& blobs, double thr, double square_size) {
    if (blobs.size() < 1) throw FcdError(FCD_E_NOPEAKS, "find_peaks: no spectral peaks above threshold");

    const std::vector<double> kr = wavenumber(H, 1.0, true), kc = wavenumber(W, 1.0, true);
    auto kvec = [&](int p) { return std::pair<double, double>(kr[p / W], kc[p % W]); };
    // rightmost = min |atan2(k_row, k_col)|; perpendicular = min |k_right . k| (fourier.py:38-39)
    size_t ir = 0;
    double best = INFINITY;
    for (size_t i = 0; i < blobs.size(); ++i) {
        auto k = kvec(blobs[i].peak);
        const double a = std::fabs(std::atan2(k.first, k.second));
        if (a < best) {
            best = a;
            ir = i;
        }
    }
    const auto k0 = kvec(blobs[ir].peak);
    size_t ip = 0;
    best = INFINITY;
    for (size_t i = 0; i < blobs.size(); ++i) {
        auto k = kvec(blobs[i].peak);
        const double d = std::fabs(k0.first * k.first + k0.second * k.second);
        if (d < best) {
            best = d;
            ip = i;
        }
    }
    std::memset(&info, 0, sizeof(info));
    info.n_blobs = (int)blobs.size();
    for (size_t i = 0; i < blobs.size(); ++i) {
        info.blob_peaks[i][0] = blobs[i].peak / W;
        info.blob_peaks[i][1] = blobs[i].peak % W;
    }
    info.threshold = thr;
    const int pk[2] = {blobs[ir].peak, blobs[ip].peak};
    const long prow[2] = {pk[0] / W, pk[1] / W}, pcol[2] = {pk[0] % W, pk[1] % W};
    // calibration factor (fcd.py:85-101): 2*sq / (2*pi / mean(|k_pix|))
    const double ak[4] = {std::fabs(kr[prow[0]]), std::fabs(kc[pcol[0]]), std::fabs(kr[prow[1]]),
                          std::fabs(kc[pcol[1]])};
    const double mean = (((ak[0] + ak[1]) + ak[2]) + ak[3]) / 4.0;
    const double pixel_wavelength = (2 * kPi) / mean;
    const double cf = (2 * square_size) / pixel_wavelength;
    const double dr = (double)(prow[0] - prow[1]);
    const double dc = (double)(pcol[0] - pcol[1]);
    const double radius = std::sqrt(dr * dr + dc * dc) / 2;  // fcd.py:68
    const double R[2] = {radius, radius};
    carrier_geometry(H, W, info, disk_rows_host, prow, pcol, cf, R);
}

inline void par_copy(void* dst, const void* src, size_t bytes) {
    if (bytes == 0) return;  // memcpy of 0 bytes from a null pointer is undefined (UBSan, host_logic_test)
    constexpr size_t kPiece = 8u << 20;
    const int nt = (int)std::min<size_t>(8, (bytes + kPiece - 1) / kPiece);
    if (nt <= 1) {
        std::memcpy(dst, src, bytes);
        return;
    }
    const size_t part = (bytes / nt + 4095) & ~(size_t)4095;
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) {
        const size_t o = part * t;
        if (o >= bytes) break;
        th.emplace_back([=] { std::memcpy((char*)dst + o, (const char*)src + o, std::min(part, bytes - o)); });
    }
    std::memcpy(dst, src, std::min(part, bytes));
    for (auto& x : th) x.join();
}


}  // namespace fcdh
