// Host runtime of the MI355X FCD engine: context, device buffers, the
// per-reference setup and the batched per-frame pipeline behind the C ABI of
// include/fcd.h.  All numerics run in the HIP kernels (kernels_*.hip); the
// host only computes the reference's scalar tables (wavenumbers, calibration
// factor, disk raster) and labels the handful of above-threshold spectrum
// pixels that find_peak_locations turns into carrier peaks.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <numeric>
#include <stdexcept>
#include <string>
#include <exception>
#include <thread>
#include <vector>

#include "../../include/fcd.h"
#include "fft_lds.hpp"
#include "host_logic.hpp"
#include "kernels.hpp"

namespace {

using fcdh::Blob;
using fcdh::FcdError;
using fcdh::kPi;
using fcdh::label_candidates_host;
using fcdh::par_copy;
using fcdh::wavenumber;

thread_local std::string g_last_error;

#define HIPCHK(x)                                                                                  \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) throw FcdError(FCD_E_HIP, std::string(#x ": ") + hipGetErrorString(e_)); \
    } while (0)

// Owning device allocation.
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    void ensure(size_t n) {
        if (n <= bytes) return;
        release();
        HIPCHK(hipMalloc(&p, n));
        bytes = n;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

void upload(void* dst, const void* src, size_t bytes, hipStream_t s) {
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
}

std::vector<float2> twiddles(int n) {
    std::vector<float2> t(n);
    for (int m = 0; m < n; ++m) {
        const double a = -2.0 * kPi * (double)m / (double)n;
        t[m] = make_float2((float)std::cos(a), (float)std::sin(a));
    }
    return t;
}

// Pass-major twiddles of the register FFT (regfft.hpp): the schedule of
// fcdk::Sched<n> (radix E = fft_elems(n) passes, a smaller last one), and for
// each pass p >= 1, k < L_p, r = 1..R_p-1: exp(-2 pi i r k / (L_p R_p)).
std::vector<float2> pass_twiddles(int n, int e = 0) {
    const int E = e ? e : fcdk::fft_elems(n);
    std::vector<float2> t;
    int L = 1, p = 0;
    while (L < n) {
        const int R = std::min(E, n / L);
        if (p > 0)
            for (int k = 0; k < L; ++k)
                for (int r = 1; r < R; ++r) {
                    const double a = -2.0 * kPi * (double)r * (double)k / ((double)L * (double)R);
                    t.push_back(make_float2((float)std::cos(a), (float)std::sin(a)));
                }
        L *= R;
        ++p;
    }
    t.resize(std::max<size_t>(t.size(), (size_t)n), make_float2(0.f, 0.f));  // kernels copy n entries
    return t;
}

// Pass-major twiddles of the group FFT (gfft.hpp, GSched<B>): radix min(16, B/L)
// passes; for each pass p >= 1, k < L_p, r = 1..R_p-1: exp(-2 pi i r k / (L_p R_p)).
std::vector<float2> group_twiddles(int B) {
    std::vector<float2> t;
    int L = 1, p = 0;
    while (L < B) {
        const int R = std::min(16, B / L);
        if (p > 0)
            for (int k = 0; k < L; ++k)
                for (int r = 1; r < R; ++r) {
                    const double a = -2.0 * kPi * (double)r * (double)k / ((double)L * (double)R);
                    t.push_back(make_float2((float)std::cos(a), (float)std::sin(a)));
                }
        L *= R;
        ++p;
    }
    if (t.empty()) t.push_back(make_float2(1.f, 0.f));
    return t;
}

// Pre-twiddles of the band-pruned inverse (kernels_band.hip): lane l of a row
// (group g = l / G, lane t = l % G, G = B / 16) multiplies band slot
// j = t + G q by exp(+2 pi i j g / W).
std::vector<float2> band_pretwiddles(int W, int B) {
    const int G = B / 16, RL = W / 16;
    std::vector<float2> t((size_t)RL * 16);
    for (int l = 0; l < RL; ++l) {
        const int g = l / G, tt = l % G;
        for (int q = 0; q < 16; ++q) {
            const long j = tt + (long)G * q;
            const double a = 2.0 * kPi * (double)((j * g) % W) / (double)W;
            t[(size_t)l * 16 + q] = make_float2((float)std::cos(a), (float)std::sin(a));
        }
    }
    return t;
}

// the smallest frame side fcd_create accepts (any larger one up to kMrMaxLen = 16384, see mr_supported)
constexpr int kMinSide = 16;

int fcd_env_int(const char* name, int dflt) {
    const char* v = std::getenv(name);
    return (v && *v) ? std::atoi(v) : dflt;
}

// Host-pointer pipeline state (fcd_process with host frames, heights only).
struct HostPipe {
    int nb = 0;                 // frames per slot
    size_t in_bytes = 0;        // raw bytes per input slot
    hipStream_t h2d = nullptr, d2h = nullptr;
    void* pin_in[2] = {nullptr, nullptr};
    float* pin_out[2] = {nullptr, nullptr};
    DevBuf dev_raw[2], dev_out[2];
    hipEvent_t ev_h2d[2] = {}, ev_free[2] = {}, ev_comp[2] = {}, ev_d2h[2] = {};
    ~HostPipe() {
        for (int i = 0; i < 2; ++i) {
            if (pin_in[i]) (void)hipHostFree(pin_in[i]);
            if (pin_out[i]) (void)hipHostFree(pin_out[i]);
            for (hipEvent_t e : {ev_h2d[i], ev_free[i], ev_comp[i], ev_d2h[i]})
                if (e) (void)hipEventDestroy(e);
        }
        if (h2d) (void)hipStreamDestroy(h2d);
        if (d2h) (void)hipStreamDestroy(d2h);
    }
};

// Page-locked host buffer that only grows (the census readback of every call).
struct PinBuf {
    void* p = nullptr;
    size_t cap = 0;
    void ensure(size_t n) {
        if (n <= cap) return;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        if (hipHostMalloc(&p, n, hipHostMallocDefault) != hipSuccess) throw std::runtime_error("hipHostMalloc failed");
        cap = n;
    }
    ~PinBuf() {
        if (p) (void)hipHostFree(p);
    }
};

// The exact (MST) unwrap's workspace: Boruvka arrays, component-graph edge records, the
// residue counts and scan offsets of the maps it is handed, the MST slot of each map, the
// copies of maps padded to multiples of 64.  The context holds two, so the two halves of
// an exact-first chunk unwrap side by side (process_impl).
struct MstSpace {
    DevBuf comp, off, rel, cw, ce, bw, be, link, hooks, ids;
    DevBuf rootof, offk, lb0, lb1, lr0, lr1, ll0, cnt, mb0, mb1;  // two-level rounds
    DevBuf cg_ncomp, cg_ecnt, cg_ea, cg_eb, cg_ew, cg_ec, cg_ed, cg_lcol;  // component-graph rounds
    DevBuf slot;                // map -> MST slot (-1: not in it) for k_int_rows2 kmode 3
    DevBuf rescnt, colk;        // residue counts, the scan's column-0 offsets
    DevBuf pad_w, pad_k, pad_ids;  // maps with residues padded to multiples of 64, their k and indices
    size_t cap = 0;
};

}  // namespace

struct fcd_ctx {
    int device = 0, H = 0, W = 0;
    // a side is not a power of two: every per-frame call takes the generic chain on the
    // mixed-radix transforms (kernels_mr.hip), the reference's own sequence of 2-D FFTs
    bool generic = false;
    fcdk::MrPlan mr_row{}, mr_col{};
    DevBuf mr_scratch;  // the mixed-radix column transforms' transposed copy (chunk frames)
    DevBuf gb_tables;   // generic chain's band columns (build_demod_tables)
    DevBuf gk_flag;     // generic chain: per map of a chunk, 1 if its k-field came from the MST
    int gb_NU = 0;      // columns in either carrier's disk
    hipStream_t own = nullptr;
    DevBuf tw_row, tw_col;        // plain tables exp(-2 pi i m / n) (generic LDS FFT kernels)
    DevBuf mr_gs;                 // the generic chain's global-scratch rows (sides / Bluestein M above 8192)
    DevBuf twp_row, twp_col;      // pass-major tables (register FFT kernels)
    DevBuf twp_col16;             // the column table for 16 elements per lane (k_int_cols / k_demod_cols at 1024)

    // reference state
    bool has_ref = false;
    fcd_ref_info info{};
    DevBuf theta;          // float [2][H][W] angle of ifft2(F_ref * mask)
    DevBuf refsig;         // float2 [2][H][W] ifft2(F_ref * mask), unnormalised
    DevBuf disk_rows;      // int [2][2W]
    std::vector<int> disk_rows_host;
    DevBuf integ_tab;      // float kxe[W], kye[H], kx2[W], ky2[H]
    double integ_cf = -1;

    // band-pruned demodulation tables (DemodTables) and the fast path's workspace
    DevBuf dt_hc, dt_outs, dt_outrows, dt_nouts, dt_colslot;
    int NC = 0, NCc[2] = {0, 0}, NCA = 0;
    int fchunk = 1;                  // frames per fast-path chunk (the workspace budget's capacity)
    int ws_nb = 0;                   // frames the fast-path chunk workspace is allocated for (<= fchunk)
    DevBuf Xb, Ab, Zt, Ht, fk, fres; // per-chunk intermediates; fk: k-fields for the fix-up pass
    int band_B = 0;                  // band window of the pruned inverse (0: full-length k_demod_phase)
    int fused_B = 0;                 // band window of the fused kernel (= band_B, or 512 at 4096-point rows)
    DevBuf band_pre, band_ptw, theta_b;  // its pre-twiddles, pass twiddles, reference angle of the band
    DevBuf theta_p;                      // theta_b in the phase kernels' lane-contiguous order
    int band_T = 0;                      // their group transform length (band_B, or 256 folded at 4096)
    bool fused_ok = false;           // k_phase_rows applies (height-only calls)
    bool force_unfused = false;      // FCD_UNFUSED=1: take the unfused chain (A/B measurement)
    int nstreams = 2;                // FCD_STREAMS: device-path chunks split over 1 or 2 streams
    int fused_split = 2;             // ... for the fused chain (default: 2 up to 1024-wide rows, 1 above)
    bool early_census = true;        // FCD_EARLY_CENSUS: device calls read the census back before the integration
    // the two halves' "census copied" events: each half copies its flags to `census` on its
    // own stream as soon as they are final (first_pass_chunk)
    hipEvent_t ev_cen[2] = {nullptr, nullptr};
    hipEvent_t ev_done = nullptr;    // end of the last device call's work on its (caller's) stream
    hipStream_t done_stream = nullptr;  // that stream, while the work may still be running
    bool done_pending = false;
    hipStream_t aux = nullptr;       // the second stream of the two-halves chains and its fork / join events (get_aux)
    hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_join0 = nullptr;
    DevBuf ir_seam;                  // k_int_rows2's seam rows (tile-range edges), one region per stream
    DevBuf ztw, col0, seam;          // its 1024-point group-FFT twiddles; column-0 wrapped values [f][2][H];
                                     // first/last unwrapped rows of every tile [f][H/tile][2][W]
    size_t fres_cap = 0;
    PinBuf census;                   // the census readback, page-locked: one DMA, no staging copy

    // workspace
    int chunk = 1;
    DevBuf spec, work, wrapped, kbuf, colk, rescnt, frames_in, out_h, scalar;
    DevBuf cand_idx, cand_val, pk_small, pk_F, pk_work;  // reference setup: candidates, scalars, spectra
    pf::Plan pf_row{}, pf_col{};      // scipy pocketfft's plans of the exact reference spectrum (float32)
    DevBuf pf_rtw, pf_ctw, pf_sums;   // their tables; numpy's chunk sums
    pf::Plan pf_row64{}, pf_col64{};  // the same for float64 images (FCD_IMG_F64), built on first use
    DevBuf pf_rtw64, pf_ctw64, pf_scratch;
    bool pf64_ready = false;
    DevBuf ref32;                     // a float64 reference rounded to float32 (the per-frame carriers)
    DevBuf fix_raw;  // raw samples of the frames redone by the exact pass
    DevBuf fix_h, fix_res;  // first-pass heights / census of an exact-first call's residue-free frames
    // temporal analysis: staged block, exp table, bins, partial sums, output, window
    DevBuf t_stage, t_tab, t_bins, t_part, t_out, t_win, t_wsum, t_slices;
    DevBuf t_chirp, t_bhat, t_work, t_gpart, t_zo, t_bad;  // the FFT path of the mean spectrum
    HostPipe pipe;
    MstSpace ms[2];  // MST workspaces (the second: the other half of an exact-first chunk)

    // stage timing: 4 events per chunk (start, after demod, after unwrap, after integrate)
    bool profiling = false;
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
    long prof_frames = 0;
    double prof_fix_ms = 0;   // host wall time of the exact fix-up pass (it synchronises)
    bool exact_first = false;  // most frames of the last device call had residues (process_impl)
    long prof_fix_frames = 0;

    hipStream_t pick(void* s) const { return s ? static_cast<hipStream_t>(s) : own; }
    hipEvent_t next_event() {
        if (ev_used == ev_pool.size()) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) throw std::runtime_error("hipEventCreate failed");
            ev_pool.push_back(e);
        }
        return ev_pool[ev_used++];
    }
    long hw() const { return (long)H * W; }
};

namespace {

void ensure_chunk_buffers(fcd_ctx* c) {
    const long hw = c->hw();
    const size_t n = (size_t)c->chunk;
    c->spec.ensure(n * hw * sizeof(float2));
    c->wrapped.ensure(n * 2 * hw * sizeof(float));
    c->colk.ensure(n * 2 * c->H * sizeof(int));
    c->rescnt.ensure(n * 2 * sizeof(int));
}

// The full-transform chain's second plane and k-field staging (the generic chain, and the
// fcd_phases_from_spectrum / fcd_unwrap / fcd_integrate entry points): allocated on first
// use, so the power-of-two fast path never holds them.
void ensure_aux_buffers(fcd_ctx* c) {
    const long hw = c->hw();
    const size_t n = (size_t)c->chunk;
    c->work.ensure(n * hw * sizeof(float2));
    c->kbuf.ensure(n * 2 * hw * sizeof(int32_t));
}

void ensure_mst(fcd_ctx* c, MstSpace& S, int nact, long hw) {
    const size_t nv = (size_t)nact * hw;
    S.ids.ensure(sizeof(int) * 2 * (size_t)std::max(c->chunk, c->fchunk) + 64);
    if (nv <= S.cap) return;
    S.comp.ensure(nv * 4);
    S.off.ensure(nv * 4);
    S.rel.ensure(nv * 8);
    S.cw.ensure(nv * 8);
    S.ce.ensure(nv * 4);
    S.bw.ensure(nv * 8);
    S.be.ensure(nv * 4);
    S.link.ensure(nv * 8);
    S.hooks.ensure((2 + fcdk::kCgRounds) * sizeof(int));  // hooks this round; graph overflow; graph rounds' hooks
    const size_t ne = (size_t)fcdk::mst_cg_edge_capacity((long)nv);
    const size_t nt = (size_t)nact * hw / 1024 + 1;  // tiles (at most one per 1024 pixels)
    S.cg_ncomp.ensure(nt * 4);
    S.cg_lcol.ensure(nt * 64 * 4);  // tile height <= 64
    S.cg_ecnt.ensure(nt * 4);
    for (DevBuf* b : {&S.cg_ea, &S.cg_eb, &S.cg_ec, &S.cg_ed}) b->ensure(ne * 4);
    S.cg_ew.ensure(ne * 8);
    for (DevBuf* b : {&S.rootof, &S.offk, &S.lb0, &S.lb1, &S.lr0, &S.lr1, &S.ll0}) b->ensure(nv * 4);
    S.cnt.ensure((size_t)fcdk::mst_level_counts() * sizeof(int));
    S.mb0.ensure(nv);
    S.mb1.ensure(nv);
    S.cap = nv;
}

fcdk::MstWork mst_work(fcd_ctx* c, MstSpace& S) {
    fcdk::MstWork m;
    m.comp = S.comp.as<int>();
    m.off = S.off.as<int>();
    m.crank = S.comp.as<unsigned char>();
    m.coff = S.off.as<short>();
    m.rel = S.rel.as<double>();
    m.cand_w = S.cw.as<double>();
    m.cand_e = S.ce.as<int>();
    m.best_w = S.bw.as<unsigned long long>();
    m.best_e = S.be.as<int>();
    m.link = S.link.as<unsigned long long>();
    m.nhooks = S.hooks.as<int>();
    m.rootof = S.rootof.as<int>();
    m.offk = S.offk.as<int>();
    m.listB[0] = S.lb0.as<int>();
    m.listB[1] = S.lb1.as<int>();
    m.listR[0] = S.lr0.as<int>();
    m.listR[1] = S.lr1.as<int>();
    m.listL0 = S.ll0.as<int>();
    m.cnt = S.cnt.as<int>();
    m.maskB[0] = S.mb0.as<unsigned char>();
    m.maskB[1] = S.mb1.as<unsigned char>();
    m.cg_ncomp = S.cg_ncomp.as<int>();
    m.cg_lcol = S.cg_lcol.as<unsigned>();
    m.cg_ecnt = S.cg_ecnt.as<int>();
    m.cg_ea = S.cg_ea.as<int>();
    m.cg_eb = S.cg_eb.as<int>();
    m.cg_ew = S.cg_ew.as<unsigned long long>();
    m.cg_ec = S.cg_ec.as<int>();
    m.cg_ed = S.cg_ed.as<int>();
    m.Hr = c->H;
    m.Wr = c->W;
    m.Hs = c->H;
    m.Ws = c->W;
    return m;
}

// Row / column transforms of the generic chain: the power-of-two LDS FFTs of
// kernels_fft.hip, or the mixed-radix ones of kernels_mr.hip for other sides.
void rows_fft(fcd_ctx* c, bool inv, fcdk::RowIn im, fcdk::RowOut om, const void* in, void* out, long nrows, float sub,
              const fcdk::PhaseOut* ph, hipStream_t s) {
    if (c->generic)
        fcdk::mr_rows(c->mr_row, inv, im, om, in, out, nrows, c->H, sub, c->tw_row.as<float2>(), ph, s, c->mr_gs.as<float2>());
    else
        fcdk::row_fft(c->W, inv, im, om, in, out, nrows, c->H, sub, c->tw_row.as<float2>(), ph, s);
}

void cols_fft(fcd_ctx* c, bool inv, float2* data, int nb, hipStream_t s) {
    if (c->generic) {
        if ((size_t)nb * c->hw() * sizeof(float2) > c->mr_scratch.bytes)
            throw FcdError(FCD_E_INTERNAL, "mixed-radix scratch too small");
        fcdk::mr_cols(c->mr_col, c->W, inv, data, nb, c->tw_col.as<float2>(), c->mr_scratch.as<float2>(), s,
                      c->mr_gs.as<float2>());
    } else {
        fcdk::col_fft(c->H, c->W, inv, data, nb, c->tw_col.as<float2>(), s);
    }
}

// 2-D forward FFT of nb real images (row pass from real input) into `out`.
void fft2_real(fcd_ctx* c, const float* in, float2* out, int nb, float sub, hipStream_t s) {
    rows_fft(c, false, fcdk::ROW_IN_REAL, fcdk::ROW_OUT_COMPLEX, in, out, (long)nb * c->H, sub, nullptr, s);
    cols_fft(c, false, out, nb, s);
}

// Wrapped phases of nb spectra (in `spec`) for both carriers, fcd.py:116-118.
void demod_phases(fcd_ctx* c, const float2* spec, int nb, float* wrapped, hipStream_t s) {
    float2* A = c->work.as<float2>();
    for (int car = 0; car < 2; ++car) {
        fcdk::DiskTable t{c->disk_rows.as<int>() + (size_t)car * 2 * c->W};
        fcdk::disk_mask(spec, A, nb, c->H, c->W, t, s);
        cols_fft(c, true, A, nb, s);
        fcdk::PhaseOut ph{c->theta.as<float>() + (size_t)car * c->hw(), wrapped, car};
        rows_fft(c, true, fcdk::ROW_IN_COMPLEX, fcdk::ROW_OUT_PHASE, A, nullptr, (long)nb * c->H, 0.f, &ph, s);
    }
}

// The exact pass builds level-0 components inside 64 x 64 tiles and then runs Boruvka
// rounds on their contracted graph (kernels_unwrap.hip).  FCD_MST_LEVEL (A/B checks):
// 2: the tiles, then rounds over the boundary-pixel lists; 1: one pixel round instead
// of the tiles, then the list rounds; 0: every round at pixel level.
int mst_level() {
    const char* e = std::getenv("FCD_MST_LEVEL");
    return e && e[0] >= '0' && e[0] <= '2' && !e[1] ? e[0] - '0' : 3;
}

// k-fields of nmaps wrapped maps (skimage unwrap_phase, fcd.py:119).  Synchronises.
// all_mst: every map goes through the MST pass without a residue count (the
// exact fix-up of frames already known to carry residues; on a residue-free map
// the MST integration equals the scan, k(0, 0) = 0 in both).
// mk (nullable): when the component-graph MST runs, its maps' k is left to the caller
// through *mk (k_int_rows2 kmode 3, no k-field pass; mk->map_slot null otherwise).
// any_res: the residue counts only as "has residues" (> 0), which lets the count skip
// the rest of a map once it has found one
// H x W: the maps' (padded) size, multiples of 64 for the tile passes; Hr x Wr: the
// frame's own size (the reliabilities' border, MstWork::Hr / Wr).
// frame_ids (the generic chain's copy-free pass, H x W the padded size, Hr x Wr the
// frame's): the maps listed (indices into w and k, both in the frame's own layout) go
// through the tile pass and the component-graph rounds with no padded copies -- the tiles'
// clamped loads replicate the last row / column as the copy would, the k-field is written
// in the frame's layout; returns false, with nothing written, if a tile graph exceeds its
// capacity (the caller then takes the padded copy and the list rounds).
bool unwrap_core(fcd_ctx* c, MstSpace& S, const float* w, int nmaps, int H, int W, int Hr, int Wr, int32_t* k,
                 int* res_host, hipStream_t s, bool all_mst, fcdk::MstK* mk, bool any_res, bool colk_only = false,
                 const std::vector<int>* frame_ids = nullptr) {
    if (mk) mk->map_slot = nullptr;
    const long hw = (long)H * W;
    std::vector<int> active;
    if (frame_ids) {
        active = *frame_ids;
    } else if (all_mst) {
        for (int i = 0; i < nmaps; ++i) active.push_back(i);
    } else {
        S.rescnt.ensure((size_t)nmaps * sizeof(int));
        int* res = S.rescnt.as<int>();
        fcdk::residues(w, nmaps, H, W, res, s, any_res);
        std::vector<int> counts(nmaps);
        HIPCHK(hipMemcpyAsync(counts.data(), res, sizeof(int) * nmaps, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        if (res_host) std::copy(counts.begin(), counts.end(), res_host);
        for (int i = 0; i < nmaps; ++i)
            if (counts[i] > 0) active.push_back(i);
    }
    // the scan unwrap for the residue-free maps (the MST pass overwrites the others);
    // skipped when every map has residues (the fix-up groups of camera frames)
    if (!frame_ids && (int)active.size() < nmaps) {
        S.colk.ensure((size_t)nmaps * H * sizeof(int));
        if (colk_only) fcdk::unwrap_colk(w, nmaps, H, W, S.colk.as<int>(), s);
        else fcdk::unwrap_scan(w, nmaps, H, W, S.colk.as<int>(), k, s);
    }
    if (active.empty()) return true;
    ensure_mst(c, S, (int)active.size(), hw);
    fcdk::MstWork m = mst_work(c, S);
    m.Hr = Hr;
    m.Wr = Wr;
    m.Hs = frame_ids ? Hr : H;
    m.Ws = frame_ids ? Wr : W;
    const int nact = (int)active.size();
    upload(S.ids.p, active.data(), sizeof(int) * nact, s);
    const int max_rounds = 64;
    int rounds = 0;
    // Boruvka halves the component count every round; check convergence every
    // third round (a round after convergence hooks nothing and changes nothing).
    int level = mst_level();
    int tile_h = 0;
    const int tile_w = fcdk::mst_tile_shape(H, W, &tile_h);
    if (frame_ids && !(level == 3 && tile_w > 0)) return false;
    if (level == 3 && tile_w > 0) {
        HIPCHK(hipMemsetAsync(m.nhooks + 1, 0, (1 + fcdk::kCgRounds) * sizeof(int), s));
        fcdk::mst_tile_level0(w, S.ids.as<int>(), nact, H, W, m, s, true);
        bool fits = true;
#ifdef FCD_DIAGNOSTIC
        static const bool cg_dbg = std::getenv("FCD_MST_DEBUG") != nullptr;  // (diagnostic builds only)
#else
        constexpr bool cg_dbg = false;
#endif
        auto cg_dump = [&](int r) {  // diagnostic: components and contracted edges entering round r
            const size_t nt = (size_t)nact * (H / tile_h) * (W / tile_w);
            std::vector<int> nc(nt), ne(nt);
            HIPCHK(hipMemcpyAsync(nc.data(), m.cg_ncomp, nt * 4, hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(ne.data(), m.cg_ecnt, nt * 4, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            long sc = 0, se = 0;
            int mc = 0, me = 0;
            for (size_t t = 0; t < nt; ++t) {
                sc += nc[t];
                se += ne[t];
                mc = std::max(mc, nc[t]);
                me = std::max(me, ne[t]);
            }
            std::fprintf(stderr, "[mst-cg] tiles %zu round %d: level-0 components %ld (max/tile %d), edges %ld (max/tile %d)\n",
                         nt, r, sc, mc, se, me);
        };
        // the first check after FCD_CG_FIRST rounds (camera frames converge in 7-9, and a
        // round of finished tiles costs one load per tile), then every third: each check
        // is a host round trip with the GPU idle
        constexpr int first = 9;  // (rounds < kCgRounds; 6 / 7 / 12 measured no better, r04k)
        for (int step = first; rounds < max_rounds; rounds += step, step = 3) {
            for (int g = 0; g < step; ++g) {
                if (cg_dbg) cg_dump(rounds + g);
                fcdk::mst_cg_round(nact, H, W, m, rounds + g, s);
            }
            // nhooks[1]: a tile graph over its capacity; nhooks[2 + r]: hooks in round r
            const int last = rounds + step - 1;
            int flags[2 + fcdk::kCgRounds] = {};
            HIPCHK(hipMemcpyAsync(flags, m.nhooks, (3 + last) * sizeof(int), hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            if (flags[1]) {
                fits = false;
                break;
            }
            if (flags[2 + last] == 0) break;
        }
        if (fits) {
            if (rounds >= max_rounds) throw FcdError(FCD_E_INTERNAL, "unwrap: Boruvka did not converge");
            if (mk) {
                std::vector<int> slot(nmaps, -1);
                for (int i = 0; i < nact; ++i) slot[active[i]] = i;
                S.slot.ensure(slot.size() * sizeof(int));
                upload(S.slot.p, slot.data(), slot.size() * sizeof(int), s);
                *mk = fcdk::MstK{m.crank, m.coff, m.offk, S.slot.as<int>(), fcdk::mst_cg_geom(H, W)};
                return true;
            }
            fcdk::mst_cg_finalize(S.ids.as<int>(), nact, H, W, m, k, s, frame_ids != nullptr);
            return true;
        }
        if (frame_ids) return false;
        level = 2;  // the boundary-list rounds need no capacity bound
        rounds = 0;
    }
    if (level >= 1) {
        if (level >= 2 && tile_w > 0) {
            // level-0 components from Boruvka inside 32 x 32 tiles (LDS)
            fcdk::mst_tile_level0(w, S.ids.as<int>(), nact, H, W, m, s);
        } else {
            // one pixel round
            fcdk::mst_init(w, S.ids.as<int>(), nact, H, W, m, s);
            fcdk::mst_round(w, S.ids.as<int>(), nact, H, W, m, s, true);
        }
        // then rounds over the boundary / root lists only
        fcdk::mst_level_setup(nact, H, W, m, s);
#ifdef FCD_DIAGNOSTIC
        static const bool dbg = std::getenv("FCD_MST_DEBUG") != nullptr;
#else
        constexpr bool dbg = false;
#endif
        auto dump = [&](int r) {  // diagnostic: list sizes (B, R) entering round r
            std::vector<int> cnt((size_t)fcdk::mst_level_counts());
            HIPCHK(hipMemcpyAsync(cnt.data(), m.cnt, cnt.size() * 4, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            const size_t nb = cnt.size() / 5;
            long tot[5] = {0, 0, 0, 0, 0};
            for (int l = 0; l < 5; ++l)
                for (size_t g = 0; g < nb; ++g) tot[l] += cnt[l * nb + g];
            std::fprintf(stderr, "[mst] nv %ld round %d: B %ld R %ld L0 %ld\n", (long)nact * hw, r,
                         tot[r & 1], tot[2 + (r & 1)], tot[4]);
        };
        for (; rounds < max_rounds; rounds += 3) {
            for (int g = 0; g < 3; ++g) {
                if (dbg) dump(rounds + g);
                fcdk::mst_level_round(w, S.ids.as<int>(), nact, H, W, m, rounds + g, s);
            }
            int hooks = 0;
            HIPCHK(hipMemcpyAsync(&hooks, m.nhooks, sizeof(int), hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            if (hooks == 0) break;
        }
        if (rounds >= max_rounds) throw FcdError(FCD_E_INTERNAL, "unwrap: Boruvka did not converge");
        fcdk::mst_level_finalize(S.ids.as<int>(), nact, H, W, m, k, s);
        return true;
    }
    fcdk::mst_init(w, S.ids.as<int>(), nact, H, W, m, s);
    for (; rounds < max_rounds; rounds += 3) {
        for (int g = 0; g < 3; ++g)
            fcdk::mst_round(w, S.ids.as<int>(), nact, H, W, m, s, rounds + g == 0);
        int hooks = 0;
        HIPCHK(hipMemcpyAsync(&hooks, m.nhooks, sizeof(int), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        if (hooks == 0) break;
    }
    if (rounds == max_rounds) throw FcdError(FCD_E_INTERNAL, "unwrap: Boruvka did not converge");
    fcdk::mst_finalize(S.ids.as<int>(), nact, H, W, m, k, s);
    return true;
}

// k-fields of nmaps wrapped maps of the context's frame size (unwrap_core).  A frame whose
// sides are not multiples of 64: the residue census and the scan of the residue-free maps
// run on the maps themselves; the maps with residues go to the MST tiles in copies padded
// by replicating their last row and column (kernels_unwrap.hip pad_maps: same residues,
// same k on the frame's pixels).
// colk_only: the residue-free maps get only their column-0 offsets (ms[space].colk), no
// k-field: the generic chain's z rows scan them themselves (PhaseOut::kflag).
void unwrap_maps(fcd_ctx* c, const float* w, int nmaps, int32_t* k, int* res_host, hipStream_t s,
                 bool all_mst = false, fcdk::MstK* mk = nullptr, bool any_res = false, int space = 0,
                 bool colk_only = false) {
    const int H = c->H, W = c->W;
    MstSpace& S = c->ms[space];
    if (H % 64 == 0 && W % 64 == 0) {
        unwrap_core(c, S, w, nmaps, H, W, H, W, k, res_host, s, all_mst, mk, any_res, colk_only);
        return;
    }
    if (mk) mk->map_slot = nullptr;
    std::vector<int> active;
    if (all_mst) {
        for (int i = 0; i < nmaps; ++i) active.push_back(i);
    } else {
        S.rescnt.ensure((size_t)nmaps * sizeof(int));
        int* res = S.rescnt.as<int>();
        fcdk::residues(w, nmaps, H, W, res, s, any_res);
        std::vector<int> counts(nmaps);
        HIPCHK(hipMemcpyAsync(counts.data(), res, sizeof(int) * nmaps, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        if (res_host) std::copy(counts.begin(), counts.end(), res_host);
        for (int i = 0; i < nmaps; ++i)
            if (counts[i] > 0) active.push_back(i);
        if ((int)active.size() < nmaps) {
            S.colk.ensure((size_t)nmaps * H * sizeof(int));
            if (colk_only) fcdk::unwrap_colk(w, nmaps, H, W, S.colk.as<int>(), s);
            else fcdk::unwrap_scan(w, nmaps, H, W, S.colk.as<int>(), k, s);
        }
    }
    if (active.empty()) return;
    const int nact = (int)active.size();
    const int Hp = (H + 63) / 64 * 64, Wp = (W + 63) / 64 * 64;
    // the tile pass and the component-graph rounds straight on the maps (no padded copy of
    // the phases, the k-field written in the frame's layout: 1080 x 1920 with residues,
    // pad_maps + unpad_k were ~0.53 ms of a 32-frame chunk's ~7 ms); the padded copy below
    // only for the other MST levels or a tile graph over its capacity
    if (unwrap_core(c, S, w, nmaps, Hp, Wp, H, W, k, nullptr, s, true, nullptr, false, false, &active)) {
        HIPCHK(hipStreamSynchronize(s));  // (active, the ids' host copy, dies here)
        return;
    }
    const size_t np = (size_t)nact * Hp * Wp;
    S.pad_w.ensure(np * sizeof(float));
    S.pad_k.ensure(np * sizeof(int32_t));
    S.pad_ids.ensure((size_t)nact * sizeof(int));
    upload(S.pad_ids.p, active.data(), (size_t)nact * sizeof(int), s);
    fcdk::pad_maps(w, nact, H, W, Hp, Wp, S.pad_w.as<float>(), s, S.pad_ids.as<int>());
    unwrap_core(c, S, S.pad_w.as<float>(), nact, Hp, Wp, H, W, S.pad_k.as<int32_t>(), nullptr, s, true, nullptr, false);
    fcdk::unpad_k(S.pad_k.as<int32_t>(), nact, Hp, Wp, H, W, k, s, S.pad_ids.as<int>());
    HIPCHK(hipStreamSynchronize(s));  // (active, the ids' host copy, dies here)
}

// Integration tables for calibration factor cf (fourier.py:128-131, 75-92).
void ensure_integ_tables(fcd_ctx* c, double cf, hipStream_t s) {
    if (c->integ_cf == cf) return;
    const int H = c->H, W = c->W;
    std::vector<double> kx = wavenumber(W, cf, false), ky = wavenumber(H, cf, false);
    std::vector<double> kxm = kx, kym = ky;
    if (W % 2 == 0) kxm[W / 2 + 1] = 0;  // remove_degeneracy, literally N/2+1 (fourier.py:88-92)
    if (H % 2 == 0) kym[H / 2 + 1] = 0;
    std::vector<float> tab(2 * (size_t)(W + H));
    float* kxe = tab.data();
    float* kye = kxe + W;
    float* kx2 = kye + H;
    float* ky2 = kx2 + W;
    for (int j = 0; j < W; ++j) {
        kxe[j] = (float)((kxm[j] - kxm[(W - j) % W]) / 2);
        kx2[j] = (float)(kx[j] * kx[j]);
    }
    for (int i = 0; i < H; ++i) {
        kye[i] = (float)((kym[i] - kym[(H - i) % H]) / 2);
        ky2[i] = (float)(ky[i] * ky[i]);
    }
    c->integ_tab.ensure(tab.size() * sizeof(float));
    upload(c->integ_tab.p, tab.data(), tab.size() * sizeof(float), s);
    HIPCHK(hipStreamSynchronize(s));  // tab is a host temporary
    c->integ_cf = cf;
}

fcdk::IntegCoef integ_coef(fcd_ctx* c, double a0, double b0, double a1, double b1) {
    fcdk::IntegCoef k;
    const float* t = c->integ_tab.as<float>();
    k.kxe = t;
    k.kye = t + c->W;
    k.kx2 = t + c->W + c->H;
    k.ky2 = t + 2 * c->W + c->H;
    k.a0 = (float)a0;
    k.b0 = (float)b0;
    k.a1 = (float)a1;
    k.b1 = (float)b1;
    k.norm = (float)(1.0 / ((double)c->H * (double)c->W));
    return k;
}

// The generic chain with its spectra kept transposed between the forward and the inverse
// column passes: kernels_mr.hip's column pass is a transpose, row transforms of the
// columns and a transpose back, so a transposed spectrum saves half the transposes (10 ->
// 5 per chunk).  Same transforms, same arithmetic as fft2_real / demod_phases / integrate_z.
// Buffers: spec (row layout), mr_scratch (transposed spectrum), work.
// Forward 2-D FFT of the frames kept at the band columns only (the union of both
// carriers' disk columns, NU of W): rows, gather-transpose of those columns, their column
// transforms: specT [nb][NU][H].  The demodulation reads no other column of the spectrum.
void generic_fft2_t(fcd_ctx* c, const float* in, int nb, float2* specT, hipStream_t s) {
    float2* tmp = c->spec.as<float2>();
    const int NU = c->gb_NU;
    fcdk::PhaseOut bo{};  // two rows per transform, their band columns only stored: [nb][H][NU]
    bo.bslot = c->gb_tables.as<int>() + NU + 2 * (c->NCc[0] + c->NCc[1]) + 2 * (size_t)c->W;
    bo.bnc = NU;
    fcdk::mr_rows(c->mr_row, false, fcdk::ROW_IN_REAL2, fcdk::ROW_OUT_BAND2, in, tmp, (long)nb * c->H, c->H, 0.f,
                  c->tw_row.as<float2>(), &bo, s, c->mr_gs.as<float2>());
    fcdk::mr_transpose(tmp, specT, nb, c->H, NU, s);
    fcdk::mr_rows(c->mr_col, false, fcdk::ROW_IN_COMPLEX, fcdk::ROW_OUT_COMPLEX, specT, specT, (long)nb * c->gb_NU, c->gb_NU,
                  0.f, c->tw_col.as<float2>(), nullptr, s, c->mr_gs.as<float2>());
}

// Per carrier: the disk-masked band columns [nb][NCc][H], their inverse column
// transforms, then the inverse row transforms with the phase, whose loads gather the band
// columns of their row (the other columns of ifft_cols(D * mask) are zero).
void generic_demod_t(fcd_ctx* c, const float2* specT, int nb, float* wrapped, hipStream_t s) {
    float2* AT = c->work.as<float2>();
    const int* g = c->gb_tables.as<int>();
    const int NU = c->gb_NU, n0 = c->NCc[0], n1 = c->NCc[1];
    const int* cols[2] = {g + NU, g + NU + n0};
    const int* uslot[2] = {g + NU + n0 + n1, g + NU + 2 * n0 + n1};
    const int* colslot = g + NU + 2 * (n0 + n1);
    for (int car = 0; car < 2; ++car) {
        const int nc = c->NCc[car];
        fcdk::DiskTable t{c->disk_rows.as<int>() + (size_t)car * 2 * c->W};
        fcdk::disk_band_t(specT, AT, nb, c->H, c->W, NU, cols[car], uslot[car], nc, t, s);
        if (nc > 0)
            fcdk::mr_rows(c->mr_col, true, fcdk::ROW_IN_COMPLEX, fcdk::ROW_OUT_COMPLEX, AT, AT, (long)nb * nc, nc, 0.f,
                          c->tw_col.as<float2>(), nullptr, s, c->mr_gs.as<float2>());
        fcdk::PhaseOut ph{c->theta.as<float>() + (size_t)car * c->hw(), wrapped, car};
        // the inverse rows gather their band columns themselves (scattering the band into
        // zero-filled rows first measured 7.68 k vs 8.18 k frames/s at 1024 x 1280, r04w)
        ph.bslot = colslot + (size_t)car * c->W;
        ph.bnc = nc;
        fcdk::mr_rows(c->mr_row, true, fcdk::ROW_IN_BAND, fcdk::ROW_OUT_PHASE, AT, nullptr, (long)nb * c->H, c->H, 0.f,
                      c->tw_row.as<float2>(), &ph, s, c->mr_gs.as<float2>());
    }
}

// z of the maps (w + 2 pi k, make_z's arithmetic) built in the row transform's load
// kflag / colk (nullable, device): per map, its k-field in kf (MST) or its scan in the z rows
void generic_integrate_t(fcd_ctx* c, int nb, const float* w, const int32_t* kf, const fcdk::IntegCoef& k, float* h_out,
                         hipStream_t s, const int* kflag = nullptr, const int* colk = nullptr) {
    float2* Z = c->spec.as<float2>();
    const float2* twc = c->tw_col.as<float2>();
    fcdk::PhaseOut zin{};
    zin.kin = kf;
    zin.kflag = kflag;
    zin.colk = colk;
    fcdk::mr_rows(c->mr_row, false, fcdk::ROW_IN_Z, fcdk::ROW_OUT_COMPLEX, w, Z, (long)nb * c->H, c->H, 0.f,
                  c->tw_row.as<float2>(), &zin, s, c->mr_gs.as<float2>());
    if (fcdk::mr_int_cols_supported(c->mr_col)) {  // the column pairs in place
        fcdk::mr_int_cols(c->mr_col, Z, nb, c->W, twc, k, s);
    } else {  // (a prime factor of H above 7 but <= 61) transposed, the spectrum kept transposed between the passes
        float2* ZT = c->mr_scratch.as<float2>();
        float2* HT = c->work.as<float2>();
        fcdk::mr_transpose(Z, ZT, nb, c->H, c->W, s);
        fcdk::mr_rows(c->mr_col, false, fcdk::ROW_IN_COMPLEX, fcdk::ROW_OUT_COMPLEX, ZT, ZT, (long)nb * c->W, c->W, 0.f,
                      twc, nullptr, s, c->mr_gs.as<float2>());
        fcdk::integ_multiply(ZT, HT, nb, c->H, c->W, k, s, true);
        fcdk::mr_rows(c->mr_col, true, fcdk::ROW_IN_COMPLEX, fcdk::ROW_OUT_COMPLEX, HT, HT, (long)nb * c->W, c->W, 0.f,
                      twc, nullptr, s, c->mr_gs.as<float2>());
        fcdk::mr_transpose(HT, Z, nb, c->W, c->H, s);
    }
    // two Hermitian rows per inverse transform
    fcdk::mr_rows(c->mr_row, true, fcdk::ROW_IN_COMPLEX2, fcdk::ROW_OUT_REAL2, Z, h_out, (long)nb * c->H, c->H, 0.f,
                  c->tw_row.as<float2>(), nullptr, s, c->mr_gs.as<float2>());
}

// h = real(ifft2(multiplier * fft2(z)))  for nb fields z (in c->spec).
void integrate_z(fcd_ctx* c, int nb, const fcdk::IntegCoef& k, float* h_out, hipStream_t s) {
    float2* Z = c->spec.as<float2>();
    float2* Hh = c->work.as<float2>();
    rows_fft(c, false, fcdk::ROW_IN_COMPLEX, fcdk::ROW_OUT_COMPLEX, Z, Z, (long)nb * c->H, 0.f, nullptr, s);
    if (c->generic && fcdk::mr_int_cols_supported(c->mr_col)) {  // the column pairs in place (kernels_mr.hip)
        fcdk::mr_int_cols(c->mr_col, Z, nb, c->W, c->tw_col.as<float2>(), k, s);
        rows_fft(c, true, fcdk::ROW_IN_COMPLEX, fcdk::ROW_OUT_REAL, Z, h_out, (long)nb * c->H, 0.f, nullptr, s);
        return;
    }
    cols_fft(c, false, Z, nb, s);
    fcdk::integ_multiply(Z, Hh, nb, c->H, c->W, k, s);
    cols_fft(c, true, Hh, nb, s);
    rows_fft(c, true, fcdk::ROW_IN_COMPLEX, fcdk::ROW_OUT_REAL, Hh, h_out, (long)nb * c->H, 0.f, nullptr, s);
}

// The column kernels' pass-major tables (their element counts may differ from fft_elems)
const float2* col_tw(fcd_ctx* c, int elems) {
    if (elems == fcdk::fft_elems(c->H)) return c->twp_col.as<float2>();
    if (elems != 16 || !c->twp_col16.p) throw FcdError(FCD_E_INTERNAL, "no pass table for this element count");
    return c->twp_col16.as<float2>();
}
const float2* ic_tw(fcd_ctx* c) { return col_tw(c, fcdk::int_cols_elems(c->H)); }
const float2* dc_tw(fcd_ctx* c) { return col_tw(c, fcdk::demod_cols_elems(c->H)); }

// A device call on a caller stream may return with its integration kernels still queued
// on that stream (early census readback).  A later device call on the same stream is
// ordered after them on the device: the stream waits on the call's end event, which also
// covers a stream the caller destroyed and whose handle the runtime handed out again.
// Any other entry point (another stream, host pointers, the context's own stream, state
// changes such as a new reference) first waits for them on the host, since it may touch
// the workspace and tables those kernels read.
void settle(fcd_ctx* c, hipStream_t same = nullptr) {
    if (!c->done_pending) return;
    if (same && same == c->done_stream) {
        HIPCHK(hipStreamWaitEvent(same, c->ev_done, 0));
        return;
    }
    HIPCHK(hipEventSynchronize(c->ev_done));
    c->done_pending = false;
}

void check_ctx(fcd_ctx* c, bool settle_pending = true) {
    if (!c) throw FcdError(FCD_E_INVALID, "null context");
    HIPCHK(hipSetDevice(c->device));
    if (settle_pending) settle(c);
}

// The fast path's chunk workspace (Xb, Ab, Zt, Ht, the k-field, seams, staging) for nb
// frames, nb <= fchunk, grown on demand: a one-frame compute_height_map pins one frame's
// workspace (tens of MB at 1024^2), not the 16 GiB throughput budget a 256-frame batch
// uses.  Sizes follow the current reference's band tables.
void ensure_fast_ws(fcd_ctx* c, int nb) {
    nb = std::max(1, std::min(nb, c->fchunk));
    if (nb <= c->ws_nb) return;
    // growing frees buffers the integration of an earlier asynchronous device call may
    // still be reading on the caller's stream (early census, settle())
    if (c->done_pending) {
        HIPCHK(hipEventSynchronize(c->ev_done));
        c->done_pending = false;
    }
    const long H = c->H, W = c->W, hw = c->hw();
    const size_t n = (size_t)nb, nw = std::max(n, (size_t)c->chunk);
    c->Xb.ensure(n * H * c->NC * sizeof(float2));
    c->Ab.ensure(n * 2 * H * c->NCA * sizeof(float2));
    c->Zt.ensure(n * hw * sizeof(float2));
    c->Ht.ensure(n * H * (W / 2 + 1) * sizeof(float2));
    c->wrapped.ensure(nw * 2 * hw * sizeof(float));
    c->colk.ensure(nw * 2 * H * sizeof(int));
    c->fk.ensure(n * 2 * hw * sizeof(int32_t));
    c->col0.ensure(n * 2 * (size_t)H * sizeof(float));
    if (c->fused_ok) c->seam.ensure(n * (size_t)(H / fcdk::phase_rows_tile(W)) * 2 * W * sizeof(float2));
    c->ir_seam.ensure(2 * fcdk::int_rows_seam_bytes(W, H, nb));
    c->rescnt.ensure(nw * 2 * sizeof(int));
    c->ws_nb = nb;
}

// Band-pruned demodulation tables: which unshifted columns each carrier disk
// covers, the half-spectrum column each one is read from (directly, or as the
// conjugate mirror of column W - uc of the real input's spectrum), and the
// per-carrier column slots of the inverse-transform planes.
void build_demod_tables(fcd_ctx* c, hipStream_t s) {
    const int H = c->H, W = c->W;
    std::vector<int> colslot(2 * (size_t)W, -1);
    struct Out { int carrier, cslot, mirror, uc, lo, hi; };
    std::vector<std::vector<Out>> per_hc(W / 2 + 1);
    for (int q = 0; q < 2; ++q) {
        const int* rows = c->disk_rows_host.data() + (size_t)q * 2 * W;
        int n = 0;
        for (int sc = 0; sc < W; ++sc) {
            if (rows[2 * sc] > rows[2 * sc + 1]) continue;
            const int uc = (sc + W - W / 2) % W;  // ifftshift: shifted column -> unshifted (any W)
            colslot[(size_t)q * W + uc] = n;
            const int hc = uc <= W / 2 ? uc : W - uc;
            per_hc[hc].push_back(Out{q, n, uc > W / 2 ? 1 : 0, uc, rows[2 * sc], rows[2 * sc + 1]});
            ++n;
        }
        c->NCc[q] = n;
    }
    (void)H;
    std::vector<int> hc_list, nouts;
    std::vector<int4> outs;
    std::vector<int2> outrows;
    for (int hc = 0; hc <= W / 2; ++hc) {
        if (per_hc[hc].empty()) continue;
        if (per_hc[hc].size() > 4) throw FcdError(FCD_E_INTERNAL, "demod tables: > 4 outputs per column");
        hc_list.push_back(hc);
        nouts.push_back((int)per_hc[hc].size());
        for (int e = 0; e < 4; ++e) {
            if (e < (int)per_hc[hc].size()) {
                const Out& o = per_hc[hc][e];
                outs.push_back(make_int4(o.carrier, o.cslot, o.mirror, o.uc));
                outrows.push_back(make_int2(o.lo, o.hi));
            } else {
                outs.push_back(make_int4(0, 0, 0, 0));
                outrows.push_back(make_int2(1, 0));
            }
        }
    }
    c->NC = (int)hc_list.size();
    c->NCA = std::max(std::max(c->NCc[0], c->NCc[1]), 1);
    if (c->NC == 0) throw FcdError(FCD_E_NOPEAKS, "carrier disks are empty");
    if (c->generic) {  // no band-pruned fast path; the generic chain's column subsets
        c->band_B = c->fused_B = 0;
        c->fused_ok = false;
        // [NU union columns][carrier 0 columns][carrier 1 columns][their union slots (2)]
        // [colslot: 2 x W] (generic_demod_t) [union slot of each column: W] (generic_fft2_t)
        std::vector<int> uslot_of(W, -1), ucols, cols[2], uslot[2];
        for (int uc = 0; uc < W; ++uc)
            if (colslot[uc] >= 0 || colslot[(size_t)W + uc] >= 0) {
                uslot_of[uc] = (int)ucols.size();
                ucols.push_back(uc);
            }
        for (int q = 0; q < 2; ++q) {
            cols[q].assign(c->NCc[q], 0);
            uslot[q].assign(c->NCc[q], 0);
            for (int uc = 0; uc < W; ++uc) {
                const int n = colslot[(size_t)q * W + uc];
                if (n < 0) continue;
                cols[q][n] = uc;
                uslot[q][n] = uslot_of[uc];
            }
        }
        c->gb_NU = (int)ucols.size();
        std::vector<int> gb(ucols);
        for (int q = 0; q < 2; ++q) gb.insert(gb.end(), cols[q].begin(), cols[q].end());
        for (int q = 0; q < 2; ++q) gb.insert(gb.end(), uslot[q].begin(), uslot[q].end());
        gb.insert(gb.end(), colslot.begin(), colslot.end());
        gb.insert(gb.end(), uslot_of.begin(), uslot_of.end());
        c->gb_tables.ensure(gb.size() * sizeof(int));
        upload(c->gb_tables.p, gb.data(), gb.size() * sizeof(int), s);
        return;
    }
    c->dt_hc.ensure(hc_list.size() * sizeof(int));
    c->dt_nouts.ensure(nouts.size() * sizeof(int));
    c->dt_outs.ensure(outs.size() * sizeof(int4));
    c->dt_outrows.ensure(outrows.size() * sizeof(int2));
    c->dt_colslot.ensure(colslot.size() * sizeof(int));
    upload(c->dt_hc.p, hc_list.data(), hc_list.size() * sizeof(int), s);
    upload(c->dt_nouts.p, nouts.data(), nouts.size() * sizeof(int), s);
    upload(c->dt_outs.p, outs.data(), outs.size() * sizeof(int4), s);
    upload(c->dt_outrows.p, outrows.data(), outrows.size() * sizeof(int2), s);
    upload(c->dt_colslot.p, colslot.data(), colslot.size() * sizeof(int), s);
    // band-pruned inverse: smallest power-of-two window >= 16 holding either carrier's band
    int B = 16;
    while (B < std::max(c->NCc[0], c->NCc[1])) B *= 2;
    c->band_B = fcdk::band_supported(W, B) ? B : 0;
    // the fused wide kernel has its own band transform: at 4096-point rows it takes the
    // 512-bin window the unfused band kernel does not (that path keeps k_demod_phase)
    c->fused_B = (c->band_B || W == 4096) && fcdk::phase_rows_supported(W, B, H) ? B : 0;
    std::vector<float2> pre, ptw;
    // the group transforms' length: the window, or at 4096-point rows its halves folded
    // per group (kernels_phase_rows_wide.hip / kernels_band.hip FOLD)
    c->band_T = c->band_B ? c->band_B : (c->fused_B ? fcdk::phase_rows_wide_bt(W) : 0);
    if (c->band_B || c->fused_B) {
        pre = band_pretwiddles(W, c->band_T);
        ptw = group_twiddles(c->band_T);
        c->band_pre.ensure(pre.size() * sizeof(float2));
        c->band_ptw.ensure(ptw.size() * sizeof(float2));
        upload(c->band_pre.p, pre.data(), pre.size() * sizeof(float2), s);
        upload(c->band_ptw.p, ptw.data(), ptw.size() * sizeof(float2), s);
        c->theta_b.ensure(2 * (size_t)c->hw() * sizeof(float));
        c->theta_p.ensure(2 * (size_t)c->hw() * sizeof(float));
    }
    c->fused_ok = c->fused_B != 0;
    std::vector<float2> ztw;
    if (c->fused_ok) {
        ztw = group_twiddles(std::min(W, 1024));
        // wider rows: the join of the W / 1024 wave-local 1024-point transforms
        // (kernels_phase_rows_wide.hip), w^(h k) = exp(-2 pi i h k / W), h = 1 .. W/1024 - 1
        for (int h = 1; h < W / 1024; ++h)
            for (int k = 0; k < 1024; ++k) {
                const double a = -2.0 * kPi * (double)h * (double)k / (double)W;
                ztw.push_back(make_float2((float)std::cos(a), (float)std::sin(a)));
            }
        c->ztw.ensure(ztw.size() * sizeof(float2));
        upload(c->ztw.p, ztw.data(), ztw.size() * sizeof(float2), s);
    }
    HIPCHK(hipStreamSynchronize(s));  // host vectors die here
    // workspace per frame: Xb + Ab + wrapped + Zt + Ht + k (fix-up path)
    const long hw = c->hw();
    const long per_frame = 8L * H * c->NC + 16L * H * c->NCA + 8L * hw + 8L * hw + 8L * H * (W / 2 + 1) + 8L * hw;
    // frames per launch: large launches amortise every kernel's tail wave; at
    // 1024^2 (bench.py, 256 frames) 8 / 32 / 128 / 256 frames per launch gave
    // 50.5k / 63.5k / 68.1k / 68.9k frames/s.  16 GiB of workspace by default
    // (of 288 GB HBM): 256 frames at 1024^2, 128 at 2048^2, 32 at 4096^2 (8 GiB, 16 frames
    // at 4096^2: c5 3.40 k -> 3.49 k; 24 GiB measured 3.43 k, r05zd / r05ze).
    // (round 6, 4096-point rows: 32 GiB, 64 frames per launch: c5 3.75 k -> 3.90 k frames/s,
    // fused stage 130 -> 122 us/frame; 16 frames 3.82 k, 47 frames 3.79 k, r06 ck / ck2.  At
    // 2048^2 256 frames per launch gave +2 % frames/s but the demod group's roofline 0.32 ->
    // 0.31, so 2048-point rows keep 16 GiB)
    const long budget = (long)fcd_env_int("FCD_CHUNK_MB", W >= 4096 ? 32768 : 16384) << 20;
    c->fchunk = (int)std::max(1L, std::min((long)fcd_env_int("FCD_CHUNK_MAX", 256), budget / per_frame));
    // the workspace itself is allocated per call, for the frames the call launches at once
    // (ensure_fast_ws): the reference's own setup below needs one frame's
    c->ws_nb = 0;
    c->ms[0].cap = c->ms[1].cap = 0;  // re-size the MST workspaces for the new chunk on next use
    ensure_fast_ws(c, 1);
}

fcdk::DemodTables demod_tables(fcd_ctx* c) {
    fcdk::DemodTables t;
    t.hc = c->dt_hc.as<int>();
    t.outs = c->dt_outs.as<int4>();
    t.outrows = c->dt_outrows.as<int2>();
    t.nouts = c->dt_nouts.as<int>();
    t.colslot = c->dt_colslot.as<int>();
    t.NC = c->NC;
    t.NCc[0] = c->NCc[0];
    t.NCc[1] = c->NCc[1];
    return t;
}

// The second stream of the two-halves chains (fused and exact-first) and the fork / join
// events, created on first use.  One stream for both: every stream a context adds shifts the
// runtime's round-robin dealing of default-priority streams over GPU_MAX_HW_QUEUES (4)
// hardware queues, and a second stream that lands on the caller's queue serialises the
// halves (a separate exact-chain stream did so under tools/fixup_bench.py: 10.5 k -> 8.6 k
// camera frames/s, r06z; at the highest priority its half ran ahead of the caller's, r06 ax).
hipStream_t get_aux(fcd_ctx* c) {
    if (!c->aux) {
        HIPCHK(hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&c->ev_join0, hipEventDisableTiming));
    }
    return c->aux;
}

// Fast path for nb frames (device pointer): band-pruned demod -> wrapped (c->wrapped).
// fo: first workspace frame (as first_pass_chunk).
void fast_demod(fcd_ctx* c, const float* frames, int nb, hipStream_t s, int fo = 0) {
    const fcdk::DemodTables T = demod_tables(c);
    const long H = c->H;
    float2* Xb = c->Xb.as<float2>() + fo * H * c->NC;
    float2* Ab = c->Ab.as<float2>() + fo * 2 * H * c->NCA;
    float* wrapped = c->wrapped.as<float>() + fo * 2 * c->hw();
    fcdk::demod_rows(c->W, frames, c->H, nb, T, Xb, c->twp_row.as<float2>(), s);
    fcdk::demod_cols(c->H, Xb, nb, T, Ab, c->NCA, dc_tw(c), s);
    // band-pruned inverse: band_B up to 2048-point rows; at 4096-point rows the fused
    // kernel's 512-bin window (its REF mode made theta_b) as two 256-bin halves folded per
    // group (band_phase_fold)
    if (c->band_B)
        fcdk::band_phase(c->W, c->band_B, false, Ab, c->H, nb, c->NCA, c->NCc[0], c->NCc[1], c->theta_p.as<float>(),
                         wrapped, c->band_pre.as<float2>(), c->band_ptw.as<float2>(), s);
    else if (c->fused_B == 512 && c->band_T == 256 && fcd_env_int("FCD_WIDE_BAND", 1))
        fcdk::band_phase_fold(c->W, Ab, c->H, nb, c->NCA, c->NCc[0], c->NCc[1], c->theta_p.as<float>(), wrapped,
                              c->band_pre.as<float2>(), c->band_ptw.as<float2>(), s);
    else
        fcdk::demod_phase(c->W, Ab, c->H, nb, c->NCA, T, c->theta.as<float>(), wrapped, c->twp_row.as<float2>(), s);
}

// Reference angle of the band-pruned inverse: the same band pipeline run on
// the reference image, angle(y_ref) (kernels_band.hip REF mode).
void band_reference(fcd_ctx* c, const float* dref, hipStream_t s) {
    if (!c->band_B && !c->fused_B) return;
    const fcdk::DemodTables T = demod_tables(c);
    fcdk::demod_rows(c->W, dref, c->H, 1, T, c->Xb.as<float2>(), c->twp_row.as<float2>(), s);
    fcdk::demod_cols(c->H, c->Xb.as<float2>(), 1, T, c->Ab.as<float2>(), c->NCA, dc_tw(c), s);
    if (c->band_B)
        fcdk::band_phase(c->W, c->band_B, true, c->Ab.as<float2>(), c->H, 1, c->NCA, c->NCc[0], c->NCc[1], nullptr,
                         c->theta_b.as<float>(), c->band_pre.as<float2>(), c->band_ptw.as<float2>(), s);
    else  // 4096-point rows: the fused kernel's own band transform in its REF mode
        fcdk::phase_rows_wide_ref(c->W, c->Ab.as<float2>(), c->H, c->NCA, c->NCc[0], c->NCc[1],
                                  c->band_pre.as<float2>(), c->band_ptw.as<float2>(), c->theta_b.as<float>(), s);
    fcdk::band_theta_lanes(c->W, c->band_T, c->theta_b.as<float>(), 2 * c->H, c->theta_p.as<float>(), s);
}

// Everything the per-frame path needs from the reference once c->info and
// c->disk_rows_host hold the carrier geometry: the disk tables, the band-pruned
// demodulation tables, and per carrier q the reference signal ifft2(fft2(ref_q) *
// mask_q) (Carrier._ccsgn, carriers.py:22-24, kept as its angle theta and as the
// band kernels' theta_b / theta_p).  Carrier q's signal comes from image dref[q]
// (both usually the same reference; distinct Carrier objects may carry distinct
// ones).  Synchronises.
void reference_state(fcd_ctx* c, const float* dref0, const float* dref1, hipStream_t s) {
    const long hw = c->hw();
    c->disk_rows.ensure(c->disk_rows_host.size() * sizeof(int));
    upload(c->disk_rows.p, c->disk_rows_host.data(), c->disk_rows_host.size() * sizeof(int), s);
    build_demod_tables(c, s);
    c->refsig.ensure(2 * hw * sizeof(float2));
    c->theta.ensure(2 * hw * sizeof(float));
    float2* F = c->spec.as<float2>();
    const float* drefs[2] = {dref0, dref1};
    const int passes = dref1 == dref0 ? 1 : 2;
    DevBuf keep;  // carrier 0's planes from pass 0 (theta, theta_p, refsig) when the images differ
    for (int pass = 0; pass < passes; ++pass) {
        const float* dref = drefs[pass];
        band_reference(c, dref, s);
        fft2_real(c, dref, F, 1, 0.f, s);
        for (int q = 0; q < 2; ++q) {
            float2* R = c->refsig.as<float2>() + q * hw;
            fcdk::DiskTable t{c->disk_rows.as<int>() + (size_t)q * 2 * c->W};
            fcdk::disk_mask(F, R, 1, c->H, c->W, t, s);
            cols_fft(c, true, R, 1, s);
            rows_fft(c, true, fcdk::ROW_IN_COMPLEX, fcdk::ROW_OUT_COMPLEX, R, R, c->H, 0.f, nullptr, s);
            fcdk::angle(R, c->theta.as<float>() + q * hw, hw, s);
        }
        const size_t tb = (size_t)hw * sizeof(float), rb = (size_t)hw * sizeof(float2);
        const bool band = c->band_B != 0 || c->fused_B != 0;
        if (passes == 2 && pass == 0) {
            keep.ensure(2 * tb + rb + (band ? 2 * tb : 0));
            char* k = static_cast<char*>(keep.p);
            HIPCHK(hipMemcpyAsync(k, c->theta.p, tb, hipMemcpyDeviceToDevice, s));
            HIPCHK(hipMemcpyAsync(k + tb, c->refsig.p, rb, hipMemcpyDeviceToDevice, s));
            if (band) {
                HIPCHK(hipMemcpyAsync(k + tb + rb, c->theta_b.p, tb, hipMemcpyDeviceToDevice, s));
                HIPCHK(hipMemcpyAsync(k + 2 * tb + rb, c->theta_p.p, tb, hipMemcpyDeviceToDevice, s));
            }
        } else if (passes == 2) {
            const char* k = static_cast<const char*>(keep.p);
            HIPCHK(hipMemcpyAsync(c->theta.p, k, tb, hipMemcpyDeviceToDevice, s));
            HIPCHK(hipMemcpyAsync(c->refsig.p, k + tb, rb, hipMemcpyDeviceToDevice, s));
            if (band) {
                HIPCHK(hipMemcpyAsync(c->theta_b.p, k + tb + rb, tb, hipMemcpyDeviceToDevice, s));
                HIPCHK(hipMemcpyAsync(c->theta_p.p, k + 2 * tb + rb, tb, hipMemcpyDeviceToDevice, s));
            }
        }
    }
    HIPCHK(hipStreamSynchronize(s));
}

// The float64 plans (FCD_IMG_F64 images), built on first use.
void ensure_pf64(fcd_ctx* c) {
    if (c->pf64_ready) return;
    std::vector<double> rtw, ctw;
    c->pf_row64 = pf::make_plan<double>(c->W, true, rtw);
    c->pf_col64 = pf::make_plan<double>(c->H, false, ctw);
    c->pf_rtw64.ensure(rtw.size() * sizeof(double));
    c->pf_ctw64.ensure(ctw.size() * sizeof(double));
    HIPCHK(hipMemcpy(c->pf_rtw64.p, rtw.data(), rtw.size() * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->pf_ctw64.p, ctw.data(), ctw.size() * sizeof(double), hipMemcpyHostToDevice));
    c->pf64_ready = true;
}

// scipy.fft.fft2 of nb device-resident real images (float32 -> complex64, float64 ->
// complex128) with the reference's own rounding (kernels_pocketfft.hip).
void exact_fft2(fcd_ctx* c, const void* in, bool f64, int nb, void* F, hipStream_t s) {
    if (f64) ensure_pf64(c);
    const pf::Plan& rp = f64 ? c->pf_row64 : c->pf_row;
    const pf::Plan& cp = f64 ? c->pf_col64 : c->pf_col;
    c->pf_scratch.ensure(std::max<size_t>(fcdk::pf_scratch_bytes(rp, cp, f64), 16));
    fcdk::pf_fft2(in, f64, nb, c->H, c->W, rp, f64 ? c->pf_rtw64.p : c->pf_rtw.p, cp, f64 ? c->pf_ctw64.p : c->pf_ctw.p,
                  F, c->pf_scratch.p, s);
}

// fourier.find_peaks + compute_calibration_factor + the carrier disks for nb
// device-resident images (fcd.py:53-101, fourier.py:7-41), every image-sized stage
// batched on the device in the image's precision: numpy's mean and centring, scipy's
// fft2 (kernels_pocketfft.hip), |F| * highpass and its maximum, the above-threshold
// candidates (any number: every pixel has a slot), and for float32 spectra the
// 8-connected labelling and the 4-blob pick (kernels_fft.hip); the host finishes each
// image from its <= 4 peaks.  Images whose candidates exceed the device labelling's
// capacity (4096), and float64 spectra, are labelled on the host from their candidate
// list (host_logic.hpp).  c->info and c->disk_rows_host end up describing the last image;
// infos[i] (nullable) gets each.
int find_peaks_batch_max(const fcd_ctx* c, bool f64) {
    const long es = f64 ? 8 : 4;
    const long per = c->hw() * (2 * es + 2 * es + 4 + es);  // spectrum, centred + |F|, candidates
    return (int)std::max(1L, (512L << 20) / per);
}

void find_peaks_batch(fcd_ctx* c, const void* dimgs, bool f64, int nb, double square_size, fcd_ref_info* infos,
                      hipStream_t s) {
    const long hw = c->hw();
    const int H = c->H, W = c->W;
    if (nb <= 0) return;
    const size_t es = f64 ? sizeof(double) : sizeof(float);
    const long cap = hw;  // every pixel may be above the threshold (fourier.py:152)
    c->pk_F.ensure((size_t)nb * hw * 2 * es);
    c->pk_work.ensure((size_t)nb * hw * 2 * es);
    char* centered = static_cast<char*>(c->pk_work.p);
    char* mag = centered + (size_t)nb * hw * es;
    c->pk_small.ensure((size_t)nb * (8 + 4 + 32) + (size_t)(H + W) * 8 + 64);
    unsigned long long* maxbits = c->pk_small.as<unsigned long long>();
    double* ktab = reinterpret_cast<double*>(maxbits + nb);
    int* counts = reinterpret_cast<int*>(ktab + H + W);
    int* res = counts + nb;
    const std::vector<double> krs = wavenumber(H, 1.0, true), kcs = wavenumber(W, 1.0, true);
    upload(ktab, krs.data(), H * sizeof(double), s);
    upload(ktab + H, kcs.data(), W * sizeof(double), s);
    c->cand_idx.ensure((size_t)nb * cap * sizeof(int));
    c->cand_val.ensure((size_t)nb * cap * es);
    const double kmin = 4 * kPi / (double)std::min(H, W);  // fourier.py:22
    // image - np.mean(image) and scipy's fft2 with the reference's own rounding
    // (kernels_pocketfft.hip): exact ties between carrier blobs break as they do there
    c->pf_sums.ensure((size_t)nb * fcdk::pf_chunk_count(hw) * es);
    fcdk::pf_center(dimgs, f64, nb, hw, c->pf_sums.p, centered, s);
    exact_fft2(c, centered, f64, nb, c->pk_F.p, s);
    fcdk::spectrum_candidates_b(c->pk_F.p, f64, nb, H, W, ktab, ktab + H, kmin * kmin, mag, maxbits, counts,
                                c->cand_idx.as<int>(), c->cand_val.p, cap, s);
    if (!f64) fcdk::label_peaks(counts, c->cand_idx.as<int>(), c->cand_val.as<float>(), cap, nb, H, W, res, s);
    std::vector<unsigned long long> mb(nb);
    std::vector<int> rs((size_t)nb * 8, 0), cnt(nb);
    HIPCHK(hipMemcpyAsync(mb.data(), maxbits, nb * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(cnt.data(), counts, nb * sizeof(int), hipMemcpyDeviceToHost, s));
    if (!f64) HIPCHK(hipMemcpyAsync(rs.data(), res, rs.size() * sizeof(int), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    const bool host_label = std::getenv("FCD_HOST_LABEL") != nullptr;  // A/B: the host labelling for all
    for (int b = 0; b < nb; ++b) {
        double mx;
        if (f64) {
            std::memcpy(&mx, &mb[b], 8);
        } else {
            float m32;
            const unsigned u = (unsigned)mb[b];
            std::memcpy(&m32, &u, 4);
            mx = m32;
        }
        const int* r = rs.data() + (size_t)b * 8;
        std::vector<Blob> blobs;
        if (f64 || r[0] != 0 || host_label) {
            const int n = cnt[b];  // <= cap = H * W
            std::vector<int> cidx(n);
            std::vector<double> cval(n);
            if (n) {
                HIPCHK(hipMemcpy(cidx.data(), c->cand_idx.as<int>() + (size_t)b * cap, n * sizeof(int),
                                 hipMemcpyDeviceToHost));
                if (f64) {
                    HIPCHK(hipMemcpy(cval.data(), c->cand_val.as<double>() + (size_t)b * cap, n * sizeof(double),
                                     hipMemcpyDeviceToHost));
                } else {
                    std::vector<float> v32(n);
                    HIPCHK(hipMemcpy(v32.data(), c->cand_val.as<float>() + (size_t)b * cap, n * sizeof(float),
                                     hipMemcpyDeviceToHost));
                    std::copy(v32.begin(), v32.end(), cval.begin());
                }
            }
            blobs = label_candidates_host(H, W, cidx, cval);
        } else {
            for (int e = 0; e < r[2]; ++e) blobs.push_back(Blob{r[3 + e], r[3 + e], 0.0});
        }
        fcdh::carriers_from_blobs(H, W, c->info, c->disk_rows_host, blobs, 0.5 * mx, square_size);
        if (infos) infos[b] = c->info;
    }
}

}  // namespace

// ====================================================================== C ABI
#define FCD_API extern "C" __attribute__((visibility("default")))

#define FCD_TRY(...)                                                            \
    try {                                                                       \
        __VA_ARGS__;                                                            \
        return FCD_OK;                                                          \
    } catch (const FcdError& e) {                                               \
        g_last_error = e.what();                                                \
        return e.code;                                                          \
    } catch (const std::exception& e) {                                         \
        g_last_error = e.what();                                                \
        return FCD_E_INTERNAL;                                                  \
    } catch (...) {                                                             \
        g_last_error = "unknown error";                                         \
        return FCD_E_INTERNAL;                                                  \
    }

FCD_API int fcd_abi_version(void) { return FCD_ABI_VERSION; }

FCD_API const char* fcd_last_error(void) { return g_last_error.c_str(); }

FCD_API int fcd_create(int device, int rows, int cols, fcd_ctx** out) {
    FCD_TRY({
        if (!out) throw FcdError(FCD_E_INVALID, "out is null");
        *out = nullptr;
        const bool pow2 = fcdk::fft_size_supported(rows) && fcdk::fft_size_supported(cols);
        if (!pow2 && !(rows >= kMinSide && cols >= kMinSide && fcdk::mr_supported(rows) && fcdk::mr_supported(cols)))
            throw FcdError(FCD_E_UNSUPPORTED, "frame sides must be in [" + std::to_string(kMinSide) + ", " +
                                                  std::to_string(fcdk::kMrMaxLen) + "], got " + std::to_string(rows) +
                                                  "x" + std::to_string(cols));
        int ndev = 0;
        HIPCHK(hipGetDeviceCount(&ndev));
        if (device < 0 || device >= ndev) throw FcdError(FCD_E_INVALID, "bad device ordinal");
        HIPCHK(hipSetDevice(device));
        std::unique_ptr<fcd_ctx> c(new fcd_ctx());
        c->device = device;
        c->force_unfused = fcd_env_int("FCD_UNFUSED", 0) != 0;
        c->nstreams = fcd_env_int("FCD_STREAMS", 2) >= 2 ? 2 : 1;
        // the fused chain at 2048- / 4096-wide rows: one stream (its kernels fill the chip
        // alone; with 32-frame chunks c5 3.48 k -> 3.52 k, c3 18.29 k -> 18.35 k, r05ze/zf)
        c->fused_split = fcd_env_int("FCD_STREAMS", 0) ? c->nstreams : (cols <= 1024 ? 2 : 1);
        c->early_census = fcd_env_int("FCD_EARLY_CENSUS", 1) != 0;
        c->H = rows;
        c->W = cols;
        c->generic = !pow2;
        if (c->generic) {
            c->mr_row = fcdk::mr_plan(cols);
            c->mr_col = fcdk::mr_plan(rows);
            const size_t gsb = std::max(fcdk::mr_long_scratch_bytes(c->mr_row), fcdk::mr_long_scratch_bytes(c->mr_col));
            if (gsb) c->mr_gs.ensure(gsb);
        }
        HIPCHK(hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking));
        get_aux(c.get());  // right after `own`: the two get different hardware queues (process_impl)
        // plain tables exp(-2 pi i m / n) (power-of-two LDS kernels), or the mixed-radix plans'
        // tables (with Bluestein's chirp and convolution spectra)
        const std::vector<float2> tr = c->generic ? fcdk::mr_tables(c->mr_row) : twiddles(cols),
                                  tc = c->generic ? fcdk::mr_tables(c->mr_col) : twiddles(rows);
        c->tw_row.ensure(tr.size() * sizeof(float2));
        c->tw_col.ensure(tc.size() * sizeof(float2));
        HIPCHK(hipMemcpy(c->tw_row.p, tr.data(), tr.size() * sizeof(float2), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(c->tw_col.p, tc.data(), tc.size() * sizeof(float2), hipMemcpyHostToDevice));
        if (!c->generic) {  // the register FFTs' pass-major tables (power-of-two fast path)
            const std::vector<float2> pr = pass_twiddles(cols), pc = pass_twiddles(rows);
            c->twp_row.ensure(pr.size() * sizeof(float2));
            c->twp_col.ensure(pc.size() * sizeof(float2));
            HIPCHK(hipMemcpy(c->twp_row.p, pr.data(), pr.size() * sizeof(float2), hipMemcpyHostToDevice));
            HIPCHK(hipMemcpy(c->twp_col.p, pc.data(), pc.size() * sizeof(float2), hipMemcpyHostToDevice));
        }
        if (!c->generic && (fcdk::int_cols_elems(rows) == 16 || fcdk::demod_cols_elems(rows) == 16)) {
            const std::vector<float2> pi = pass_twiddles(rows, 16);
            c->twp_col16.ensure(pi.size() * sizeof(float2));
            HIPCHK(hipMemcpy(c->twp_col16.p, pi.data(), pi.size() * sizeof(float2), hipMemcpyHostToDevice));
        }
        {
            std::vector<float> rtw, ctw;  // the plans' tables (complex entries as (re, im) pairs)
            c->pf_row = pf::make_plan<float>(cols, true, rtw);
            c->pf_col = pf::make_plan<float>(rows, false, ctw);
            c->pf_rtw.ensure(rtw.size() * sizeof(float));
            c->pf_ctw.ensure(ctw.size() * sizeof(float));
            HIPCHK(hipMemcpy(c->pf_rtw.p, rtw.data(), rtw.size() * sizeof(float), hipMemcpyHostToDevice));
            HIPCHK(hipMemcpy(c->pf_ctw.p, ctw.data(), ctw.size() * sizeof(float), hipMemcpyHostToDevice));
        }
        // chunk: ~48 B of workspace per pixel per frame; keep the working set near the 256 MiB MALL
        // (the generic chain streams every stage through HBM anyway: up to 32 frames
        // in 4 GiB, its transposes' scratch included)
        const long per_frame = 48L * rows * cols;
        c->chunk = c->generic ? (int)std::max(1L, std::min(32L, (4L << 30) / (per_frame + 8L * rows * cols)))
                              : (int)std::max(1L, std::min(64L, (256L << 20) / per_frame));
        ensure_chunk_buffers(c.get());
        if (c->generic) c->mr_scratch.ensure((size_t)c->chunk * c->hw() * sizeof(float2));
        c->scalar.ensure(64);
        *out = c.release();
    })
}

FCD_API int fcd_destroy(fcd_ctx* ctx) {
    FCD_TRY({
        if (!ctx) return FCD_OK;
        (void)hipSetDevice(ctx->device);
        // a device call may return with its integration still queued on the caller's
        // stream (early census): wait for it before the workspace goes
        if (ctx->ev_done) (void)hipEventSynchronize(ctx->ev_done);
        (void)hipStreamSynchronize(ctx->own);
        (void)hipStreamDestroy(ctx->own);
        for (hipEvent_t e : ctx->ev_cen)
            if (e) (void)hipEventDestroy(e);
        if (ctx->ev_done) (void)hipEventDestroy(ctx->ev_done);
        if (ctx->aux) {
            (void)hipStreamSynchronize(ctx->aux);
            (void)hipStreamDestroy(ctx->aux);
            (void)hipEventDestroy(ctx->ev_fork);
            (void)hipEventDestroy(ctx->ev_join);
            (void)hipEventDestroy(ctx->ev_join0);
        }
        delete ctx;
    })
}

FCD_API int fcd_synchronize(fcd_ctx* ctx) {
    FCD_TRY({
        check_ctx(ctx);
        if (ctx->ev_done) HIPCHK(hipEventSynchronize(ctx->ev_done));
        ctx->done_pending = false;
        HIPCHK(hipStreamSynchronize(ctx->own));
    })
}

FCD_API int fcd_set_reference(fcd_ctx* c, const float* reference, int flags, double square_size,
                              fcd_ref_info* info) {
    FCD_TRY({
        check_ctx(c);
        if (!reference) throw FcdError(FCD_E_INVALID, "reference is null");
        if (flags & ~(FCD_DEVICE_PTRS | FCD_IMG_F64)) throw FcdError(FCD_E_INVALID, "bad flags");
        hipStream_t s = c->own;
        const long hw = c->hw();
        const bool f64 = flags & FCD_IMG_F64;
        const size_t es = f64 ? sizeof(double) : sizeof(float);
        c->has_ref = false;
        const void* dref = reference;
        if (!(flags & FCD_DEVICE_PTRS)) {
            c->frames_in.ensure(hw * es);
            upload(c->frames_in.p, reference, hw * es, s);
            dref = c->frames_in.p;
        }
        // the carrier picks from the reference's own precision (fourier.py:18)
        find_peaks_batch(c, dref, f64, 1, square_size, nullptr, s);
        c->pk_F.release();  // (the exact spectrum: a one-off per reference, not kept)
        const float* dref32 = static_cast<const float*>(dref);
        if (f64) {  // the per-frame demodulation's carrier signals from its float32 rounding
            c->ref32.ensure(hw * sizeof(float));
            fcdk::convert_f64(static_cast<const double*>(dref), hw, c->ref32.as<float>(), s);
            dref32 = c->ref32.as<float>();
        }
        reference_state(c, dref32, dref32, s);
        c->has_ref = true;
        if (info) *info = c->info;
    })
}

FCD_API int fcd_set_carriers(fcd_ctx* c, const float* ref0, const float* ref1, int flags, double calibration_factor,
                             const int64_t* peaks, const double* radius, fcd_ref_info* info) {
    FCD_TRY({
        check_ctx(c);
        if (!ref0 || !peaks || !radius) throw FcdError(FCD_E_INVALID, "null argument");
        if (!ref1) ref1 = ref0;
        if (!std::isfinite(calibration_factor) || calibration_factor == 0.0)
            throw FcdError(FCD_E_INVALID, "calibration factor must be finite and non-zero");
        long prow[2], pcol[2];
        double R[2];
        for (int q = 0; q < 2; ++q) {
            prow[q] = (long)peaks[2 * q];
            pcol[q] = (long)peaks[2 * q + 1];
            R[q] = radius[q];
            if (prow[q] < 0 || prow[q] >= c->H || pcol[q] < 0 || pcol[q] >= c->W)
                throw FcdError(FCD_E_INVALID, "carrier peak outside the image");
            if (!(R[q] > 0.0) || !std::isfinite(R[q])) throw FcdError(FCD_E_INVALID, "carrier radius must be > 0");
        }
        hipStream_t s = c->own;
        const long hw = c->hw();
        c->has_ref = false;
        const float* d0 = ref0;
        const float* d1 = ref1;
        if (flags != FCD_DEVICE_PTRS) {
            const bool two = ref1 != ref0;
            c->frames_in.ensure((two ? 2 : 1) * hw * sizeof(float));
            upload(c->frames_in.p, ref0, hw * sizeof(float), s);
            d0 = d1 = c->frames_in.as<float>();
            if (two) {
                upload(c->frames_in.as<float>() + hw, ref1, hw * sizeof(float), s);
                d1 = c->frames_in.as<float>() + hw;
            }
        }
        std::memset(&c->info, 0, sizeof(c->info));
        fcdh::carrier_geometry(c->H, c->W, c->info, c->disk_rows_host, prow, pcol, calibration_factor, R);
        reference_state(c, d0, d1, s);
        c->has_ref = true;
        if (info) *info = c->info;
    })
}

FCD_API int fcd_find_peaks(fcd_ctx* c, const float* images, int n, int flags, double square_size,
                           fcd_ref_info* infos) {
    FCD_TRY({
        check_ctx(c);
        if (!images || !infos || n < 0) throw FcdError(FCD_E_INVALID, "bad arguments");
        if (flags & ~(FCD_DEVICE_PTRS | FCD_IMG_F64)) throw FcdError(FCD_E_INVALID, "bad flags");
        hipStream_t s = c->own;
        const long hw = c->hw();
        const bool f64 = flags & FCD_IMG_F64;
        const size_t es = f64 ? sizeof(double) : sizeof(float);
        // the context's reference (if any) is kept: its per-reference host state is
        // restored afterwards; the device state find_peaks_batch touches is workspace
        const fcd_ref_info keep_info = c->info;
        const std::vector<int> keep_rows = c->disk_rows_host;
        struct Restore {
            fcd_ctx* c;
            const fcd_ref_info& info;
            const std::vector<int>& rows;
            ~Restore() {
                c->info = info;
                c->disk_rows_host = rows;
            }
        } restore{c, keep_info, keep_rows};
        const int bmax = find_peaks_batch_max(c, f64);
        for (int i0 = 0; i0 < n; i0 += bmax) {
            const int nb = std::min(bmax, n - i0);
            const void* img = reinterpret_cast<const char*>(images) + (size_t)i0 * hw * es;
            if (!(flags & FCD_DEVICE_PTRS)) {
                c->frames_in.ensure((size_t)nb * hw * es);
                upload(c->frames_in.p, img, (size_t)nb * hw * es, s);
                img = c->frames_in.p;
            }
            find_peaks_batch(c, img, f64, nb, square_size, infos + i0, s);
        }
    })
}

FCD_API int fcd_get_carriers(fcd_ctx* c, float* ccsgn, uint8_t* mask) {
    FCD_TRY({
        check_ctx(c);
        if (!c->has_ref) throw FcdError(FCD_E_STATE, "no reference set");
        const long hw = c->hw();
        if (ccsgn) {
            HIPCHK(hipMemcpy(ccsgn, c->refsig.p, 2 * hw * sizeof(float2), hipMemcpyDeviceToHost));
            const float sc = (float)(1.0 / (double)hw);
            for (long i = 0; i < 2 * hw; ++i) {
                ccsgn[2 * i] *= sc;
                ccsgn[2 * i + 1] *= -sc;  // conj
            }
        }
        if (mask) {
            for (int q = 0; q < 2; ++q) {
                const int* rows = c->disk_rows_host.data() + (size_t)q * 2 * c->W;
                for (int i = 0; i < c->H; ++i)
                    for (int j = 0; j < c->W; ++j) {
                        const int si = (i + c->H / 2) % c->H, sj = (j + c->W / 2) % c->W;
                        mask[(size_t)q * hw + (size_t)i * c->W + j] = si >= rows[2 * sj] && si <= rows[2 * sj + 1];
                    }
            }
        }
    })
}

namespace {

// First pass of one chunk: nb device-resident float32 frames through the
// band-pruned pipeline with the residue-free unwrap, heights to hdst (device).
// fo: first workspace frame of the chunk (the fused chain's per-frame
// intermediates are frame-strided, so disjoint frame ranges of one workspace can
// run concurrently on different streams).
// census_ev (fused chain only): recorded once the chunk's census flags are final (fused
// kernel + tile-range census, which then runs right after it), before the integration.
void first_pass_chunk(fcd_ctx* c, const float* fr, int nb, bool unwrap, bool fused, int* res, float* hdst,
                      int32_t* kdst, const fcdk::IntegCoef& coef, hipStream_t s, int fo = 0,
                      hipEvent_t census_ev = nullptr, const int* census_src = nullptr, int* census_host = nullptr,
                      size_t census_n = 0) {
    if (fused) {
        // height only: band transforms, phase, unwrap and the z-row FFT in one
        // pass (kernels_phase_rows.hip); colk lands in the spectra's DC bins
        const fcdk::DemodTables T = demod_tables(c);
        const long H = c->H, W = c->W;
        float2* Xb = c->Xb.as<float2>() + fo * H * c->NC;
        float2* Ab = c->Ab.as<float2>() + fo * 2 * H * c->NCA;
        float* col0 = c->col0.as<float>() + fo * 2 * H;
        int* colk = c->colk.as<int>() + fo * 2 * H;
        float2* Zt = c->Zt.as<float2>() + fo * H * W;
        float2* seam = c->seam.as<float2>() + fo * (H / fcdk::phase_rows_tile(c->W)) * 2 * W;
        float2* Ht = c->Ht.as<float2>() + fo * H * (W / 2 + 1);
        if (c->profiling) HIPCHK(hipEventRecord(c->next_event(), s));
        fcdk::demod_rows(c->W, fr, c->H, nb, T, Xb, c->twp_row.as<float2>(), s);
        fcdk::demod_cols(c->H, Xb, nb, T, Ab, c->NCA, dc_tw(c), s);
        if (c->profiling) HIPCHK(hipEventRecord(c->next_event(), s));
        const bool defer = !census_ev;
        fcdk::phase_rows(c->W, unwrap, Ab, c->H, nb, c->NCA, c->NCc[0], c->NCc[1], c->theta_p.as<float>(),
                         c->band_pre.as<float2>(), c->band_ptw.as<float2>(), c->ztw.as<float2>(), col0, res, Zt, seam,
                         s, defer);
        // early census: the flags go to the page-locked readback buffer on this stream as soon
        // as they are final (a copy on a stream of its own waited behind whatever shared its
        // hardware queue), and the event marks their arrival
        if (census_ev && census_n)
            HIPCHK(hipMemcpyAsync(census_host, census_src, census_n * sizeof(int), hipMemcpyDeviceToHost, s));
        if (census_ev) HIPCHK(hipEventRecord(census_ev, s));
        if (unwrap) fcdk::unwrap_colk_compact(col0, 2 * nb, c->H, colk, s);
        if (c->profiling) HIPCHK(hipEventRecord(c->next_event(), s));
        fcdk::int_cols(c->H, Zt, c->W, nb, coef, Ht, ic_tw(c), s, unwrap ? colk : nullptr);
        fcdk::int_c2r(c->W, Ht, c->H, nb, hdst, c->twp_row.as<float2>(), s);
        // the census of the tile-range edges: its flags are read only when the call ends,
        // so it runs last instead of holding the integration kernels behind it (a small
        // grid waiting for CUs the other stream's fused kernel holds)
        if (unwrap && defer) fcdk::phase_rows_seam(c->W, c->H, nb, seam, res, s);
    } else {
        const long H = c->H, W = c->W;
        float* wrapped = c->wrapped.as<float>() + fo * 2 * H * W;
        int* colk = c->colk.as<int>() + fo * 2 * H;
        float2* Zt = c->Zt.as<float2>() + fo * H * W;
        float2* Ht = c->Ht.as<float2>() + fo * H * (W / 2 + 1);
        if (c->profiling) HIPCHK(hipEventRecord(c->next_event(), s));
        fast_demod(c, fr, nb, s, fo);
        if (c->profiling) HIPCHK(hipEventRecord(c->next_event(), s));
        if (unwrap) fcdk::unwrap_colk(wrapped, 2 * nb, c->H, c->W, colk, s);
        if (c->profiling) HIPCHK(hipEventRecord(c->next_event(), s));
        // the second concurrent half (fo > 0) has its own seam region
        float2* seam = c->ir_seam.as<float2>() +
                       (fo ? fcdk::int_rows_seam_bytes(c->W, c->H, c->ws_nb) / sizeof(float2) : 0);
        fcdk::int_rows(c->W, unwrap ? 1 : 0, wrapped, colk, nullptr, kdst, res, c->H, nb, Zt, c->twp_row.as<float2>(),
                       seam, s);
        fcdk::int_cols(c->H, Zt, c->W, nb, coef, Ht, ic_tw(c), s);
        fcdk::int_c2r(c->W, Ht, c->H, nb, hdst, c->twp_row.as<float2>(), s);
    }
    if (c->profiling) {
        HIPCHK(hipEventRecord(c->next_event(), s));
        c->prof_frames += nb;
    }
}

// Caller memory that is page-locked (fcd_host_alloc, hipHostRegister, torch
// pin_memory) is copied by DMA straight from / to its own pages.
bool host_pinned(const void* p) {
    if (!p) return false;
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// memcpy between pageable and pinned host memory, split over threads (one
// host thread moves ~10 GB/s; the PCIe link ~50 GB/s per direction).
void ensure_host_pipe(fcd_ctx* c, int format) {
    HostPipe& P = c->pipe;
    const long hw = c->hw();
    if (!P.h2d) {
        HIPCHK(hipStreamCreateWithFlags(&P.h2d, hipStreamNonBlocking));
        HIPCHK(hipStreamCreateWithFlags(&P.d2h, hipStreamNonBlocking));
        for (int i = 0; i < 2; ++i)
            for (hipEvent_t* e : {&P.ev_h2d[i], &P.ev_free[i], &P.ev_comp[i], &P.ev_d2h[i]})
                HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
    }
    // 128 MiB of float32 frames per slot (32 frames at 1024^2): two slots in flight
    // overlap the H2D copy, the compute and the D2H copy.  Never more frames than the
    // chunk workspace of the current reference holds (fchunk changes with it).
    const long budget = (long)fcd_env_int("FCD_PIPE_MB", 128) << 20;
    const int nb = (int)std::max(1L, std::min((long)c->fchunk, budget / (hw * 4)));
    if (nb != P.nb) {
        for (int i = 0; i < 2; ++i) {
            if (P.pin_out[i]) (void)hipHostFree(P.pin_out[i]);
            if (P.pin_in[i]) (void)hipHostFree(P.pin_in[i]);
            P.pin_out[i] = nullptr;
            P.pin_in[i] = nullptr;
        }
        P.in_bytes = 0;
        P.nb = nb;
        const size_t out_b = (size_t)nb * hw * 4;
        for (int i = 0; i < 2; ++i) {
            HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&P.pin_out[i]), out_b, hipHostMallocDefault));
            P.dev_out[i].ensure(out_b);
        }
    }
    const size_t in_b = (size_t)P.nb * fcdk::raw_frame_bytes(format, c->H, c->W);
    if (in_b > P.in_bytes) {
        for (int i = 0; i < 2; ++i) {
            if (P.pin_in[i]) (void)hipHostFree(P.pin_in[i]);
            P.pin_in[i] = nullptr;
            HIPCHK(hipHostMalloc(&P.pin_in[i], in_b, hipHostMallocDefault));
            P.dev_raw[i].ensure(in_b);
        }
        P.in_bytes = in_b;
    }
}

// Host frames, heights only: three-stage pipeline over two slots.  While chunk
// i computes on the context stream, chunk i+1's samples cross PCIe on the H2D
// stream and chunk i-1's heights on the D2H stream; pageable caller memory is
// staged through pinned slots by parallel memcpy, pinned caller memory is
// DMA'd directly.
void host_pipeline(fcd_ctx* c, const void* frames, int format, int n_frames, bool unwrap, bool fused, int* res,
                   float* height_out, const fcdk::IntegCoef& coef, hipStream_t s) {
    ensure_host_pipe(c, format);
    HostPipe& P = c->pipe;
    const long hw = c->hw();
    // on any exit (an error included) no copy may still target the caller's memory
    struct Drain {
        HostPipe& P;
        hipStream_t s;
        ~Drain() {
            (void)hipStreamSynchronize(s);
            (void)hipStreamSynchronize(P.h2d);
            (void)hipStreamSynchronize(P.d2h);
        }
    } drain{P, s};
    const size_t rb = fcdk::raw_frame_bytes(format, c->H, c->W);
    const bool pin_src = host_pinned(frames), pin_dst = host_pinned(height_out);
    ensure_fast_ws(c, std::min(P.nb, n_frames));
    const int nchunks = (n_frames + P.nb - 1) / P.nb;
    auto chunk_frames = [&](int i) { return std::min(P.nb, n_frames - i * P.nb); };
    auto retire = [&](int i) {  // chunk i's heights: pinned slot -> caller memory
        if (pin_dst || !height_out) return;
        HIPCHK(hipEventSynchronize(P.ev_d2h[i & 1]));
        par_copy(height_out + (size_t)i * P.nb * hw, P.pin_out[i & 1], (size_t)chunk_frames(i) * hw * 4);
    };
    for (int i = 0; i < nchunks; ++i) {
        const int slot = i & 1, nb = chunk_frames(i);
        const size_t f0 = (size_t)i * P.nb;
        const char* src = static_cast<const char*>(frames) + f0 * rb;
        if (!pin_src) {
            if (i >= 2) HIPCHK(hipEventSynchronize(P.ev_h2d[slot]));  // slot's previous upload has left
            par_copy(P.pin_in[slot], src, (size_t)nb * rb);
            src = static_cast<const char*>(P.pin_in[slot]);
        }
        if (i >= 2) HIPCHK(hipStreamWaitEvent(P.h2d, P.ev_free[slot], 0));  // device slot consumed
        HIPCHK(hipMemcpyAsync(P.dev_raw[slot].p, src, (size_t)nb * rb, hipMemcpyHostToDevice, P.h2d));
        HIPCHK(hipEventRecord(P.ev_h2d[slot], P.h2d));
        HIPCHK(hipStreamWaitEvent(s, P.ev_h2d[slot], 0));
        const float* fr = P.dev_raw[slot].as<float>();
        if (format != FCD_FMT_F32) {
            fcdk::ingest(format, P.dev_raw[slot].p, nb, c->H, c->W, c->frames_in.as<float>(), s);
            fr = c->frames_in.as<float>();
            HIPCHK(hipEventRecord(P.ev_free[slot], s));
        }
        if (i >= 2) HIPCHK(hipStreamWaitEvent(s, P.ev_d2h[slot], 0));  // heights slot drained
        first_pass_chunk(c, fr, nb, unwrap, fused, res ? res + f0 * 2 : nullptr, P.dev_out[slot].as<float>(),
                         nullptr, coef, s);
        if (format == FCD_FMT_F32) HIPCHK(hipEventRecord(P.ev_free[slot], s));
        HIPCHK(hipEventRecord(P.ev_comp[slot], s));
        if (height_out) {
            HIPCHK(hipStreamWaitEvent(P.d2h, P.ev_comp[slot], 0));
            float* dst = pin_dst ? height_out + f0 * hw : P.pin_out[slot];
            HIPCHK(hipMemcpyAsync(dst, P.dev_out[slot].p, (size_t)nb * hw * 4, hipMemcpyDeviceToHost, P.d2h));
            HIPCHK(hipEventRecord(P.ev_d2h[slot], P.d2h));
        }
        if (i >= 1) retire(i - 1);
    }
    if (nchunks >= 1) retire(nchunks - 1);
    HIPCHK(hipStreamSynchronize(P.d2h));
    HIPCHK(hipStreamSynchronize(P.h2d));
}

// Frames `idx` of a (host or device, any format) batch -> float32 in frames_in.
void stage_frames(fcd_ctx* c, const void* frames, int format, bool dev, const int* idx, int n, hipStream_t s) {
    const long hw = c->hw();
    const size_t rb = fcdk::raw_frame_bytes(format, c->H, c->W);
    const hipMemcpyKind kind = dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    void* dst = c->frames_in.p;
    if (format != FCD_FMT_F32) {
        c->fix_raw.ensure((size_t)n * rb);
        dst = c->fix_raw.p;
    }
    for (int i = 0; i < n; ++i)
        HIPCHK(hipMemcpyAsync(static_cast<char*>(dst) + (size_t)i * rb,
                              static_cast<const char*>(frames) + (size_t)idx[i] * rb, rb, kind, s));
    if (format != FCD_FMT_F32) fcdk::ingest(format, dst, n, c->H, c->W, c->frames_in.as<float>(), s);
    (void)hw;
}

// The generic chain (a frame side that is not a power of two): per chunk of c->chunk
// frames the reference's own sequence -- fft2 of the frames (fcd.py:28), per carrier the
// disk mask, ifft2 and phase step (fcd.py:116-118), the unwrap of both maps (fcd.py:119:
// residue census, scan or exact MST), phi0 + i phi1 and its spectral integration with the
// displacement solve folded in (fcd.py:30-33, fourier.py:115-137) -- on the mixed-radix
// transforms.  Synchronous on `s`.
int process_generic(fcd_ctx* c, const void* frames, int format, int n_frames, bool dev, bool unwrap,
                    const fcdk::IntegCoef& coef, float* height_out, float* wrapped_out, int32_t* k_out, hipStream_t s) {
    ensure_aux_buffers(c);
    const long hw = c->hw();
    const hipMemcpyKind kind = dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    c->frames_in.ensure((size_t)c->chunk * hw * sizeof(float));
    c->out_h.ensure((size_t)c->chunk * hw * sizeof(float));
    double unwrap_ms = 0;
    long nres = 0;
    for (int f0 = 0; f0 < n_frames; f0 += c->chunk) {
        const int nb = std::min(c->chunk, n_frames - f0);
        const float* fr = reinterpret_cast<const float*>(frames) + (size_t)f0 * hw;
        if (!dev || format != FCD_FMT_F32) {
            std::vector<int> idx(nb);
            std::iota(idx.begin(), idx.end(), f0);
            stage_frames(c, frames, format, dev, idx.data(), nb, s);
            fr = c->frames_in.as<float>();
        }
        if (c->profiling) HIPCHK(hipEventRecord(c->next_event(), s));
        float* w = c->wrapped.as<float>();
        if ((size_t)nb * hw * sizeof(float2) > c->mr_scratch.bytes)
            throw FcdError(FCD_E_INTERNAL, "mixed-radix scratch too small");
        float2* specT = c->mr_scratch.as<float2>();
        generic_fft2_t(c, fr, nb, specT, s);
        generic_demod_t(c, specT, nb, w, s);
        if (c->profiling) HIPCHK(hipEventRecord(c->next_event(), s));
        int32_t* k = nullptr;
        const int* kflag = nullptr;
        std::vector<int> flags;
        if (unwrap) {
            std::vector<int> counts(2 * (size_t)nb);
            k = c->kbuf.as<int32_t>();
            const auto tu = std::chrono::steady_clock::now();
            // heights only: the residue-free maps' scan runs in the z rows (no k-field pass)
            const bool zscan = k_out == nullptr;
            unwrap_maps(c, w, 2 * nb, k, counts.data(), s, false, nullptr, true, 0, zscan);
            if (zscan) {
                flags.resize(2 * (size_t)nb);
                for (size_t m = 0; m < flags.size(); ++m) flags[m] = counts[m] > 0;
                // (the scanned maps' column-0 offsets were computed iff some map is residue-free)
                bool any_scan = false;
                for (int f : flags) any_scan |= f == 0;
                if (any_scan && !c->ms[0].colk.p) throw FcdError(FCD_E_INTERNAL, "column offsets missing");
                c->gk_flag.ensure(flags.size() * sizeof(int));
                upload(c->gk_flag.p, flags.data(), flags.size() * sizeof(int), s);
                kflag = c->gk_flag.as<int>();
            }
            if (c->profiling) {  // the unwrap span (it synchronises), counted as the exact pass's time
                HIPCHK(hipStreamSynchronize(s));
                unwrap_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tu).count();
            }
            for (int i = 0; i < nb; ++i) nres += counts[2 * (size_t)i] || counts[2 * (size_t)i + 1];
        }
        if (c->profiling) HIPCHK(hipEventRecord(c->next_event(), s));
        float* hdst = dev && height_out ? height_out + (size_t)f0 * hw : c->out_h.as<float>();
        generic_integrate_t(c, nb, w, k, coef, hdst, s, kflag, kflag ? c->ms[0].colk.as<int>() : nullptr);
        if (c->profiling) {
            HIPCHK(hipEventRecord(c->next_event(), s));
            c->prof_frames += nb;
        }
        if (height_out && !dev) HIPCHK(hipMemcpyAsync(height_out + (size_t)f0 * hw, hdst, (size_t)nb * hw * 4, kind, s));
        if (wrapped_out)
            HIPCHK(hipMemcpyAsync(wrapped_out + (size_t)f0 * 2 * hw, w, (size_t)nb * 2 * hw * 4, kind, s));
        if (k_out && k) {
            HIPCHK(hipMemcpyAsync(k_out + (size_t)f0 * 2 * hw, k, (size_t)nb * 2 * hw * 4, kind, s));
        } else if (k_out) {
            if (dev) HIPCHK(hipMemsetAsync(k_out + (size_t)f0 * 2 * hw, 0, (size_t)nb * 2 * hw * 4, s));
            else std::memset(k_out + (size_t)f0 * 2 * hw, 0, (size_t)nb * 2 * hw * 4);
        }
        HIPCHK(hipStreamSynchronize(s));  // the chunk's workspace is reused by the next
    }
    if (c->profiling) {  // frames with residues (their maps took the exact MST unwrap) and the unwrap's time
        c->prof_fix_ms += unwrap_ms;
        c->prof_fix_frames += nres;
    }
    return FCD_OK;
}

// The first pass's heights (the fused chain when fused_ok, as pass 1 of process_impl runs it)
// of the frames f0 + idx[i] of a batch, written to hdst + idx[i] * H * W (device) for each
// frame whose census of that chain is clean; a frame the chain's census flags (a wrapped
// difference of exactly fl(pi)) keeps the exact chain's heights, as pass 2 would give it.
void first_pass_heights(fcd_ctx* c, const void* frames, int format, bool dev, int f0, const std::vector<int>& idx,
                        bool fused_allowed, const fcdk::IntegCoef& coef, float* hdst, hipStream_t s) {
    const long hw = c->hw();
    const int n = (int)idx.size();
    const bool fused = c->fused_ok && fused_allowed && !c->force_unfused;
    std::vector<int> abs_idx(n);
    for (int i = 0; i < n; ++i) abs_idx[i] = f0 + idx[i];
    const bool run = abs_idx[n - 1] - abs_idx[0] == n - 1;
    const float* fr;
    if (run && dev && format == FCD_FMT_F32) {
        fr = reinterpret_cast<const float*>(frames) + (size_t)abs_idx[0] * hw;
    } else {
        stage_frames(c, frames, format, dev, abs_idx.data(), n, s);
        fr = c->frames_in.as<float>();
    }
    c->fix_h.ensure((size_t)n * hw * sizeof(float));
    c->fix_res.ensure((size_t)n * 2 * sizeof(int));
    int* res = c->fix_res.as<int>();
    HIPCHK(hipMemsetAsync(res, 0, (size_t)n * 2 * sizeof(int), s));
    first_pass_chunk(c, fr, n, true, fused, res, c->fix_h.as<float>(), nullptr, coef, s);
    std::vector<int> flags((size_t)n * 2);
    HIPCHK(hipMemcpyAsync(flags.data(), res, flags.size() * sizeof(int), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    for (int i = 0; i < n; ++i)
        if (!flags[2 * (size_t)i] && !flags[2 * (size_t)i + 1])
            HIPCHK(hipMemcpyAsync(hdst + (size_t)idx[i] * hw, c->fix_h.as<float>() + (size_t)i * hw, hw * sizeof(float),
                                  hipMemcpyDeviceToDevice, s));
}

int process_impl(fcd_ctx* c, const void* frames, int format, int n_frames, int flags, double height, int unwrap,
                 float* height_out, float* wrapped_out, int32_t* k_out, void* stream) {
    check_ctx(c, false);
    // the previous call's queued work: ordered on the device for a device call on the same
    // caller stream, waited for on the host otherwise
    settle(c, flags == FCD_DEVICE_PTRS && stream ? static_cast<hipStream_t>(stream) : nullptr);
    if (!c->has_ref) throw FcdError(FCD_E_STATE, "no reference set");
    if (!frames || n_frames < 0) throw FcdError(FCD_E_INVALID, "bad frames");
    if (fcdk::raw_frame_bytes(format, c->H, c->W) == 0) throw FcdError(FCD_E_INVALID, "unknown frame format");
    if (!(height != 0.0)) throw FcdError(FCD_E_INVALID, "height must be non-zero");
    if (n_frames == 0) return FCD_OK;
    hipStream_t s = c->pick(stream);
    const long hw = c->hw();
    const bool dev = flags == FCD_DEVICE_PTRS;
    const size_t rb = fcdk::raw_frame_bytes(format, c->H, c->W);
    const fcd_ref_info& in = c->info;
    const double det = in.frequencies[0][1] * in.frequencies[1][0] - in.frequencies[0][0] * in.frequencies[1][1];
    const double sc = 1.0 / (det * height);
    ensure_integ_tables(c, in.calibration_factor, s);
    // h_hat = i/k^2 [(kx f1[0] - ky f1[1]) Phi0 + (ky f0[1] - kx f0[0]) Phi1] / (det * height)
    const fcdk::IntegCoef coef = integ_coef(c, in.frequencies[1][0] * sc, -in.frequencies[1][1] * sc,
                                            -in.frequencies[0][0] * sc, in.frequencies[0][1] * sc);
    if (c->generic)
        return process_generic(c, frames, format, n_frames, dev, unwrap != 0, coef, height_out, wrapped_out, k_out, s);
    // frames launched at once: the call's own, up to the workspace budget's fchunk
    const int nbmax = std::max(1, std::min(c->fchunk, n_frames));
    ensure_fast_ws(c, nbmax);
    c->frames_in.ensure((size_t)nbmax * hw * sizeof(float));
    c->out_h.ensure((size_t)nbmax * hw * sizeof(float));
    const hipMemcpyKind out_kind = dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    int* res = nullptr;
    if (unwrap) {  // residue census of every map of the call
        c->fres.ensure((size_t)n_frames * 2 * sizeof(int) + 16);
        res = c->fres.as<int>();
        HIPCHK(hipMemsetAsync(res, 0, (size_t)n_frames * 2 * sizeof(int), s));
    }
    // ---- residue-heavy input (camera frames: every map carries residues): when most
    // frames of the previous call needed the exact pass, the fused first pass would only
    // produce heights that pass 2 throws away, so this call runs the exact chain at once:
    // demod, residue count, the scan unwrap for residue-free maps and the MST for the
    // others, integration.  Frames with residues: the same kernels and k-fields as pass 2
    // (bit-identical heights); residue-free frames: redone by the first pass's chain
    // (first_pass_heights), so every frame's heights are those of the two-pass form whatever
    // the previous call held.  FCD_EXACT_FIRST=0 / 1 forces either mode.
    const int ef_env = fcd_env_int("FCD_EXACT_FIRST", -1);  // (read per call: tests switch it)
    if (unwrap && !wrapped_out && (ef_env >= 0 ? ef_env == 1 : c->exact_first)) {
        const auto t0 = std::chrono::steady_clock::now();
        long nres = 0;
        std::vector<int> counts;
        for (int f0 = 0; f0 < n_frames; f0 += nbmax) {
            const int nb = std::min(nbmax, n_frames - f0);
            const float* fr = reinterpret_cast<const float*>(static_cast<const char*>(frames) + (size_t)f0 * rb);
            if (!dev || format != FCD_FMT_F32) {
                std::vector<int> idx(nb);
                std::iota(idx.begin(), idx.end(), f0);
                stage_frames(c, frames, format, dev, idx.data(), nb, s);
                fr = c->frames_in.as<float>();
            }
            int32_t* kf = dev && k_out ? k_out + (size_t)f0 * 2 * hw : c->fk.as<int32_t>();
            counts.assign((size_t)2 * nb, 0);
            float* hdst = dev && height_out ? height_out + (size_t)f0 * hw : c->out_h.as<float>();
            // frames fo .. fo + n - 1 of the chunk: demod, unwrap (census, scan / MST in MST
            // workspace h), integration, all on stream hs
            auto half = [&](int h, int fo, int n, hipStream_t hs) {
                float* wr = c->wrapped.as<float>() + (size_t)fo * 2 * hw;
                int32_t* kh = kf + (size_t)fo * 2 * hw;
                float2* Zt = c->Zt.as<float2>() + (size_t)fo * hw;
                float2* Ht = c->Ht.as<float2>() + (size_t)fo * c->H * (c->W / 2 + 1);
                fast_demod(c, fr + (size_t)fo * hw, n, hs, fo);
                fcdk::MstK mk{};
                unwrap_maps(c, wr, 2 * n, kh, counts.data() + 2 * (size_t)fo, hs, false, k_out ? nullptr : &mk, true, h);
                fcdk::int_rows(c->W, mk.map_slot ? 3 : 2, wr, nullptr, kh, nullptr, nullptr, c->H, n, Zt,
                               c->twp_row.as<float2>(), nullptr, hs, mk.map_slot ? &mk : nullptr);
                fcdk::int_cols(c->H, Zt, c->W, n, coef, Ht, ic_tw(c), hs);
                fcdk::int_c2r(c->W, Ht, c->H, n, hdst + (size_t)fo * hw, c->twp_row.as<float2>(), hs);
            };
            if (c->nstreams < 2 || nb < 8) {
                half(0, 0, nb, s);
            } else {
                // Two halves side by side, each driven by its own host thread on its own stream
                // and MST workspace: one half's census read-back, graph-round convergence checks
                // and small graph-round kernels overlap the other half's kernels, instead of
                // leaving the chip idle (the camera frames' exact chain, r04ap trace).
                // Both halves on the context's own two streams (created one after the other at
                // fcd_create, so the runtime deals them different hardware queues), the caller's
                // stream only forking and joining them: with the caller's stream as the first
                // half's, whether the halves overlapped depended on how many streams the process
                // had created before the second (camera frames 9.86 k / 10.4 k frames/s in two
                // process layouts, r06)
                const int nb0 = (nb + 1) / 2;
                hipStream_t const ax = get_aux(c);
                hipStream_t const h0 = c->own;
                HIPCHK(hipEventRecord(c->ev_fork, s));
                if (h0 != s) HIPCHK(hipStreamWaitEvent(h0, c->ev_fork, 0));
                HIPCHK(hipStreamWaitEvent(ax, c->ev_fork, 0));
                std::exception_ptr err1;
                std::thread t1([&] {
                    try {
                        HIPCHK(hipSetDevice(c->device));
                        half(1, nb0, nb - nb0, ax);
                    } catch (...) {
                        err1 = std::current_exception();
                    }
                });
                std::exception_ptr err0;
                try {
                    half(0, 0, nb0, h0);
                } catch (...) {
                    err0 = std::current_exception();
                }
                t1.join();
                HIPCHK(hipEventRecord(c->ev_join, ax));
                HIPCHK(hipStreamWaitEvent(s, c->ev_join, 0));
                if (h0 != s) {
                    HIPCHK(hipEventRecord(c->ev_join0, h0));
                    HIPCHK(hipStreamWaitEvent(s, c->ev_join0, 0));
                }
                if (err0) std::rethrow_exception(err0);
                if (err1) std::rethrow_exception(err1);
            }
            // The chunk's residue-free frames get the first pass's heights, as when this call
            // had not followed a residue-heavy one: a frame's heights never depend on what
            // earlier calls held (the reference is a pure function of its inputs, fcd.py:13-35).
            std::vector<int> clean;
            for (int i = 0; i < nb; ++i)
                if (!counts[2 * (size_t)i] && !counts[2 * (size_t)i + 1]) clean.push_back(i);
            if (!clean.empty()) first_pass_heights(c, frames, format, dev, f0, clean, k_out == nullptr, coef, hdst, s);
            if (!dev && height_out)
                HIPCHK(hipMemcpyAsync(height_out + (size_t)f0 * hw, hdst, (size_t)nb * hw * 4, out_kind, s));
            if (!dev && k_out)
                HIPCHK(hipMemcpyAsync(k_out + (size_t)f0 * 2 * hw, kf, (size_t)nb * 2 * hw * 4, out_kind, s));
            if (!dev) HIPCHK(hipStreamSynchronize(s));
            for (int i = 0; i < nb; ++i) nres += counts[2 * (size_t)i] || counts[2 * (size_t)i + 1];
        }
        if (dev && !c->profiling) {  // the integration stays queued on the caller's stream, as in pass 1 below
            if (!c->ev_done) HIPCHK(hipEventCreateWithFlags(&c->ev_done, hipEventDisableTiming));
            HIPCHK(hipEventRecord(c->ev_done, s));
            c->done_stream = s;
            c->done_pending = true;
        } else {
            HIPCHK(hipStreamSynchronize(s));
        }
        if (4 * nres < n_frames) c->exact_first = false;  // mostly residue-free again
        if (c->profiling) {
            c->prof_fix_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            c->prof_fix_frames += nres;
        }
        return FCD_OK;
    }
    // ---- pass 1: every frame through the band-pruned pipeline with the residue-free unwrap
    const bool fused = c->fused_ok && !wrapped_out && !k_out && !c->force_unfused;
    // device-pointer calls of the fused chain read the census back as soon as its flags
    // are final: the call returns while the integration kernels still run on `stream`
    // (asynchronous as every device-pointer call, fcd.h), so the caller's next batch is
    // queued behind them instead of after a host round trip with the GPU idle
    const bool early = c->early_census && dev && fused && unwrap && height_out != nullptr;
    int cen_halves = 0;
    if (!dev && !wrapped_out && !k_out) {
        host_pipeline(c, frames, format, n_frames, unwrap != 0, fused, res, height_out, coef, s);
    } else {
        for (int f0 = 0; f0 < n_frames; f0 += nbmax) {
            const int nb = std::min(nbmax, n_frames - f0);
            const char* raw = static_cast<const char*>(frames) + (size_t)f0 * rb;
            const float* fr = reinterpret_cast<const float*>(raw);
            if (!dev || format != FCD_FMT_F32) {
                std::vector<int> idx(nb);
                std::iota(idx.begin(), idx.end(), 0);
                stage_frames(c, raw, format, dev, idx.data(), nb, s);
                fr = c->frames_in.as<float>();
            }
            float* hdst = (dev && height_out) ? height_out + (size_t)f0 * hw : c->out_h.as<float>();
            int32_t* kdst = k_out && unwrap ? (dev ? k_out + (size_t)f0 * 2 * hw : c->fk.as<int32_t>()) : nullptr;
            int* rs = res ? res + (size_t)f0 * 2 : nullptr;
            // the fused chain only: split (the unfused chain at 2048^2 / 4096^2 measured 1-2 %
            // slower split, r01br, though its workspace offsets allow it)
            const int nsplit = fused && !c->profiling && nb >= 2 ? c->fused_split : 1;
            // early census: the last chunk's halves mark when their census flags are final,
            // and the readback below waits for those marks only, not for the integration
            const bool last = f0 + nb >= n_frames;
            hipEvent_t cen0 = nullptr, cen1 = nullptr;
            if (early && last) {
                if (!c->ev_cen[0])
                    for (auto& e : c->ev_cen) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
                c->census.ensure((size_t)n_frames * 2 * sizeof(int));
                cen0 = c->ev_cen[0];
                cen1 = nsplit == 2 ? c->ev_cen[1] : nullptr;
                cen_halves = nsplit;
            }
            if (nsplit == 2) {
                // two halves of the chunk on two streams: kernels bound by different
                // resources (HBM-bound c2r / demod_rows, latency-bound phase_rows /
                // int_cols) overlap instead of running back to back
                hipStream_t const ax = get_aux(c);
                const int na = (nb + 1) / 2, nb2 = nb - na;
                // (r01bh/bi, 1024^2 x 256: 74.5k -> 75.7-76.3k frames/s; starting the
                // second half after the first half's demod kernels instead: no gain)
                HIPCHK(hipEventRecord(c->ev_fork, s));
                HIPCHK(hipStreamWaitEvent(ax, c->ev_fork, 0));
                // early census: half 0 reads back every earlier frame's flags too (the earlier
                // chunks' halves joined this stream), half 1 its own
                int* const ch = cen0 ? static_cast<int*>(c->census.p) : nullptr;
                first_pass_chunk(c, fr, na, unwrap != 0, fused, rs, hdst, nullptr, coef, s, 0, cen0, res, ch,
                                 cen0 ? 2 * ((size_t)f0 + na) : 0);
                first_pass_chunk(c, fr + (size_t)na * hw, nb2, unwrap != 0, fused, rs ? rs + 2 * na : nullptr,
                                 hdst + (size_t)na * hw, nullptr, coef, ax, na, cen1, rs ? rs + 2 * na : nullptr,
                                 ch ? ch + 2 * ((size_t)f0 + na) : nullptr, cen1 ? 2 * (size_t)nb2 : 0);
                HIPCHK(hipEventRecord(c->ev_join, ax));
                HIPCHK(hipStreamWaitEvent(s, c->ev_join, 0));
            } else {
                first_pass_chunk(c, fr, nb, unwrap != 0, fused, rs, hdst, kdst, coef, s, 0, cen0, res,
                                 cen0 ? static_cast<int*>(c->census.p) : nullptr, cen0 ? 2 * ((size_t)f0 + nb) : 0);
            }
            if (height_out && !dev)
                HIPCHK(hipMemcpyAsync(height_out + (size_t)f0 * hw, hdst, (size_t)nb * hw * 4, out_kind, s));
            if (wrapped_out)
                HIPCHK(hipMemcpyAsync(wrapped_out + (size_t)f0 * 2 * hw, c->wrapped.p, (size_t)nb * 2 * hw * 4,
                                      out_kind, s));
            if (k_out && unwrap && !dev)
                HIPCHK(hipMemcpyAsync(k_out + (size_t)f0 * 2 * hw, kdst, (size_t)nb * 2 * hw * 4, out_kind, s));
            if (k_out && !unwrap) {
                if (dev)
                    HIPCHK(hipMemsetAsync(k_out + (size_t)f0 * 2 * hw, 0, (size_t)nb * 2 * hw * 4, s));
                else
                    std::memset(k_out + (size_t)f0 * 2 * hw, 0, (size_t)nb * 2 * hw * 4);
            }
            if (!dev) HIPCHK(hipStreamSynchronize(s));
        }
    }
    if (dev) {  // the call's last work on the caller's stream so far (fcd_destroy / fcd_synchronize wait on it)
        if (!c->ev_done) HIPCHK(hipEventCreateWithFlags(&c->ev_done, hipEventDisableTiming));
        HIPCHK(hipEventRecord(c->ev_done, s));
        c->done_stream = s;
        c->done_pending = true;
    }
    if (!unwrap) return FCD_OK;
    // ---- pass 2: frames whose maps have residues are redone with the Boruvka (MST) unwrap
    // into page-locked memory: a pageable destination went through the runtime's staging
    // copy (a blit kernel, then a host memcpy before the stream reports completion)
    std::vector<int> counts((size_t)n_frames * 2);
    c->census.ensure(counts.size() * sizeof(int));
    int* cdst = static_cast<int*>(c->census.p);
    // early census: the halves copied their flags on their own streams and marked them
    // (first_pass_chunk); otherwise one copy on the caller's stream after everything
    if (cen_halves == 0) HIPCHK(hipMemcpyAsync(cdst, res, counts.size() * sizeof(int), hipMemcpyDeviceToHost, s));
    auto ready = [&]() {
        if (cen_halves == 0) return hipStreamQuery(s);
        for (int h = 0; h < cen_halves; ++h) {
            const hipError_t e = hipEventQuery(c->ev_cen[h]);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    };
    // polled rather than a blocking wait: the caller's next batch is enqueued as soon
    // as this one's census is back (a blocking wait's wake-up sat in every bench step,
    // ~17 us per 256-frame step at 1024^2).  The poll yields the core between queries
    // and gives up after 20 ms (a 1024^2 chunk's first pass takes ~3 ms, a 4096^2 one
    // ~6 ms), then blocks.
    constexpr long spin_us = 20000;
    hipError_t qe = hipErrorNotReady;
    {
        const auto t_end = std::chrono::steady_clock::now() + std::chrono::microseconds(spin_us);
        while ((qe = ready()) == hipErrorNotReady && std::chrono::steady_clock::now() < t_end)
            std::this_thread::yield();
    }
    if (qe == hipErrorNotReady) {
        if (cen_halves == 0) {
            qe = hipStreamSynchronize(s);
        } else {
            qe = hipSuccess;
            for (int h = 0; h < cen_halves && qe == hipSuccess; ++h) qe = hipEventSynchronize(c->ev_cen[h]);
        }
    }
    HIPCHK(qe);
    std::memcpy(counts.data(), cdst, counts.size() * sizeof(int));
    std::vector<int> redo;
    for (int f = 0; f < n_frames; ++f)
        if (counts[2 * (size_t)f] || counts[2 * (size_t)f + 1]) redo.push_back(f);
    if (2 * redo.size() >= (size_t)n_frames) c->exact_first = true;  // the next call skips pass 1
    const auto fix_t0 = std::chrono::steady_clock::now();
    struct FixTimer {
        fcd_ctx* c;
        std::chrono::steady_clock::time_point t0;
        size_t n;
        ~FixTimer() {
            if (c->profiling) {
                c->prof_fix_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                c->prof_fix_frames += (long)n;
            }
        }
    } fix_timer{c, fix_t0, redo.size()};
    for (size_t g0 = 0; g0 < redo.size(); g0 += nbmax) {
        const int ng = (int)std::min<size_t>(nbmax, redo.size() - g0);
        const int* gi = redo.data() + g0;
        // a group of consecutive frames (every frame of a batch of camera frames has
        // residues) is read in place and its heights are written in place: no
        // per-frame staging copies, whose host-side enqueueing left the GPU idle
        const bool run = gi[ng - 1] - gi[0] == ng - 1;
        const float* fr;
        if (run && dev && format == FCD_FMT_F32) {
            fr = reinterpret_cast<const float*>(frames) + (size_t)gi[0] * hw;
        } else {
            stage_frames(c, frames, format, dev, gi, ng, s);
            fr = c->frames_in.as<float>();
        }
        fast_demod(c, fr, ng, s);
        int32_t* kf = c->fk.as<int32_t>();
        unwrap_maps(c, c->wrapped.as<float>(), 2 * ng, kf, nullptr, s, true);
        fcdk::int_rows(c->W, 2, c->wrapped.as<float>(), nullptr, kf, nullptr, nullptr, c->H, ng, c->Zt.as<float2>(),
                       c->twp_row.as<float2>(), nullptr, s);
        fcdk::int_cols(c->H, c->Zt.as<float2>(), c->W, ng, coef, c->Ht.as<float2>(), ic_tw(c), s);
        const bool direct = run && dev && height_out;
        float* hdst = direct ? height_out + (size_t)gi[0] * hw : c->out_h.as<float>();
        fcdk::int_c2r(c->W, c->Ht.as<float2>(), c->H, ng, hdst, c->twp_row.as<float2>(), s);
        if (run) {
            if (height_out && !direct)
                HIPCHK(hipMemcpyAsync(height_out + (size_t)gi[0] * hw, hdst, (size_t)ng * hw * 4, out_kind, s));
            if (k_out)
                HIPCHK(hipMemcpyAsync(k_out + (size_t)gi[0] * 2 * hw, kf, (size_t)ng * 2 * hw * 4, out_kind, s));
        } else {
            for (int i = 0; i < ng; ++i) {
                const size_t f = (size_t)gi[i];
                if (height_out)
                    HIPCHK(hipMemcpyAsync(height_out + f * hw, hdst + (size_t)i * hw, hw * 4, out_kind, s));
                if (k_out) HIPCHK(hipMemcpyAsync(k_out + f * 2 * hw, kf + (size_t)i * 2 * hw, 2 * hw * 4, out_kind, s));
            }
        }
        HIPCHK(hipStreamSynchronize(s));
    }
    return FCD_OK;
}

}  // namespace

// Only a device call on a caller stream returns with work still queued: with a null
// stream the work runs on the context's own (non-blocking) stream, which no caller stream
// is ordered with, so the call waits for it before returning (fcd.h).
static int process_entry(fcd_ctx* c, const void* frames, int format, int n_frames, int flags, double height, int unwrap,
                  float* height_out, float* wrapped_out, int32_t* k_out, void* stream) {
    const int rc = process_impl(c, frames, format, n_frames, flags, height, unwrap, height_out, wrapped_out, k_out,
                                stream);
    if (!stream) settle(c);
    return rc;
}

FCD_API int fcd_process(fcd_ctx* c, const float* frames, int n_frames, int flags, double height, int unwrap,
                        float* height_out, float* wrapped_out, int32_t* k_out, void* stream) {
    FCD_TRY(return process_entry(c, frames, FCD_FMT_F32, n_frames, flags, height, unwrap, height_out, wrapped_out,
                                 k_out, stream))
}

FCD_API int fcd_process_raw(fcd_ctx* c, const void* frames, int format, int n_frames, int flags, double height,
                            int unwrap, float* height_out, float* wrapped_out, int32_t* k_out, void* stream) {
    FCD_TRY(return process_entry(c, frames, format, n_frames, flags, height, unwrap, height_out, wrapped_out, k_out,
                                 stream))
}

FCD_API int fcd_frame_bytes(fcd_ctx* c, int format, int64_t* bytes) {
    FCD_TRY({
        check_ctx(c);
        if (!bytes) throw FcdError(FCD_E_INVALID, "bytes is null");
        const size_t b = fcdk::raw_frame_bytes(format, c->H, c->W);
        if (!b) throw FcdError(FCD_E_INVALID, "unknown frame format");
        *bytes = (int64_t)b;
    })
}

FCD_API int fcd_host_alloc(int64_t bytes, void** out) {
    FCD_TRY({
        if (!out || bytes < 0) throw FcdError(FCD_E_INVALID, "bad arguments");
        *out = nullptr;
        HIPCHK(hipHostMalloc(out, (size_t)std::max<int64_t>(bytes, 1), hipHostMallocDefault));
    })
}

FCD_API int fcd_host_free(void* p) {
    FCD_TRY({
        if (p) HIPCHK(hipHostFree(p));
    })
}

FCD_API int fcd_phases_from_spectrum(fcd_ctx* c, const float* spectrum, int n, int flags, int unwrap,
                                     float* wrapped_out, int32_t* k_out, void* stream) {
    FCD_TRY({
        check_ctx(c);
        ensure_aux_buffers(c);
        if (!c->has_ref) throw FcdError(FCD_E_STATE, "no reference set");
        if (!spectrum || n < 0) throw FcdError(FCD_E_INVALID, "bad spectrum");
        hipStream_t s = c->pick(stream);
        const long hw = c->hw();
        const bool dev = flags == FCD_DEVICE_PTRS;
        for (int f0 = 0; f0 < n; f0 += c->chunk) {
            const int nb = std::min(c->chunk, n - f0);
            const float2* sp = reinterpret_cast<const float2*>(spectrum) + (size_t)f0 * hw;
            if (!dev) {
                upload(c->spec.p, sp, (size_t)nb * hw * sizeof(float2), s);
                sp = c->spec.as<float2>();
            }
            float* w = c->wrapped.as<float>();
            demod_phases(c, sp, nb, w, s);
            int32_t* k = nullptr;
            if (unwrap) {
                k = c->kbuf.as<int32_t>();
                unwrap_maps(c, w, 2 * nb, k, nullptr, s);
            }
            const hipMemcpyKind kind = dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
            if (wrapped_out)
                HIPCHK(hipMemcpyAsync(wrapped_out + (size_t)f0 * 2 * hw, w, (size_t)nb * 2 * hw * 4, kind, s));
            if (k_out && k)
                HIPCHK(hipMemcpyAsync(k_out + (size_t)f0 * 2 * hw, k, (size_t)nb * 2 * hw * 4, kind, s));
            else if (k_out && dev)
                HIPCHK(hipMemsetAsync(k_out + (size_t)f0 * 2 * hw, 0, (size_t)nb * 2 * hw * 4, s));
            else if (k_out)
                std::memset(k_out + (size_t)f0 * 2 * hw, 0, (size_t)nb * 2 * hw * 4);
            if (!dev) HIPCHK(hipStreamSynchronize(s));
        }
    })
}

FCD_API int fcd_unwrap(fcd_ctx* c, const float* wrapped, int n_maps, int flags, int32_t* k_out,
                       int32_t* residues_out, void* stream) {
    FCD_TRY({
        check_ctx(c);
        ensure_aux_buffers(c);
        if (!wrapped || !k_out || n_maps < 0) throw FcdError(FCD_E_INVALID, "bad arguments");
        hipStream_t s = c->pick(stream);
        const long hw = c->hw();
        const bool dev = flags == FCD_DEVICE_PTRS;
        const int per = 2 * c->chunk;
        for (int m0 = 0; m0 < n_maps; m0 += per) {
            const int nm = std::min(per, n_maps - m0);
            const float* w = wrapped + (size_t)m0 * hw;
            if (!dev) {
                upload(c->wrapped.p, w, (size_t)nm * hw * 4, s);
                w = c->wrapped.as<float>();
            }
            int32_t* k = dev ? k_out + (size_t)m0 * hw : c->kbuf.as<int32_t>();
            std::vector<int> res(nm);
            unwrap_maps(c, w, nm, k, res.data(), s);
            if (residues_out) std::copy(res.begin(), res.end(), residues_out + m0);
            if (!dev) {
                HIPCHK(hipMemcpyAsync(k_out + (size_t)m0 * hw, k, (size_t)nm * hw * 4, hipMemcpyDeviceToHost, s));
                HIPCHK(hipStreamSynchronize(s));
            }
        }
        HIPCHK(hipStreamSynchronize(s));
    })
}

FCD_API int fcd_integrate(fcd_ctx* c, const float* gx, const float* gy, int n, double cf, int flags, float* h_out,
                          void* stream) {
    FCD_TRY({
        check_ctx(c);
        ensure_aux_buffers(c);
        if (!gx || !gy || !h_out || n < 0) throw FcdError(FCD_E_INVALID, "bad arguments");
        hipStream_t s = c->pick(stream);
        const long hw = c->hw();
        const bool dev = flags == FCD_DEVICE_PTRS;
        ensure_integ_tables(c, cf, s);
        // h_hat = (-i kx gx_hat - i ky gy_hat) / k^2  ->  a0 = -1, b1 = -1
        const fcdk::IntegCoef coef = integ_coef(c, -1.0, 0.0, 0.0, -1.0);
        if (!dev) {
            c->frames_in.ensure((size_t)c->chunk * hw * 4 * 2);
            c->out_h.ensure((size_t)c->chunk * hw * 4);
        }
        for (int f0 = 0; f0 < n; f0 += c->chunk) {
            const int nb = std::min(c->chunk, n - f0);
            const float* x = gx + (size_t)f0 * hw;
            const float* y = gy + (size_t)f0 * hw;
            if (!dev) {
                float* st = c->frames_in.as<float>();
                upload(st, x, (size_t)nb * hw * 4, s);
                upload(st + (size_t)nb * hw, y, (size_t)nb * hw * 4, s);
                x = st;
                y = st + (size_t)nb * hw;
            }
            fcdk::pack_z(x, y, c->spec.as<float2>(), (long)nb * hw, s);
            float* dst = dev ? h_out + (size_t)f0 * hw : c->out_h.as<float>();
            integrate_z(c, nb, coef, dst, s);
            if (!dev) {
                HIPCHK(hipMemcpyAsync(h_out + (size_t)f0 * hw, dst, (size_t)nb * hw * 4, hipMemcpyDeviceToHost, s));
                HIPCHK(hipStreamSynchronize(s));
            }
        }
    })
}

FCD_API int fcd_fft2(fcd_ctx* c, const float* in, int n, int flags, float* out, void* stream) {
    FCD_TRY({
        check_ctx(c);
        if (!in || !out || n < 0) throw FcdError(FCD_E_INVALID, "bad arguments");
        if (flags & ~(FCD_DEVICE_PTRS | FCD_IMG_F64)) throw FcdError(FCD_E_INVALID, "bad flags");
        hipStream_t s = c->pick(stream);
        const long hw = c->hw();
        const bool dev = flags & FCD_DEVICE_PTRS, f64 = flags & FCD_IMG_F64;
        const size_t es = f64 ? sizeof(double) : sizeof(float);
        if (!dev) {
            c->frames_in.ensure((size_t)c->chunk * hw * es);
            c->pk_F.ensure((size_t)c->chunk * hw * 2 * es);
        }
        for (int f0 = 0; f0 < n; f0 += c->chunk) {
            const int nb = std::min(c->chunk, n - f0);
            const void* x = reinterpret_cast<const char*>(in) + (size_t)f0 * hw * es;
            if (!dev) {
                upload(c->frames_in.p, x, (size_t)nb * hw * es, s);
                x = c->frames_in.p;
            }
            void* dst = dev ? reinterpret_cast<char*>(out) + (size_t)f0 * hw * 2 * es : c->pk_F.p;
            exact_fft2(c, x, f64, nb, dst, s);
            if (!dev) {
                HIPCHK(hipMemcpyAsync(reinterpret_cast<char*>(out) + (size_t)f0 * hw * 2 * es, dst,
                                      (size_t)nb * hw * 2 * es, hipMemcpyDeviceToHost, s));
                HIPCHK(hipStreamSynchronize(s));
            }
        }
        if (dev && n > 0) {  // the pocketfft scratch stays in use on the caller's stream: any
            // other entry point (find_peaks / set_reference on c->own reuse it) settles first
            if (!c->ev_done) HIPCHK(hipEventCreateWithFlags(&c->ev_done, hipEventDisableTiming));
            HIPCHK(hipEventRecord(c->ev_done, s));
            c->done_stream = s;
            c->done_pending = true;
        }
    })
}

namespace {

// The block [r0, r0 + bh) x [c0, c0 + bw) of a [T][rows][cols] float32 (or, with
// FCD_STACK_F64 in flags, float64) stack on the device: the caller's own memory
// (device pointers) or a staged copy of just the block (host pointers).  Returns
// the block origin and its pitches in elements.
struct BlockView {
    fcdk::Samples p;
    long frame_pitch, row_pitch;
};

BlockView stage_block(fcd_ctx* c, const void* stack, int T, int rows, int cols, int r0, int c0, int bh, int bw,
                      int flags, hipStream_t s) {
    if (!stack || T <= 0 || rows <= 0 || cols <= 0 || bh <= 0 || bw <= 0 || r0 < 0 || c0 < 0 || r0 + bh > rows ||
        c0 + bw > cols)
        throw FcdError(FCD_E_INVALID, "bad stack / block arguments");
    if (flags & ~(FCD_DEVICE_PTRS | FCD_STACK_F64)) throw FcdError(FCD_E_INVALID, "bad flags");
    const bool dev = flags & FCD_DEVICE_PTRS, f64 = flags & FCD_STACK_F64;
    const size_t es = f64 ? sizeof(double) : sizeof(float);
    const char* src = static_cast<const char*>(stack);
    if (dev) return {{src + ((size_t)r0 * cols + c0) * es, f64}, (long)rows * cols, cols};
    c->t_stage.ensure((size_t)T * bh * bw * es);
    char* d = static_cast<char*>(c->t_stage.p);
    for (int t = 0; t < T; ++t)
        HIPCHK(hipMemcpy2DAsync(d + (size_t)t * bh * bw * es, (size_t)bw * es,
                                src + (((size_t)t * rows + r0) * cols + c0) * es, (size_t)cols * es, (size_t)bw * es,
                                bh, hipMemcpyHostToDevice, s));
    return {{d, f64}, (long)bh * bw, bw};
}

// exp(-2 pi i j / n), j < n, in f64 (the DFT kernels index it by (f t) mod n)
void upload_exp_table(fcd_ctx* c, DevBuf& buf, int n, hipStream_t s) {
    std::vector<double2> tab(n);
    for (int j = 0; j < n; ++j) {
        const double a = -2.0 * kPi * (double)j / (double)n;
        tab[j] = make_double2(std::cos(a), std::sin(a));
    }
    buf.ensure((size_t)n * sizeof(double2));
    upload(buf.p, tab.data(), (size_t)n * sizeof(double2), s);
    HIPCHK(hipStreamSynchronize(s));  // tab dies here
}

}  // namespace

FCD_API int fcd_temporal_spectrum(fcd_ctx* c, const void* stack, int T, int rows, int cols, int r0, int c0, int bh,
                                  int bw, int flags, int nf, double* sum_count, void* stream) {
    FCD_TRY({
        check_ctx(c);
        if (!sum_count || nf <= 0 || nf > T) throw FcdError(FCD_E_INVALID, "bad spectrum arguments");
        hipStream_t s = c->pick(stream);
        const BlockView v = stage_block(c, stack, T, rows, cols, r0, c0, bh, bw, flags, s);
        const int P = bh * bw;
        fcdk::TfftPlan pl;
        int tiles = 1;
        bool fft = fcdk::temporal_spectrum_uses_fft(T, nf) && fcdk::temporal_fft_plan(T, P, &pl);
        if (fft && pl.pair) {
            // per-pixel NaN / infinity flags; a series with an infinity keeps the block on
            // one series per transform (kernels_tfft.hip k_tfft_flags)
            c->t_bad.ensure((size_t)P * sizeof(int) + 64);
            const int ninf = fcdk::temporal_inf_pixels(v.p, v.frame_pitch, v.row_pitch, bw, P, T, c->t_bad.as<int>(),
                                                       c->t_bad.as<int>() + P, s);
            if (ninf > 0) fcdk::temporal_fft_plan(T, P, &pl, false);
        }
        if (fft) {
            // Bluestein + four-step FFT: chirp, twiddles and B = FFT(b) / M from the host in f64
            std::vector<double2> chirp, tw, bhat;
            fcdk::temporal_fft_tables(T, pl, chirp, tw, bhat);
            c->t_tab.ensure(tw.size() * sizeof(double2));
            c->t_chirp.ensure(chirp.size() * sizeof(double2));
            c->t_bhat.ensure(bhat.size() * sizeof(double2));
            c->t_work.ensure((size_t)pl.work_elems * sizeof(double2));
            c->t_gpart.ensure((size_t)pl.ngroups * nf * sizeof(double2));
            if (pl.pair) c->t_zo.ensure((size_t)pl.zo_elems * sizeof(double2));
            c->t_part.ensure((size_t)nf * 2 * sizeof(double));
            upload(c->t_tab.p, tw.data(), tw.size() * sizeof(double2), s);
            upload(c->t_chirp.p, chirp.data(), chirp.size() * sizeof(double2), s);
            upload(c->t_bhat.p, bhat.data(), bhat.size() * sizeof(double2), s);
            const fcdk::TfftWork wk{c->t_work.as<double2>(), pl.pair ? c->t_zo.as<double2>() : nullptr,
                                    c->t_gpart.as<double2>(), pl.pair ? c->t_bad.as<int>() : nullptr};
            fcdk::temporal_spectrum_fft(v.p, v.frame_pitch, v.row_pitch, bw, P, T, nf, pl, c->t_chirp.as<double2>(),
                                        c->t_tab.as<double2>(), c->t_bhat.as<double2>(), wk, c->t_part.as<double>(), s);
            HIPCHK(hipStreamSynchronize(s));  // the host tables die here
        } else {
            upload_exp_table(c, c->t_tab, T, s);
            tiles = fcdk::temporal_spectrum_tiles(P, T);
            c->t_part.ensure((size_t)tiles * nf * 2 * sizeof(double));
            fcdk::temporal_dft(v.p, v.frame_pitch, v.row_pitch, bw, P, T, c->t_tab.as<double2>(), nullptr, nf,
                               nullptr, c->t_part.as<double>(), nullptr, s);
        }
        std::vector<double> part((size_t)tiles * nf * 2);
        HIPCHK(hipMemcpyAsync(part.data(), c->t_part.p, part.size() * sizeof(double), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        for (int f = 0; f < nf; ++f) {  // fixed-order sum over the pixel tiles (deterministic)
            double a = 0.0, n = 0.0;
            for (int i = 0; i < tiles; ++i) {
                a += part[((size_t)i * nf + f) * 2];
                n += part[((size_t)i * nf + f) * 2 + 1];
            }
            sum_count[2 * f] = a;
            sum_count[2 * f + 1] = n;
        }
    })
}

FCD_API int fcd_temporal_bins(fcd_ctx* c, const void* stack, int T, int rows, int cols, int r0, int c0, int bh,
                              int bw, int flags, const int* bins, int nbins, double* x_out, void* stream) {
    FCD_TRY({
        check_ctx(c);
        if (!bins || !x_out || nbins <= 0) throw FcdError(FCD_E_INVALID, "bad bins arguments");
        for (int i = 0; i < nbins; ++i)
            if (bins[i] < 0 || bins[i] >= T) throw FcdError(FCD_E_INVALID, "bin out of range");
        hipStream_t s = c->pick(stream);
        const bool dev = flags & FCD_DEVICE_PTRS;
        const BlockView v = stage_block(c, stack, T, rows, cols, r0, c0, bh, bw, flags, s);
        upload_exp_table(c, c->t_tab, T, s);
        c->t_bins.ensure((size_t)nbins * sizeof(int));
        upload(c->t_bins.p, bins, (size_t)nbins * sizeof(int), s);
        const int P = bh * bw;
        double2* out = reinterpret_cast<double2*>(x_out);
        if (!dev) {
            c->t_out.ensure((size_t)P * nbins * sizeof(double2));
            out = c->t_out.as<double2>();
        }
        const int nz = fcdk::temporal_bins_slices(P, nbins, T);
        if (nz > 1) c->t_slices.ensure((size_t)nz * P * nbins * sizeof(double2));
        fcdk::temporal_dft(v.p, v.frame_pitch, v.row_pitch, bw, P, T, c->t_tab.as<double2>(), c->t_bins.as<int>(),
                           nbins, out, nullptr, nz > 1 ? c->t_slices.as<double2>() : nullptr, s);
        if (!dev) {
            HIPCHK(hipMemcpyAsync(x_out, out, (size_t)P * nbins * sizeof(double2), hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
        } else {
            HIPCHK(hipStreamSynchronize(s));  // the bins buffer is reused by the next call
        }
    })
}

FCD_API int fcd_spectrogram(fcd_ctx* c, const void* stack, int T, int rows, int cols, int r0, int c0, int bh, int bw,
                            int flags, int nperseg, int noverlap, const double* window, double fs, double* s_out,
                            void* stream) {
    FCD_TRY({
        check_ctx(c);
        if (!window || !s_out || nperseg < 1 || nperseg > T || noverlap < 0 || noverlap >= nperseg || !(fs > 0))
            throw FcdError(FCD_E_INVALID, "bad spectrogram arguments");
        if (nperseg > fcdk::spectro_max_nperseg()) throw FcdError(FCD_E_UNSUPPORTED, "nperseg too large");
        hipStream_t s = c->pick(stream);
        const bool dev = flags & FCD_DEVICE_PTRS;
        const BlockView v = stage_block(c, stack, T, rows, cols, r0, c0, bh, bw, flags, s);
        const int step = nperseg - noverlap, nseg = (T - nperseg) / step + 1, nf = nperseg / 2 + 1;
        // window, its DFT W_f (the mean-removal term) and the density scale, in f64
        std::vector<double2> tab(nperseg), wsum(nf);
        double w2 = 0.0;
        for (int j = 0; j < nperseg; ++j) {
            const double a = -2.0 * kPi * (double)j / (double)nperseg;
            tab[j] = make_double2(std::cos(a), std::sin(a));
            w2 += window[j] * window[j];
        }
        for (int f = 0; f < nf; ++f) {
            double re = 0.0, im = 0.0;
            for (int n = 0; n < nperseg; ++n) {
                const double2 e = tab[(size_t)((long)f * n % nperseg)];
                re += window[n] * e.x;
                im += window[n] * e.y;
            }
            wsum[f] = make_double2(re, im);
        }
        c->t_tab.ensure((size_t)nperseg * sizeof(double2));
        c->t_win.ensure((size_t)nperseg * sizeof(double));
        c->t_wsum.ensure((size_t)nf * sizeof(double2));
        upload(c->t_tab.p, tab.data(), (size_t)nperseg * sizeof(double2), s);
        upload(c->t_win.p, window, (size_t)nperseg * sizeof(double), s);
        upload(c->t_wsum.p, wsum.data(), (size_t)nf * sizeof(double2), s);
        const int P = bh * bw;
        double* out = s_out;
        if (!dev) {
            c->t_out.ensure((size_t)P * nf * nseg * sizeof(double));
            out = c->t_out.as<double>();
        }
        fcdk::spectrogram(v.p, v.frame_pitch, v.row_pitch, bw, P, nperseg, step, nseg, c->t_win.as<double>(),
                          c->t_tab.as<double2>(), c->t_wsum.as<double2>(), nf, 1.0 / (fs * w2), out, s);
        if (!dev)
            HIPCHK(hipMemcpyAsync(s_out, out, (size_t)P * nf * nseg * sizeof(double), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));  // host vectors die here
    })
}

FCD_API int fcd_profile(fcd_ctx* c, int enable) {
    FCD_TRY({
        check_ctx(c);
        HIPCHK(hipStreamSynchronize(c->own));
        c->profiling = enable != 0;
        c->ev_used = 0;
        c->prof_frames = 0;
    })
}

FCD_API int fcd_stage_times(fcd_ctx* c, double* out4, int64_t* frames) {
    FCD_TRY({
        check_ctx(c);
        if (!out4) throw FcdError(FCD_E_INVALID, "out8 is null");
        for (int i = 0; i < 4; ++i) out4[i] = 0;
        out4[4] = c->prof_fix_ms;
        out4[5] = (double)c->prof_fix_frames;
        out4[6] = (double)(c->ev_used / 4);  // launch groups (chunks) covered
        out4[7] = (double)c->fchunk;         // frames per launch group
        c->prof_fix_ms = 0;
        c->prof_fix_frames = 0;
        if (c->ev_used) HIPCHK(hipEventSynchronize(c->ev_pool[c->ev_used - 1]));
        for (size_t q = 0; q + 3 < c->ev_used; q += 4) {
            float ms[3];
            for (int i = 0; i < 3; ++i) HIPCHK(hipEventElapsedTime(&ms[i], c->ev_pool[q + i], c->ev_pool[q + i + 1]));
            for (int i = 0; i < 3; ++i) out4[i] += ms[i];
            out4[3] += (double)ms[0] + ms[1] + ms[2];
        }
        if (frames) *frames = c->prof_frames;
        c->ev_used = 0;
        c->prof_frames = 0;
    })
}
