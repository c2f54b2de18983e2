// Launch wrappers for the FCD HIP kernels (gfx950).  Host-callable; every
// wrapper is asynchronous on the given stream and dispatches on the
// power-of-two transform length at run time.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdlib>
#include <vector>

#include "pocketfft.hpp"  // pf::Plan

namespace fcdk {

// the current device's CU count, cached once per process (kernels_fast.hip)
int device_cu_count();

// Row-FFT input / output modes.
// ROW_IN_Z (mr_rows only): z = (w0 + 2 pi k0) + i (w1 + 2 pi k1) of the two maps' rows, in =
// wrapped [nb][2][H][W], PhaseOut::kin the k-fields (null: none), as make_z
// ROW_IN_BAND (mr_rows only): row (b, i) of the band columns held transposed, in = [nb][bnc][H]
// complex, column j = in[b][bslot[j]][i] (bslot[j] < 0: zero)
// ROW_IN_REAL2 / ROW_IN_COMPLEX2 (mr_rows only, with ROW_OUT_BAND2 / ROW_OUT_REAL2): rows 2p and
// 2p + 1 of a frame (nrows a multiple of H; an odd H's last row alone) in one complex
// transform -- two real rows as re + i im (their spectra split by Hermitian symmetry), or
// the real parts of two rows' inverses as those of ifft(Herm(A) + i Herm(B)),
// Herm(Y)(k) = (Y(k) + conj Y(-k)) / 2
enum RowIn { ROW_IN_COMPLEX = 0, ROW_IN_REAL = 1, ROW_IN_Z = 2, ROW_IN_BAND = 3, ROW_IN_REAL2 = 4, ROW_IN_COMPLEX2 = 5 };
// ROW_OUT_BAND2 (mr_rows only): the band columns of each row, out = [nrows][bnc] complex,
// column j to slot bslot[j] (bslot[j] < 0: not stored)
enum RowOut { ROW_OUT_COMPLEX = 0, ROW_OUT_REAL = 1, ROW_OUT_PHASE = 2, ROW_OUT_BAND2 = 4, ROW_OUT_REAL2 = 5 };

struct PhaseOut {          // ROW_OUT_PHASE: w = wrap(theta - atan2(A))
    const float* theta;    // [H][W] reference angle of this carrier
    float* wrapped;        // output base; row r of batch b -> wrapped + ((b*2 + carrier)*H + r)*W
    int carrier;
    const int32_t* kin = nullptr;  // ROW_IN_Z's k-fields
    const int* bslot = nullptr;    // ROW_IN_BAND's / ROW_OUT_BAND2's column slots [W] and their count
    int bnc = 0;
    // ROW_IN_Z with kflag: map m takes kin where kflag[m] != 0 (its MST k-field), else its
    // residue-free scan k(i, j) = colk[m][i] - sum_{j' < j} find_wrap(w(i, j'), w(i, j' + 1)),
    // computed in the row's load (k_rowscan's integers)
    const int* kflag = nullptr;
    const int* colk = nullptr;
};

// Disk band-pass of one carrier (skimage.draw.disk raster in fftshifted
// coordinates): per shifted column sc the inclusive shifted-row range
// [rows[2*sc], rows[2*sc+1]] inside the disk (empty when lo > hi).
struct DiskTable {
    const int* rows;       // device, length 2*W
};

// Integration multipliers: h_hat = i*((kxe*a0 + kye*b0)*Phi0 + (kxe*a1 + kye*b1)*Phi1)/k2 * norm
struct IntegCoef {
    const float* kxe;      // [W] odd-symmetrised column wavenumbers
    const float* kye;      // [H] odd-symmetrised row wavenumbers
    const float* kx2;      // [W] unmodified column wavenumber squared
    const float* ky2;      // [H]
    float a0, b0, a1, b1, norm;
};

// Band-pruned demodulation tables (built once per reference on the host).
struct DemodTables {
    const int* hc;         // [NC] half-spectrum columns (0..W/2) the carrier disks need
    const int4* outs;      // [NC][4] (carrier, cslot, mirror, unshifted column) per output column
    const int2* outrows;   // [NC][4] shifted-row range [lo, hi] of the disk in that column
    const int* nouts;      // [NC] outputs per half column (<= 4)
    const int* colslot;    // [2][W] carrier column slot of each unshifted column, or -1
    int NC;
    int NCc[2];
};

// Zt (row spectra of phi0 + i phi1) tile height at W <= 1024: every column
// segment of a tile is one run of FCD_ZT_1024 * 8 bytes (shared by the fused
// kernel's write-out, k_int_rows2 and the column kernels).  16 rows: a run is one
// 128-byte line, so k_int_cols reads each line once (8 rows: two columns per line,
// 1.45x the compulsory reads, PMC r04e; 1.00x with 16, r04n, same step time).
#ifndef FCD_ZT_1024
#define FCD_ZT_1024 16
#endif
// Zt layout tile at 4096-point rows (rows per column run; k_int_rows2 holds 4 rows per
// tile in LDS, the fused wide kernel 2).  16 makes k_int_cols read whole 128-byte lines
// (1.37x -> 1.00x the compulsory reads, int_cols + c2r 123.6 -> 107.7 us/frame), but the
// fused wide kernel then writes 16-byte pieces of 8-tile runs: plain stores read every
// line back (152.9 -> 202.7 us/frame), streaming ones crawl (396.9); c5 3.14k -> 2.83k /
// 1.78k frames/s (r04q / r04r).  With 4 the fused kernel's 2-row tiles write half runs
// (PMC: 2.08x the Zt bytes written).  2 (the fused tile writes whole layout tiles, one
// contiguous 64 KB region; k_int_cols reads 16-byte runs in groups of 8 blocks on one XCD
// taking a line's 8 columns together): fused 152.8 -> 144.6 us/frame but int_cols + c2r
// 124.2 -> 147.3, c5 3.13k -> 2.98k frames/s (r05).  So 4.
#ifndef FCD_ZT_4096
#define FCD_ZT_4096 4
#endif
// Zt layout: rows per column run at row length W
__host__ __device__ constexpr int zt_layout(int W) { return W <= 1024 ? FCD_ZT_1024 : (W == 2048 ? 8 : FCD_ZT_4096); }
// Zt keeps the natural column order inside a tile.  (A mirror-paired order, every
// column next to its Hermitian mirror so that a 128-byte line is exactly the pair one
// k_int_cols item reads, cut Zt reads by 30 % but measured slower: kbench r03k1, int_cols
// 3.02 vs 2.86, int_rows 4.47 vs 4.33, phase_rows 5.92 vs 5.86 us/frame)
bool fft_size_supported(int n);
// frame ingest (kernels_ingest.hip): raw samples (FCD_FMT_*) -> float32 frames
size_t raw_frame_bytes(int format, int H, int W);
void ingest(int format, const void* raw, int nframes, int H, int W, float* out, hipStream_t s);
// float64 -> float32, rounded to nearest (numpy astype)
void convert_f64(const double* in, long n, float* out, hipStream_t s);

// ---- band-pruned per-frame pipeline (kernels_fast.hip) ----
void demod_rows(int W, const float* frames, int H, int nb, const DemodTables& T, float2* Xb, const float2* tw,
                hipStream_t s);
void demod_cols(int H, const float2* Xb, int nb, const DemodTables& T, float2* Ab, int NCA, const float2* tw,
                hipStream_t s);
void demod_phase(int W, const float2* Ab, int H, int nb, int NCA, const DemodTables& T, const float* theta,
                 float* wrapped, const float2* tw, hipStream_t s);
// seam: kmode 1's buffer of the tile ranges' first / last unwrapped rows
// (int_rows_seam_bytes(W, H, nb) bytes; may be null for kmodes 0 and 2)
void int_rows(int W, int kmode, const float* w, const int* colk, const int32_t* kin, int32_t* kout, int* rescount,
              int H, int nb, float2* Zt, const float2* tw, float2* seam, hipStream_t s,
              const struct MstK* mk = nullptr);
size_t int_rows_seam_bytes(int W, int H, int nb);
struct IntegCoef;
// colk (nullable): per (frame, map, row) column-0 unwrap offsets still to be
// added (the fused path adds 2 pi W (colk0 + i colk1) to each row's DC bin).
void int_cols(int H, const float2* Zt, int W, int nb, const IntegCoef& c, float2* Ht, const float2* tw,
              hipStream_t s, const int* colk = nullptr);
void int_c2r(int W, const float2* Ht, int H, int nb, float* h, const float2* tw, hipStream_t s);
int c2r_rows_per_block(int W);
// band-pruned inverse row transform + phase (kernels_band.hip): B-point window
// of the carrier band, W/B pre-twiddled group transforms per row.
// theta [rows][W] (band_phase REF output) -> the lane-contiguous copy that
// band_phase (REF = false) and phase_rows read as their `theta`
void band_theta_lanes(int W, int B, const float* theta, int rows, float* thp, hipStream_t s);
bool band_supported(int W, int B);
void band_phase_fold(int W, const float2* Ab, int H, int nb, int NCA, int ncc0, int ncc1, const float* theta,
                     float* out, const float2* pre, const float2* ptw, hipStream_t s);
void band_phase(int W, int B, bool ref, const float2* Ab, int H, int nb, int NCA, int ncc0, int ncc1,
                const float* theta, float* out, const float2* pre, const float2* ptw, hipStream_t s);
// column-0 prefix of the residue-free unwrap (kernels_unwrap.hip)
void unwrap_colk(const float* w, int nmaps, int H, int W, int* colk, hipStream_t s);
// the same over compact column-0 values col0[map][H] (the fused path's side output)
void unwrap_colk_compact(const float* col0, int nmaps, int H, int* colk, hipStream_t s);
// fused band transform + phase + unwrap + z-row FFT (kernels_phase_rows.hip)
// W = 1024 (B = 128), 2048 (B = 256) and 4096 (B = 512; kernels_phase_rows_wide.hip).  ztw:
// group_twiddles(W) at 1024; wider: the 1024-point table followed by the join twiddles
// exp(-2 pi i h k / W), h = 1 .. W/1024 - 1, k < 1024.
bool phase_rows_supported(int W, int B, int H);
int phase_rows_tile(int W);  // rows per fused tile (seam buffer: nb * H / tile * 2 * W float2)
// defer_seam: the census of the edges between the blocks' tile ranges is left to a
// later phase_rows_seam on the same stream (its flags are read only at the end of the
// call, so the headline chain launches it after the integration kernels).
void phase_rows(int W, bool unwrap, const float2* Ab, int H, int nb, int NCA, int ncc0, int ncc1, const float* theta,
                const float2* pre, const float2* ptw, const float2* ztw, float* col0, int* flags, float2* Zt,
                float2* seam, hipStream_t s, bool defer_seam = false);
void phase_rows_seam(int W, int H, int nb, const float2* seam, int* flags, hipStream_t s);

// In-place or out-of-place batched row FFT over nrows rows of length W.
void row_fft(int W, bool inverse, RowIn in_mode, RowOut out_mode, const void* in, void* out, long nrows,
             int H, float sub, const float2* tw, const PhaseOut* ph, hipStream_t s);
// In-place batched column FFT of nbatch [H][W] complex arrays.
void col_fft(int H, int W, bool inverse, float2* data, int nbatch, const float2* tw, hipStream_t s);
// Mixed-radix row / column transforms (kernels_mr.hip) of the generic chain for sides that
// are not powers of two: radix 8 / 4 / 2 / 3 / 5 / 7 codelets, a generic pass for odd
// primes <= kMrMaxRadix, Bluestein (power-of-two M) otherwise.  Any side in [2, kMrMaxLen]
// (rows beyond 8192 complex in global scratch).
constexpr int kMrMaxRadix = 61;
constexpr int kMrMaxLen = 16384;  // longest side of the generic chain
struct MrPlan {
    int n, nf;
    int fct[24];  // radices in pass order (of n; of M with Bluestein)
    int blue, M;  // Bluestein: convolution length
    int tM, tc, tgf, tgi;  // offsets into the table of mr_tables (Bluestein)
};
bool mr_supported(int n);
MrPlan mr_plan(int n);
// the plan's table: exp(-2 pi i m / n), m < n, then (Bluestein) the M-point table, the chirp
// and the convolution kernels' spectra
std::vector<float2> mr_tables(const MrPlan& p);
// as row_fft (same modes; tw: mr_tables(p) on the device)
// gs: the caller's global scratch of mr_long_scratch_bytes(p) bytes (rows longer than the
// LDS holds; null when that is 0) -- per context, so contexts on one device never share it
void mr_rows(const MrPlan& p, bool inverse, RowIn in_mode, RowOut out_mode, const void* in, void* out, long nrows,
             int H, float sub, const float2* tw, const PhaseOut* ph, hipStream_t s, float2* gs);
size_t mr_long_scratch_bytes(const MrPlan& p);
// [nb][R][C] -> [nb][C][R]
void mr_transpose(const float2* in, float2* out, int nb, int R, int C, hipStream_t s);
// column subset: [nb][R][C] -> [nb][NS][R] (columns cols[])
void mr_gather_cols(const float2* in, float2* out, int nb, int R, int C, const int* cols, int NS, hipStream_t s);
// The spectral integration's column stage of the generic chain, in place on Z [nb][p.n][W]
// (the row spectra of phi0 + i phi1): per workgroup a run of columns in LDS, forward column
// transforms, the multiplier (m1 + i m0) Z -- integ_multiply's h_hat up to its real part
// after the inverse, which ROW_IN_COMPLEX2 takes --, inverse column transforms: no
// transposes, one read and one write of Z.
// (column lengths whose plan has radices <= 8 only, mr_int_cols_supported)
bool mr_int_cols_supported(const MrPlan& p);
void mr_int_cols(const MrPlan& p, float2* Z, int nb, int W, const float2* tw, const IntegCoef& c, hipStream_t s);
// in-place column transforms of [nb][p.n][W] (through scratch: nb * p.n * W complex)
void mr_cols(const MrPlan& p, int W, bool inverse, float2* data, int nb, const float2* tw, float2* scratch,
             hipStream_t s, float2* gs);

// out[b] = in[b] * disk (unshifted spectrum index)
// the generic chain's band columns: out[b][k][i] = spec_t[b][uslot[k]][i] inside carrier's disk
// at unshifted column cols[k], else 0 (spec_t: [nb][NU][H] transposed band spectra)
void disk_band_t(const float2* spec_t, float2* out, int nbatch, int H, int W, int NU, const int* cols,
                 const int* uslot, int nc, DiskTable t, hipStream_t s);
// transposed: in / out column-major per image ([b][j][i]: the generic chain's transposed spectra)
void disk_mask(const float2* in, float2* out, int nbatch, int H, int W, DiskTable t, hipStream_t s, bool transposed = false);
// theta = atan2(R)  (reference carrier angle)
void angle(const float2* in, float* out, long n, hipStream_t s);
// Batched reference setup (fourier.find_peaks for nb images): |F| (np.abs's formula for
// complex64 / complex128) * highpass per image with its maximum (as unsigned bits of the
// float / double, zero-extended) and the above-threshold candidates (cap per image,
// border excluded); 8-connected labelling and the 4 dimmest blobs' peaks per image for
// float32 spectra (res: 8 ints per image, see kernels_fft.hip).
void spectrum_candidates_b(const void* F, bool f64, int nb, int H, int W, const double* krow_s, const double* kcol_s,
                           double kmin2, void* mag, unsigned long long* maxbits, int* count, int* idx, void* val,
                           long cap, hipStream_t s);
void label_peaks(const int* counts, const int* idx, const float* val, long cap, int nb, int H, int W, int* res,
                 hipStream_t s);
// The reference's spectrum bit for bit (kernels_pocketfft.hip, pocketfft.hpp): numpy's
// mean and centring, scipy 1.7.1 pocketfft's fft2 of real images of any shape, float32
// or float64 (f64).  Plans and tables from pf::make_plan (rows real, columns complex).
int pf_chunk_count(long hw);  // sums: nb * pf_chunk_count(hw) elements
// global scratch the transforms need when a row's / column's buffers exceed LDS
size_t pf_scratch_bytes(const pf::Plan& rows, const pf::Plan& cols, bool f64);
void pf_center(const void* img, bool f64, int nb, long hw, void* sums, void* out, hipStream_t s);
void pf_fft2(const void* in, bool f64, int nb, int H, int W, const pf::Plan& rows, const void* rtab, const pf::Plan& cols,
             const void* ctab, void* F, void* scratch, hipStream_t s);

// kernels_phase_rows_wide.hip: the fused kernel at 2048- and 4096-point rows, and its
// REF mode (4096: the reference's band angles into theta_b, [2][H][W])
void phase_rows_wide(int W, bool unwrap, const float2* Ab, int H, int nb, int NCA, int ncc0, int ncc1, const float* theta,
                     const float2* pre, const float2* ptw, const float2* ztw, float* col0, int* flags, float2* Zt,
                     float2* seam, hipStream_t s, bool defer_seam = false);
void phase_rows_wide_seam(int W, int H, int nb, const float2* seam, int* flags, hipStream_t s);
void phase_rows_wide_ref(int W, const float2* Ab, int H, int NCA, int ncc0, int ncc1, const float2* pre,
                         const float2* ptw, float* theta_b, hipStream_t s);
int phase_rows_wide_bt(int W);  // its band group transform length (the window, or half of it folded)

// ---- unwrap ----
// counts[m] = residues of map m; any_only: counts[m] > 0 iff map m has residues (blocks of
// an already-counted map skip their strips)
void residues(const float* w, int nmaps, int H, int W, int* counts, hipStream_t s, bool any_only = false);
void unwrap_scan(const float* w, int nmaps, int H, int W, int* colk, int32_t* k, hipStream_t s);
// frames whose sides are not multiples of 64: unwrapped in a copy padded to Hp x Wp by
// replicating the last row / column (kernels_unwrap.hip), k copied back
// ids (nullable): padded map m is map ids[m] of w / k
void pad_maps(const float* w, int nmaps, int H, int W, int Hp, int Wp, float* out, hipStream_t s,
              const int* ids = nullptr);
void unpad_k(const int32_t* kp, int nmaps, int Hp, int Wp, int H, int W, int32_t* k, hipStream_t s,
             const int* ids = nullptr);

// The component-graph path's tile geometry: level-0 component of pixel v (vertex id slot *
// H * W + pixel) = tile_of(v) * ccap + crank[v]
struct CgGeom {
    int W, tw, th, tiles_x, tiles, ccap;
    long hw;
    __host__ __device__ __forceinline__ int tile_of(long v) const {
        const int slot = (int)(v / hw), p = (int)(v % hw);
        return slot * tiles + (p / W) / th * tiles_x + (p % W) / tw;
    }
};
// k of the maps the component-graph MST unwrapped, read where it is used (k_int_rows2
// kmode 3) instead of a k-field pass: k(v) = offk[comp(v)] + coff[v] - (the same at the
// map's pixel 0); map_slot[map] = its MST slot or -1 (then k comes from kin)
struct MstK {
    const unsigned char* crank;
    const short* coff;
    const int* offk;
    const int* map_slot;
    CgGeom geo;
};
struct MstWork {
    int* comp; int* off; double* rel; double* cand_w; int* cand_e;
    unsigned long long* best_w; int* best_e; unsigned long long* link; int* nhooks;
    // two-level rounds (mst_level_*): per level-0 root its current root and
    // offset; boundary-pixel lists (ping-pong), current-root lists (ping-pong),
    // the level-0 root list, all segmented by block; cnt: mst_level_counts() ints
    int* rootof; int* offk; int* listB[2]; int* listR[2]; int* listL0; int* cnt;
    unsigned char* maskB[2];  // per boundary entry: its neighbours still outside its component
    // component-graph rounds (mst_cg_round): per tile its level-0 component count and
    // contracted-edge count, the edge records (SoA) in per-tile segments; nhooks[1]:
    // set if a tile's graph did not fit (never, by the planar bound; the host falls back);
    // nhooks[2 + r]: hooks in graph round r (r < kCgRounds; zeroed once per MST pass, so
    // the rounds need no per-round reset)
    int* cg_ncomp; int* cg_ecnt; int* cg_ea; int* cg_eb; unsigned long long* cg_ew; int* cg_ec; int* cg_ed;
    // per tile its column-0 pixels' labels, row by row (rank | offset << 16): the far ends
    // of the edges into a tile from its left neighbour, read as one run instead of one
    // cache line per row of crank / coff
    unsigned* cg_lcol;
    // the component-graph path's level-0 labels, compact (aliases of comp / off): per pixel
    // its component's rank in its tile (< cg_ccap <= 256) and K(pixel) - K(component)
    unsigned char* crank; short* coff;
    // the frame's own size when the maps were padded to multiples of 64 (fcd_engine.cpp
    // unwrap_maps): the reference's border reliabilities lie on rows / columns 0 and Hr - 1
    // / Wr - 1, and every pad pixel gets kPadRel, so every edge touching a pad pixel is
    // heavier than every edge of the frame and the frame's MST is the padded graph's
    // restricted to the frame (the k-field of the frame's pixels is unchanged)
    int Hr, Wr;
    // the layout the tile pass loads the wrapped phases from: the maps as given (Hs x Ws =
    // the unwrap's H x W), or (the generic chain's level-3 pass) the frame's own maps,
    // Hr x Wr, whose clamped loads replicate the last row / column exactly as the padded
    // copy does
    int Hs, Ws;
};
constexpr double kPadRel = 1e300;
// Maps listed in map_ids (device int[nact]) of the wrapped stack w.
void mst_init(const float* w, const int* map_ids, int nact, int H, int W, MstWork m, hipStream_t s);
// first: the round right after mst_init (every component a single vertex)
void mst_round(const float* w, const int* map_ids, int nact, int H, int W, MstWork m, hipStream_t s, bool first = false);
void mst_finalize(const int* map_ids, int nact, int H, int W, MstWork m, int32_t* k, hipStream_t s);
// Two-level Boruvka: after mst_init + one mst_round(first) every pixel has a
// level-0 component; mst_level_setup lists the level-0 roots and the pixels on
// a component boundary, and every later round walks only those lists
// (round r reads list parity r & 1).  mst_level_finalize writes k.
int mst_level_counts();
// Level-0 components from Boruvka inside each 32 x 32 tile (LDS), with the
// reliabilities; replaces mst_init + the first pixel round before mst_level_setup.
int mst_tile_shape(int H, int W, int* th);  // tile width (64 / 32) and height, 0: no tile pass
// graph: write the tile's contracted component graph for mst_cg_round instead of the
// per-pixel state of the boundary-list rounds (mst_level_setup / mst_level_round).
void mst_tile_level0(const float* w, const int* map_ids, int nact, int H, int W, MstWork m, hipStream_t s,
                     bool graph = false);
long mst_cg_edge_capacity(long nv);  // edge records for nv vertices (any tile side)
// Round r of the component-graph Boruvka (r = 0: the candidates come from the tile pass; its
// hooks resolve the cross-tile edges).
constexpr int kCgRounds = 72;
void mst_cg_round(int nact, int H, int W, MstWork m, int r, hipStream_t s);
// k of the component-graph path (every level-0 component's offk final)
// frame_layout: k is the frame's own layout (maps of m.Hr x m.Wr, map_ids index it), the
// pad pixels dropped; else the unwrap's H x W layout
void mst_cg_finalize(const int* map_ids, int nact, int H, int W, MstWork m, int32_t* k, hipStream_t s,
                     bool frame_layout = false);
CgGeom mst_cg_geom(int H, int W);
void mst_level_setup(int nact, int H, int W, MstWork m, hipStream_t s);
void mst_level_round(const float* w, const int* map_ids, int nact, int H, int W, MstWork m, int r, hipStream_t s);
void mst_level_finalize(const int* map_ids, int nact, int H, int W, MstWork m, int32_t* k, hipStream_t s);

// ---- integration ----
// z = (w0 + 2pi k0) + i (w1 + 2pi k1)   (k may be null)
void make_z(const float* w, const int32_t* k, float2* z, int nbatch, int H, int W, hipStream_t s);
// z = gx + i gy
void pack_z(const float* gx, const float* gy, float2* z, long n, hipStream_t s);
void integ_multiply(const float2* Z, float2* Hh, int nbatch, int H, int W, IntegCoef c, hipStream_t s,
                    bool transposed = false);
// phases f32 = w + 2pi k
void compose_phase(const float* w, const int32_t* k, float* out, long n, hipStream_t s);

// temporal analysis of a map stack (kernels_temporal.hip): samples float32 or
// float64 (the reference keeps a float64 series in float64)
struct Samples {
    const void* p;
    bool f64;
};
void temporal_dft(Samples stack, long frame_pitch, long row_pitch, int bw, int P, int T, const double2* tab,
                  const int* freqs, int nf, double2* out, double* partial, double2* slices, hipStream_t s);
int temporal_dft_tiles(int P);
int temporal_spectrum_tiles(int P, int T);  // partial-sum rows of a mean-spectrum call
int temporal_bins_slices(int P, int nf, int T);  // slices[slices][P][nf] workspace of a bins call
int spectro_max_nperseg();
// mean spectrum of a long series by Bluestein + four-step FFT (kernels_tfft.hip)
struct TfftPlan {
    int logM, M, log1, log2, M1, M2;  // M = 2^logM >= 2T - 1 = M1 x M2
    int Pb, ngroups;                  // pixels per batch, partial-sum rows (64 or 128 pixels each)
    bool pair;                        // two real series per transform (x_p + i x_q)
    long work_elems, zo_elems;        // double2 workspace sizes
};
struct TfftWork {
    double2* work;   // [work_elems]
    double2* zo;     // [zo_elems] (pair)
    double2* gpart;  // [ngroups][nf]
    int* bad;        // [P] (pair): pixel has a non-finite sample
};
bool temporal_spectrum_uses_fft(int T, int nf);
// allow_pair = false: one series per transform (a block with an infinity in some series)
bool temporal_fft_plan(int T, int P, TfftPlan* pl, bool allow_pair = true);  // false: T too long
// bad[P] per-pixel flags (1 NaN, 2 infinity) of the block; returns the pixels with an
// infinity and no NaN.  Synchronises.
int temporal_inf_pixels(Samples stack, long frame_pitch, long row_pitch, int bw, int P, int T, int* bad, int* count,
                        hipStream_t s);
void temporal_fft_tables(int T, const TfftPlan& pl, std::vector<double2>& chirp, std::vector<double2>& tw,
                         std::vector<double2>& bhat);
// partial [nf][2] (sum of |X|, count) over the block
void temporal_spectrum_fft(Samples stack, long frame_pitch, long row_pitch, int bw, int P, int T, int nf,
                           const TfftPlan& pl, const double2* chirp, const double2* tw, const double2* bhat,
                           const TfftWork& wk, double* partial, hipStream_t s);
void spectrogram(Samples stack, long frame_pitch, long row_pitch, int bw, int P, int nperseg, int step, int nseg,
                 const double* win, const double2* tab, const double2* wsum, int nf, double scale, double* out,
                 hipStream_t s);

}  // namespace fcdk
