// Phase unwrapping on the device: the reference's
//   phases[i] = unwrap_phase(phase_angles)        /root/reference/pyfcd/fcd.py:119
// (scikit-image 0.18.3, Herraez et al. 2002; restated in oracle/herraez_unwrap.c).
//
// Herraez's greedy merge over edges sorted by reliability accepts exactly the
// edges of the unique minimum spanning tree under the total order
// (reliability, edge index), and the result is w + 2*pi*k with k integrated
// along that tree (k2 - k1 = -find_wrap(w1, w2) across every tree edge),
// up to one global constant.  Two device paths produce that k-field:
//
//  * residue-free maps (no plaquette with non-zero wrap-count circulation):
//    every path integrates to the same k, so a column-0 prefix scan plus a
//    per-row prefix scan (one wave per row) gives it exactly;
//  * maps with residues: Boruvka MST on the 4-connected pixel grid with the
//    reference's f64 reliabilities and edge-index tie-break, carrying each
//    vertex's k-offset to its component root through every hook and pointer
//    jump, so the tree integration falls out of the MST construction itself.
//
// Both normalise k(0, 0) = 0 (the reference's constant depends on its merge
// history).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <algorithm>
#include <stdexcept>
#include <string>

#include "kernels.hpp"

namespace fcdk {

#define FCD_HIPCHK(x)                                                               \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) throw std::runtime_error(std::string(#x ": ") + hipGetErrorString(e_)); \
    } while (0)
#define FCD_CHECK_LAUNCH()                                                          \
    do {                                                                            \
        hipError_t e_ = hipGetLastError();                                          \
        if (e_ != hipSuccess) throw std::runtime_error(std::string("kernel launch: ") + hipGetErrorString(e_)); \
    } while (0)

constexpr double kPi = 3.141592653589793;      // skimage unwrap's PI (probed: double M_PI)
constexpr double kTwoPi = 6.283185307179586;
constexpr double kBorderRel = 9999999.0;
#ifndef FCD_T0_REL_UNROLL
#define FCD_T0_REL_UNROLL 2  // reliability loop trips unrolled (A/B r04t: 1 8.46-8.50k, 2 8.56k, 5 8.39-8.44k frames/s)
#endif
#ifndef FCD_T0_ROUNDS_DEFAULT
#define FCD_T0_ROUNDS_DEFAULT 2  // tile hook rounds before the cap (k_mst_tile0); large: none
#endif

// find_wrap of the reference unwrapper: -1 if w1 - w2 > pi, +1 if < -pi.
__device__ __forceinline__ int find_wrap(float a, float b) {
    const double d = (double)a - (double)b;  // exact in f64
    return d > kPi ? -1 : (d < -kPi ? 1 : 0);
}

__device__ __forceinline__ double wrapd(double x) {
    return x > kPi ? __dsub_rn(x, kTwoPi) : (x < -kPi ? __dadd_rn(x, kTwoPi) : x);
}

// XCD-aware block id for the one-thread-per-pixel stencil kernels: workgroups are
// dealt round-robin to the 8 XCDs (block b -> XCD b % 8), each with its own L2, so
// consecutive blocks (consecutive quarter rows) land on different L2s and every
// row's neighbours above and below are fetched again by other XCDs.  Renumbering
// b -> (b % 8) * (G / 8) + b / 8 keeps runs of consecutive rows on one XCD.
__device__ __forceinline__ long xcd_block() {
    const unsigned G = gridDim.x, b = blockIdx.x;
    return (G % 8 == 0) ? (long)(b % 8) * (G / 8) + b / 8 : (long)b;
}

// ------------------------------------------------------------------ residues
// find_wrap in f32: fl(a - b) > fl(pi) only if a - b > M_PI; |fl(a - b)| = fl(pi) is
// flagged for the exact f64 test (kernels_fast.hip fw_fast)
__device__ __forceinline__ int find_wrap_f(float a, float b, bool& amb) {
    const float d = a - b;
    constexpr float P = 3.14159274f;
    amb |= fabsf(d) == P;
    return d > P ? -1 : (d < -P ? 1 : 0);
}

// Residue count per map: each thread walks a strip of kResRows plaquette rows down 4
// columns (16-byte loads of each row once, the next row's loads issued before the
// current pair's tests), blockIdx.y = map.
constexpr int kResRows = 16;
__device__ __forceinline__ int residues_quad(const float (&ra)[5], const float (&rc)[5], int nk) {
    bool amb = false;
    int r = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        // plaquette (i, j + k): a -> b -> c -> d -> a, a = (i, j+k), b = (i, j+k+1), c = (i+1, j+k+1), d = (i+1, j+k)
        const int s = find_wrap_f(ra[k], ra[k + 1], amb) + find_wrap_f(ra[k + 1], rc[k + 1], amb) +
                      find_wrap_f(rc[k + 1], rc[k], amb) + find_wrap_f(rc[k], ra[k], amb);
        r += k < nk && s != 0;
    }
    if (amb) {  // some difference is exactly fl(pi) apart: the f64 tests for this quad
        r = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            r += k < nk && (find_wrap(ra[k], ra[k + 1]) + find_wrap(ra[k + 1], rc[k + 1]) + find_wrap(rc[k + 1], rc[k]) +
                            find_wrap(rc[k], ra[k])) != 0;
    }
    return r;
}

// Blocks are numbered map-fastest (block b: map b % nmaps, strip block b / nmaps), so the
// first blocks in flight sample every map.  any_only: a map's count is then only "> 0 iff
// it has residues", and a block whose map is already counted skips its strip (camera
// frames: most blocks, their maps flagged by the first wave of blocks).
__global__ __launch_bounds__(256) void k_residues(const float* __restrict__ w, int H, int W, int nmaps, int* counts,
                                                  bool any_only) {
    const int map = (int)(blockIdx.x % (unsigned)nmaps);
    if (any_only && __hip_atomic_load(counts + map, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > 0) return;
    const int q = (W + 3) / 4;  // column quads per row
    const long idx = (long)(blockIdx.x / (unsigned)nmaps) * 256 + threadIdx.x;
    const int strip = (int)(idx / q), j = (int)(idx % q) * 4;
    const int i0 = strip * kResRows, i1 = min(i0 + kResRows, H - 1);  // plaquette rows [i0, i1)
    int r = 0;
    if (i0 < i1) {
        const float* m = w + (long)map * H * W + (long)i0 * W + j;
        const int nk = min(4, W - 1 - j);  // plaquettes j .. j + nk - 1 (the row's last one is W - 2)
        auto load = [&](const float* p, float (&v)[5]) {
            if ((W & 3) == 0) {  // 16-byte aligned quads
                const float4 a = *reinterpret_cast<const float4*>(p);
                v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k) v[k] = j + k < W ? p[k] : 0.f;
            }
            v[4] = j + 4 < W ? p[4] : 0.f;
        };
        float ra[5], rc[5], rn[5] = {};
        load(m, ra);
        load(m + W, rc);
        for (int i = i0; i < i1; ++i) {
            if (i + 2 <= i1) load(m + 2L * W, rn);  // row i + 2 (the next pair's lower row)
            r += residues_quad(ra, rc, nk);
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                ra[k] = rc[k];
                rc[k] = rn[k];
            }
            m += W;
        }
    }
    // one atomic per block with residues: a map's count word takes one add per block
    // (the camera frames' 1.6 k residues per map would otherwise queue ~1.6 k adds on it)
    __shared__ int bc;
    if (threadIdx.x == 0) bc = 0;
    __syncthreads();
    int wave_cnt = r;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) wave_cnt += __shfl_xor(wave_cnt, o, 64);
    if ((threadIdx.x & 63) == 0 && wave_cnt) atomicAdd(&bc, wave_cnt);
    __syncthreads();
    if (threadIdx.x == 0 && bc) atomicAdd(counts + map, bc);
}

void residues(const float* w, int nmaps, int H, int W, int* counts, hipStream_t s, bool any_only) {
    FCD_HIPCHK(hipMemsetAsync(counts, 0, sizeof(int) * nmaps, s));
    const long threads = (long)(H - 1 + kResRows - 1) / kResRows * ((W + 3) / 4);
    const long blocks = (threads + 255) / 256 * nmaps;
    if (blocks > 0x7fffffffL) throw std::runtime_error("residues: too many maps in one launch");
    hipLaunchKernelGGL(k_residues, dim3((unsigned)blocks), dim3(256), 0, s, w, H, W, nmaps, counts, any_only);
    FCD_CHECK_LAUNCH();
}

// ------------------------------------------------------------------ residue-free scan path
// colk[map][i] = k(i, 0) = -sum_{i' < i} find_wrap(w[i'][0], w[i'+1][0])
// One wave per map (a 64-thread block), 8 rows per lane and chunk, a wave scan of the
// lanes' sums, the running total carried over chunks.  At most 32 VGPRs and no LDS, so its
// blocks fit beside the other stream's fused kernel (2 waves / SIMD at 235 VGPRs) instead
// of waiting for that kernel's CUs: the 256-thread form (loc[64], ~80 VGPRs) ran 6-188 us
// per launch in the two-stream headline chain, ahead of the integration (r05c).
// CONTIG: the compact column-0 copy (row stride 1: immediate load offsets, ~30 VGPRs).
constexpr int COLK_R = 8;
template <bool CONTIG>
__global__ __launch_bounds__(64) void k_colk(const float* __restrict__ w, int H, long map_stride, long W_,
                                             int* __restrict__ colk) {
    const long W = CONTIG ? 1 : W_;
    const int map = blockIdx.x, lane = threadIdx.x;
    const float* m = w + (long)map * map_stride;
    int* out = colk + (long)map * H;
    int carry = 0;
    for (int i0 = 0; i0 < H; i0 += 64 * COLK_R) {
        const int r0 = i0 + lane * COLK_R;
        float v[COLK_R + 1];
#pragma unroll
        for (int q = 0; q <= COLK_R; ++q) v[q] = r0 + q < H ? m[(long)(r0 + q) * W] : 0.f;
        int loc[COLK_R];  // exclusive: sum of d over rows r0 .. r0 + q - 1
        int sum = 0;
#pragma unroll
        for (int q = 0; q < COLK_R; ++q) {
            loc[q] = sum;
            if (r0 + q + 1 < H) sum -= find_wrap(v[q], v[q + 1]);
        }
        int incl = sum;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int t = __shfl_up(incl, off, 64);
            if (lane >= off) incl += t;
        }
        const int base = carry + incl - sum;
#pragma unroll
        for (int q = 0; q < COLK_R; ++q)
            if (r0 + q < H) out[r0 + q] = base + loc[q];
        carry += __shfl(incl, 63, 64);
    }
}

// One wave per row: k(i, j) = colk[i] - sum_{j' < j} find_wrap(w[i][j'], w[i][j'+1]),
// in 64-pixel chunks (lane l holds pixel c + l: coalesced loads and stores, the next
// chunk's load issued before this one's scan; the right neighbour of lane 63 is the next
// chunk's lane 0), an exclusive wave scan per chunk and the running total carried.  (One
// contiguous run of W / 64 pixels per lane read 0.38 TB/s at 1024 x 1280, r04u.)
__global__ __launch_bounds__(256) void k_rowscan(const float* __restrict__ w, long nrows, int H, int W,
                                                 const int* __restrict__ colk, int32_t* __restrict__ k) {
    const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= nrows) return;  // wave-uniform
    const float* r = w + row * W;
    int32_t* ko = k + row * W;
    int acc = colk[row];  // row index == map * H + i == colk layout
    float cur = lane < W ? r[lane] : 0.f;
    for (int c0 = 0; c0 < W; c0 += 64) {
        const float nxt = c0 + 64 + lane < W ? r[c0 + 64 + lane] : 0.f;
        float right = __shfl_down(cur, 1, 64);
        const float n0 = __shfl(nxt, 0, 64);
        if (lane == 63) right = n0;
        bool amb = false;
        int fw = find_wrap_f(cur, right, amb);
        if (amb) fw = find_wrap(cur, right);
        const int d = c0 + lane + 1 < W ? -fw : 0;  // k(j + 1) - k(j)
        int incl = d;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int v = __shfl_up(incl, off, 64);
            if (lane >= off) incl += v;
        }
        if (c0 + lane < W) ko[c0 + lane] = acc + incl - d;
        acc += __shfl(incl, 63, 64);
        cur = nxt;
    }
}

void unwrap_colk(const float* w, int nmaps, int H, int W, int* colk, hipStream_t s) {
    hipLaunchKernelGGL(k_colk<false>, dim3(nmaps), dim3(64), 0, s, w, H, (long)H * W, (long)W, colk);
    FCD_CHECK_LAUNCH();
}

void unwrap_colk_compact(const float* col0, int nmaps, int H, int* colk, hipStream_t s) {
    hipLaunchKernelGGL(k_colk<true>, dim3(nmaps), dim3(64), 0, s, col0, H, (long)H, 1L, colk);
    FCD_CHECK_LAUNCH();
}

void unwrap_scan(const float* w, int nmaps, int H, int W, int* colk, int32_t* k, hipStream_t s) {
    if (H > 16384) throw std::runtime_error("unwrap_scan: H too large");
    hipLaunchKernelGGL(k_colk<false>, dim3(nmaps), dim3(64), 0, s, w, H, (long)H * W, (long)W, colk);
    FCD_CHECK_LAUNCH();
    const long nrows = (long)nmaps * H;
    hipLaunchKernelGGL(k_rowscan, dim3((unsigned)((nrows + 3) / 4)), dim3(256), 0, s, w, nrows, H, W, colk, k);
    FCD_CHECK_LAUNCH();
}

// ------------------------------------------------------------------ frames padded to multiples of 64
// The unwrap's tiles, residue strips and row scans work on sides that are multiples of 64;
// a frame of any other size is unwrapped in a copy padded by replicating its last row /
// column.  A pad plaquette then has zero wrap circulation (find_wrap is antisymmetric), the
// residue-free scan integrates the frame's pixels from their own left / upper neighbours
// only, and the MST pass gives pad pixels the reliability kPadRel (MstWork::Hr / Wr).
__global__ __launch_bounds__(256) void k_pad_maps(const float* __restrict__ w, long n, int H, int W, int Hp, int Wp,
                                                  const int* __restrict__ ids, float* __restrict__ out) {
    for (long g = (long)blockIdx.x * 256 + threadIdx.x; g < n; g += (long)gridDim.x * 256) {
        const long m = g / ((long)Hp * Wp), p = g - m * Hp * Wp;
        const int i = (int)(p / Wp), j = (int)(p % Wp);
        const long src = ids ? ids[m] : m;
        out[g] = w[(src * H + min(i, H - 1)) * W + min(j, W - 1)];
    }
}

__global__ __launch_bounds__(256) void k_unpad_k(const int32_t* __restrict__ kp, long n, int H, int W, int Hp, int Wp,
                                                 const int* __restrict__ ids, int32_t* __restrict__ k) {
    for (long g = (long)blockIdx.x * 256 + threadIdx.x; g < n; g += (long)gridDim.x * 256) {
        const long m = g / ((long)H * W), p = g - m * H * W;
        const int i = (int)(p / W), j = (int)(p % W);
        const long dst = ids ? ids[m] : m;
        k[dst * H * W + p] = kp[(m * Hp + i) * Wp + j];
    }
}

static unsigned grid_of(long n) { return (unsigned)std::min<long>(std::max<long>((n + 255) / 256, 1), 16384); }

void pad_maps(const float* w, int nmaps, int H, int W, int Hp, int Wp, float* out, hipStream_t s, const int* ids) {
    const long n = (long)nmaps * Hp * Wp;
    hipLaunchKernelGGL(k_pad_maps, dim3(grid_of(n)), dim3(256), 0, s, w, n, H, W, Hp, Wp, ids, out);
    FCD_CHECK_LAUNCH();
}

void unpad_k(const int32_t* kp, int nmaps, int Hp, int Wp, int H, int W, int32_t* k, hipStream_t s, const int* ids) {
    const long n = (long)nmaps * H * W;
    hipLaunchKernelGGL(k_unpad_k, dim3(grid_of(n)), dim3(256), 0, s, kp, n, H, W, Hp, Wp, ids, k);
    FCD_CHECK_LAUNCH();
}

// ------------------------------------------------------------------ Boruvka MST path
// Vertex ids are slot*H*W + pixel for the nact active maps (slot -> map_ids[slot]).
__device__ __forceinline__ unsigned long long pack_link(int parent, int off) {
    return ((unsigned long long)(unsigned)parent << 32) | (unsigned)off;
}
__device__ __forceinline__ int link_parent(unsigned long long l) { return (int)(l >> 32); }
__device__ __forceinline__ int link_off(unsigned long long l) { return (int)(unsigned)(l & 0xffffffffull); }

__global__ void k_mst_rel(const float* __restrict__ w, const int* __restrict__ map_ids, int nact, int H, int W,
                          int Hr, int Wr, double* __restrict__ rel, int* comp, int* off) {
    const long hw = (long)H * W;
    const long v = xcd_block() * blockDim.x + threadIdx.x;
    if (v >= nact * hw) return;
    const int slot = (int)(v / hw);
    const long p = v % hw;
    const int i = (int)(p / W), j = (int)(p % W);
    const float* m = w + (long)map_ids[slot] * hw;
    double r = (i >= Hr || j >= Wr) ? kPadRel : kBorderRel;
    if (i > 0 && j > 0 && i < Hr - 1 && j < Wr - 1) {
        const double c = m[p];
        const double h = __dsub_rn(wrapd(__dsub_rn((double)m[p - 1], c)), wrapd(__dsub_rn(c, (double)m[p + 1])));
        const double vv = __dsub_rn(wrapd(__dsub_rn((double)m[p - W], c)), wrapd(__dsub_rn(c, (double)m[p + W])));
        const double d1 =
            __dsub_rn(wrapd(__dsub_rn((double)m[p - W - 1], c)), wrapd(__dsub_rn(c, (double)m[p + W + 1])));
        const double d2 =
            __dsub_rn(wrapd(__dsub_rn((double)m[p - W + 1], c)), wrapd(__dsub_rn(c, (double)m[p + W - 1])));
        double s = __dadd_rn(__dmul_rn(h, h), __dmul_rn(vv, vv));
        s = __dadd_rn(s, __dmul_rn(d1, d1));
        s = __dadd_rn(s, __dmul_rn(d2, d2));
        r = s;
    }
    rel[v] = r;
    comp[v] = (int)v;
    off[v] = 0;
}

// Candidate: the lightest (rel_e, edge index) edge of v leaving its component.
template <bool FIRST>
__global__ void k_mst_cand(const int* __restrict__ map_ids, int nact, int H, int W, MstWork m) {
    const long hw = (long)H * W;
    const long v = xcd_block() * blockDim.x + threadIdx.x;
    if (v >= nact * hw) return;
    (void)map_ids;
    const long base = (v / hw) * hw;
    const long p = v - base;
    const int i = (int)(p / W), j = (int)(p % W);
    const int cv = m.comp[v];
    const double rv = m.rel[v];
    const int nh = H * (W - 1);
    double bw = __longlong_as_double(0x7ff0000000000000ll);  // +inf
    int be = 0x7fffffff;
    auto consider = [&](long u, int eidx) {
        if (m.comp[u] == cv) return;
        const double we = (u > v) ? __dadd_rn(rv, m.rel[u]) : __dadd_rn(m.rel[u], rv);  // rel(p1) + rel(p2)
        if (we < bw || (we == bw && eidx < be)) {
            bw = we;
            be = eidx;
        }
    };
    if (j + 1 < W) consider(v + 1, i * (W - 1) + j);
    if (j > 0) consider(v - 1, i * (W - 1) + j - 1);
    if (i + 1 < H) consider(v + W, nh + i * W + j);
    if (i > 0) consider(v - W, nh + (i - 1) * W + j);
    if constexpr (FIRST) {  // every component is one vertex: its candidate IS its best edge
        m.best_w[v] = (unsigned long long)__double_as_longlong(bw);
        m.best_e[v] = be;
        return;
    }
    m.cand_e[v] = be;
    const bool has = be != 0x7fffffff;
    if (has) m.cand_w[v] = bw;  // interior vertices (no outgoing edge) skip the weight store: cand2 reads it only here
    // One atomicMin per run of consecutive lanes in the same component (a wave is
    // 64 consecutive pixels of a row, so components cross it in runs): segmented
    // suffix-min over the run, then the run's first lane updates the root.  Without
    // it every boundary vertex of round 2 hit a device-scope atomic.
    const int lane = threadIdx.x & 63;
    const int cprev = __shfl_up(cv, 1, 64);
    const unsigned long long heads = __ballot(lane == 0 || cprev != cv);
    unsigned long long key = has ? (unsigned long long)__double_as_longlong(bw) : ~0ull;  // +doubles order as uints
#pragma unroll
    for (int sft = 1; sft < 64; sft <<= 1) {
        const unsigned lo = __shfl_down((unsigned)key, sft, 64), hi = __shfl_down((unsigned)(key >> 32), sft, 64);
        const unsigned long long other = ((unsigned long long)hi << 32) | lo;
        // lane + sft is in this run iff no run starts in (lane, lane + sft]
        const unsigned long long between = (lane + sft < 64) ? (heads >> (lane + 1)) & ((1ull << sft) - 1) : 1ull;
        if (between == 0 && other < key) key = other;
    }
    if (((heads >> lane) & 1) && key != ~0ull) atomicMin(m.best_w + cv, key);
}

__global__ void k_mst_cand2(int nact, int H, int W, MstWork m) {
    const long v = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= nact * (long)H * W) return;
    const int be = m.cand_e[v];
    if (be == 0x7fffffff) return;
    const int cv = m.comp[v];
    if ((unsigned long long)__double_as_longlong(m.cand_w[v]) == m.best_w[cv]) atomicMin(m.best_e + cv, be);
}

__device__ __forceinline__ bool mst_hook_one(const float* __restrict__ w, const int* __restrict__ map_ids, int H, int W,
                                             MstWork& m, long c);

__device__ __forceinline__ void count_hook(bool hooked, int* nhooks) {
    // The host only needs "any hook this round" (convergence).  Even one atomic per
    // wave serialises ~1.5 M times on one word in round 1 of a 96-map batch (half the
    // fix-up pass); a wave that sees the flag already raised skips its atomic.
    const unsigned long long b = __ballot(hooked);
    if ((threadIdx.x & 63) == 0 && b &&
        __hip_atomic_load(nhooks, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
        atomicOr(nhooks, 1);
}

__global__ void k_mst_hook(const float* __restrict__ w, const int* __restrict__ map_ids, int nact, int H, int W,
                           MstWork m) {
    const long hw = (long)H * W;
    const long c = (long)blockIdx.x * blockDim.x + threadIdx.x;
    bool hooked = false;
    if (c < nact * hw && m.comp[c] == (int)c) {
        // only roots carry a link (read by k_mst_jump / k_mst_update): self unless hooked
        hooked = mst_hook_one(w, map_ids, H, W, m, c);
        if (!hooked) m.link[c] = pack_link((int)c, 0);
    }
    count_hook(hooked, m.nhooks);
}

__device__ __forceinline__ bool mst_hook_one(const float* __restrict__ w, const int* __restrict__ map_ids, int H, int W,
                                             MstWork& m, long c) {
    const long hw = (long)H * W;
    const int e = m.best_e[c];
    if (e == 0x7fffffff) return false;
    const long base = (c / hw) * hw;
    const int nh = H * (W - 1);
    long p1, p2;
    if (e < nh) {
        p1 = base + (long)(e / (W - 1)) * W + (e % (W - 1));
        p2 = p1 + 1;
    } else {
        p1 = base + (e - nh);
        p2 = p1 + W;
    }
    const float* mw = w + (long)map_ids[c / hw] * hw;
    const int inc = find_wrap(mw[p1 - base], mw[p2 - base]);
    long x, y;
    int delta;  // k(y) - k(x) across the edge
    if (m.comp[p1] == (int)c) {
        x = p1; y = p2; delta = -inc;
    } else {
        x = p2; y = p1; delta = inc;
    }
    const int d = m.comp[y];
    if (m.best_e[d] == e && c < d) return false;  // mutual pair: the smaller root stays a root
    const int poff = m.off[y] - m.off[x] - delta;  // K_c - K_d
    m.link[c] = pack_link(d, poff);
    return true;
}

// Pointer jumping with path compression.  Concurrent threads may read a link
// before or after another thread compressed it; both are valid chains to the
// same final root (the offsets add up either way), so 64-bit atomic loads and
// stores of workgroup scope suffice: a stale L2 copy on another XCD only makes
// a chain longer, never wrong.
__global__ void k_mst_jump(int nact, int H, int W, MstWork m) {
    const long c = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nact * (long)H * W) return;
    if (m.comp[c] != (int)c) return;
    unsigned long long l = __hip_atomic_load(m.link + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    int p = link_parent(l), o = link_off(l);
    if (p == (int)c) return;
    for (;;) {
        const unsigned long long l2 = __hip_atomic_load(m.link + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const int pp = link_parent(l2);
        if (pp == p) break;
        o += link_off(l2);
        p = pp;
        __hip_atomic_store(m.link + c, pack_link(p, o), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

__global__ void k_mst_update(int nact, int H, int W, MstWork m) {
    const long v = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= nact * (long)H * W) return;
    const int c = m.comp[v];
    const unsigned long long l = m.link[c];  // final after k_mst_jump (kernel boundary)
    const int r = link_parent(l);
    if (r != c) {
        m.comp[v] = r;
        m.off[v] += link_off(l);
    }
    if (c == (int)v) {  // the next round's roots are among this round's: reset only those
        m.best_w[v] = 0x7ff0000000000000ull;  // bits of +inf (positive doubles order as uints)
        m.best_e[v] = 0x7fffffff;
    }
}

static inline unsigned nblk(long n) { return (unsigned)((n + 255) / 256); }

void mst_init(const float* w, const int* map_ids, int nact, int H, int W, MstWork m, hipStream_t s) {
    const long n = (long)nact * H * W;
    hipLaunchKernelGGL(k_mst_rel, dim3(nblk(n)), dim3(256), 0, s, w, map_ids, nact, H, W, m.Hr, m.Wr, m.rel, m.comp,
                       m.off);
    FCD_CHECK_LAUNCH();
    // no reset of best_w / best_e: the first round (k_mst_cand<true>) writes every
    // vertex's entry before anything reads it
}

void mst_round(const float* w, const int* map_ids, int nact, int H, int W, MstWork m, hipStream_t s, bool first) {
    const long n = (long)nact * H * W;
    FCD_HIPCHK(hipMemsetAsync(m.nhooks, 0, sizeof(int), s));
    if (first) {
        hipLaunchKernelGGL(k_mst_cand<true>, dim3(nblk(n)), dim3(256), 0, s, map_ids, nact, H, W, m);
        FCD_CHECK_LAUNCH();
    } else {
        hipLaunchKernelGGL(k_mst_cand<false>, dim3(nblk(n)), dim3(256), 0, s, map_ids, nact, H, W, m);
        FCD_CHECK_LAUNCH();
        hipLaunchKernelGGL(k_mst_cand2, dim3(nblk(n)), dim3(256), 0, s, nact, H, W, m);
        FCD_CHECK_LAUNCH();
    }
    hipLaunchKernelGGL(k_mst_hook, dim3(nblk(n)), dim3(256), 0, s, w, map_ids, nact, H, W, m);
    FCD_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_mst_jump, dim3(nblk(n)), dim3(256), 0, s, nact, H, W, m);
    FCD_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_mst_update, dim3(nblk(n)), dim3(256), 0, s, nact, H, W, m);
    FCD_CHECK_LAUNCH();
}

__global__ void k_mst_finalize(const int* __restrict__ map_ids, int nact, int H, int W, MstWork m, int32_t* k) {
    const long hw = (long)H * W;
    const long v = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= nact * hw) return;
    const int slot = (int)(v / hw);
    const long base = slot * hw;
    k[(long)map_ids[slot] * hw + (v - base)] = m.off[v] - m.off[base];
}

void mst_finalize(const int* map_ids, int nact, int H, int W, MstWork m, int32_t* k, hipStream_t s) {
    const long n = (long)nact * H * W;
    hipLaunchKernelGGL(k_mst_finalize, dim3(nblk(n)), dim3(256), 0, s, map_ids, nact, H, W, m, k);
    FCD_CHECK_LAUNCH();
}

// ------------------------------------------------------------------ two-level Boruvka
// After the first pixel round (mst_round first = true) every pixel v belongs to a
// level-0 component comp[v] with k(v) = K[comp[v]] + off[v].  The later rounds
// never touch every pixel again: each level-0 root c carries its current root
// rootof[c] and offk[c] = K[c] - K[rootof[c]], so
//   k(v) = K[root] + offk[comp[v]] + off[v],
// candidates come from the pixels on a component boundary (a list that only
// shrinks: a pixel whose four neighbours share its component never gets an
// outgoing edge again), hooks and pointer jumps run over the list of current
// roots, and the per-round relabelling over the level-0 roots (about a third of
// the pixels after the first round).  Same edges, weights, tie-break and hook rule
// as the pixel rounds, so the same unique MST and k-field.

// The lists are SEGMENTED: block g of the fixed LVL_BLOCKS grid owns the pixel
// range [g * seg, (g + 1) * seg) and segment g of every list (capacity seg, count
// cnt[g]), appends through a workgroup counter in LDS and never touches a global
// counter (one word would serialise millions of appends per round).  Within a
// wave the appended entries keep lane order, so the boundary list stays in pixel
// order run by run, which the per-root segmented minimum of k_lvl_cand uses.
constexpr int LVL_BLOCKS = 4096;

__device__ __forceinline__ int block_append(bool pred, int* lds_counter) {
    const unsigned long long b = __ballot(pred);
    if (!b) return -1;
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((long long)b) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(lds_counter, __popcll(b));
    base = __shfl(base, leader, 64);
    return pred ? base + __popcll(b & ((1ull << lane) - 1)) : -1;
}

// cnt layout: [list][LVL_BLOCKS] for list = B0, B1, R0, R1, L0
__device__ __forceinline__ int* lvl_cnt(int* cnt, int list) { return cnt + (long)list * LVL_BLOCKS; }

__global__ __launch_bounds__(256) void k_lvl_setup(int nact, int H, int W, MstWork m, long seg) {
    __shared__ int nroot, nbnd;
    if (threadIdx.x == 0) nroot = nbnd = 0;
    __syncthreads();
    const long hw = (long)H * W, nv = nact * hw;
    const long s0 = (long)blockIdx.x * seg, s1 = std::min(nv, s0 + seg);
    for (long base = s0; base < s1; base += blockDim.x) {
        const long v = base + threadIdx.x;
        const bool in = v < s1;
        bool root = false, bnd = false;
        unsigned mask = 0;
        if (in) {
            const long p = v % hw;
            const int i = (int)(p / W), j = (int)(p % W);
            const int c = m.comp[v];
            root = c == (int)v;
            mask = (unsigned)(j + 1 < W && m.comp[v + 1] != c) | ((unsigned)(j > 0 && m.comp[v - 1] != c) << 1) |
                   ((unsigned)(i + 1 < H && m.comp[v + W] != c) << 2) | ((unsigned)(i > 0 && m.comp[v - W] != c) << 3);
            bnd = mask != 0;
            if (root) {
                m.rootof[v] = (int)v;
                m.offk[v] = 0;
            }
        }
        const int pl = block_append(root, &nroot);
        if (pl >= 0) {
            m.listL0[s0 + pl] = (int)v;
            m.listR[0][s0 + pl] = (int)v;
        }
        const int pb = block_append(bnd, &nbnd);
        if (pb >= 0) {
            m.listB[0][s0 + pb] = (int)v;
            m.maskB[0][s0 + pb] = (unsigned char)mask;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        lvl_cnt(m.cnt, 0)[blockIdx.x] = nbnd;
        lvl_cnt(m.cnt, 2)[blockIdx.x] = nroot;
        lvl_cnt(m.cnt, 4)[blockIdx.x] = nroot;
    }
}

// Candidates over segment g of the boundary list B[par]; survivors (pixels that
// still have an outgoing edge) go to segment g of B[par ^ 1] with their candidate
// edge and root; per-root minimum weight by one atomicMin per run of consecutive
// lanes with the same root.  LVL_U entries per thread per iteration, their gathers
// (B -> comp -> rootof, four neighbours each) issued together: the chain of
// dependent loads, not bandwidth, bounds this kernel.
constexpr int LVL_U = 4;

__global__ __launch_bounds__(256) void k_lvl_cand(int H, int W, MstWork m, int par, long seg) {
    __shared__ int nout;
    if (threadIdx.x == 0) nout = 0;
    __syncthreads();
    const int nh = H * (W - 1);
    const long hw = (long)H * W;
    const long s0 = (long)blockIdx.x * seg;
    const int n = lvl_cnt(m.cnt, par)[blockIdx.x];
    const int* B = m.listB[par] + s0;
    int* B2 = m.listB[par ^ 1] + s0;
    double* cw = m.cand_w + s0;
    int* ce = m.cand_e + s0;
    int* cr = m.listB[par] + s0;  // the candidates' roots overwrite the consumed entries of B[par]
    const unsigned char* M = m.maskB[par] + s0;
    unsigned char* M2 = m.maskB[par ^ 1] + s0;
    const int lane = threadIdx.x & 63;
    for (int base = 0; base < n; base += 256 * LVL_U) {
        int v[LVL_U], c0[LVL_U], cv[LVL_U], cn[LVL_U][4], rn[LVL_U][4], eix[LVL_U][4];
        long nb[LVL_U][4];
        bool in[LVL_U];
        unsigned mk[LVL_U];
#pragma unroll
        for (int u = 0; u < LVL_U; ++u) {
            const int i = base + u * 256 + threadIdx.x;
            in[u] = i < n;
            v[u] = in[u] ? B[i] : 0;
            mk[u] = in[u] ? M[i] : 0u;
        }
#pragma unroll
        for (int u = 0; u < LVL_U; ++u) {
            // only the neighbours outside v's component when it entered the list: a
            // neighbour inside it stays inside (components only merge)
            const int p = (int)(v[u] % hw);
            const int pi = p / W, pj = p - pi * W;
            nb[u][0] = (mk[u] & 1) ? v[u] + 1 : -1;
            nb[u][1] = (mk[u] & 2) ? v[u] - 1 : -1;
            nb[u][2] = (mk[u] & 4) ? v[u] + W : -1;
            nb[u][3] = (mk[u] & 8) ? v[u] - W : -1;
            eix[u][0] = pi * (W - 1) + pj;
            eix[u][1] = pi * (W - 1) + pj - 1;
            eix[u][2] = nh + pi * W + pj;
            eix[u][3] = nh + (pi - 1) * W + pj;
            c0[u] = m.comp[v[u]];
#pragma unroll
            for (int d = 0; d < 4; ++d) cn[u][d] = nb[u][d] >= 0 ? m.comp[nb[u][d]] : -1;
        }
#pragma unroll
        for (int u = 0; u < LVL_U; ++u) {
            cv[u] = m.rootof[c0[u]];
#pragma unroll
            for (int d = 0; d < 4; ++d) rn[u][d] = cn[u][d] >= 0 ? m.rootof[cn[u][d]] : -1;
        }
        double bw[LVL_U];
        int be[LVL_U];
#pragma unroll
        for (int u = 0; u < LVL_U; ++u) {
            bw[u] = __longlong_as_double(0x7ff0000000000000ll);
            be[u] = 0x7fffffff;
            if (!in[u]) {
                cv[u] = -1 - lane;  // distinct per idle lane: never part of a run
                continue;
            }
            const double rv = m.rel[v[u]];
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                if (rn[u][d] < 0 || rn[u][d] == cv[u]) {
                    mk[u] &= ~(1u << d);
                    continue;
                }
                const double we = __dadd_rn(rv, m.rel[nb[u][d]]);
                if (we < bw[u] || (we == bw[u] && eix[u][d] < be[u])) {
                    bw[u] = we;
                    be[u] = eix[u][d];
                }
            }
        }
        // every lane has read its B entries before any is overwritten (survivors never
        // outnumber the entries read so far; the barrier orders the reads first)
        __syncthreads();
#pragma unroll
        for (int u = 0; u < LVL_U; ++u) {
            const bool has = be[u] != 0x7fffffff;
            const int pos = block_append(has, &nout);
            if (pos >= 0) {
                B2[pos] = v[u];
                M2[pos] = (unsigned char)mk[u];
                ce[pos] = be[u];
                cw[pos] = bw[u];
                cr[pos] = cv[u];
            }
            const int cprev = __shfl_up(cv[u], 1, 64);
            const unsigned long long heads = __ballot(lane == 0 || cprev != cv[u]);
            unsigned long long key = has ? (unsigned long long)__double_as_longlong(bw[u]) : ~0ull;
#pragma unroll
            for (int sft = 1; sft < 64; sft <<= 1) {
                const unsigned lo = __shfl_down((unsigned)key, sft, 64), hi = __shfl_down((unsigned)(key >> 32), sft, 64);
                const unsigned long long other = ((unsigned long long)hi << 32) | lo;
                const unsigned long long between =
                    (lane + sft < 64) ? (heads >> (lane + 1)) & ((1ull << sft) - 1) : 1ull;
                if (between == 0 && other < key) key = other;
            }
            if (((heads >> lane) & 1) && key != ~0ull) atomicMin(m.best_w + cv[u], key);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) lvl_cnt(m.cnt, par ^ 1)[blockIdx.x] = nout;
}

// Edge-index tie-break among the candidates of minimum weight (B[par ^ 1]).
__global__ __launch_bounds__(256) void k_lvl_cand2(MstWork m, int par, long seg) {
    const long s0 = (long)blockIdx.x * seg;
    const int n = lvl_cnt(m.cnt, par ^ 1)[blockIdx.x];
    const int* cr = m.listB[par] + s0;  // roots stored by k_lvl_cand
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int cv = cr[i];
        if ((unsigned long long)__double_as_longlong(m.cand_w[s0 + i]) == m.best_w[cv])
            atomicMin(m.best_e + cv, m.cand_e[s0 + i]);
    }
}

// Hooks of the current roots (R[par]); the roots that stay roots go to R[par ^ 1].
__global__ __launch_bounds__(256) void k_lvl_hook(const float* __restrict__ w, const int* __restrict__ map_ids, int H,
                                                  int W, MstWork m, int par, long seg) {
    __shared__ int nout;
    if (threadIdx.x == 0) nout = 0;
    __syncthreads();
    const long hw = (long)H * W;
    const int nh = H * (W - 1);
    const long s0 = (long)blockIdx.x * seg;
    const int n = lvl_cnt(m.cnt, 2 + par)[blockIdx.x];
    const int* R = m.listR[par] + s0;
    int* R2 = m.listR[par ^ 1] + s0;
    for (int base = 0; base < n; base += blockDim.x) {
        const int i = base + threadIdx.x;
        bool hooked = false, stays = false;
        int c = 0;
        if (i < n) {
            c = R[i];
            const int e = m.best_e[c];
            if (e == 0x7fffffff) {
                stays = true;
            } else {
                const long mb = ((long)c / hw) * hw;
                long p1, p2;
                if (e < nh) {
                    p1 = mb + (long)(e / (W - 1)) * W + (e % (W - 1));
                    p2 = p1 + 1;
                } else {
                    p1 = mb + (e - nh);
                    p2 = p1 + W;
                }
                const float* mw = w + (long)map_ids[c / hw] * hw;
                const int inc = find_wrap(mw[p1 - mb], mw[p2 - mb]);
                long x, y;
                int delta;  // k(y) - k(x) across the edge
                if (m.rootof[m.comp[p1]] == c) {
                    x = p1; y = p2; delta = -inc;
                } else {
                    x = p2; y = p1; delta = inc;
                }
                const int d = m.rootof[m.comp[y]];
                if (m.best_e[d] == e && c < d) {
                    stays = true;  // mutual pair: the smaller root stays a root
                } else {
                    const int kx = m.offk[m.comp[x]] + m.off[x], ky = m.offk[m.comp[y]] + m.off[y];
                    m.link[c] = pack_link(d, ky - kx - delta);  // K_c - K_d
                    hooked = true;
                }
            }
            if (stays) m.link[c] = pack_link(c, 0);
        }
        const int pos = block_append(stays, &nout);
        if (pos >= 0) R2[pos] = c;
        count_hook(hooked, m.nhooks);
    }
    __syncthreads();
    if (threadIdx.x == 0) lvl_cnt(m.cnt, 2 + (par ^ 1))[blockIdx.x] = nout;
}

// Pointer jumping over this round's roots (as k_mst_jump).
__global__ __launch_bounds__(256) void k_lvl_jump(MstWork m, int par, long seg) {
    const long s0 = (long)blockIdx.x * seg;
    const int n = lvl_cnt(m.cnt, 2 + par)[blockIdx.x];
    const int* R = m.listR[par] + s0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int c = R[i];
        unsigned long long l = __hip_atomic_load(m.link + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        int p = link_parent(l), o = link_off(l);
        if (p == c) continue;
        for (;;) {
            const unsigned long long l2 = __hip_atomic_load(m.link + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const int pp = link_parent(l2);
            if (pp == p) break;
            o += link_off(l2);
            p = pp;
            __hip_atomic_store(m.link + c, pack_link(p, o), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
}

// Relabel the level-0 roots; reset the candidate slots of this round's roots.
__global__ __launch_bounds__(256) void k_lvl_update(MstWork m, long seg) {
    const long s0 = (long)blockIdx.x * seg;
    const int n = lvl_cnt(m.cnt, 4)[blockIdx.x];
    const int* L0 = m.listL0 + s0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int c = L0[i];
        const int r = m.rootof[c];
        const unsigned long long l = m.link[r];
        const int p = link_parent(l);
        if (p != r) {
            m.rootof[c] = p;
            m.offk[c] += link_off(l);
        }
        if (c == r) {
            m.best_w[c] = 0x7ff0000000000000ull;
            m.best_e[c] = 0x7fffffff;
        }
    }
}

__global__ void k_lvl_finalize(const int* __restrict__ map_ids, int nact, int H, int W, MstWork m, int32_t* k) {
    const long hw = (long)H * W;
    const long v = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= nact * hw) return;
    const int slot = (int)(v / hw);
    const long base = slot * hw;
    const int kv = m.offk[m.comp[v]] + m.off[v];
    const int kb = m.offk[m.comp[base]] + m.off[base];
    k[(long)map_ids[slot] * hw + (v - base)] = kv - kb;
}

static long lvl_seg(long n) { return (n + LVL_BLOCKS - 1) / LVL_BLOCKS; }

int mst_level_counts() { return 5 * LVL_BLOCKS; }

void mst_level_setup(int nact, int H, int W, MstWork m, hipStream_t s) {
    const long n = (long)nact * H * W, seg = lvl_seg(n);
    hipLaunchKernelGGL(k_lvl_setup, dim3(LVL_BLOCKS), dim3(256), 0, s, nact, H, W, m, seg);
    FCD_CHECK_LAUNCH();
}

void mst_level_round(const float* w, const int* map_ids, int nact, int H, int W, MstWork m, int r, hipStream_t s) {
    const long n = (long)nact * H * W, seg = lvl_seg(n);
    const int par = r & 1;
    FCD_HIPCHK(hipMemsetAsync(m.nhooks, 0, sizeof(int), s));
    const dim3 g(LVL_BLOCKS), b(256);
    hipLaunchKernelGGL(k_lvl_cand, g, b, 0, s, H, W, m, par, seg);
    FCD_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_lvl_cand2, g, b, 0, s, m, par, seg);
    FCD_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_lvl_hook, g, b, 0, s, w, map_ids, H, W, m, par, seg);
    FCD_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_lvl_jump, g, b, 0, s, m, par, seg);
    FCD_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_lvl_update, g, b, 0, s, m, seg);
    FCD_CHECK_LAUNCH();
}

void mst_level_finalize(const int* map_ids, int nact, int H, int W, MstWork m, int32_t* k, hipStream_t s) {
    const long n = (long)nact * H * W;
    hipLaunchKernelGGL(k_lvl_finalize, dim3(nblk(n)), dim3(256), 0, s, map_ids, nact, H, W, m, k);
    FCD_CHECK_LAUNCH();
}

// ------------------------------------------------------------------ tile-local first level
// Level-0 components from a Boruvka run inside each 32 x 32 tile, in LDS: by the
// cut property, the lightest edge (under the total order (weight, edge index)) leaving
// ANY vertex set is an edge of the unique MST, so a tile component whose lightest
// outgoing edge -- over all its edges, the ones leaving the tile included -- ends
// inside the tile may hook along it; a component whose lightest edge leaves the tile
// waits (another component may still hook into it, and then the union's lightest
// edge can be inside again).  The rounds stop when no component hooks.  Every hook
// is an MST edge, so the components are subtrees of the MST and the two-level rounds
// finish the same tree (same k-field as the all-pixel rounds).  The tile also
// writes the f64 reliabilities (k_mst_rel's arithmetic) the later rounds read.
// Tiles of TW x TH = 64 x 64 (4096 pixels, 1024 threads, 65 KB of LDS: one workgroup
// per CU at 128 VGPRs), 64 x 32 (512 threads, 33 KB: two) or 32 x 32 (256 threads, 17 KB:
// four); 4 pixels per thread.
// diagnostic (FCD_T0_STAMPS builds): per-phase cycles of the first 256 tiles (thread 0)
// and their round counts; phases 7-11 split the graph write-out
#ifdef FCD_T0_STAMPS
constexpr int kT0Phases = 13;
__device__ unsigned long long g_t0_stamps[256 * (kT0Phases + 1)];
extern "C" __attribute__((visibility("default"))) int fcd_debug_t0_stamps(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_t0_stamps), sizeof(g_t0_stamps)) == hipSuccess ? 0 : -1;
}
struct T0Clock {
    unsigned long long tprev = __builtin_readcyclecounter(), ph[kT0Phases] = {};
    __device__ __forceinline__ void stamp(int i) {
        const unsigned long long t = __builtin_readcyclecounter();
        ph[i] += t - tprev;
        tprev = t;
    }
};
#else
struct T0Clock {
    __device__ __forceinline__ void stamp(int) {}
};
#endif
// Edges of a tile by a local code that keeps the global edge order (horizontal edges
// first, each kind row-major; li in [-1, TH], lj in [-1, TW] relative to the tile origin):
// horizontal (li, lj)-(li, lj + 1) -> (li + 1) << 7 | (lj + 1), vertical (li, lj)-(li + 1, lj)
// -> 1 << 14 | (li + 1) << 7 | (lj + 1).  Decoding is shifts and masks.
__device__ __forceinline__ int t0_hcode(int li, int lj) { return ((li + 1) << 7) | (lj + 1); }
__device__ __forceinline__ int t0_vcode(int li, int lj) { return (1 << 14) | ((li + 1) << 7) | (lj + 1); }
// a root's link: parent (local index) in the high half, K_c - K_parent (|.| <= T0N) low
__device__ __forceinline__ unsigned t0_link(int parent, int off) { return ((unsigned)parent << 16) | (unsigned short)off; }
__device__ __forceinline__ int t0_parent(unsigned l) { return (int)(l >> 16); }
__device__ __forceinline__ int t0_off(unsigned l) { return (int)(short)(l & 0xffffu); }

// ------------------------------------------------------------------ component graph
// The level rounds after the tile pass on the CONTRACTED graph: nodes are the level-0
// components, edges the lightest edge between each pair of adjacent components
// (contracting subtrees of the MST keeps the MST: of parallel edges between two
// components only the lightest (weight, edge index) can be in it, by the cycle property
// of the contracted graph).  When a tile's Boruvka stops, every component's lightest
// edge leaves the tile, so every component holds a tile-border pixel: V <= 2 (TW + TH) - 4
// components (a tile stopped by the round cap checks V <= cg_ccap itself), and the
// contracted tile graph is planar, so at most 3 V - 6 distinct adjacent pairs inside the
// tile, plus the TH + TW edges leaving it to the right and downwards (the other two sides
// are the neighbours' right / down edges).  Hence the fixed per-tile capacities below and
// an LDS hash table that never fills.
//
// Per tile tg (= blockIdx.x of the tile pass): components tg * cg_ccap + rank, edges in
// [tg * cg_ecap, + cg_ecnt[tg]) as records (ea, eb, weight bits, global edge index,
// ed = K_ea - K_eb from the pixel offsets and the edge's wrap count).  An edge to a
// neighbour tile is written with eb = -1 - (neighbour pixel's vertex id) and the
// neighbour's offset missing; the first round's hooks resolve it (comp[], off[] of the pixel).
// For a TW x TH tile: V <= 2 (TW + TH) - 4, edges <= 3 V - 6 + TW + TH.
__host__ __device__ constexpr int cg_ccap(int tw, int th) { return 2 * (tw + th); }
__host__ __device__ constexpr int cg_pow2(int n) { return n <= 1 ? 1 : 2 * cg_pow2((n + 1) / 2); }
__host__ __device__ constexpr int cg_ecap(int tw, int th) { return cg_pow2(3 * (2 * (tw + th) - 4) - 6 + tw + th); }
static_assert(cg_ecap(64, 64) == 1024 && cg_ecap(64, 32) == 1024 && cg_ecap(32, 32) == 512, "capacities");

__device__ __forceinline__ void cg_write_edge(MstWork& m, long e, int ea, int eb, unsigned long long ew, int ec, int ed) {
    m.cg_ea[e] = ea;
    m.cg_eb[e] = eb;
    m.cg_ew[e] = ew;
    m.cg_ec[e] = ec;
    m.cg_ed[e] = ed;
}

// Positions in a block-wide list for N predicates per lane: one LDS atomic per wave
// (a block_append per predicate serialised ~200 atomics per tile on one word).
template <int N>
__device__ __forceinline__ void wave_append(const bool (&pred)[N], int* lds_counter, int (&pos)[N]) {
    unsigned long long b[N];
    int tot = 0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        b[j] = __ballot(pred[j]);
        tot += __popcll(b[j]);
    }
    const int lane = threadIdx.x & 63;
    int base = 0;
    if (tot) {  // wave-uniform
        if (lane == 0) base = atomicAdd(lds_counter, tot);
        base = __shfl(base, 0, 64);
    }
    const unsigned long long lt = (1ull << lane) - 1;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        pos[j] = pred[j] ? base + __popcll(b[j] & lt) : -1;
        base += __popcll(b[j]);
    }
}

// After the tile's rounds: lc / lo (labels, offsets) valid, the rest of the pool free.
template <int TW, int TH>
__device__ __forceinline__ void tile0_graph(unsigned char* pool, const unsigned long long (&ekey)[4][4], unsigned incs,
                                            int H, int W, int gi0, int gj0, long vbase, MstWork& m, T0Clock& clk) {
    constexpr int T0N = TW * TH, NT = T0N / 4;
    constexpr int HS = T0N / 2;  // hash slots: >= 2.7x the pairs a tile can have
    constexpr int HB = HS == 2048 ? 11 : (HS == 1024 ? 10 : 9);
    static_assert((1 << HB) == HS && 3 * (2 * (TW + TH) - 4) - 6 < HS, "hash size: more slots than pairs");
    constexpr int ECAP = cg_ecap(TW, TH);
    static_assert(16 * HS <= 8 * T0N, "hash table in the minimum-weight region");
    unsigned* const hkey = reinterpret_cast<unsigned*>(pool);  // pair (a, b), a < b, + 1; 0: empty
    unsigned* const hcode = hkey + HS;
    unsigned long long* const hwt = reinterpret_cast<unsigned long long*>(pool + 8 * HS);
    int* const rk = reinterpret_cast<int*>(pool + 8 * T0N);  // rank of each root (the links' region)
    const short* const lc = reinterpret_cast<const short*>(pool + 12 * T0N);
    const short* const lo = reinterpret_cast<const short*>(pool + 14 * T0N);
    const long tg = blockIdx.x;
    const int cb = (int)(tg * cg_ccap(TW, TH));
    const long eb0 = tg * ECAP;
    const int nh = H * (W - 1);
    // Round 0 of the component-graph rounds comes out of the tile's last round: every
    // component's lightest outgoing edge (after a full run all of them leave the tile;
    // after a capped one some end inside it) is its minimum (bw, be) there, be as a local
    // edge code (t0_hcode / t0_vcode).
    const unsigned long long* const bw = reinterpret_cast<const unsigned long long*>(pool);
    const int* const be = reinterpret_cast<const int*>(pool + 8 * T0N);
    unsigned long long rbw[4];
    int rbe[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int c = threadIdx.x + NT * k;
        const bool root = lc[c] == c;
        rbw[k] = root ? bw[c] : ~0ull;
        rbe[k] = root ? be[c] : 0x7fffffff;
    }
    __shared__ int ncnt[2];  // roots, edges
    if (threadIdx.x == 0) ncnt[0] = ncnt[1] = 0;
    __syncthreads();  // the minima are read before the hash table overwrites them
    for (int i = threadIdx.x; i < HS; i += NT) {
        hkey[i] = 0u;
        hcode[i] = 0x7fffffffu;
        hwt[i] = ~0ull;
    }
    __syncthreads();
    clk.stamp(7);
    {
        bool root[4];
        int r[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) root[k] = lc[threadIdx.x + NT * k] == threadIdx.x + NT * k;
        wave_append(root, &ncnt[0], r);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (r[k] < 0) continue;
            rk[threadIdx.x + NT * k] = r[k];
            const int code = rbe[k];  // local code -> global edge index (k_mst_cand's numbering)
            int ge = 0x7fffffff;
            if (code != 0x7fffffff) {
                const int gi = gi0 + ((code >> 7) & 127) - 1, gj = gj0 + (code & 127) - 1;
                ge = (code >> 14) ? nh + gi * W + gj : gi * (W - 1) + gj;
            }
            m.best_w[cb + r[k]] = rbw[k];
            m.best_e[cb + r[k]] = ge;
        }
    }
    __syncthreads();
    clk.stamp(8);
    // Every global store of the write-out comes after the last barrier: a barrier is a
    // workgroup release and would wait for the stores in flight (about a quarter of the
    // tile's time when the comp / off stores preceded the hash phases).
    int slot[8], pos[8];
    bool cross[8];
    unsigned key[8];  // the pair of an edge between two components of the tile, 0: none
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int i = threadIdx.x + NT * k;
        const int li = i / TW, lj = i % TW;
        const int c = lc[i];
#pragma unroll
        for (int h = 0; h < 2; ++h) {  // h = 0: right edge (d = 0), 1: down edge (d = 2)
            const int j = 2 * k + h;
            const bool exists = ekey[k][2 * h] != ~0ull;
            const int ni = li + h, nj = lj + 1 - h;
            const bool inside = ni < TH && nj < TW;
            cross[j] = exists && !inside;  // into the neighbour tile: resolved by the first round
            const int cy = lc[inside ? ni * TW + nj : i];
            key[j] = exists && inside && cy != c ? ((unsigned)min(c, cy) << 12 | (unsigned)max(c, cy)) + 1u : 0u;
        }
    }
    // the eight lookups' first probes issued together, then the rare collisions in turn
    unsigned cur[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        slot[j] = (int)((key[j] * 2654435761u) >> (32 - HB));
        cur[j] = key[j] ? hkey[slot[j]] : 0u;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if (!key[j]) {
            slot[j] = -1;
            continue;
        }
        unsigned hs = (unsigned)slot[j], c0 = cur[j];
        slot[j] = -1;
        for (int probe = 0; probe < HS; ++probe) {
            if (c0 == 0u) c0 = atomicCAS(hkey + hs, 0u, key[j]);
            if (c0 == 0u || c0 == key[j]) {
                slot[j] = (int)hs;
                break;
            }
            hs = (hs + 1) & (HS - 1);
            c0 = hkey[hs];
        }
        if (slot[j] < 0) atomicOr(m.nhooks + 1, 1);  // cannot happen (planar bound); the host falls back
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
        if (slot[j] >= 0) atomicMin(hwt + slot[j], ekey[j >> 1][2 * (j & 1)]);
    auto code_of = [&](int j) {
        const int i = threadIdx.x + NT * (j >> 1), gi = gi0 + i / TW, gj = gj0 + i % TW;
        return (j & 1) ? nh + gi * W + gj : gi * (W - 1) + gj;
    };
    wave_append(cross, &ncnt[1], pos);
    __syncthreads();
    clk.stamp(9);
#pragma unroll
    for (int j = 0; j < 8; ++j)
        if (slot[j] >= 0 && hwt[slot[j]] == ekey[j >> 1][2 * (j & 1)]) atomicMin(hcode + slot[j], (unsigned)code_of(j));
    __syncthreads();
    {
        bool win[8];
        int wpos[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            win[j] = slot[j] >= 0 && hwt[slot[j]] == ekey[j >> 1][2 * (j & 1)] && hcode[slot[j]] == (unsigned)code_of(j);
        wave_append(win, &ncnt[1], wpos);
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (win[j]) pos[j] = wpos[j];  // an edge is either inside the tile or leaves it
    }
    __syncthreads();
    clk.stamp(10);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int i = threadIdx.x + NT * k;
        const int li = i / TW, lj = i % TW;
        const long v = vbase + (long)(gi0 + li) * W + gj0 + lj;
        const int c = lc[i];
        const int id = cb + rk[c];
        m.crank[v] = (unsigned char)rk[c];  // (a rank >= 256 sets the overflow flag below)
        m.coff[v] = lo[i];
        if (lj == 0) m.cg_lcol[tg * TH + li] = ((unsigned)rk[c] & 0xffu) | ((unsigned)(unsigned short)lo[i] << 16);
        if (c == i) {  // (its round-0 minimum is written above)
            m.rootof[id] = id;
            m.offk[id] = 0;
            m.link[id] = pack_link(id, 0);
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int j = 2 * k + h;
            if (pos[j] < 0 || pos[j] >= ECAP) continue;
            const int delta = -((int)((incs >> (8 * k + 4 * h)) & 3u) - 1);  // k(y) - k(x)
            if (cross[j]) {
                cg_write_edge(m, eb0 + pos[j], id, (int)(-1 - (v + (h ? W : 1))), ekey[k][2 * h], code_of(j), -lo[i] - delta);
            } else {
                const int y = (li + h) * TW + lj + 1 - h;
                cg_write_edge(m, eb0 + pos[j], id, cb + rk[lc[y]], ekey[k][2 * h], code_of(j), lo[y] - lo[i] - delta);
            }
        }
    }
    if (threadIdx.x == 0) {
        m.cg_ncomp[tg] = ncnt[0];
        m.cg_ecnt[tg] = min(ncnt[1], ECAP);
        if (ncnt[1] > ECAP || ncnt[0] > cg_ccap(TW, TH)) atomicOr(m.nhooks + 1, 1);
    }
    clk.stamp(11);
}

// cap (CG only): after `cap` hook rounds the tile stops as soon as it holds at most
// cg_ccap components, its last candidates (every component's lightest edge, inside the
// tile or leaving it) becoming round 0 of the component-graph rounds.  The components
// are MST subtrees after any number of rounds, so the tree is the same; the late tile
// rounds (few hooks, a full round's barriers and atomics each) move to the contracted
// graph, which is then only a few per cent larger (tools/diag/t0_rounds_sim.py on the
// camera frames: 17.0 k components and 32 k tile pairs per map after the full run,
// 17.6 k / 33 k after 3 rounds, 20.5 k / 42 k after 2).  At most cg_ccap components
// keep the capacities: the contracted tile graph is planar (a minor of the grid), so
// at most 3 V - 6 pairs.
template <int TW, int TH, bool CG>
__global__ __launch_bounds__(TW * TH / 4, 4) void k_mst_tile0(const float* __restrict__ w, const int* __restrict__ map_ids,
                                                          int nact, int H, int W, MstWork m, int cap) {
    constexpr int T0N = TW * TH;  // pixels per tile
    constexpr int T0W = TW + 4;   // wrapped-phase image with a 2-pixel halo
    constexpr int T0R = TW + 2;   // reliabilities with a 1-pixel halo
    constexpr int NT = T0N / 4;   // threads, 4 pixels each
    static_assert((TW == 64 || TW == 32) && TH <= 64 && T0N % 256 == 0, "16-bit local indices and 7-bit edge-code fields");
    // 16 bytes per pixel (64 KB at 64 x 64: two workgroups per CU): the rounds' arrays;
    // before them the same bytes hold the wrapped phases and reliabilities.  A root's
    // link replaces its edge code once every hook decision is made (step (c)).
    __shared__ __attribute__((aligned(16))) unsigned char pool[16 * T0N];
    unsigned long long* const bw = reinterpret_cast<unsigned long long*>(pool);  // component minima (f64 bits)
    int* const be = reinterpret_cast<int*>(pool + 8 * T0N);                      // their edge codes
    // the roots' links (their own array, so the hooks write them directly and the minima's
    // reset needs no barrier of its own; 1 workgroup per CU by registers, LDS to spare)
    __shared__ unsigned lnk[T0N];
    short* const lc = reinterpret_cast<short*>(pool + 12 * T0N);                 // component of each pixel
    short* const lo = reinterpret_cast<short*>(pool + 14 * T0N);                 // K(pixel) - K(component)
    float* const ws = reinterpret_cast<float*>(pool);
    double* const rs = reinterpret_cast<double*>(pool + ((T0W * (TH + 4) * 4 + 15) & ~15));
    static_assert(((T0W * (TH + 4) * 4 + 15) & ~15) + T0R * (TH + 2) * 8 <= 16 * T0N, "phases + reliabilities fit the pool");
    T0Clock clk;
#define T0_STAMP(i) clk.stamp(i)
    const long hw = (long)H * W;
    const int tiles_x = W / TW, tiles = (H / TH) * tiles_x;
    const int slot = blockIdx.x / tiles, tile = blockIdx.x % tiles;
    const int gi0 = (tile / tiles_x) * TH, gj0 = (tile % tiles_x) * TW;
    const float* mw = w + (long)map_ids[slot] * ((long)m.Hs * m.Ws);
    const long vbase = (long)slot * hw;
    // wrapped phases, 2-pixel halo (outside the map: never read for an existing edge).
    // All of a thread's loads are issued before the first LDS store (clamped addresses,
    // unconditional loads): as a loop, each trip waited for its load (vmcnt(0) before
    // the ds_write), five HBM round trips in a row, 11 % of the tile (stamps r04p).
    constexpr int NL = (T0W * (TH + 4) + NT - 1) / NT;
    float v[NL];
#pragma unroll
    for (int u = 0; u < NL; ++u) {
        const int i = threadIdx.x + u * NT;
        const int gi = gi0 - 2 + i / T0W, gj = gj0 - 2 + i % T0W;
        const int ci = min(max(gi, 0), m.Hs - 1), cj = min(max(gj, 0), m.Ws - 1);
        v[u] = mw[(long)ci * m.Ws + cj];
    }
#pragma unroll
    for (int u = 0; u < NL; ++u) asm volatile("" ::"v"(v[u]));  // (keeps the last load up here)
#pragma unroll
    for (int u = 0; u < NL; ++u) {
        const int i = threadIdx.x + u * NT;
        if (i < T0W * (TH + 4)) ws[i] = v[u];
    }
    __syncthreads();
    T0_STAMP(12);
    // reliabilities of the tile and its 1-pixel halo (k_mst_rel's operation order)
#pragma unroll FCD_T0_REL_UNROLL
    for (int i = threadIdx.x; i < T0R * (TH + 2); i += NT) {
        const int li = i / T0R, lj = i % T0R;  // ws index (li + 1, lj + 1)
        const int gi = gi0 - 1 + li, gj = gj0 - 1 + lj;
        double r = (gi >= m.Hr || gj >= m.Wr) ? kPadRel : kBorderRel;
        if (gi > 0 && gj > 0 && gi < m.Hr - 1 && gj < m.Wr - 1) {
            const float* q = ws + (li + 1) * T0W + (lj + 1);
            const double c = q[0];
            const double h = __dsub_rn(wrapd(__dsub_rn((double)q[-1], c)), wrapd(__dsub_rn(c, (double)q[1])));
            const double vv = __dsub_rn(wrapd(__dsub_rn((double)q[-T0W], c)), wrapd(__dsub_rn(c, (double)q[T0W])));
            const double d1 =
                __dsub_rn(wrapd(__dsub_rn((double)q[-T0W - 1], c)), wrapd(__dsub_rn(c, (double)q[T0W + 1])));
            const double d2 =
                __dsub_rn(wrapd(__dsub_rn((double)q[-T0W + 1], c)), wrapd(__dsub_rn(c, (double)q[T0W - 1])));
            double s = __dadd_rn(__dmul_rn(h, h), __dmul_rn(vv, vv));
            s = __dadd_rn(s, __dmul_rn(d1, d1));
            s = __dadd_rn(s, __dmul_rn(d2, d2));
            r = s;
        }
        rs[i] = r;
        if (!CG && li >= 1 && li <= TH && lj >= 1 && lj <= TW) m.rel[vbase + (long)gi * W + gj] = r;
    }
    __syncthreads();
    T0_STAMP(0);
    auto relat = [&](int li, int lj) { return rs[(li + 1) * T0R + (lj + 1)]; };  // li in [-1, TH], lj in [-1, TW]
    // the 4 incident edges of each of this thread's pixels, once: weight rel(p) + rel(q)
    // (f64, as k_mst_rel / k_mst_round) as its bit pattern (non-negative doubles order
    // as unsigned integers), ~0 for an edge past the map border; the rounds then only
    // compare integers (weight, then edge code).  With them the edges' find_wrap values
    // (2 bits each, + 1), so a hook needs no phase reads.
    unsigned long long ekey[4][4];
    unsigned incs = 0;
    auto wat = [&](int li, int lj) { return ws[(li + 2) * T0W + (lj + 2)]; };
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int i = threadIdx.x + NT * k;
        const int li = i / TW, lj = i % TW, gi = gi0 + li, gj = gj0 + lj;
        const double rv = relat(li, lj);
        const float wc = wat(li, lj);
        incs |= (unsigned)(find_wrap(wc, wat(li, lj + 1)) + 1) << (8 * k);
        incs |= (unsigned)(find_wrap(wat(li, lj - 1), wc) + 1) << (8 * k + 2);
        incs |= (unsigned)(find_wrap(wc, wat(li + 1, lj)) + 1) << (8 * k + 4);
        incs |= (unsigned)(find_wrap(wat(li - 1, lj), wc) + 1) << (8 * k + 6);
        auto edge = [&](int d, bool exists, int ni, int nj) {
            ekey[k][d] = exists ? (unsigned long long)__double_as_longlong(__dadd_rn(rv, relat(ni, nj))) : ~0ull;
        };
        edge(0, gj + 1 < W, li, lj + 1);
        edge(1, gj > 0, li, lj - 1);
        edge(2, gi + 1 < H, li + 1, lj);
        edge(3, gi > 0, li - 1, lj);
    }
    __syncthreads();  // every phase / reliability read before the rounds' arrays overwrite them
    for (int i = threadIdx.x; i < T0N; i += NT) {
        lc[i] = (short)i;
        lo[i] = 0;
        bw[i] = 0x7ff0000000000000ull;
        be[i] = 0x7fffffff;
        lnk[i] = t0_link(i, 0);  // (a root's link stays its own: only hooked roots' links change)
    }
    __shared__ int t0roots[2];  // the capped rounds' component counts (by round parity)
    if (threadIdx.x == 0) t0roots[0] = t0roots[1] = 0;
    __syncthreads();
    T0_STAMP(1);
    [[maybe_unused]] int nrounds = 0;
    int lor[4] = {0, 0, 0, 0};  // this thread's pixels' lo (LDS keeps the copy the others read)
    for (;;) {
        ++nrounds;
        const bool capped = CG && nrounds > cap;  // block-uniform
        // (a) each pixel's lightest edge to another tile component or out of the tile
        // (the five component labels loaded unconditionally, then selects)
        unsigned long long key[4];
        int ke[4], kd[4], cs[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int i = threadIdx.x + NT * k;
            const int li = i / TW, lj = i % TW;
            int nbc[4];
            bool in[4];
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                const int ni = li + (d == 2) - (d == 3), nj = lj + (d == 0) - (d == 1);
                in[d] = ni >= 0 && ni < TH && nj >= 0 && nj < TW;
                nbc[d] = lc[in[d] ? ni * TW + nj : i];
            }
            const int c = lc[i];
            cs[k] = c;
            unsigned long long bk = ~0ull;
            int bev = 0x7fffffff, bd = 0;
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                const unsigned long long kk = (in[d] && nbc[d] == c) ? ~0ull : ekey[k][d];
                const int code = d == 0 ? t0_hcode(li, lj)
                                        : (d == 1 ? t0_hcode(li, lj - 1) : (d == 2 ? t0_vcode(li, lj) : t0_vcode(li - 1, lj)));
                const bool better = kk < bk || (kk == bk && kk != ~0ull && code < bev);
                bk = better ? kk : bk;
                bev = better ? code : bev;
                bd = better ? d : bd;
            }
            key[k] = bk;
            ke[k] = bev;
            kd[k] = bd;
            // (skipping the atomicMin when the minimum is already lower measured slower,
            // 13.67 -> 13.9 ms per 96 frames, r03cg6)
            if (bk != ~0ull) atomicMin(bw + c, bk);
        }
        if (capped) {  // count this round's components (one LDS atomic per wave)
            int tot = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) tot += __popcll(__ballot(cs[k] == (int)threadIdx.x + NT * k));
            if ((threadIdx.x & 63) == 0) atomicAdd(&t0roots[nrounds & 1], tot);
            if (threadIdx.x == 0) t0roots[(nrounds + 1) & 1] = 0;  // read two rounds ago, added to next round
        }
        __syncthreads();
        T0_STAMP(2);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (key[k] != ~0ull && key[k] == bw[cs[k]]) atomicMin(be + cs[k], ke[k]);
        __syncthreads();
        T0_STAMP(3);
        // (the minima are final: with few enough components they are round 0 of the graph)
        if (capped && t0roots[nrounds & 1] <= cg_ccap(TW, TH)) break;
        // (c) hooks: the pixel holding its component's lightest edge (unique: weight,
        // then edge code) decides, if that edge ends inside the tile, and writes the
        // component's link (every current root's link is its own until then)
        int hooked = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int i = threadIdx.x + NT * k, c = cs[k];
            // the component's lightest edge by its (tile-unique) code alone: an edge has one
            // end in c, so no other pixel of c holds it as a candidate
            if (key[k] == ~0ull || ke[k] != be[c]) continue;
            const int li = i / TW, lj = i % TW, d = kd[k];
            const int ni = li + (d == 2) - (d == 3), nj = lj + (d == 0) - (d == 1);
            if (!(ni >= 0 && ni < TH && nj >= 0 && nj < TW)) continue;  // leaves the tile: the level rounds take it
            const int y = ni * TW + nj;
            const int inc = (int)((incs >> (8 * k + 2 * d)) & 3u) - 1;
            const int delta = (d == 0 || d == 2) ? -inc : inc;  // k(y) - k(i) across the edge
            const int dr = lc[y];
            if (be[dr] == ke[k] && c < dr) continue;  // mutual pair: the smaller root stays
            lnk[c] = t0_link(dr, lo[y] - lor[k] - delta);  // K_c - K_dr
            hooked = 1;
        }
        const int any = __syncthreads_or(hooked);
        if (!any) break;
        T0_STAMP(4);
        // the minima's reset for the next round (nothing reads them after the hooks)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int i = threadIdx.x + NT * k;
            bw[i] = 0x7ff0000000000000ull;
            be[i] = 0x7fffffff;
        }
        // (d) every hooked root to its final root (a root's link is one 32-bit word, so
        // parent and offset are read together)
        // each root walks to its final root, publishing the shortcuts as it goes (lockstep
        // pointer jumping with a barrier per pass measured 9.0 k vs 9.9 k frames/s, r04aj;
        // every pixel walking, no barrier before the relabel: 10.45 k -> 10.12 k, r05t)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int c = threadIdx.x + NT * k;
            if (cs[k] != c) continue;
            const unsigned l = __hip_atomic_load(lnk + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            int p = t0_parent(l), o = t0_off(l);
            if (p == c) continue;
            for (;;) {
                const unsigned l2 = __hip_atomic_load(lnk + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                const int pp = t0_parent(l2);
                if (pp == p) break;
                o += t0_off(l2);
                p = pp;
                __hip_atomic_store(lnk + c, t0_link(p, o), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        __syncthreads();
        T0_STAMP(5);
        // labels and offsets (this phase reads only links)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int i = threadIdx.x + NT * k;
            const unsigned l = lnk[cs[k]];
            lc[i] = (short)t0_parent(l);
            lo[i] = (short)(lor[k] + t0_off(l));
            lor[k] = (short)(lor[k] + t0_off(l));
        }
        __syncthreads();
        T0_STAMP(6);
    }
    if constexpr (CG) {
        tile0_graph<TW, TH>(pool, ekey, incs, H, W, gi0, gj0, vbase, m, clk);
    } else {
    // level-0 components: global ids of the tile roots, offsets to them; candidate
    // slots of every pixel reset for the level rounds
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int i = threadIdx.x + NT * k;
        const int li = i / TW, lj = i % TW;
        const long v = vbase + (long)(gi0 + li) * W + (gj0 + lj);
        const int c = lc[i];
        m.comp[v] = (int)(vbase + (long)(gi0 + c / TW) * W + (gj0 + c % TW));
        m.off[v] = lo[i];
        m.best_w[v] = 0x7ff0000000000000ull;
        m.best_e[v] = 0x7fffffff;
    }
    }
#ifdef FCD_T0_STAMPS
    if constexpr (!CG) T0_STAMP(7);
    if (blockIdx.x < 256 && threadIdx.x == 0) {
        for (int i = 0; i < kT0Phases; ++i) g_t0_stamps[blockIdx.x * (kT0Phases + 1) + i] = clk.ph[i];
        g_t0_stamps[blockIdx.x * (kT0Phases + 1) + kT0Phases] = nrounds;
    }
#endif
}

// ---- component-graph rounds: over each tile's edge segment (edges), then over each
// tile's level-0 components (relabel).  Same weights, tie-break and hook rule as the
// pixel rounds, so the same unique MST and k-field.

// The graph-round kernels take one WAVE per tile segment (the tiles of a 4-wave block run
// independently): the compaction is a wave ballot prefix, with no workgroup barrier or LDS
// counter, and a segment's ~300-450 edges fill a wave's lanes 8 deep instead of leaving
// most of a 256-thread block idle (graph rounds 2.55 -> 2.22 ms per 96 real frames, 8.46-
// 8.63 k -> 8.73-8.78 k frames/s, r04ab).
#define CG_TILES_LOOP(t)                                                                 \
    const int lane = threadIdx.x & 63;                                                   \
    const int wpb = blockDim.x >> 6;                                                     \
    for (int t = blockIdx.x * wpb + (threadIdx.x >> 6); t < ntiles; t += gridDim.x * wpb)
#define CG_STRIDE 64

// Candidates (rounds >= 1): per edge between different current roots, atomicMin of its
// weight into both roots; the segment is compacted in place (edges inside a root are
// gone for good).
constexpr int CGW_U = 8;  // edges per lane per pass: 512 of a segment
// Each wave first takes its segment's minima per root in a small LDS table (the segment's
// edges meet a few dozen roots; the global 64-bit atomics of later rounds queue on those
// roots), then one global atomicMin per table entry.
constexpr int CGH = 256;  // root slots per wave
__global__ __launch_bounds__(256) void k_cg_cand(MstWork m, int ntiles, int ecap) {
    const unsigned long long lt = (1ull << (threadIdx.x & 63)) - 1;
    __shared__ unsigned hkey_s[4][CGH];  // root + 1, 0: empty
    __shared__ unsigned long long hval_s[4][CGH];
    unsigned* const hk = hkey_s[(threadIdx.x >> 6) & 3];
    unsigned long long* const hv = hval_s[(threadIdx.x >> 6) & 3];
    auto root_min = [&](int r, unsigned long long w) {
        const unsigned key = (unsigned)r + 1u;
        unsigned h = (key * 2654435761u) >> 24;
        for (int probe = 0; probe < 8; ++probe) {
            const unsigned cur = atomicCAS(hk + h, 0u, key);
            if (cur == 0u || cur == key) {
                atomicMin(hv + h, w);
                return;
            }
            h = (h + 1) & (CGH - 1);
        }
        atomicMin(m.best_w + r, w);  // a crowded table: straight to the root's minimum
    };
    CG_TILES_LOOP(t) {
        const int n = m.cg_ecnt[t];
        if (n == 0) continue;  // wave-uniform: a finished tile costs one load per round
        const long b0 = (long)t * ecap;
        int nout = 0;
#pragma unroll
        for (int q = 0; q < CGH / 64; ++q) {
            hk[lane + 64 * q] = 0u;
            hv[lane + 64 * q] = ~0ull;
        }
        __builtin_amdgcn_wave_barrier();
        for (int base = 0; base < n; base += 64 * CGW_U) {
            int ea[CGW_U], eb[CGW_U], ec[CGW_U], ed[CGW_U], ra[CGW_U], rb[CGW_U];
            unsigned long long ew[CGW_U];
            bool keep[CGW_U];
#pragma unroll
            for (int u = 0; u < CGW_U; ++u) {
                const int i = base + u * 64 + lane;
                keep[u] = i < n;
                ea[u] = eb[u] = ec[u] = ed[u] = 0;
                ew[u] = 0;
                if (keep[u]) {
                    ea[u] = m.cg_ea[b0 + i];
                    eb[u] = m.cg_eb[b0 + i];
                    ew[u] = m.cg_ew[b0 + i];
                    ec[u] = m.cg_ec[b0 + i];
                    ed[u] = m.cg_ed[b0 + i];
                }
            }
#pragma unroll
            for (int u = 0; u < CGW_U; ++u) {
                ra[u] = keep[u] ? m.rootof[ea[u]] : 0;
                rb[u] = keep[u] ? m.rootof[eb[u]] : 0;
                keep[u] = keep[u] && ra[u] != rb[u];
            }
            // in-order compaction: a survivor moves to pos <= its index, a slot this wave
            // has read already (its loads precede every store, and return in order)
#pragma unroll
            for (int u = 0; u < CGW_U; ++u) {
                const unsigned long long bal = __ballot(keep[u]);
                const int pos = nout + __popcll(bal & lt);
                nout += __popcll(bal);
                if (!keep[u]) continue;
                if (pos != base + u * 64 + lane) cg_write_edge(m, b0 + pos, ea[u], eb[u], ew[u], ec[u], ed[u]);
                root_min(ra[u], ew[u]);
                root_min(rb[u], ew[u]);
            }
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int q = 0; q < CGH / 64; ++q) {
            const unsigned key = hk[lane + 64 * q];
            if (key) atomicMin(m.best_w + (key - 1u), hv[lane + 64 * q]);
        }
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) m.cg_ecnt[t] = nout;
    }
}
// Edge-index tie-break among each root's edges of minimum weight.
__global__ __launch_bounds__(256) void k_cg_cand2(MstWork m, int ntiles, int ecap) {
    CG_TILES_LOOP(t) {
        const int n = m.cg_ecnt[t];
        const long b0 = (long)t * ecap;
        for (int i = lane; i < n; i += CG_STRIDE) {
            const unsigned long long w = m.cg_ew[b0 + i];
            const int ra = m.rootof[m.cg_ea[b0 + i]], rb = m.rootof[m.cg_eb[b0 + i]], c = m.cg_ec[b0 + i];
            if (m.best_w[ra] == w) atomicMin(m.best_e + ra, c);
            if (m.best_w[rb] == w) atomicMin(m.best_e + rb, c);
        }
    }
}

// Hooks: the (unique) edge that is a root's lightest links it to the other root;
// of a mutual pair the larger root hooks onto the smaller.
// FIRST (round 0, whose minima the tile pass wrote): the edges into a neighbour tile
// are resolved here (and written back) instead of in k_cg_cand.
// A pixel's level-0 component id in the component-graph path: its tile's segment base
// plus its rank there (crank).
CgGeom mst_cg_geom(int H, int W) {
    int th = 0;
    const int tw = mst_tile_shape(H, W, &th);
    if (!tw) throw std::runtime_error("component graph: frame not a multiple of the tile");
    return CgGeom{W, tw, th, W / tw, (H / th) * (W / tw), cg_ccap(tw, th), (long)H * W};
}

template <bool FIRST>
__global__ __launch_bounds__(256) void k_cg_hook(MstWork m, int ntiles, int ecap, CgGeom geo, int* hflag) {
    CG_TILES_LOOP(t) {
        const int n = m.cg_ecnt[t];
        const long b0 = (long)t * ecap;
        for (int base = 0; base < n; base += CG_STRIDE) {
            const int i = base + lane;
            bool hooked = false;
            if (i < n) {
                const unsigned long long w = m.cg_ew[b0 + i];
                const int a = m.cg_ea[b0 + i], c = m.cg_ec[b0 + i];
                int b = m.cg_eb[b0 + i];
                int ed = m.cg_ed[b0 + i];
                if (FIRST && b < 0) {
                    // the far end y of an edge into the right / lower neighbour tile: a
                    // column-0 pixel from that tile's cg_lcol run (the right-hand edges of a
                    // tile then read 256 contiguous bytes, not 64 cache lines of crank and
                    // of coff: ~2/3 of this kernel's 1.2 GB per 96 frames, PMC r04ay)
                    const long y = -1 - (long)b;
                    const int tl = geo.tile_of(y);
                    const int p = (int)(y % geo.hw), py = p / geo.W, px = p - py * geo.W;
                    int rk, of;
                    if (px % geo.tw == 0) {
                        const unsigned lv = m.cg_lcol[(long)tl * geo.th + py % geo.th];
                        rk = (int)(lv & 0xffu);
                        of = (int)(short)(lv >> 16);
                    } else {
                        rk = m.crank[y];
                        of = m.coff[y];
                    }
                    b = tl * geo.ccap + rk;
                    ed += of;
                    m.cg_eb[b0 + i] = b;
                    m.cg_ed[b0 + i] = ed;
                }
                // (round 0: every level-0 component is its own root, offset 0)
                const int ra = FIRST ? a : m.rootof[a], rb = FIRST ? b : m.rootof[b];
                const bool wa = m.best_w[ra] == w && m.best_e[ra] == c;
                const bool wb = m.best_w[rb] == w && m.best_e[rb] == c;
                if (wa || wb) {
                    const int kab = FIRST ? ed : ed - m.offk[a] + m.offk[b];  // K_ra - K_rb
                    if (wa && (!wb || ra > rb)) m.link[ra] = pack_link(rb, kab);
                    else m.link[rb] = pack_link(ra, -kab);
                    hooked = true;
                }
            }
            count_hook(hooked, hflag);
        }
    }
}

// Every level-0 component to its new root (pointer jumping with path compression,
// as k_mst_jump: a root's link is only ever replaced by a link to a further ancestor
// with the offsets summed); the roots reset their candidate slots.
__global__ __launch_bounds__(256) void k_cg_relabel(MstWork m, int ntiles, int ccap) {
    CG_TILES_LOOP(t) {
        const int n = m.cg_ncomp[t];
        for (int i = lane; i < n; i += CG_STRIDE) {
            const int c = t * ccap + i;
            const int r = m.rootof[c];
            const unsigned long long l = __hip_atomic_load(m.link + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            int p = link_parent(l);
            if (p != r) {
                int o = link_off(l);
                for (;;) {
                    const unsigned long long l2 = __hip_atomic_load(m.link + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const int pp = link_parent(l2);
                    if (pp == p) break;
                    o += link_off(l2);
                    p = pp;
                    __hip_atomic_store(m.link + r, pack_link(p, o), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                m.rootof[c] = p;
                m.offk[c] += o;
            }
            if (p == c) {
                m.best_w[c] = 0x7ff0000000000000ull;
                m.best_e[c] = 0x7fffffff;
            }
        }
    }
}

long mst_cg_edge_capacity(long nv) { return nv / 2 + 1024; }
static_assert(cg_ecap(32, 32) * 2 <= 32 * 32 && cg_ecap(64, 32) * 2 <= 64 * 32 && cg_ecap(64, 64) * 2 <= 64 * 64,
              "edge records: nv / 2 covers every tile shape");

void mst_cg_round(int nact, int H, int W, MstWork m, int r, hipStream_t s) {
    int th = 0;
    const int tw = mst_tile_shape(H, W, &th);
    if (!tw) throw std::runtime_error("mst_cg_round: frame not a multiple of the tile");
    const int ntiles = nact * (H / th) * (W / tw);
    const int ecap = cg_ecap(tw, th), ccap = cg_ccap(tw, th);
    const CgGeom geo = mst_cg_geom(H, W);
    if (r >= kCgRounds) throw std::runtime_error("mst_cg_round: round past the hook-flag slots");
    int* const hflag = m.nhooks + 2 + r;  // zeroed with the MST pass (no per-round reset)
    const dim3 g((unsigned)std::min((ntiles + 3) / 4, 4096)), b(256);  // 4 tiles per block at a time
    if (r == 0) {  // the candidates of round 0 came with the tile pass
        hipLaunchKernelGGL(k_cg_hook<true>, g, b, 0, s, m, ntiles, ecap, geo, hflag);
        FCD_CHECK_LAUNCH();
    } else {
        hipLaunchKernelGGL(k_cg_cand, g, b, 0, s, m, ntiles, ecap);
        FCD_CHECK_LAUNCH();
        hipLaunchKernelGGL(k_cg_cand2, g, b, 0, s, m, ntiles, ecap);
        FCD_CHECK_LAUNCH();
        hipLaunchKernelGGL(k_cg_hook<false>, g, b, 0, s, m, ntiles, ecap, geo, hflag);
        FCD_CHECK_LAUNCH();
    }
    hipLaunchKernelGGL(k_cg_relabel, g, b, 0, s, m, ntiles, ccap);
    FCD_CHECK_LAUNCH();
}

// k(v) = K[component] + off(v) - (the same at the map's pixel 0): 4 pixels per thread.
template <bool FRAME>
__global__ __launch_bounds__(256) void k_cg_finalize(const int* __restrict__ map_ids, int nact, MstWork m, CgGeom geo,
                                                     int32_t* __restrict__ k) {
    const long v = 4 * ((long)blockIdx.x * blockDim.x + threadIdx.x);
    if (v >= nact * geo.hw) return;
    const int slot = (int)(v / geo.hw);
    const long base = slot * geo.hw;
    const int kb = m.offk[geo.tile_of(base) * geo.ccap + m.crank[base]] + m.coff[base];
    const int cb = geo.tile_of(v) * geo.ccap;  // 4 pixels of one row of one tile (tw % 4 == 0)
    const uchar4 r = *reinterpret_cast<const uchar4*>(m.crank + v);
    const short4 o = *reinterpret_cast<const short4*>(m.coff + v);
    const int4 kv = make_int4(m.offk[cb + r.x] + o.x - kb, m.offk[cb + r.y] + o.y - kb, m.offk[cb + r.z] + o.z - kb,
                              m.offk[cb + r.w] + o.w - kb);
    if constexpr (FRAME) {  // the frame's own layout: pixels past Hr x Wr are pad
        const long p = v - base;
        const int i = (int)(p / geo.W), j = (int)(p % geo.W);
        if (i >= m.Hr) return;
        int32_t* kr = k + (long)map_ids[slot] * ((long)m.Hr * m.Wr) + (long)i * m.Wr;
        const int kk[4] = {kv.x, kv.y, kv.z, kv.w};
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (j + q < m.Wr) kr[j + q] = kk[q];
    } else {
        *reinterpret_cast<int4*>(k + (long)map_ids[slot] * geo.hw + (v - base)) = kv;
    }
}

void mst_cg_finalize(const int* map_ids, int nact, int H, int W, MstWork m, int32_t* k, hipStream_t s,
                     bool frame_layout) {
    const CgGeom geo = mst_cg_geom(H, W);
    const long n4 = (long)nact * H * W / 4;
    const dim3 g((unsigned)((n4 + 255) / 256));
    if (frame_layout) hipLaunchKernelGGL(k_cg_finalize<true>, g, dim3(256), 0, s, map_ids, nact, m, geo, k);
    else hipLaunchKernelGGL(k_cg_finalize<false>, g, dim3(256), 0, s, map_ids, nact, m, geo, k);
    FCD_CHECK_LAUNCH();
}

int mst_tile_shape(int H, int W, int* th) {
    // 64 x 64 tiles (a frame of another size reaches the unwrap padded to multiples of 64,
    // unwrap_maps; 32 x 32 and 64 x 32 tiles measured slower and were removed, r04x)
    if (H % 64 == 0 && W % 64 == 0) return *th = 64, 64;
    return *th = 0, 0;
}

void mst_tile_level0(const float* w, const int* map_ids, int nact, int H, int W, MstWork m, hipStream_t s, bool graph) {
    int th = 0;
    const int tw = mst_tile_shape(H, W, &th);
    if (!tw) throw std::runtime_error("mst_tile_level0: frame not a multiple of the tile");
    const dim3 g((unsigned)((long)nact * (H / th) * (W / tw)));
    const dim3 b((unsigned)(tw * th / 4));
    // FCD_T0_ROUNDS (read per call; tests/test_gpu_parity.py runs 0 / 1 / 2 / 99 against the
    // default): the tile rounds before the cap applies
    const char* e = std::getenv("FCD_T0_ROUNDS");
    const int cap = e ? std::atoi(e) : FCD_T0_ROUNDS_DEFAULT;
    if (graph)
        hipLaunchKernelGGL((k_mst_tile0<64, 64, true>), g, b, 0, s, w, map_ids, nact, H, W, m, cap);
    else
        hipLaunchKernelGGL((k_mst_tile0<64, 64, false>), g, b, 0, s, w, map_ids, nact, H, W, m, cap);
    FCD_CHECK_LAUNCH();
}

}  // namespace fcdk
