/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into the product library.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.
 *
 * CPU restatement of the 2-D phase unwrapper the reference calls at
 * /root/reference/pyfcd/fcd.py:119 (`unwrap_phase(phase_angles)`), i.e.
 * scikit-image 0.18.3 `skimage.restoration.unwrap_phase` (non-wrap-around,
 * no mask).  Its C core ships only as a compiled .so in the survey container,
 * so this file restates the published algorithm (Herraez et al., Applied
 * Optics 41(35), 2002: "Fast two-dimensional phase-unwrapping algorithm based
 * on sorting by reliability following a noncontinuous path") as pinned by
 * probing the .so (see tests/golden/make_golden.py and SURVEY.md §8a row H1):
 *
 *   - PI is the double M_PI (probed: a step of 3.1415927 wraps, 3.14159265
 *     does not), TWOPI = 2*M_PI.
 *   - reliability of an interior pixel = H^2 + V^2 + D1^2 + D2^2 (f64, summed
 *     left to right, no FMA), H = wrap(w[l]-w) - wrap(w-w[r]) and the same for
 *     the vertical and the two diagonal neighbour pairs.
 *   - border pixels: the reference draws 9999999 + rand() (unseeded, so it
 *     varies from call to call); this restatement uses the constant 9999999,
 *     which only changes border pixels next to residues.
 *   - edges: all horizontal (row-major), then all vertical; reliab =
 *     rel(p1) + rel(p2); increment = find_wrap(v1, v2).  Sorted ascending,
 *     ties by edge index (the reference's quicksort leaves ties unspecified;
 *     interior ties do not occur in practice).
 *   - greedy merge: singleton p2 joins p1's group, else singleton p1 joins
 *     p2's group, else the strictly larger group absorbs the other (size tie:
 *     group 1 is absorbed into group 2).  Output = w + 2*pi*k.
 *
 * The merge bookkeeping (which pixel keeps k = 0) is reproduced literally, so
 * this restatement also reproduces the reference's global 2*pi offset.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_PI 3.141592653589793
#define ORC_TWOPI 6.283185307179586
#define ORC_BORDER_REL 9999999.0

static double orc_wrap(double x) {
    if (x > ORC_PI) return x - ORC_TWOPI;
    if (x < -ORC_PI) return x + ORC_TWOPI;
    return x;
}

static int orc_find_wrap(double a, double b) {
    double d = a - b;
    if (d > ORC_PI) return -1;
    if (d < -ORC_PI) return 1;
    return 0;
}

typedef struct {
    double rel;
    int32_t idx; /* edge index: horizontal edges first, then vertical */
} orc_key;

static int orc_cmp(const void* a, const void* b) {
    const orc_key* x = (const orc_key*)a;
    const orc_key* y = (const orc_key*)b;
    if (x->rel < y->rel) return -1;
    if (x->rel > y->rel) return 1;
    return (x->idx > y->idx) - (x->idx < y->idx);
}

/* Per-pixel reliability, f64.  Exported so tests can check the GPU's values. */
void orc_reliability(const double* w, int H, int W, double* rel) {
    for (int i = 0; i < H * W; ++i) rel[i] = ORC_BORDER_REL;
    for (int i = 1; i < H - 1; ++i) {
        for (int j = 1; j < W - 1; ++j) {
            const double* c = w + (size_t)i * W + j;
            double h = orc_wrap(c[-1] - c[0]) - orc_wrap(c[0] - c[1]);
            double v = orc_wrap(c[-W] - c[0]) - orc_wrap(c[0] - c[W]);
            double d1 = orc_wrap(c[-W - 1] - c[0]) - orc_wrap(c[0] - c[W + 1]);
            double d2 = orc_wrap(c[-W + 1] - c[0]) - orc_wrap(c[0] - c[W - 1]);
            double hh = h * h, vv = v * v, dd1 = d1 * d1, dd2 = d2 * d2;
            double s = hh + vv;
            s = s + dd1;
            s = s + dd2;
            rel[(size_t)i * W + j] = s;
        }
    }
}

/*
 * Unwrap one H x W map.  wrapped: f32 (as the reference feeds float32 angles,
 * promoted to f64 exactly).  k_out: int32 wrap counts; unwrapped_out (nullable):
 * f64 w + 2*pi*k.  Returns 0 on success, -1 on allocation failure.
 */
int orc_unwrap2d(const float* wrapped, int H, int W, int32_t* k_out, double* unwrapped_out) {
    size_t n = (size_t)H * W;
    size_t nh = (size_t)H * (W - 1), nv = (size_t)(H - 1) * W, ne = nh + nv;
    double* w = (double*)malloc(n * sizeof(double));
    double* rel = (double*)malloc(n * sizeof(double));
    orc_key* keys = (orc_key*)malloc(ne * sizeof(orc_key));
    int32_t* head = (int32_t*)malloc(n * sizeof(int32_t));
    int32_t* next = (int32_t*)malloc(n * sizeof(int32_t));
    int32_t* last = (int32_t*)malloc(n * sizeof(int32_t));
    int32_t* size = (int32_t*)malloc(n * sizeof(int32_t));
    if (!w || !rel || !keys || !head || !next || !last || !size) {
        free(w); free(rel); free(keys); free(head); free(next); free(last); free(size);
        return -1;
    }
    for (size_t i = 0; i < n; ++i) w[i] = (double)wrapped[i];
    orc_reliability(w, H, W, rel);

    size_t e = 0;
    for (int i = 0; i < H; ++i)
        for (int j = 0; j < W - 1; ++j, ++e) {
            size_t p = (size_t)i * W + j;
            keys[e].rel = rel[p] + rel[p + 1];
            keys[e].idx = (int32_t)e;
        }
    for (int i = 0; i < H - 1; ++i)
        for (int j = 0; j < W; ++j, ++e) {
            size_t p = (size_t)i * W + j;
            keys[e].rel = rel[p] + rel[p + W];
            keys[e].idx = (int32_t)e;
        }
    qsort(keys, ne, sizeof(orc_key), orc_cmp);

    for (size_t i = 0; i < n; ++i) {
        head[i] = (int32_t)i; next[i] = -1; last[i] = (int32_t)i; size[i] = 1; k_out[i] = 0;
    }
    for (size_t t = 0; t < ne; ++t) {
        int32_t ei = keys[t].idx;
        int32_t p1, p2;
        if ((size_t)ei < nh) {
            int i = ei / (W - 1), j = ei % (W - 1);
            p1 = i * W + j; p2 = p1 + 1;
        } else {
            int32_t v = ei - (int32_t)nh;
            p1 = v; p2 = v + W;
        }
        int32_t g1 = head[p1], g2 = head[p2];
        if (g1 == g2) continue;
        int inc = orc_find_wrap(w[p1], w[p2]);
        if (next[p2] < 0 && head[p2] == p2) {            /* p2 alone: join group 1 */
            next[last[g1]] = p2; last[g1] = p2; size[g1]++;
            head[p2] = g1; k_out[p2] = k_out[p1] - inc;
        } else if (next[p1] < 0 && head[p1] == p1) {     /* p1 alone: join group 2 */
            next[last[g2]] = p1; last[g2] = p1; size[g2]++;
            head[p1] = g2; k_out[p1] = k_out[p2] + inc;
        } else if (size[g1] > size[g2]) {                /* group 2 into group 1 */
            int32_t d = k_out[p1] - inc - k_out[p2];
            next[last[g1]] = g2; last[g1] = last[g2]; size[g1] += size[g2];
            for (int32_t q = g2; q >= 0; q = next[q]) { head[q] = g1; k_out[q] += d; }
        } else {                                         /* group 1 into group 2 */
            int32_t d = k_out[p2] + inc - k_out[p1];
            next[last[g2]] = g1; last[g2] = last[g1]; size[g2] += size[g1];
            for (int32_t q = g1; q >= 0; q = next[q]) { head[q] = g2; k_out[q] += d; }
        }
    }
    if (unwrapped_out)
        for (size_t i = 0; i < n; ++i) unwrapped_out[i] = w[i] + ORC_TWOPI * (double)k_out[i];
    free(w); free(rel); free(keys); free(head); free(next); free(last); free(size);
    return 0;
}

/* Number of residues (plaquettes with non-zero wrap-count circulation). */
long orc_count_residues(const float* wrapped, int H, int W) {
    long r = 0;
    for (int i = 0; i < H - 1; ++i)
        for (int j = 0; j < W - 1; ++j) {
            size_t p = (size_t)i * W + j;
            double a = wrapped[p], b = wrapped[p + 1], c = wrapped[p + W + 1], d = wrapped[p + W];
            int s = orc_find_wrap(a, b) + orc_find_wrap(b, c) + orc_find_wrap(c, d) + orc_find_wrap(d, a);
            r += (s != 0);
        }
    return r;
}
