/*
 * fcd.h — C ABI of the MI355X fast-checkerboard-demodulation engine.
 *
 * This is the drop-in boundary for the reference's hot path
 * (/root/reference/pyfcd/).  The reference is pure Python and
 * has no FFI of its own; each entry point below replaces the Python-level
 * interface cited next to it, and the ctypes binding in
 * trapped-modes-ltg_amd/pyfcd/_lib.py (shown in INTEGRATION.md) keeps the
 * reference's classmethod signatures on top of it.
 *
 * Conventions
 *   - Every function returns FCD_OK (0) or a negative FCD_E_* code; the
 *     message is available from fcd_last_error() (per host thread).
 *   - Buffers are caller-owned.  flags = FCD_HOST_PTRS: all array arguments
 *     are host pointers (the call copies and synchronises); FCD_DEVICE_PTRS:
 *     all array arguments are device pointers on the context's device and the
 *     call is asynchronous on `stream` (NULL = the context's own stream),
 *     except where a function says it synchronises.
 *   - Images are row-major float32 [rows][cols] (float64 where FCD_IMG_F64
 *     says so); complex arrays are interleaved complex64 (complex128).  rows and
 *     cols are any sides in [16, 16384] (the reference's scipy FFTs take any
 *     length): powers of two in [64, 4096] take the band-pruned fast path, every
 *     other shape (1920 x 1080, 1000 x 1000, 1023 x 1021, 4099 x 96 ...) the
 *     generic chain (the reference's own sequence of 2-D FFTs on mixed-radix /
 *     Bluestein transforms), with the same results and tolerances.  Larger
 *     sides return FCD_E_UNSUPPORTED (the exact unwrap's 32-bit vertex ids).
 *   - A context belongs to one device and one host thread at a time.
 */
#ifndef FCD_H
#define FCD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FCD_ABI_VERSION 7

enum {
    FCD_OK = 0,
    FCD_E_INVALID = -1,      /* bad argument (null pointer, size mismatch, ...) */
    FCD_E_UNSUPPORTED = -2,  /* shape not supported (a side outside [16, 16384]) */
    FCD_E_HIP = -3,          /* HIP runtime / launch failure */
    FCD_E_STATE = -4,        /* no reference set */
    FCD_E_NOPEAKS = -5,      /* < 2 carrier peaks: the reference raises ValueError/IndexError */
    FCD_E_INTERNAL = -6
};

enum { FCD_HOST_PTRS = 0, FCD_DEVICE_PTRS = 1 };

/* Flag bit of the temporal-analysis calls (OR-ed into flags): the stack holds
 * float64 samples instead of float32.  The reference hands a float64 series to
 * scipy / numpy unchanged (analyze.py:486-527), so it is not rounded to float32
 * on the way in. */
enum { FCD_STACK_F64 = 2 };

/* Flag bit of fcd_set_reference / fcd_find_peaks / fcd_fft2 (OR-ed into flags): the
 * images are float64 instead of float32.  The reference computes find_peaks' spectrum in
 * the image's own precision (fourier.py:18: a float64 image -> complex128 FFTs, as
 * pyval/val.py:98 hands compute_height_map), so the carrier picks of a float64 reference
 * come from the float64 spectrum, bit for bit; fcd_fft2 then writes complex128.  The
 * per-frame demodulation of fcd_process stays float32 (the reference image rounded to
 * float32 for the carrier signals). */
enum { FCD_IMG_F64 = 4 };

/* Frame sample formats (fcd_process_raw).  The reference decodes every frame
 * to float32 on the host (analyze.load_image, analyze.py:25-40); these let the
 * raw camera samples cross PCIe and be widened on the device instead.
 *   FCD_FMT_F32  float32 [rows][cols]
 *   FCD_FMT_U8   uint8   [rows][cols]          (8-bit PNG / BMP)
 *   FCD_FMT_U16  uint16  [rows][cols]          (16-bit, host byte order)
 *   FCD_FMT_P10  10-bit samples packed MSB-first, each row padded to a whole
 *                byte: rows * ceil(10 * cols / 8) bytes (TIFF BitsPerSample=10,
 *                FillOrder=1, the examples' reference_df.tif / prueba1_*.tif) */
enum { FCD_FMT_F32 = 0, FCD_FMT_U8 = 1, FCD_FMT_U16 = 2, FCD_FMT_P10 = 3 };

typedef struct fcd_ctx fcd_ctx;

/* Reference-derived state (fcd.compute_carriers, fcd.py:53-70). */
typedef struct {
    int64_t peaks[2][2];        /* fftshifted (row, col): [0] rightmost, [1] perpendicular (fourier.py:38-39) */
    double radius;              /* |p0 - p1| / 2 (fcd.py:68) */
    double calibration_factor;  /* fcd.compute_calibration_factor (fcd.py:87-101) */
    double frequencies[2][2];   /* Carrier.frequencies, (k_row, k_col) (carriers.py:12) */
    int32_t mask_count[2];      /* pixels inside each disk band-pass (carriers.py:17-20) */
    int32_t n_blobs;            /* blobs kept by find_peak_locations (<= 4, fourier.py:166-168) */
    int64_t blob_peaks[4][2];   /* their peak pixels, ascending intensity */
    double threshold;           /* 0.5 * max |F| after the high-pass (fourier.py:35; a float32 value for
                                   float32 images, float64 for FCD_IMG_F64) */
} fcd_ref_info;

int fcd_abi_version(void);
const char* fcd_last_error(void);

/* Allocate a context for `rows` x `cols` frames on HIP device `device`. */
int fcd_create(int device, int rows, int cols, fcd_ctx** out);
int fcd_destroy(fcd_ctx* ctx);
/* Waits for the context's own stream and for the last device-pointer call's work on
 * the stream it was given (fcd_process may return before its integration kernels
 * finish, see there). */
int fcd_synchronize(fcd_ctx* ctx);

/* Replaces fcd.compute_carriers(reference, square_size) (fcd.py:53-70) and,
 * inside it, fcd.compute_calibration_factor (fcd.py:72-101), fourier.find_peaks
 * (fourier.py:7-41) and Carrier.__init__ (carriers.py:10-24).  Synchronises. */
int fcd_set_reference(fcd_ctx* ctx, const float* reference, int flags, double square_size, fcd_ref_info* info);

/* Replaces Carrier(reference_image, calibration_factor, peak, peak_radius)
 * (carriers.py:10-24) for both carriers at once, with caller-chosen geometry
 * instead of fourier.find_peaks: peaks int64 [2][2] fftshifted (row, col),
 * radius double [2] (each carrier's own disk), the calibration factor of
 * Carrier.frequencies (carriers.py:12).  Carrier q's ccsgn comes from image
 * ref_q (ref1 may equal ref0 or be NULL: the same image).  Afterwards
 * fcd_process / fcd_phases_from_spectrum demodulate against these carriers and
 * info reports them (n_blobs = 0, threshold = 0).  Synchronises. */
int fcd_set_carriers(fcd_ctx* ctx, const float* ref0, const float* ref1, int flags, double calibration_factor,
                     const int64_t* peaks, const double* radius, fcd_ref_info* info);

/* fourier.find_peaks (fourier.py:7-41) + fcd.compute_calibration_factor
 * (fcd.py:72-101) for n images (many-reference workloads)
 * WITHOUT replacing the context's reference: infos[i] gets what
 * fcd_set_reference(images[i]) would report (peaks, radius, calibration factor,
 * carrier frequencies, disk pixel counts, blobs, threshold).  Batches of images
 * run every image-sized stage on the device (means, FFTs, |F| high-pass and its
 * maximum, thresholded candidates, 8-connected labelling, the 4 dimmest blobs'
 * peaks); the host finishes each image from its <= 4 peaks (an image with more than
 * 4096 above-threshold pixels is labelled on the host from its candidate list).
 * Synchronises. */
int fcd_find_peaks(fcd_ctx* ctx, const float* images, int n, int flags, double square_size, fcd_ref_info* infos);

/* Carrier arrays for the Python mirror: ccsgn complex64 [2][rows][cols]
 * (carriers.py:22-24, normalised like scipy ifft2) and the ifftshifted disk
 * masks uint8 [2][rows][cols] (carriers.py:17-20).  Host pointers, either may
 * be NULL.  Synchronises. */
int fcd_get_carriers(fcd_ctx* ctx, float* ccsgn, uint8_t* mask);

/* Replaces fcd.compute_height_map(reference, displaced, square_size, layers,
 * height, unwrap) (fcd.py:13-35) for a batch of n_frames frames against the
 * reference set by fcd_set_reference.  `height` is the effective height
 * (fcd.py:16-25; the caller folds layers via fcd.height_from_layers).
 * Outputs (any may be NULL):
 *   height_out  float32 [n][rows][cols]
 *   wrapped_out float32 [n][2][rows][cols]  -angle(ifft2(D*mask)*ccsgn) (fcd.py:118)
 *   k_out       int32   [n][2][rows][cols]  2*pi multiples: phases = wrapped + 2*pi*k (fcd.py:119)
 * With unwrap == 0 the phases are the wrapped angles (k_out is zero-filled).
 * Synchronises on the residue census when unwrap != 0.  Device pointers and only
 * height_out (the fused chain): the census is read back as soon as its flags are final,
 * so the call returns with the integration kernels still queued on `stream` (order later
 * work on that stream, or call fcd_synchronize); frames with residues are then redone by
 * the exact pass before the call returns.  A later call on another stream, and every
 * other entry point of the context, first waits for that queued work. */
int fcd_process(fcd_ctx* ctx, const float* frames, int n_frames, int flags, double height, int unwrap,
                float* height_out, float* wrapped_out, int32_t* k_out, void* stream);

/* fcd_process for frames stored in a raw sample format (FCD_FMT_*): the same
 * computation on the frames widened to float32 (exact: all samples < 2^24).
 * With host pointers and only height_out requested the call pipelines host
 * memory -> PCIe -> compute -> PCIe -> host memory over two slots and three
 * streams; page-locked caller buffers (fcd_host_alloc) are DMA'd directly,
 * pageable ones are staged through the context's pinned slots.  Replaces the
 * analyze.folder loop body (analyze.py:216-246: load_image + compute_height_map). */
int fcd_process_raw(fcd_ctx* ctx, const void* frames, int format, int n_frames, int flags, double height,
                    int unwrap, float* height_out, float* wrapped_out, int32_t* k_out, void* stream);

/* Bytes of one frame in `format` for this context's shape. */
int fcd_frame_bytes(fcd_ctx* ctx, int format, int64_t* bytes);

/* Page-locked host memory for frame / height stacks (no reference counterpart). */
int fcd_host_alloc(int64_t bytes, void** out);
int fcd_host_free(void* p);

/* Replaces fcd.compute_phases(displaced_fft, carriers, unwrap) (fcd.py:103-120)
 * for n spectra (complex64 [n][rows][cols], unshifted fft2 output). */
int fcd_phases_from_spectrum(fcd_ctx* ctx, const float* spectrum, int n, int flags, int unwrap, float* wrapped_out,
                             int32_t* k_out, void* stream);

/* Replaces skimage.restoration.unwrap_phase as called at fcd.py:119, for
 * n_maps float32 maps.  k_out int32 [n][rows][cols]; residues_out (nullable)
 * int32 [n] residue count per map.  Synchronises. */
int fcd_unwrap(fcd_ctx* ctx, const float* wrapped, int n_maps, int flags, int32_t* k_out, int32_t* residues_out,
               void* stream);

/* Replaces fourier.integrate_in_fourier(gx, gy, calibration_factor)
 * (fourier.py:115-137) for n gradient pairs (float32, result float32). */
int fcd_integrate(fcd_ctx* ctx, const float* gx, const float* gy, int n, double calibration_factor, int flags,
                  float* h_out, void* stream);

/* scipy.fft.fft2 of n real float32 images -> complex64 (as fcd.py:28). */
int fcd_fft2(fcd_ctx* ctx, const float* in, int n, int flags, float* out, void* stream);

/* Temporal analysis of a height-map stack.  `stack` is
 * float32 [T][rows][cols], or float64 with FCD_STACK_F64 in flags (frame pitch
 * rows*cols, row pitch cols, in elements; any shape,
 * not the context's); the block is [r0, r0 + bh) x [c0, c0 + bw), pixel
 * p = i * bw + j.  Host pointers: only the block is copied to the device.
 * All three accumulate in f64 and synchronise.
 *
 * fcd_temporal_spectrum — the mean spectrum of analyze.block_amplitude
 * (analyze.py:566-577: np.nanmean(|np.fft.fft(maps, axis=-1)|) over the
 * block's pixels, bins f < nf): sum_count (host) [nf][2] = sum of |X_p(f)|
 * over the pixels whose X_p(f) is not NaN, and their number. */
int fcd_temporal_spectrum(fcd_ctx* ctx, const void* stack, int T, int rows, int cols, int r0, int c0, int bh, int bw,
                          int flags, int nf, double* sum_count, void* stream);

/* The harmonic bins of analyze.block_amplitude (analyze.py:579-587):
 * x_out [bh*bw][nbins] complex128 = sum_t x_p(t) exp(-2 pi i bins[k] t / T)
 * (bins host memory; x_out host or device per flags). */
int fcd_temporal_bins(fcd_ctx* ctx, const void* stack, int T, int rows, int cols, int r0, int c0, int bh, int bw,
                      int flags, const int* bins, int nbins, double* x_out, void* stream);

/* analyze.spectrogram on a block (analyze.py:486-527: scipy.signal.spectrogram
 * of every pixel's series, detrend='constant', scaling='density', mode='psd',
 * one-sided): window float64 [nperseg] (host), segments start every
 * nperseg - noverlap samples, nseg = (T - nperseg) / (nperseg - noverlap) + 1,
 * nf = nperseg / 2 + 1; s_out float64 [bh*bw][nf][nseg]. */
int fcd_spectrogram(fcd_ctx* ctx, const void* stack, int T, int rows, int cols, int r0, int c0, int bh, int bw,
                    int flags, int nperseg, int noverlap, const double* window, double fs, double* s_out,
                    void* stream);

/* Stage timing (no reference counterpart; measurement only).  With enable != 0,
 * fcd_process records HIP events on its stream around each stage of every
 * chunk.  fcd_stage_times synchronises and returns the accumulated device
 * milliseconds since the last call: out[0] demodulation (forward FFT, disk
 * band-pass, inverse FFTs, phase), out[1] unwrap pre-pass, out[2] unwrap scan
 * + displacement + integration, out[3] whole first pass, out[4] the exact
 * (Boruvka) fix-up pass, out[5] frames that needed it, out[6] launch groups
 * (chunks) covered, out[7] frames per launch group (the chunk size); *frames =
 * frames covered by the first pass. */
int fcd_profile(fcd_ctx* ctx, int enable);
int fcd_stage_times(fcd_ctx* ctx, double* out8, int64_t* frames);

#ifdef __cplusplus
}
#endif

#endif /* FCD_H */
