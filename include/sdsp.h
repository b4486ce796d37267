/*
 * sdsp.h — C ABI of the MI355X-native streaming filter engine (libsdsp.so).
 *
 * Drop-in boundary for juliantos/solid-dsp's hot path.  Every entry point
 * replaces one method of the reference's Rust API; the reference item it
 * replaces is cited (paths relative to the reference checkout).  A Rust shim
 * crate keeps `solid::filter::*` / `solid::dot_product::*` and forwards to
 * these symbols (INTEGRATION.md shows the bindings).
 *
 * Conventions (mirroring the reference):
 *  - Construction copies taps into the handle (DotProduct::new, alloc_zeroed,
 *    src/dot_product/mod.rs:57-87) and can fail with the reference's error
 *    enums (FIRErrorCode src/filter/fir/mod.rs:40-45, IIRErrorCode
 *    src/filter/iir/mod.rs:41-49, SecondOrderErrorCode src/filter/iir/sos.rs:19-21),
 *    returned as sdsp_status codes.  Execution cannot fail except for device
 *    errors (>= SDSP_E_DEVICE); sdsp_last_error() gives the message.
 *  - Complex samples/taps are interleaved {re, im}, the #[repr(C)] layout of
 *    num::Complex<T>.
 *  - A handle is bound to one device and owns: the tap copy, the delay-line
 *    state (the reference's `Window`, src/window/mod.rs:9-77) resident in HBM,
 *    one hipStream_t and device staging buffers.  A handle is not thread safe
 *    (the reference types are !Send); distinct handles may run concurrently.
 *  - `*_execute_block` takes HOST slices (like `&[In] -> Vec<Out>`) and is
 *    PCIe-bound; `*_execute_block_device` takes device pointers (HBM resident)
 *    and a hipStream_t and is asynchronous.  NULL = the handle's own stream;
 *    the legacy null stream is passed as hipStreamLegacy ((void*)1).  Calls on
 *    one handle must be stream-ordered (the delay line is updated in HBM at
 *    the end of every call).
 *  - No CPU fallback: with no usable gfx950 device every create call returns
 *    SDSP_E_NO_DEVICE.
 *  - Streaming calls do not filter in place: an input block that overlaps its
 *    output block is rejected with SDSP_E_INVALID_ARGUMENT (the kernels read
 *    each input window, and the delay-line update reads the block's tail, after
 *    other workgroups have started writing outputs).
 *  - Host-side state calls (reset, get/set_state, clone, set_scale) first wait
 *    for the work an earlier *_execute_block_device queued on a caller stream.
 */
#ifndef SDSP_H
#define SDSP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDSP_API __attribute__((visibility("default")))

/* (Coef, In) pairs.  Out = Coef * In (num-complex Mul). */
typedef enum {
    SDSP_RR32 = 0, /* f32  taps, f32  samples                                  */
    SDSP_RC32 = 1, /* f32  taps, c32  samples ("crcf")                         */
    SDSP_CC32 = 2, /* c32  taps, c32  samples ("cccf")                         */
    SDSP_RR64 = 3, /* f64  taps, f64  samples (the reference Filter path)      */
    SDSP_RC64 = 4, /* f64  taps, c64  samples (FIRFilter<f64, Complex<f64>>)   */
    SDSP_CC64 = 5  /* c64  taps, c64  samples                                  */
} sdsp_dtype;

/* Kernel selection for FIR-type and IIR handles.  A new handle uses SDSP_ALGO_EXACT:
 * by default every result is bit-identical to the reference algorithm at the handle's
 * precision, whatever the block size.  The fast kernels are opt-in. */
typedef enum {
    SDSP_ALGO_AUTO = 0,  /* FFT overlap-save for 32-bit complex blocks >= 65536 samples, else EXACT */
    SDSP_ALGO_EXACT = 1, /* direct form in the reference summation order, no FMA contraction:
                            bit-identical to the reference algorithm at the handle's precision */
    SDSP_ALGO_FMA = 2,   /* direct form, same order, fused multiply-add                      */
    SDSP_ALGO_FFT = 3    /* overlap-save fast convolution (N = 4096) in LDS                  */
} sdsp_algo;

typedef enum {
    SDSP_OK = 0,
    /* FIRErrorCode (src/filter/fir/mod.rs:40-45) */
    SDSP_E_COEFFICIENTS_LENGTH_ZERO = 1,
    SDSP_E_DECIMATION_LESS_THAN_ONE = 2,
    SDSP_E_INTERPOLATION_LESS_THAN_ONE = 3,
    SDSP_E_NOT_ENOUGH_FILTERS = 4,
    /* IIRErrorCode (src/filter/iir/mod.rs:41-49) */
    SDSP_E_NUMERATOR_LENGTH_ZERO = 10,
    SDSP_E_DENOMINATOR_LENGTH_ZERO = 11,
    SDSP_E_SOS_SIZE_ZERO = 12,
    SDSP_E_SOS_SIZE_MISMATCH = 13,
    SDSP_E_SOS_SIZE_NOT_MULTIPLE_OF_3 = 14,
    SDSP_E_IIR_DECIMATION_LESS_THAN_ONE = 15,
    SDSP_E_IIR_INTERPOLATION_LESS_THAN_ONE = 16,
    /* SecondOrderErrorCode (src/filter/iir/sos.rs:19-21) */
    SDSP_E_SOS_COEFFICIENTS_NOT_IN_RANGE = 20,
    /* NCOErrorCode (src/nco/mod.rs:7-10) */
    SDSP_E_NCO_BANDWIDTH_OUT_OF_RANGE = 30,
    /* AGCErrorCode (src/auto_gain_control/mod.rs:49-56) */
    SDSP_E_AGC_BANDWIDTH_OUT_OF_RANGE = 40,
    SDSP_E_AGC_SIGNAL_LEVEL_OUT_OF_RANGE = 41,
    SDSP_E_AGC_GAIN_BELOW_THRESHOLD = 42,
    SDSP_E_AGC_SCALE_BELOW_THRESHOLD = 43,
    SDSP_E_AGC_SAMPLES_TOO_LOW = 44,
    /* argument errors the reference reports by panicking */
    SDSP_E_INVALID_ARGUMENT = 90,
    SDSP_E_UNSUPPORTED = 91,
    /* device errors */
    SDSP_E_DEVICE = 100,
    SDSP_E_NO_DEVICE = 101,
    SDSP_E_OUT_OF_MEMORY = 102
} sdsp_status;

SDSP_API const char* sdsp_last_error(void);
SDSP_API const char* sdsp_version(void);
/* number of visible gfx950 devices (0 when none) */
SDSP_API int sdsp_device_count(void);
/* bytes of one sample / one tap of a dtype */
SDSP_API size_t sdsp_sample_size(int dtype);
SDSP_API size_t sdsp_coef_size(int dtype);

/* ------------------------------------------------------------------------
 * FIR and decimating FIR  (FIRFilter src/filter/fir/mod.rs:58-304,
 *                          DecimatingFIRFilter src/filter/fir/decim.rs:5-281)
 * A FIR handle is a DecimatingFIRFilter with decimation 1.  `channels`
 * independent delay lines share the taps; device/host buffers are
 * channel-major: sample i of channel c at [c * n + i].
 * ------------------------------------------------------------------------ */
typedef struct sdsp_fir sdsp_fir;

/* FIRFilter::new(&[Coef], scale)                    src/filter/fir/mod.rs:79-88 */
SDSP_API int sdsp_fir_create(sdsp_fir** out, int dtype, const void* taps, size_t len,
                             const void* scale, int device);
/* DecimatingFIRFilter::new(&[Coef], scale, M)       src/filter/fir/decim.rs:27-42 */
SDSP_API int sdsp_decim_create(sdsp_fir** out, int dtype, const void* taps, size_t len,
                               const void* scale, size_t decimation, int device);
/* channel count (default 1); resets the delay lines */
SDSP_API int sdsp_fir_set_channels(sdsp_fir* h, size_t channels);
SDSP_API int sdsp_fir_set_algo(sdsp_fir* h, int algo);
SDSP_API int sdsp_fir_get_algo(const sdsp_fir* h); /* resolved algorithm */
/* Process-wide starting algorithm of handles created afterwards (sdsp_fir_create,
 * sdsp_decim_create, the sdsp_iir_* / sdsp_sos_create family; PFB / interpolator handles take FMA
 * when it is FMA, else EXACT): SDSP_ALGO_EXACT (the default: every result bit-identical to the
 * reference), SDSP_ALGO_AUTO (blocks of >= 65536 32-bit complex samples on the overlap-save FIR,
 * >= 65536 32-bit inputs on the FMA decimator, IIR blocks of >= 8192 samples on the scans where
 * the cascade admits one; everything shorter on the reference order) or SDSP_ALGO_FMA.  Read from
 * the environment variable SDSP_DEFAULT_ALGO ("auto" / "exact" / "fma") at the first handle or
 * query unless set here first.  Not part of the reference API: it lets a deployment move an
 * unchanged caller of that API onto the fast paths.  Existing handles keep their algorithm. */
SDSP_API int sdsp_set_default_algo(int algo);
SDSP_API int sdsp_get_default_algo(void);
/* kernel-variant knobs: performance only, every accepted value computes the complete output
 * (retired keys of earlier builds are rejected with SDSP_E_INVALID_ARGUMENT). */
typedef enum {
    SDSP_TUNE_DECIM_SEG = 6,     /* FMA decimator: outputs per lane group (0 = automatic) */
    SDSP_TUNE_IIR_WAVE_SCAN = 7, /* IIR scan kernel: 0 = block scan, 1 = wave scan with 256-byte chunks (default
                                    for complex and f64 samples), 2 = 128-byte chunks (default for real f32),
                                    3/4 = paired 128/64-byte chunks (real f32), 5 = 256-byte chunks rerun
                                    instead of corrected, 6 = 128-byte chunks without the register prefetch */
    SDSP_TUNE_CHAN_STREAMING = 8, /* channeliser: streaming M=1024 kernel where it applies: 3 = 1024-thread
                                     workgroups, sixteen frames per round, the next round's samples
                                     requested before this round's stores; 1 = the same without; 2 / 4 =
                                     512-thread workgroups without / with that prefetch; 5 (default) / 6 =
                                     as 3 with eight / four frames per round (waves 0..7 / 0..3 transform);
                                     0 = per-frame kernel */
    SDSP_TUNE_CHAN_FRAMES_PER_BLOCK = 9, /* streaming channeliser: frames per workgroup (0 = automatic, 64..256) */
    SDSP_TUNE_OLS_KERNEL = 14,   /* overlap-save segments (16-byte aligned rows): 0 (default) one-shot
                                    XCD-ordered kernels: the interior segments in one launch (one halo row
                                    compiled in when L <= 257), the boundary segments and the next history
                                    in a second,
                                    1 persistent packed kernel for the interior segments (L <= 1025),
                                    2 scalar kernel, 3 the one-shot kernel with 16-byte lanes */
    SDSP_TUNE_CHAN_XCD_ORDER = 15, /* streaming channeliser: 1 (default) = each XCD walks a contiguous
                                     eighth of the frame chunks, 0 = launch order */
    SDSP_TUNE_HOST_STEP = 16,     /* FIR / decimator: 1 (default) = execute(sample), push and host blocks with
                                     n * len <= SDSP_TUNE_HOST_BLOCK_MACS run on the host against the
                                     handle's delay line (single-channel handles, not the FFT algorithm;
                                     reference arithmetic, bit-identical to the EXACT/FMA kernels);
                                     0 = every call launches device work (one-sample step kernel) */
    SDSP_TUNE_HOST_BLOCK_MACS = 17, /* host-block threshold in multiply-adds (default 65536) */
    SDSP_TUNE_FFT_GROUP = 18,      /* four-step passes on the generic pass kernel: at most this many
                                      transforms per workgroup (1..64, default 4) */
    SDSP_TUNE_FFT_WAVE1024 = 19,   /* four-step passes of 1024 points (c32): 16 (default) pipelined persistent
                                      wave-FFT kernel, 1 / 8 one-shot with 16 / 8 transforms per workgroup,
                                      0 the generic pass kernel */
    SDSP_TUNE_ACORR_KERNEL = 20,   /* AutoCorrelator: 0 (default) pipelined kernel on interior tiles (delay
                                      and window <= 128), one-shot kernel elsewhere; 1 the one-shot kernel
                                      everywhere, delayed input staged in LDS (delay <= 256); 2 the one-shot
                                      kernel with two loads per product */
    SDSP_TUNE_AGC_KERNEL = 21      /* AGC bank: 0 (default) pipelined kernel for calls < 2^22 samples per
                                      channel, 1 the plain per-sample kernel */
} sdsp_tune_key;
SDSP_API int sdsp_fir_set_tuning(sdsp_fir* h, int key, int value);
SDSP_API void sdsp_fir_destroy(sdsp_fir* h);        /* Drop */
/* Clone (derive(Clone), fir/mod.rs:58): same taps and a snapshot of the delay line */
SDSP_API int sdsp_fir_clone(const sdsp_fir* h, sdsp_fir** out);
/* set_scale / get_scale                              fir/mod.rs:103-124, decim.rs:57-78 */
SDSP_API int sdsp_fir_set_scale(sdsp_fir* h, const void* scale);
SDSP_API int sdsp_fir_get_scale(const sdsp_fir* h, void* scale);
/* len (fir/mod.rs:139-142), get_decimation (decim.rs:92-95) */
SDSP_API size_t sdsp_fir_len(const sdsp_fir* h);
SDSP_API size_t sdsp_fir_decimation(const sdsp_fir* h);
/* coefficients(): the stored (REVERSED) taps, as DotProduct::coefficents (fir/mod.rs:173-176) */
SDSP_API int sdsp_fir_coefficients(const sdsp_fir* h, void* out_len_taps);
/* number of outputs a block of n inputs produces from the current phase */
SDSP_API size_t sdsp_fir_output_count(const sdsp_fir* h, size_t n);
/* Filter::execute(sample) -> Vec<Out> (0 or 1 outputs)  fir/mod.rs:209-212, decim.rs:221-228
 * (single channel handles only) *n_out = 0/1 */
SDSP_API int sdsp_fir_execute(sdsp_fir* h, const void* sample, void* out, size_t* n_out);
/* Filter::execute_block(&[In]) -> Vec<Out>          fir/mod.rs:235-241, decim.rs:250-256
 * in: channels*n host samples; out: channels*output_count(n) host samples */
SDSP_API int sdsp_fir_execute_block(sdsp_fir* h, const void* in, size_t n, void* out, size_t* n_out);
/* device-resident variant (asynchronous on `stream`; NULL = handle stream) */
SDSP_API int sdsp_fir_execute_block_device(sdsp_fir* h, const void* d_in, size_t n, void* d_out,
                                           size_t* n_out, void* stream);
/* DecimatingFIRFilter::push / write (advance phase, no output)  decim.rs:115-118, 136-139 */
SDSP_API int sdsp_decim_push(sdsp_fir* h, const void* sample);
SDSP_API int sdsp_decim_write(sdsp_fir* h, const void* samples, size_t n);
/* reset: zero the delay lines and the phase (Window::reset, src/window/mod.rs:54-56) */
SDSP_API int sdsp_fir_reset(sdsp_fir* h);
/* delay-line state: the last len-1 inputs per channel, oldest first (+ the phase) */
SDSP_API size_t sdsp_fir_state_len(const sdsp_fir* h);
SDSP_API int sdsp_fir_get_state(const sdsp_fir* h, void* hist, size_t* phase);
SDSP_API int sdsp_fir_set_state(sdsp_fir* h, const void* hist, size_t phase);
/* Filter::frequency_response / group_delay (host f64)   fir/mod.rs:263-303 */
SDSP_API int sdsp_fir_frequency_response(const sdsp_fir* h, double f, double* re_im);
SDSP_API int sdsp_fir_group_delay(const sdsp_fir* h, double f, double* delay);
SDSP_API int sdsp_fir_synchronize(sdsp_fir* h);
/* diagnostic (no reference counterpart): how many calls on this handle queued device work or moved
   its delay line between host and device (kernel launches, async copies, history pulls / flushes);
   per-sample calls on the host step leave it unchanged */
SDSP_API unsigned long long sdsp_fir_device_ops(const sdsp_fir* h);

/* ------------------------------------------------------------------------
 * Polyphase filterbank and interpolating FIR
 *  (PolyPhaseFilterBank src/filter/fir/pfb.rs:3-91,
 *   InterpolatingFIRFilter src/filter/fir/interp.rs:6-138)
 * ------------------------------------------------------------------------ */
typedef struct sdsp_pfb sdsp_pfb;

/* PolyPhaseFilterBank::new(&[Coef], filters, scale)  pfb.rs:24-49 */
SDSP_API int sdsp_pfb_create(sdsp_pfb** out, int dtype, const void* taps, size_t len, size_t filters,
                             const void* scale, int device);
/* InterpolatingFIRFilter::new(&[Coef], M)            interp.rs:27-54 */
SDSP_API int sdsp_interp_create(sdsp_pfb** out, int dtype, const void* taps, size_t len,
                                size_t interpolation, int device);
SDSP_API void sdsp_pfb_destroy(sdsp_pfb* h);
SDSP_API int sdsp_pfb_clone(const sdsp_pfb* h, sdsp_pfb** out);
SDSP_API size_t sdsp_pfb_len(const sdsp_pfb* h);          /* number of filters M */
SDSP_API size_t sdsp_pfb_subfilter_len(const sdsp_pfb* h); /* K */
SDSP_API int sdsp_pfb_set_scale(sdsp_pfb* h, const void* scale);
SDSP_API int sdsp_pfb_get_scale(const sdsp_pfb* h, void* scale);
/* coefficents(): M x K branch coefficients (stored order) */
SDSP_API int sdsp_pfb_coefficients(const sdsp_pfb* h, void* out_mk);
/* push(sample)  pfb.rs:81-83 */
SDSP_API int sdsp_pfb_push(sdsp_pfb* h, const void* sample);
/* execute(index) on the current window  pfb.rs:85-90 */
SDSP_API int sdsp_pfb_execute(sdsp_pfb* h, size_t index, void* out);
/* reset  pfb.rs:77-79 */
SDSP_API int sdsp_pfb_reset(sdsp_pfb* h);
/* dot-product order: SDSP_ALGO_EXACT (default, the reference's sequential sum,
 * bit-identical) or SDSP_ALGO_FMA (fused multiply-add, same order) */
SDSP_API int sdsp_pfb_set_algo(sdsp_pfb* h, int algo);
/* independent channels in one handle: blocks are channel-major [channels][n]
 * in, [channels][n*M] out; resets every channel's window */
SDSP_API int sdsp_pfb_set_channels(sdsp_pfb* h, size_t channels);
/* for each input: push, then all M branch outputs -> out[n*M]
 * (InterpolatingFIRFilter::execute_block  interp.rs:102-111).  The _device form
 * rejects overlapping input and output blocks (SDSP_E_INVALID_ARGUMENT). */
SDSP_API int sdsp_pfb_execute_block(sdsp_pfb* h, const void* in, size_t n, void* out);
SDSP_API int sdsp_pfb_execute_block_device(sdsp_pfb* h, const void* d_in, size_t n, void* d_out, void* stream);
SDSP_API int sdsp_pfb_frequency_response(const sdsp_pfb* h, double f, double* re_im);
SDSP_API int sdsp_pfb_group_delay(const sdsp_pfb* h, double f, double* delay);
SDSP_API int sdsp_pfb_synchronize(sdsp_pfb* h);

/* ------------------------------------------------------------------------
 * IIR family  (IIRFilter src/filter/iir/mod.rs:62-414, SecondOrderFilter
 *  src/filter/iir/sos.rs:34-231, DecimatingIIRFilter src/filter/iir/decim.rs:5-280,
 *  InterpolatingIIRFilter src/filter/iir/interp.rs:6-268).
 * dtype: SDSP_RR32, SDSP_RC32, SDSP_RR64, SDSP_RC64 (real coefficients, like
 * the reference's Conj + Real bound).  type: 0 = Normal, 1 = SecondOrder.
 * algo: SDSP_ALGO_EXACT = reference-order serial recurrence (one lane per
 * channel, bit-identical); SDSP_ALGO_FMA = block-parallel scan (stable SOS
 * cascades); SDSP_ALGO_AUTO = scan for long blocks when the cascade admits it.
 * ------------------------------------------------------------------------ */
typedef struct sdsp_iir sdsp_iir;

/* IIRFilter::new(&ff, &fb, IIRFilterType)            mod.rs:92-164 */
SDSP_API int sdsp_iir_create(sdsp_iir** out, int dtype, const void* ff, size_t nff, const void* fb, size_t nfb,
                             int type, int device);
/* DecimatingIIRFilter::new(&ff, &fb, type, M)         decim.rs:11-30 */
SDSP_API int sdsp_iir_decim_create(sdsp_iir** out, int dtype, const void* ff, size_t nff, const void* fb,
                                   size_t nfb, int type, size_t decimation, int device);
/* InterpolatingIIRFilter::new(&ff, &fb, type, M)      interp.rs:12-31 */
SDSP_API int sdsp_iir_interp_create(sdsp_iir** out, int dtype, const void* ff, size_t nff, const void* fb,
                                    size_t nfb, int type, size_t interpolation, int device);
/* SecondOrderFilter::new(&ff, &fb) (f64)              sos.rs:55-75 */
SDSP_API int sdsp_sos_create(sdsp_iir** out, const double* ff, size_t nff, const double* fb, size_t nfb,
                             int device);
SDSP_API void sdsp_iir_destroy(sdsp_iir* h);
SDSP_API int sdsp_iir_clone(const sdsp_iir* h, sdsp_iir** out);
SDSP_API int sdsp_iir_set_channels(sdsp_iir* h, size_t channels);
SDSP_API int sdsp_iir_set_algo(sdsp_iir* h, int algo);
/* kernel-variant knob (SDSP_TUNE_IIR_WAVE_SCAN; performance only) */
SDSP_API int sdsp_iir_set_tuning(sdsp_iir* h, int key, int value);
/* scan plan of section group g: warm-up chunks (0 = scan not admissible) and chunk length */
SDSP_API int sdsp_iir_scan_info(const sdsp_iir* h, int group, int* warmup_chunks, int* chunk);
/* the wave scan a cascade group gets when the scan is requested: 0 none (serial recurrence),
 * 1 warm-up chunks (decaying state response), 2 exact inter-wave carries (non-decaying but
 * well conditioned: aggregate pass + carry scan + output pass); -1 bad handle/group */
SDSP_API int sdsp_iir_wscan_mode(const sdsp_iir* h, int group);
SDSP_API size_t sdsp_iir_output_count(const sdsp_iir* h, size_t n);
/* Filter::execute / execute_block                     mod.rs:270-316, decim.rs:203-225, interp.rs:197-214 */
SDSP_API int sdsp_iir_execute(sdsp_iir* h, const void* sample, void* out, size_t* n_out);
SDSP_API int sdsp_iir_execute_block(sdsp_iir* h, const void* in, size_t n, void* out, size_t* n_out);
SDSP_API int sdsp_iir_execute_block_device(sdsp_iir* h, const void* d_in, size_t n, void* d_out, size_t* n_out,
                                           void* stream);
SDSP_API int sdsp_iir_reset(sdsp_iir* h);
/* state: SOS (w1, w2) per section per channel; Normal the last cap-1 w values, newest first */
SDSP_API size_t sdsp_iir_state_len(const sdsp_iir* h);
SDSP_API int sdsp_iir_get_state(const sdsp_iir* h, void* state, size_t* phase);
SDSP_API int sdsp_iir_set_state(sdsp_iir* h, const void* state, size_t phase);
/* numerator_coefs() / denominator_coefs() as stored (mod.rs:123-127,156-157); which: 0 num, 1 den */
SDSP_API size_t sdsp_iir_num_coefs(const sdsp_iir* h, int which);
SDSP_API int sdsp_iir_coefficients(const sdsp_iir* h, double* num, double* den);
/* SecondOrderFilter numerator_coefs (a[1..]/a0) and denominator_coefs (b/a0) of one section */
SDSP_API int sdsp_sos_section_coefs(const sdsp_iir* h, int section, double* num2, double* den3);
/* Filter::frequency_response / group_delay (host f64)  mod.rs:336-413 */
SDSP_API int sdsp_iir_frequency_response(const sdsp_iir* h, double f, double* re_im);
SDSP_API int sdsp_iir_group_delay(const sdsp_iir* h, double f, double* delay);
SDSP_API int sdsp_iir_synchronize(sdsp_iir* h);

/* ------------------------------------------------------------------------
 * FFT  (FFT::new / FFT::execute, src/fft/mod.rs:175-215).  direction: 0 FORWARD,
 * 1 REVERSE (unnormalised, like the reference).  precision: 0 = complex f32,
 * 1 = complex f64.  Sizes 1 .. 2^24, every size the reference plans (SURVEY §8f
 * row 2).  Power-of-two sizes up to 4096 run a radix-4 Stockham FFT in LDS, larger
 * powers of two a four-step FFT (two strided LDS passes, f64 inter-pass twiddles);
 * other sizes up to 512 a direct DFT, larger ones Bluestein's chirp-z transform
 * over a power-of-two convolution (where the reference plans Rader / mixed radix,
 * src/fft/mod.rs:123-170; the results agree within the transforms' rounding).
 * ------------------------------------------------------------------------ */
typedef struct sdsp_fft sdsp_fft;
SDSP_API int sdsp_fft_create(sdsp_fft** out, size_t nfft, int direction, int precision, int device);
SDSP_API void sdsp_fft_destroy(sdsp_fft* h);
SDSP_API size_t sdsp_fft_len(const sdsp_fft* h);
/* device plan: 0 direct DFT, 1 power of two in LDS, 2 Bluestein, 3 four-step power of two */
SDSP_API int sdsp_fft_method(const sdsp_fft* h);
/* kernel-variant knobs: SDSP_TUNE_FFT_GROUP, SDSP_TUNE_FFT_WAVE1024 (performance only) */
SDSP_API int sdsp_fft_set_tuning(sdsp_fft* h, int key, int value);
/* `batch` contiguous transforms of nfft complex samples */
SDSP_API int sdsp_fft_execute(sdsp_fft* h, const void* in, void* out, size_t batch);
SDSP_API int sdsp_fft_execute_device(sdsp_fft* h, const void* d_in, void* d_out, size_t batch, void* stream);

/* ------------------------------------------------------------------------
 * PFB + FFT channeliser (build-defined composition of PolyPhaseFilterBank's
 * coefficient layout, src/filter/fir/pfb.rs:24-49, and FFT FORWARD; SURVEY
 * Appendix A.6).  M channels (power of two, 4..4096), K = len / M taps per
 * branch, branch p fed by input phase M-1-p.  dtype SDSP_RC32 or SDSP_RC64.
 * Blocks are whole frames: n (per stream) a multiple of M; out[s][frame][M].
 * ------------------------------------------------------------------------ */
typedef struct sdsp_chan sdsp_chan;
SDSP_API int sdsp_chan_create(sdsp_chan** out, int dtype, const void* taps, size_t len, size_t channels,
                              int device);
SDSP_API void sdsp_chan_destroy(sdsp_chan* h);
SDSP_API int sdsp_chan_set_streams(sdsp_chan* h, size_t streams);
/* kernel-variant knobs: SDSP_TUNE_CHAN_STREAMING, SDSP_TUNE_CHAN_FRAMES_PER_BLOCK,
 * SDSP_TUNE_CHAN_XCD_ORDER (performance only) */
SDSP_API int sdsp_chan_set_tuning(sdsp_chan* h, int key, int value);
SDSP_API int sdsp_chan_reset(sdsp_chan* h);
SDSP_API int sdsp_chan_execute_block(sdsp_chan* h, const void* in, size_t n, void* out, size_t* frames);
SDSP_API int sdsp_chan_execute_block_device(sdsp_chan* h, const void* d_in, size_t n, void* d_out,
                                            size_t* frames, void* stream);
SDSP_API int sdsp_chan_synchronize(sdsp_chan* h);

/* ------------------------------------------------------------------------
 * DotProduct (src/dot_product/mod.rs:37-171): DotProduct::new(&coefs, direction)
 * + Execute::execute(&samples), reference order (bit-identical).  direction:
 * 0 FORWARD, 1 REVERSE.  The batched form runs `batch` sample vectors of n
 * samples spaced `stride` samples apart (device pointers, current device).
 * ------------------------------------------------------------------------ */
SDSP_API int sdsp_dot_execute(int dtype, const void* coefs, size_t len, int direction, const void* samples,
                              size_t n, void* out);
SDSP_API int sdsp_dot_execute_batched_device(int dtype, const void* coefs, size_t len, int direction,
                                             const void* d_samples, size_t n, size_t stride, size_t batch,
                                             void* d_out, void* stream);

/* ------------------------------------------------------------------------
 * AutoCorrelator (src/filter/auto_correlator/mod.rs:26-214), SURVEY §8f row 3.
 * precision: 0 = Complex<f32>, 1 = Complex<f64> (the reference's push() needs
 * C = f64, :99-102; the f32 handle runs the same operations at f32).  After each
 * push the output is sum_{j < window} x[n-j] * conj(x[n-j-delay]) over the delayed
 * Window's unfilled tail (terms with j + delay >= window are zero), newest first,
 * from zero — bit-identical to the reference order.  `channels` independent
 * correlators, channel-major buffers.  Energy: sum of |x|^2 over the last
 * window_size inputs (f64; the reference's running sum agrees to rounding).
 * ------------------------------------------------------------------------ */
typedef struct sdsp_acorr sdsp_acorr;
/* AutoCorrelator::<C>::new(window_size, delay)        :51-62 */
SDSP_API int sdsp_acorr_create(sdsp_acorr** out, size_t window_size, size_t delay, int precision, int device);
SDSP_API void sdsp_acorr_destroy(sdsp_acorr* h);
SDSP_API int sdsp_acorr_set_channels(sdsp_acorr* h, size_t channels);
/* kernel-variant knob: SDSP_TUNE_ACORR_KERNEL (performance only) */
SDSP_API int sdsp_acorr_set_tuning(sdsp_acorr* h, int key, int value);
SDSP_API size_t sdsp_acorr_window_size(const sdsp_acorr* h);
SDSP_API size_t sdsp_acorr_delay(const sdsp_acorr* h);
/* reset  :76-85 */
SDSP_API int sdsp_acorr_reset(sdsp_acorr* h);
/* push (one sample, single channel)  :99-111;  write (push only)  :128-137 */
SDSP_API int sdsp_acorr_push(sdsp_acorr* h, const void* sample);
SDSP_API int sdsp_acorr_write(sdsp_acorr* h, const void* samples, size_t n);
SDSP_API int sdsp_acorr_write_device(sdsp_acorr* h, const void* d_samples, size_t n, void* stream);
/* execute() on the current windows (no push), one value per channel  :156-163 */
SDSP_API int sdsp_acorr_execute(sdsp_acorr* h, void* out);
/* execute_block: push then execute per sample  :181-191 */
SDSP_API int sdsp_acorr_execute_block(sdsp_acorr* h, const void* in, size_t n, void* out);
SDSP_API int sdsp_acorr_execute_block_device(sdsp_acorr* h, const void* d_in, size_t n, void* d_out, void* stream);
/* get_energy, one f64 per channel  :212-214 */
SDSP_API int sdsp_acorr_get_energy(sdsp_acorr* h, double* energy);
SDSP_API int sdsp_acorr_synchronize(sdsp_acorr* h);

/* ------------------------------------------------------------------------
 * NCO (src/nco/mod.rs:27-187), SURVEY §8f row 4.  Phase and frequency are u32
 * registers on the host (as in the reference); sample blocks are mixed on the
 * device with the reference's 1024-entry f64 sine table and index rule.
 * mix_block: out[i] = mix_up(x[i]) (down = 0) or mix_down(x[i]) (down = 1), then
 * step() — the loop mix_up_block / mix_down_block spell out (:153-172; the
 * reference's versions index an empty Vec and panic for any non-empty input).
 * precision 0 = Complex<f32> samples (f32 table and product), 1 = Complex<f64>
 * (bit-identical to the reference).
 * ------------------------------------------------------------------------ */
typedef struct sdsp_nco sdsp_nco;
SDSP_API int sdsp_nco_create(sdsp_nco** out, int device);                     /* NCO::new  :36-50 */
SDSP_API void sdsp_nco_destroy(sdsp_nco* h);
SDSP_API int sdsp_nco_reset(sdsp_nco* h);                                     /* :53-56 */
SDSP_API uint32_t sdsp_nco_constrain(double theta);                           /* constrain :175-187 */
SDSP_API int sdsp_nco_set_frequency(sdsp_nco* h, double delta_theta);         /* :59-61 */
SDSP_API int sdsp_nco_adjust_frequency(sdsp_nco* h, double dt);               /* :64-66 */
SDSP_API double sdsp_nco_get_frequency(const sdsp_nco* h);                    /* :69-76 */
SDSP_API int sdsp_nco_set_phase(sdsp_nco* h, double phi);                     /* :79-81 */
SDSP_API int sdsp_nco_adjust_phase(sdsp_nco* h, double delta_phi);            /* :84-86 */
SDSP_API double sdsp_nco_get_phase(const sdsp_nco* h);                        /* :89-91 */
SDSP_API int sdsp_nco_step(sdsp_nco* h);                                      /* :94-96 */
SDSP_API int sdsp_nco_sincos(const sdsp_nco* h, double* sin_cos);             /* :104-117 (sin, cos) */
SDSP_API int sdsp_nco_set_internal_pll_bandwidth(sdsp_nco* h, double bw);     /* :124-132 */
SDSP_API int sdsp_nco_pll_step(sdsp_nco* h, double delta_phi);                /* :135-138 */
SDSP_API int sdsp_nco_get_state(const sdsp_nco* h, uint32_t* theta, uint32_t* delta_theta);
SDSP_API int sdsp_nco_set_state(sdsp_nco* h, uint32_t theta, uint32_t delta_theta);
SDSP_API int sdsp_nco_mix_block(sdsp_nco* h, int down, int precision, const void* in, size_t n, void* out);
SDSP_API int sdsp_nco_mix_block_device(sdsp_nco* h, int down, int precision, const void* d_in, size_t n,
                                       void* d_out, void* stream);
SDSP_API int sdsp_nco_synchronize(sdsp_nco* h);

/* ------------------------------------------------------------------------
 * AGC (src/auto_gain_control/mod.rs:97-677), SURVEY §8f row 4.  A handle is a
 * bank of `channels` independent AGCs (channel-major sample buffers) with
 * device-resident state; one lane per channel runs the reference's per-sample
 * recurrence (execute :214-246) in f64, with the squelch state machine
 * (update_squelch_mode :631-677).  Samples are f64 (sample_type 0) or
 * Complex<f64> (1), the two types the reference's trait bounds admit.  The
 * recurrence calls exp/ln/log10 per sample: results agree with the reference to
 * libm rounding (the device's f64 exp/log are not glibc's), not bit for bit.
 * Setters apply to every channel; sdsp_agc_get_state reads one channel.
 * ------------------------------------------------------------------------ */
typedef struct sdsp_agc sdsp_agc;
typedef enum {  /* SquelchMode  :84-94 */
    SDSP_SQUELCH_UNKNOWN = 0,
    SDSP_SQUELCH_ENABLED = 1,
    SDSP_SQUELCH_RISE = 2,
    SDSP_SQUELCH_SIGNALHI = 3,
    SDSP_SQUELCH_FALL = 4,
    SDSP_SQUELCH_SIGNALLO = 5, /* the reference's SINGALLO */
    SDSP_SQUELCH_TIMEOUT = 6,
    SDSP_SQUELCH_DISABLED = 7
} sdsp_squelch_mode;
typedef struct {  /* struct AGC  :96-108 */
    double gain, scale, bandwidth, alpha, energy_estimate;
    int32_t lock, squelch_mode;
    double squelch_threshold;
    uint64_t squelch_timeout, squelch_timer;
} sdsp_agc_state;
SDSP_API int sdsp_agc_create(sdsp_agc** out, size_t channels, int device);      /* AGC::new  :136-149 */
SDSP_API void sdsp_agc_destroy(sdsp_agc* h);
SDSP_API size_t sdsp_agc_channels(const sdsp_agc* h);
/* kernel-variant knob: SDSP_TUNE_AGC_KERNEL (performance only) */
SDSP_API int sdsp_agc_set_tuning(sdsp_agc* h, int key, int value);
SDSP_API int sdsp_agc_reset(sdsp_agc* h);                                       /* :178-188 */
/* execute_block  :273-285 (execute per sample :214-246); n samples per channel */
SDSP_API int sdsp_agc_execute_block(sdsp_agc* h, int sample_type, const void* in, size_t n, void* out);
SDSP_API int sdsp_agc_execute_block_device(sdsp_agc* h, int sample_type, const void* d_in, size_t n, void* d_out,
                                           void* stream);
/* init  :568-586 — per channel: gain = 1 / (sqrt(mean |x|^2) + 1e-16); levels[c] receives the level */
SDSP_API int sdsp_agc_init(sdsp_agc* h, int sample_type, const void* in, size_t n, double* levels);
SDSP_API int sdsp_agc_lock(sdsp_agc* h);                                        /* :303-305 */
SDSP_API int sdsp_agc_unlock(sdsp_agc* h);                                      /* :322-324 */
SDSP_API int sdsp_agc_set_bandwidth(sdsp_agc* h, double bandwidth);             /* :374-386 */
SDSP_API int sdsp_agc_set_signal_level(sdsp_agc* h, double level);              /* :416-428 */
SDSP_API int sdsp_agc_set_rssi(sdsp_agc* h, double rssi);                       /* :458-466 */
SDSP_API int sdsp_agc_set_gain(sdsp_agc* h, double gain);                       /* :497-504 */
SDSP_API int sdsp_agc_set_scale(sdsp_agc* h, double scale);                     /* :535-542 */
SDSP_API int sdsp_agc_update_squelch_mode(sdsp_agc* h);                        /* :631-677, each channel */
SDSP_API int sdsp_agc_squelch_enable(sdsp_agc* h);                              /* :589-591 */
SDSP_API int sdsp_agc_squelch_disable(sdsp_agc* h);                             /* :594-596 */
SDSP_API int sdsp_agc_squelch_set_threshold(sdsp_agc* h, double threshold);     /* :612-614 */
SDSP_API int sdsp_agc_squelch_set_timeout(sdsp_agc* h, uint64_t timeout);       /* :622-624 */
SDSP_API int sdsp_agc_get_state(sdsp_agc* h, size_t channel, sdsp_agc_state* st);
SDSP_API int sdsp_agc_set_state(sdsp_agc* h, size_t channel, const sdsp_agc_state* st);
SDSP_API int sdsp_agc_synchronize(sdsp_agc* h);

/* ------------------------------------------------------------------------
 * Device utilities
 * ------------------------------------------------------------------------ */
/* Synthetic stream (build-defined): `count` f32 scalars
 * x(i) = ((mix64(seed ^ channel*G + (start+i+1)*G) >> 40) * 2^-24) * 2 - 1 */
SDSP_API int sdsp_synth_f32_device(void* d_out, uint64_t seed, uint64_t channel, uint64_t start,
                                   size_t count, void* stream);
/* STREAM-style 16-B-per-lane device copy (HBM bandwidth calibration) */
SDSP_API int sdsp_bandwidth_copy_device(const void* d_src, void* d_dst, size_t bytes, void* stream);
/* Host-side reference FIR tap design (src/filter/firdes/mod.rs:278-305) */
SDSP_API int sdsp_firdes_kaiser(size_t n, double fc, double as, double mu, double* h);
SDSP_API int sdsp_firdes_notch(size_t m, double f0, double as, double* h);
SDSP_API double sdsp_kaiser_beta(double as);
/* The rest of solid::filter::firdes (src/filter/firdes/mod.rs:46-640), host f64 like the
 * reference.  Status codes are FirdesErrorCode + 1: 1 Bandwidth, 2 StopBandLevel, 3 Mu,
 * 4 SemiLength, 5 FilterSize, 6 FFTSize.  `method`: 0 EstimationMethod::Kaiser, 1 Herrmann. */
/* estimate_required_filter_length :71-94 (the f64 estimate `as usize`, saturating) */
SDSP_API int sdsp_firdes_estimate_length(double df, double as, int method, size_t* len);
/* estimate_required_filter_length_kaiser :199-211 / _herrmann :213-240 */
SDSP_API int sdsp_firdes_estimate_length_kaiser(double df, double as, double* len);
SDSP_API int sdsp_firdes_estimate_length_herrmann(double df, double as, double* len);
/* estimate_required_filter_stop_band_attenuation :117-145 (bisection, 20 steps) */
SDSP_API int sdsp_firdes_estimate_stop_band_attenuation(double df, size_t n, int method, double* as);
/* estimate_required_filter_transition :168-196 */
SDSP_API int sdsp_firdes_estimate_transition(double as, size_t n, int method, double* df);
/* firdes_doppler :389-419 (Bessel J0 of src/math/mod.rs:102-146, Kaiser window beta 4) */
SDSP_API int sdsp_firdes_doppler(size_t n, double fd, double k, double theta, double* h);
/* filter_autocorrelation :443-456, filter_crosscorrelation :487-527 */
SDSP_API double sdsp_filter_autocorrelation(const double* h, size_t n, ptrdiff_t lag);
SDSP_API double sdsp_filter_crosscorrelation(const double* h, size_t nh, const double* g, size_t ng, ptrdiff_t lag);
/* filter_isi :552-577: (rms, max); (0, 0) when n != 2 sps delay + 1 */
SDSP_API int sdsp_filter_isi(const double* h, size_t n, size_t sps, size_t delay, double* rms, double* max);
/* filter_energy :602-640: relative out-of-band energy over fft_size bins (DotProduct FORWARD per bin) */
SDSP_API int sdsp_filter_energy(const double* h, size_t n, double fc, size_t fft_size, double* energy);
/* PLL loop filters (src/filter/iirdes/pll/mod.rs:24-99) */
SDSP_API int sdsp_active_lag(double bw, double zeta, double k, double* num3, double* den3);
SDSP_API int sdsp_active_proportional_integral(double bw, double zeta, double k, double* num3, double* den3);
/* group delay helpers (src/group_delay/mod.rs:51-129) */
SDSP_API int sdsp_fir_group_delay_taps(const double* h, size_t n, double f, double* out);
SDSP_API int sdsp_iir_group_delay_taps(const double* b, size_t nb, const double* a, size_t na, double f,
                                       double* out);

#ifdef __cplusplus
}
#endif
#endif /* SDSP_H */
