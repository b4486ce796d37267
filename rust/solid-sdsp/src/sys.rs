//! Raw declarations of include/sdsp.h (C ABI of libsdsp.so).  Every handle is
//! opaque; samples are `#[repr(C)]` `num::Complex<T>` = interleaved {re, im}.
#![allow(non_camel_case_types)]
use std::os::raw::{c_char, c_int, c_void};

#[repr(C)] pub struct sdsp_fir { _p: [u8; 0] }
#[repr(C)] pub struct sdsp_pfb { _p: [u8; 0] }
#[repr(C)] pub struct sdsp_iir { _p: [u8; 0] }
#[repr(C)] pub struct sdsp_fft { _p: [u8; 0] }
#[repr(C)] pub struct sdsp_chan { _p: [u8; 0] }
#[repr(C)] pub struct sdsp_acorr { _p: [u8; 0] }
#[repr(C)] pub struct sdsp_nco { _p: [u8; 0] }
#[repr(C)] pub struct sdsp_agc { _p: [u8; 0] }

/// struct AGC (auto_gain_control/mod.rs:96-108) as include/sdsp.h sdsp_agc_state
#[repr(C)]
#[derive(Clone, Copy, Default)]
pub struct sdsp_agc_state {
    pub gain: f64,
    pub scale: f64,
    pub bandwidth: f64,
    pub alpha: f64,
    pub energy_estimate: f64,
    pub lock: i32,
    pub squelch_mode: i32,
    pub squelch_threshold: f64,
    pub squelch_timeout: u64,
    pub squelch_timer: u64,
}

pub const SDSP_RR32: c_int = 0;
pub const SDSP_RC32: c_int = 1;
pub const SDSP_CC32: c_int = 2;
pub const SDSP_RR64: c_int = 3;
pub const SDSP_RC64: c_int = 4;
pub const SDSP_CC64: c_int = 5;

pub const SDSP_ALGO_AUTO: c_int = 0;
pub const SDSP_ALGO_EXACT: c_int = 1;
pub const SDSP_ALGO_FMA: c_int = 2;
pub const SDSP_ALGO_FFT: c_int = 3;

pub const SDSP_TUNE_HOST_STEP: c_int = 16;
pub const SDSP_TUNE_HOST_BLOCK_MACS: c_int = 17;

pub const SDSP_OK: c_int = 0;
pub const SDSP_E_COEFFICIENTS_LENGTH_ZERO: c_int = 1;
pub const SDSP_E_DECIMATION_LESS_THAN_ONE: c_int = 2;
pub const SDSP_E_INTERPOLATION_LESS_THAN_ONE: c_int = 3;
pub const SDSP_E_NOT_ENOUGH_FILTERS: c_int = 4;
pub const SDSP_E_NUMERATOR_LENGTH_ZERO: c_int = 10;
pub const SDSP_E_DENOMINATOR_LENGTH_ZERO: c_int = 11;
pub const SDSP_E_SOS_SIZE_ZERO: c_int = 12;
pub const SDSP_E_SOS_SIZE_MISMATCH: c_int = 13;
pub const SDSP_E_SOS_SIZE_NOT_MULTIPLE_OF_3: c_int = 14;
pub const SDSP_E_IIR_DECIMATION_LESS_THAN_ONE: c_int = 15;
pub const SDSP_E_IIR_INTERPOLATION_LESS_THAN_ONE: c_int = 16;
pub const SDSP_E_NCO_BANDWIDTH_OUT_OF_RANGE: c_int = 30;
pub const SDSP_E_AGC_BANDWIDTH_OUT_OF_RANGE: c_int = 40;
pub const SDSP_E_AGC_SIGNAL_LEVEL_OUT_OF_RANGE: c_int = 41;
pub const SDSP_E_AGC_GAIN_BELOW_THRESHOLD: c_int = 42;
pub const SDSP_E_AGC_SCALE_BELOW_THRESHOLD: c_int = 43;
pub const SDSP_E_AGC_SAMPLES_TOO_LOW: c_int = 44;

extern "C" {
    pub fn sdsp_last_error() -> *const c_char;
    pub fn sdsp_device_count() -> c_int;

    // FIRFilter / DecimatingFIRFilter (fir/mod.rs:58-304, fir/decim.rs:5-281)
    pub fn sdsp_fir_create(out: *mut *mut sdsp_fir, dtype: c_int, taps: *const c_void, len: usize,
                           scale: *const c_void, device: c_int) -> c_int;
    pub fn sdsp_decim_create(out: *mut *mut sdsp_fir, dtype: c_int, taps: *const c_void, len: usize,
                             scale: *const c_void, decimation: usize, device: c_int) -> c_int;
    pub fn sdsp_fir_destroy(h: *mut sdsp_fir);
    pub fn sdsp_fir_clone(h: *const sdsp_fir, out: *mut *mut sdsp_fir) -> c_int;
    pub fn sdsp_fir_set_algo(h: *mut sdsp_fir, algo: c_int) -> c_int;
    pub fn sdsp_set_default_algo(algo: c_int) -> c_int;
    pub fn sdsp_get_default_algo() -> c_int;
    pub fn sdsp_fir_set_tuning(h: *mut sdsp_fir, key: c_int, value: c_int) -> c_int;
    pub fn sdsp_fir_execute(h: *mut sdsp_fir, sample: *const c_void, out: *mut c_void, n_out: *mut usize) -> c_int;
    pub fn sdsp_fir_get_state(h: *const sdsp_fir, hist: *mut c_void, phase: *mut usize) -> c_int;
    pub fn sdsp_fir_synchronize(h: *mut sdsp_fir) -> c_int;
    pub fn sdsp_fir_set_scale(h: *mut sdsp_fir, scale: *const c_void) -> c_int;
    pub fn sdsp_fir_get_scale(h: *const sdsp_fir, scale: *mut c_void) -> c_int;
    pub fn sdsp_fir_len(h: *const sdsp_fir) -> usize;
    pub fn sdsp_fir_decimation(h: *const sdsp_fir) -> usize;
    pub fn sdsp_fir_coefficients(h: *const sdsp_fir, out: *mut c_void) -> c_int;
    pub fn sdsp_fir_output_count(h: *const sdsp_fir, n: usize) -> usize;
    pub fn sdsp_fir_execute_block(h: *mut sdsp_fir, input: *const c_void, n: usize, out: *mut c_void,
                                  n_out: *mut usize) -> c_int;
    pub fn sdsp_fir_execute_block_device(h: *mut sdsp_fir, d_in: *const c_void, n: usize, d_out: *mut c_void,
                                         n_out: *mut usize, stream: *mut c_void) -> c_int;
    pub fn sdsp_decim_push(h: *mut sdsp_fir, sample: *const c_void) -> c_int;
    pub fn sdsp_decim_write(h: *mut sdsp_fir, samples: *const c_void, n: usize) -> c_int;
    pub fn sdsp_fir_reset(h: *mut sdsp_fir) -> c_int;
    pub fn sdsp_fir_frequency_response(h: *const sdsp_fir, f: f64, re_im: *mut f64) -> c_int;
    pub fn sdsp_fir_group_delay(h: *const sdsp_fir, f: f64, delay: *mut f64) -> c_int;

    // PolyPhaseFilterBank / InterpolatingFIRFilter (fir/pfb.rs:3-91, fir/interp.rs:6-138)
    pub fn sdsp_pfb_create(out: *mut *mut sdsp_pfb, dtype: c_int, taps: *const c_void, len: usize,
                           filters: usize, scale: *const c_void, device: c_int) -> c_int;
    pub fn sdsp_interp_create(out: *mut *mut sdsp_pfb, dtype: c_int, taps: *const c_void, len: usize,
                              interpolation: usize, device: c_int) -> c_int;
    pub fn sdsp_pfb_destroy(h: *mut sdsp_pfb);
    pub fn sdsp_pfb_clone(h: *const sdsp_pfb, out: *mut *mut sdsp_pfb) -> c_int;
    pub fn sdsp_pfb_len(h: *const sdsp_pfb) -> usize;
    pub fn sdsp_pfb_subfilter_len(h: *const sdsp_pfb) -> usize;
    pub fn sdsp_pfb_set_scale(h: *mut sdsp_pfb, scale: *const c_void) -> c_int;
    pub fn sdsp_pfb_get_scale(h: *const sdsp_pfb, scale: *mut c_void) -> c_int;
    pub fn sdsp_pfb_coefficients(h: *const sdsp_pfb, out_mk: *mut c_void) -> c_int;
    pub fn sdsp_pfb_push(h: *mut sdsp_pfb, sample: *const c_void) -> c_int;
    pub fn sdsp_pfb_execute(h: *mut sdsp_pfb, index: usize, out: *mut c_void) -> c_int;
    pub fn sdsp_pfb_reset(h: *mut sdsp_pfb) -> c_int;
    pub fn sdsp_pfb_execute_block(h: *mut sdsp_pfb, input: *const c_void, n: usize, out: *mut c_void) -> c_int;
    pub fn sdsp_pfb_frequency_response(h: *const sdsp_pfb, f: f64, re_im: *mut f64) -> c_int;
    pub fn sdsp_pfb_group_delay(h: *const sdsp_pfb, f: f64, delay: *mut f64) -> c_int;

    // IIRFilter / DecimatingIIRFilter / InterpolatingIIRFilter (iir/mod.rs:62-414, iir/decim.rs, iir/interp.rs)
    pub fn sdsp_iir_create(out: *mut *mut sdsp_iir, dtype: c_int, ff: *const c_void, nff: usize,
                           fb: *const c_void, nfb: usize, kind: c_int, device: c_int) -> c_int;
    pub fn sdsp_iir_decim_create(out: *mut *mut sdsp_iir, dtype: c_int, ff: *const c_void, nff: usize,
                                 fb: *const c_void, nfb: usize, kind: c_int, decimation: usize,
                                 device: c_int) -> c_int;
    pub fn sdsp_iir_interp_create(out: *mut *mut sdsp_iir, dtype: c_int, ff: *const c_void, nff: usize,
                                  fb: *const c_void, nfb: usize, kind: c_int, interpolation: usize,
                                  device: c_int) -> c_int;
    pub fn sdsp_iir_destroy(h: *mut sdsp_iir);
    pub fn sdsp_iir_clone(h: *const sdsp_iir, out: *mut *mut sdsp_iir) -> c_int;
    pub fn sdsp_iir_set_algo(h: *mut sdsp_iir, algo: c_int) -> c_int;
    pub fn sdsp_iir_output_count(h: *const sdsp_iir, n: usize) -> usize;
    pub fn sdsp_iir_execute_block(h: *mut sdsp_iir, input: *const c_void, n: usize, out: *mut c_void,
                                  n_out: *mut usize) -> c_int;
    pub fn sdsp_iir_reset(h: *mut sdsp_iir) -> c_int;
    pub fn sdsp_iir_execute(h: *mut sdsp_iir, sample: *const c_void, out: *mut c_void, n_out: *mut usize) -> c_int;
    pub fn sdsp_iir_num_coefs(h: *const sdsp_iir, which: c_int) -> usize;
    pub fn sdsp_iir_coefficients(h: *const sdsp_iir, num: *mut f64, den: *mut f64) -> c_int;
    pub fn sdsp_sos_section_coefs(h: *const sdsp_iir, section: c_int, num2: *mut f64, den3: *mut f64) -> c_int;
    pub fn sdsp_iir_group_delay_taps(b: *const f64, nb: usize, a: *const f64, na: usize, f: f64,
                                     out: *mut f64) -> c_int;
    pub fn sdsp_iir_frequency_response(h: *const sdsp_iir, f: f64, re_im: *mut f64) -> c_int;
    pub fn sdsp_iir_group_delay(h: *const sdsp_iir, f: f64, delay: *mut f64) -> c_int;

    // FFT (fft/mod.rs:123-215), channeliser
    pub fn sdsp_fft_create(out: *mut *mut sdsp_fft, nfft: usize, direction: c_int, precision: c_int,
                           device: c_int) -> c_int;
    pub fn sdsp_fft_destroy(h: *mut sdsp_fft);
    pub fn sdsp_fft_len(h: *const sdsp_fft) -> usize;
    pub fn sdsp_fft_execute(h: *mut sdsp_fft, input: *const c_void, out: *mut c_void, batch: usize) -> c_int;
    pub fn sdsp_chan_create(out: *mut *mut sdsp_chan, dtype: c_int, taps: *const c_void, len: usize,
                            channels: usize, device: c_int) -> c_int;
    pub fn sdsp_chan_destroy(h: *mut sdsp_chan);
    pub fn sdsp_chan_execute_block(h: *mut sdsp_chan, input: *const c_void, n: usize, out: *mut c_void,
                                   frames: *mut usize) -> c_int;

    // tap / loop-filter design (firdes/mod.rs:243-368, iirdes/pll/mod.rs:24-99)
    pub fn sdsp_kaiser_beta(stop_band_attenuation: f64) -> f64;
    // the rest of firdes (firdes/mod.rs:46-640); method 0 Kaiser, 1 Herrmann
    pub fn sdsp_firdes_estimate_length(df: f64, as_: f64, method: c_int, len: *mut usize) -> c_int;
    pub fn sdsp_firdes_estimate_length_kaiser(df: f64, as_: f64, len: *mut f64) -> c_int;
    pub fn sdsp_firdes_estimate_length_herrmann(df: f64, as_: f64, len: *mut f64) -> c_int;
    pub fn sdsp_firdes_estimate_stop_band_attenuation(df: f64, n: usize, method: c_int, as_: *mut f64) -> c_int;
    pub fn sdsp_firdes_estimate_transition(as_: f64, n: usize, method: c_int, df: *mut f64) -> c_int;
    pub fn sdsp_firdes_doppler(n: usize, fd: f64, k: f64, theta: f64, h: *mut f64) -> c_int;
    pub fn sdsp_filter_autocorrelation(h: *const f64, n: usize, lag: isize) -> f64;
    pub fn sdsp_filter_crosscorrelation(h: *const f64, nh: usize, g: *const f64, ng: usize, lag: isize) -> f64;
    pub fn sdsp_filter_isi(h: *const f64, n: usize, sps: usize, delay: usize, rms: *mut f64, max: *mut f64) -> c_int;
    pub fn sdsp_filter_energy(h: *const f64, n: usize, fc: f64, fft_size: usize, energy: *mut f64) -> c_int;
    pub fn sdsp_firdes_kaiser(n: usize, fc: f64, as_: f64, mu: f64, h: *mut f64) -> c_int;
    pub fn sdsp_firdes_notch(m: usize, f0: f64, as_: f64, h: *mut f64) -> c_int;
    pub fn sdsp_active_lag(bw: f64, zeta: f64, k: f64, num3: *mut f64, den3: *mut f64) -> c_int;
    pub fn sdsp_active_proportional_integral(bw: f64, zeta: f64, k: f64, num3: *mut f64, den3: *mut f64) -> c_int;

    // AutoCorrelator (filter/auto_correlator/mod.rs:26-214); precision 0 Complex<f32>, 1 Complex<f64>
    pub fn sdsp_acorr_create(out: *mut *mut sdsp_acorr, window_size: usize, delay: usize, precision: c_int,
                             device: c_int) -> c_int;
    pub fn sdsp_acorr_destroy(h: *mut sdsp_acorr);
    pub fn sdsp_acorr_window_size(h: *const sdsp_acorr) -> usize;
    pub fn sdsp_acorr_delay(h: *const sdsp_acorr) -> usize;
    pub fn sdsp_acorr_reset(h: *mut sdsp_acorr) -> c_int;
    pub fn sdsp_acorr_push(h: *mut sdsp_acorr, sample: *const c_void) -> c_int;
    pub fn sdsp_acorr_write(h: *mut sdsp_acorr, samples: *const c_void, n: usize) -> c_int;
    pub fn sdsp_acorr_execute(h: *mut sdsp_acorr, out: *mut c_void) -> c_int;
    pub fn sdsp_acorr_execute_block(h: *mut sdsp_acorr, input: *const c_void, n: usize, out: *mut c_void) -> c_int;
    pub fn sdsp_acorr_get_energy(h: *mut sdsp_acorr, energy: *mut f64) -> c_int;

    // NCO (nco/mod.rs:27-187): u32 phase registers on the host, blocks mixed on the device
    pub fn sdsp_nco_create(out: *mut *mut sdsp_nco, device: c_int) -> c_int;
    pub fn sdsp_nco_destroy(h: *mut sdsp_nco);
    pub fn sdsp_nco_reset(h: *mut sdsp_nco) -> c_int;
    pub fn sdsp_nco_constrain(theta: f64) -> u32;
    pub fn sdsp_nco_set_frequency(h: *mut sdsp_nco, delta_theta: f64) -> c_int;
    pub fn sdsp_nco_adjust_frequency(h: *mut sdsp_nco, dt: f64) -> c_int;
    pub fn sdsp_nco_get_frequency(h: *const sdsp_nco) -> f64;
    pub fn sdsp_nco_set_phase(h: *mut sdsp_nco, phi: f64) -> c_int;
    pub fn sdsp_nco_adjust_phase(h: *mut sdsp_nco, delta_phi: f64) -> c_int;
    pub fn sdsp_nco_get_phase(h: *const sdsp_nco) -> f64;
    pub fn sdsp_nco_step(h: *mut sdsp_nco) -> c_int;
    pub fn sdsp_nco_sincos(h: *const sdsp_nco, sin_cos: *mut f64) -> c_int;
    pub fn sdsp_nco_set_internal_pll_bandwidth(h: *mut sdsp_nco, bw: f64) -> c_int;
    pub fn sdsp_nco_pll_step(h: *mut sdsp_nco, delta_phi: f64) -> c_int;
    pub fn sdsp_nco_get_state(h: *const sdsp_nco, theta: *mut u32, delta_theta: *mut u32) -> c_int;
    pub fn sdsp_nco_mix_block(h: *mut sdsp_nco, down: c_int, precision: c_int, input: *const c_void, n: usize,
                              out: *mut c_void) -> c_int;

    // AGC (auto_gain_control/mod.rs:97-677); sample_type 0 f64, 1 Complex<f64>
    pub fn sdsp_agc_create(out: *mut *mut sdsp_agc, channels: usize, device: c_int) -> c_int;
    pub fn sdsp_agc_destroy(h: *mut sdsp_agc);
    pub fn sdsp_agc_reset(h: *mut sdsp_agc) -> c_int;
    pub fn sdsp_agc_execute_block(h: *mut sdsp_agc, sample_type: c_int, input: *const c_void, n: usize,
                                  out: *mut c_void) -> c_int;
    pub fn sdsp_agc_init(h: *mut sdsp_agc, sample_type: c_int, input: *const c_void, n: usize,
                         levels: *mut f64) -> c_int;
    pub fn sdsp_agc_lock(h: *mut sdsp_agc) -> c_int;
    pub fn sdsp_agc_unlock(h: *mut sdsp_agc) -> c_int;
    pub fn sdsp_agc_set_bandwidth(h: *mut sdsp_agc, bandwidth: f64) -> c_int;
    pub fn sdsp_agc_set_signal_level(h: *mut sdsp_agc, level: f64) -> c_int;
    pub fn sdsp_agc_set_rssi(h: *mut sdsp_agc, rssi: f64) -> c_int;
    pub fn sdsp_agc_set_gain(h: *mut sdsp_agc, gain: f64) -> c_int;
    pub fn sdsp_agc_set_scale(h: *mut sdsp_agc, scale: f64) -> c_int;
    pub fn sdsp_agc_update_squelch_mode(h: *mut sdsp_agc) -> c_int;
    pub fn sdsp_agc_squelch_enable(h: *mut sdsp_agc) -> c_int;
    pub fn sdsp_agc_squelch_disable(h: *mut sdsp_agc) -> c_int;
    pub fn sdsp_agc_squelch_set_threshold(h: *mut sdsp_agc, threshold: f64) -> c_int;
    pub fn sdsp_agc_squelch_set_timeout(h: *mut sdsp_agc, timeout: u64) -> c_int;
    pub fn sdsp_agc_get_state(h: *mut sdsp_agc, channel: usize, st: *mut sdsp_agc_state) -> c_int;

    // DotProduct (dot_product/mod.rs:37-171)
    pub fn sdsp_dot_execute(dtype: c_int, coefs: *const c_void, len: usize, direction: c_int,
                            samples: *const c_void, n: usize, out: *mut c_void) -> c_int;
}
