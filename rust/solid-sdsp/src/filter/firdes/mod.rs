//! `solid::filter::firdes` (src/filter/firdes/mod.rs:1-640): FIR tap design and
//! analysis -- the length / attenuation / transition estimates, Kaiser, notch and
//! Doppler designs, auto- / cross-correlation, ISI and out-of-band energy -- computed
//! in f64 by libsdsp's host code (design.cpp), equal to the reference's arithmetic to
//! the bit (tests/test_capi.py: the oracle restatement and the doctest KATs).
pub mod filter_traits;

use crate::sys;

use std::error::Error;
use std::fmt;

/// firdes/mod.rs:17-24 (private in the reference: it only surfaces as `Box<dyn Error>`)
#[derive(Debug)]
enum FirdesErrorCode {
    Bandwidth,
    StopBandLevel,
    Mu,
    SemiLength,
    FilterSize,
    FFTSize,
}

#[derive(Debug)]
struct FirdesError(FirdesErrorCode);

impl fmt::Display for FirdesError {
    /// firdes/mod.rs:29-41
    fn fmt(&self, f: &mut fmt::Formatter) -> fmt::Result {
        let error_code = match self.0 {
            FirdesErrorCode::Bandwidth => "Invalid Bandwidth [0, 0.5]",
            FirdesErrorCode::StopBandLevel => "Invalid Stop Band Attenuation (0, inf)",
            FirdesErrorCode::Mu => "Invalid Mu Range [-0.5, 0.5]",
            FirdesErrorCode::SemiLength => "Invalid Filter Semi Length [1, 1000]",
            FirdesErrorCode::FilterSize => "Invalid Filter Size [1, inf)",
            FirdesErrorCode::FFTSize => "Invalid FFT Size [1, inf)",
        };
        write!(f, "Firdes Error: {}", error_code)
    }
}

impl Error for FirdesError {}

fn status(rc: i32) -> Result<(), Box<dyn Error>> {
    match rc {
        0 => Ok(()),
        1 => Err(Box::new(FirdesError(FirdesErrorCode::Bandwidth))),
        2 => Err(Box::new(FirdesError(FirdesErrorCode::StopBandLevel))),
        3 => Err(Box::new(FirdesError(FirdesErrorCode::Mu))),
        4 => Err(Box::new(FirdesError(FirdesErrorCode::SemiLength))),
        5 => Err(Box::new(FirdesError(FirdesErrorCode::FilterSize))),
        _ => Err(Box::new(FirdesError(FirdesErrorCode::FFTSize))),
    }
}

/// firdes/mod.rs:46-49
pub enum EstimationMethod {
    Kaiser,
    Herrmann,
}

fn method_code(method: &EstimationMethod) -> std::os::raw::c_int {
    match method {
        EstimationMethod::Kaiser => 0,
        EstimationMethod::Herrmann => 1,
    }
}

/// firdes/mod.rs:71-94
pub fn estimate_required_filter_length(
    transition_bandwidth: f64,
    stop_band_attenuation: f64,
    method: EstimationMethod,
) -> Result<usize, Box<dyn Error>> {
    let mut n = 0usize;
    status(unsafe {
        sys::sdsp_firdes_estimate_length(transition_bandwidth, stop_band_attenuation, method_code(&method), &mut n)
    })?;
    Ok(n)
}

/// firdes/mod.rs:117-145
pub fn estimate_required_filter_stop_band_attenuation(
    transition_bandwidth: f64,
    filter_length: usize,
    method: EstimationMethod,
) -> Result<f64, Box<dyn Error>> {
    let mut v = 0.0f64;
    status(unsafe {
        sys::sdsp_firdes_estimate_stop_band_attenuation(transition_bandwidth, filter_length, method_code(&method),
                                                        &mut v)
    })?;
    Ok(v)
}

/// firdes/mod.rs:168-196
pub fn estimate_required_filter_transition(
    stop_band_attenuation: f64,
    filter_length: usize,
    method: EstimationMethod,
) -> Result<f64, Box<dyn Error>> {
    let mut v = 0.0f64;
    status(unsafe {
        sys::sdsp_firdes_estimate_transition(stop_band_attenuation, filter_length, method_code(&method), &mut v)
    })?;
    Ok(v)
}

/// firdes/mod.rs:199-211
pub fn estimate_required_filter_length_kaiser(
    transition_bandwidth: f64,
    stop_band_attenuation: f64,
) -> Result<f64, Box<dyn Error>> {
    let mut v = 0.0f64;
    status(unsafe { sys::sdsp_firdes_estimate_length_kaiser(transition_bandwidth, stop_band_attenuation, &mut v) })?;
    Ok(v)
}

/// firdes/mod.rs:213-240
pub fn estimate_required_filter_length_herrmann(
    transition_bandwidth: f64,
    stop_band_attenuation: f64,
) -> Result<f64, Box<dyn Error>> {
    let mut v = 0.0f64;
    status(unsafe {
        sys::sdsp_firdes_estimate_length_herrmann(transition_bandwidth, stop_band_attenuation, &mut v)
    })?;
    Ok(v)
}

/// firdes/mod.rs:243-253
pub fn kaiser_beta(stop_band_attenuation: f64) -> f64 {
    unsafe { sys::sdsp_kaiser_beta(stop_band_attenuation) }
}

/// firdes/mod.rs:278-305
pub fn firdes_kaiser(
    filter_length: usize,
    cutoff_frequency: f64,
    stop_band_attenuation: f64,
    fractional_sample_offset: f64,
) -> Result<Vec<f64>, Box<dyn Error>> {
    let mut h = vec![0.0f64; filter_length];
    status(unsafe {
        sys::sdsp_firdes_kaiser(filter_length, cutoff_frequency, stop_band_attenuation, fractional_sample_offset,
                                h.as_mut_ptr())
    })?;
    Ok(h)
}

/// firdes/mod.rs:329-368: 2 semi_length + 1 taps
pub fn firdes_notch(
    semi_length: usize,
    notch_frequency: f64,
    stop_band_attenuation: f64,
) -> Result<Vec<f64>, Box<dyn Error>> {
    let mut h = vec![0.0f64; 2 * semi_length + 1];
    status(unsafe { sys::sdsp_firdes_notch(semi_length, notch_frequency, stop_band_attenuation, h.as_mut_ptr()) })?;
    Ok(h)
}

/// firdes/mod.rs:389-419
pub fn firdes_doppler(
    filter_length: usize,
    doppler_frequency: f64,
    rice_fading_factor: f64,
    theta: f64,
) -> Result<Vec<f64>, Box<dyn Error>> {
    let mut h = vec![0.0f64; filter_length];
    status(unsafe {
        sys::sdsp_firdes_doppler(filter_length, doppler_frequency, rice_fading_factor, theta, h.as_mut_ptr())
    })?;
    Ok(h)
}

/// firdes/mod.rs:443-456
pub fn filter_autocorrelation(filter: &[f64], lag: isize) -> f64 {
    unsafe { sys::sdsp_filter_autocorrelation(filter.as_ptr(), filter.len(), lag) }
}

/// firdes/mod.rs:487-527
pub fn filter_crosscorrelation(h: &[f64], g: &[f64], lag: isize) -> f64 {
    unsafe { sys::sdsp_filter_crosscorrelation(h.as_ptr(), h.len(), g.as_ptr(), g.len(), lag) }
}

/// firdes/mod.rs:552-577
pub fn filter_isi(filter: &[f64], samples_per_symbol: usize, filter_delay: usize) -> (f64, f64) {
    let (mut rms, mut max) = (0.0f64, 0.0f64);
    unsafe { sys::sdsp_filter_isi(filter.as_ptr(), filter.len(), samples_per_symbol, filter_delay, &mut rms, &mut max) };
    (rms, max)
}

/// firdes/mod.rs:602-640
pub fn filter_energy(
    filter: &[f64],
    cutoff_frequency: f64,
    fft_size: usize,
) -> Result<f64, Box<dyn Error>> {
    let mut e = 0.0f64;
    status(unsafe { sys::sdsp_filter_energy(filter.as_ptr(), filter.len(), cutoff_frequency, fft_size, &mut e) })?;
    Ok(e)
}
