//! `solid::filter::firdes` (src/filter/firdes/mod.rs): the Kaiser tap design chain
//! the hot path's configurations use (firdes_kaiser :278-305, firdes_notch :329-368,
//! kaiser_beta :243-253), computed in f64 by libsdsp's host code (design.cpp,
//! equal to the reference to the bit in tests/test_capi.py).
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
        _ => Err(Box::new(FirdesError(FirdesErrorCode::SemiLength))),
    }
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
