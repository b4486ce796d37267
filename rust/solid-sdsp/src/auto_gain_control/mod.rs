//! `solid::auto_gain_control` (src/auto_gain_control/mod.rs:1-693): `AGC` on
//! libsdsp.so (sdsp_agc, one channel).  The state (gain, energy estimate, lock,
//! squelch machine) lives on the device; `execute_block` runs the reference's
//! per-sample recurrence (:214-246) in the gfx950 `agc_*` kernel in f64.  The
//! recurrence's exp / ln are the device's f64 functions: outputs agree with the
//! reference to libm rounding (tests/test_gpu_rx.py), not bit for bit.
use crate::{check, device, last_error, sys};

use std::error::Error;
use std::fmt;

use num::complex::Complex;

/// auto_gain_control/mod.rs:47-54
#[derive(Debug, PartialEq, Eq)]
pub enum AGCErrorCode {
    BandwidthOutOfRange,
    SignalLevelOutOfRange,
    GainBelowThreshold,
    ScaleBelowThreshold,
    SamplesTooLow,
}

/// auto_gain_control/mod.rs:56-57
#[derive(Debug)]
pub struct AGCError(pub AGCErrorCode, f64);

impl fmt::Display for AGCError {
    /// auto_gain_control/mod.rs:59-78
    fn fmt(&self, f: &mut fmt::Formatter) -> fmt::Result {
        let error_code = match self.0 {
            AGCErrorCode::BandwidthOutOfRange => self.1.to_string() + " Bandwidth not in range [0, 1]",
            AGCErrorCode::SignalLevelOutOfRange => self.1.to_string() + " Level is too low (0, inf)",
            AGCErrorCode::GainBelowThreshold => self.1.to_string() + " Gain is below Threshold (0, inf)",
            AGCErrorCode::ScaleBelowThreshold => self.1.to_string() + " Scale is below Threshold (0, inf)",
            AGCErrorCode::SamplesTooLow => "Need more than 0 Samples to operate".to_string(),
        };
        write!(f, "AGC Error {}", error_code)
    }
}

impl Error for AGCError {}

/// auto_gain_control/mod.rs:82-92 (SINGALLO as spelled there)
#[derive(PartialEq, Eq, Copy, Clone, Debug)]
pub enum SquelchMode {
    UNKNOWN,
    ENABLED,
    RISE,
    SIGNALHI,
    FALL,
    SINGALLO,
    TIMEOUT,
    DISABLED,
}

const MODES: [SquelchMode; 8] = [
    SquelchMode::UNKNOWN,
    SquelchMode::ENABLED,
    SquelchMode::RISE,
    SquelchMode::SIGNALHI,
    SquelchMode::FALL,
    SquelchMode::SINGALLO,
    SquelchMode::TIMEOUT,
    SquelchMode::DISABLED,
];

/// The sample types the reference's bounds admit (`Mul<f64> + Conj + Real<Output = f64>`):
/// f64 (sample_type 0) and Complex<f64> (1).
pub trait AgcSample: private::Sealed + Copy {
    const SAMPLE_TYPE: std::os::raw::c_int;
}
mod private {
    pub trait Sealed {}
}
impl private::Sealed for f64 {}
impl private::Sealed for Complex<f64> {}
impl AgcSample for f64 {
    const SAMPLE_TYPE: std::os::raw::c_int = 0;
}
impl AgcSample for Complex<f64> {
    const SAMPLE_TYPE: std::os::raw::c_int = 1;
}

/// auto_gain_control/mod.rs:95-107
pub struct AGC {
    h: *mut sys::sdsp_agc,
}

fn agc_err(rc: i32, v: f64) -> Box<dyn Error> {
    match rc {
        sys::SDSP_E_AGC_BANDWIDTH_OUT_OF_RANGE => Box::new(AGCError(AGCErrorCode::BandwidthOutOfRange, v)),
        sys::SDSP_E_AGC_SIGNAL_LEVEL_OUT_OF_RANGE => Box::new(AGCError(AGCErrorCode::SignalLevelOutOfRange, v)),
        sys::SDSP_E_AGC_GAIN_BELOW_THRESHOLD => Box::new(AGCError(AGCErrorCode::GainBelowThreshold, v)),
        sys::SDSP_E_AGC_SCALE_BELOW_THRESHOLD => Box::new(AGCError(AGCErrorCode::ScaleBelowThreshold, v)),
        sys::SDSP_E_AGC_SAMPLES_TOO_LOW => Box::new(AGCError(AGCErrorCode::SamplesTooLow, v)),
        _ => Box::new(last_error(rc)),
    }
}

impl AGC {
    /// :136-149
    pub fn new() -> Self {
        let mut h = std::ptr::null_mut();
        check(unsafe { sys::sdsp_agc_create(&mut h, 1, device()) });
        AGC { h }
    }

    fn state(&self) -> sys::sdsp_agc_state {
        let mut st = sys::sdsp_agc_state::default();
        check(unsafe { sys::sdsp_agc_get_state(self.h, 0, &mut st) });
        st
    }

    /// :178-188
    pub fn reset(&mut self) {
        check(unsafe { sys::sdsp_agc_reset(self.h) })
    }

    /// :214-246
    pub fn execute<T: AgcSample>(&mut self, input: T) -> T {
        let mut out = input;
        check(unsafe {
            sys::sdsp_agc_execute_block(self.h, T::SAMPLE_TYPE, &input as *const T as _, 1, &mut out as *mut T as _)
        });
        out
    }

    /// :273-285
    pub fn execute_block<T: AgcSample>(&mut self, input: &[T]) -> Vec<T> {
        let mut out = input.to_vec();
        check(unsafe {
            sys::sdsp_agc_execute_block(self.h, T::SAMPLE_TYPE, input.as_ptr() as _, input.len(),
                                        out.as_mut_ptr() as _)
        });
        out
    }

    /// :303-305
    pub fn lock(&mut self) {
        check(unsafe { sys::sdsp_agc_lock(self.h) })
    }

    /// :322-324
    pub fn unlock(&mut self) {
        check(unsafe { sys::sdsp_agc_unlock(self.h) })
    }

    /// :341-343 (returns the lock flag, as the reference does)
    pub fn is_unlocked(&self) -> bool {
        self.state().lock != 0
    }

    /// :357-359
    pub fn get_bandwidth(&self) -> f64 {
        self.state().bandwidth
    }

    /// :374-386
    pub fn set_bandwidth(&mut self, bandwidth: f64) -> Result<f64, Box<dyn Error>> {
        match unsafe { sys::sdsp_agc_set_bandwidth(self.h, bandwidth) } {
            0 => Ok(bandwidth),
            rc => Err(agc_err(rc, bandwidth)),
        }
    }

    /// :400-402
    pub fn get_signal_level(&self) -> f64 {
        1.0 / self.state().gain
    }

    /// :416-428
    pub fn set_signal_level(&mut self, level: f64) -> Result<f64, Box<dyn Error>> {
        match unsafe { sys::sdsp_agc_set_signal_level(self.h, level) } {
            0 => Ok(level),
            rc => Err(agc_err(rc, level)),
        }
    }

    /// :442-444
    pub fn get_rssi(&self) -> f64 {
        self.state().gain.log10() * -20.0
    }

    /// :458-466
    pub fn set_rssi(&mut self, rssi: f64) {
        check(unsafe { sys::sdsp_agc_set_rssi(self.h, rssi) })
    }

    /// :480-482
    pub fn get_gain(&self) -> f64 {
        self.state().gain
    }

    /// :497-504
    pub fn set_gain(&mut self, gain: f64) -> Result<f64, Box<dyn Error>> {
        match unsafe { sys::sdsp_agc_set_gain(self.h, gain) } {
            0 => Ok(gain),
            rc => Err(agc_err(rc, gain)),
        }
    }

    /// :518-520
    pub fn get_scale(&self) -> f64 {
        self.state().scale
    }

    /// :535-542
    pub fn set_scale(&mut self, scale: f64) -> Result<f64, Box<dyn Error>> {
        match unsafe { sys::sdsp_agc_set_scale(self.h, scale) } {
            0 => Ok(scale),
            rc => Err(agc_err(rc, scale)),
        }
    }

    /// :568-586: the linear signal level, sqrt(mean |x|^2) + 1e-16
    pub fn init<T: AgcSample>(&mut self, input: &[T]) -> Result<f64, Box<dyn Error>> {
        let mut level = 0.0f64;
        match unsafe { sys::sdsp_agc_init(self.h, T::SAMPLE_TYPE, input.as_ptr() as _, input.len(), &mut level) } {
            0 => Ok(level),
            rc => Err(agc_err(rc, 0.0)),
        }
    }

    /// :589-591
    pub fn squelch_enable(&mut self) {
        check(unsafe { sys::sdsp_agc_squelch_enable(self.h) })
    }

    /// :594-596
    pub fn squelch_disable(&mut self) {
        check(unsafe { sys::sdsp_agc_squelch_disable(self.h) })
    }

    /// :598-604
    pub fn is_squelch_enabled(&self) -> bool {
        self.squelch_get_mode() != SquelchMode::DISABLED
    }

    /// :607-609
    pub fn squelch_get_threshold(&self) -> f64 {
        self.state().squelch_threshold
    }

    /// :612-614
    pub fn squelch_set_threshold(&mut self, threshold: f64) {
        check(unsafe { sys::sdsp_agc_squelch_set_threshold(self.h, threshold) })
    }

    /// :617-619
    pub fn squelch_get_timeout(&self) -> usize {
        self.state().squelch_timeout as usize
    }

    /// :622-624
    pub fn squelch_set_timeout(&mut self, timeout: usize) {
        check(unsafe { sys::sdsp_agc_squelch_set_timeout(self.h, timeout as u64) })
    }

    /// :627-629
    pub fn squelch_get_mode(&self) -> SquelchMode {
        MODES[(self.state().squelch_mode as usize) & 7]
    }

    /// :631-677
    pub fn update_squelch_mode(&mut self) {
        check(unsafe { sys::sdsp_agc_update_squelch_mode(self.h) })
    }
}

impl Default for AGC {
    fn default() -> Self {
        Self::new()
    }
}

impl Drop for AGC {
    fn drop(&mut self) {
        unsafe { sys::sdsp_agc_destroy(self.h) }
    }
}

impl fmt::Display for AGC {
    /// auto_gain_control/mod.rs:686-693
    fn fmt(&self, f: &mut fmt::Formatter) -> fmt::Result {
        let s = self.state();
        write!(f, "AGC [Gain={:.5}] [Scale={:.5}] [Bandwidth={:.5}] [Alpha={:.5}] [Energy={:.5}]",
               s.gain, s.scale, s.bandwidth, s.alpha, s.energy_estimate)
    }
}
