//! `solid::nco` (src/nco/mod.rs:1-203): the numerically controlled oscillator on
//! libsdsp.so (sdsp_nco).  The u32 phase registers live in the handle on the host
//! and move exactly as the reference's (`constrain`, wrapping adds); blocks are
//! mixed on the gfx950 device with the reference's 1024-entry sine table and index
//! rule, bit-identical at Complex<f64> (tests/test_gpu_rx.py).  Single-sample
//! `mix_up` / `mix_down` form `complex_exponential() * input` on the host, as the
//! reference does.
use crate::{check, device, last_error, sys};

use std::error::Error;
use std::fmt;

use num::complex::Complex;

/// nco/mod.rs:7-10
#[derive(Debug, PartialEq, Eq)]
pub enum NCOErrorCode {
    BandwidthOutOfRange,
}

/// nco/mod.rs:12-13
#[derive(Debug)]
pub struct NCOError(pub NCOErrorCode);

impl fmt::Display for NCOError {
    /// nco/mod.rs:15-22
    fn fmt(&self, f: &mut fmt::Formatter) -> fmt::Result {
        let error_code = match self.0 {
            NCOErrorCode::BandwidthOutOfRange => "Bandwidth out Range [0, inf)",
        };
        write!(f, "NCO Error {}", error_code)
    }
}

impl Error for NCOError {}

/// nco/mod.rs:27-34 (alpha / beta mirrored here for Display; the handle holds its own)
#[derive(Debug)]
pub struct NCO {
    h: *mut sys::sdsp_nco,
    alpha: f64,
    beta: f64,
}

impl NCO {
    /// :36-50
    pub fn new() -> Self {
        let mut h = std::ptr::null_mut();
        check(unsafe { sys::sdsp_nco_create(&mut h, device()) });
        let a = 0.1f64;
        NCO { h, alpha: a, beta: a.sqrt() }
    }

    /// :53-56
    pub fn reset(&mut self) {
        check(unsafe { sys::sdsp_nco_reset(self.h) })
    }

    /// :59-61
    pub fn set_frequency(&mut self, delta_theta: f64) {
        check(unsafe { sys::sdsp_nco_set_frequency(self.h, delta_theta) })
    }

    /// :64-66
    pub fn adjust_frequency(&mut self, dt: f64) {
        check(unsafe { sys::sdsp_nco_adjust_frequency(self.h, dt) })
    }

    /// :69-76
    pub fn get_frequency(&self) -> f64 {
        unsafe { sys::sdsp_nco_get_frequency(self.h) }
    }

    /// :79-81
    pub fn set_phase(&mut self, phi: f64) {
        check(unsafe { sys::sdsp_nco_set_phase(self.h, phi) })
    }

    /// :84-86
    pub fn adjust_phase(&mut self, delta_phi: f64) {
        check(unsafe { sys::sdsp_nco_adjust_phase(self.h, delta_phi) })
    }

    /// :89-91
    pub fn get_phase(&self) -> f64 {
        unsafe { sys::sdsp_nco_get_phase(self.h) }
    }

    /// :94-96
    pub fn step(&mut self) {
        check(unsafe { sys::sdsp_nco_step(self.h) })
    }

    /// :104-107
    pub fn sin(&self) -> f64 {
        self.sincos().0
    }

    /// :109-113
    pub fn cos(&self) -> f64 {
        self.sincos().1
    }

    /// :115-117: (sin, cos) from the 1024-entry table
    pub fn sincos(&self) -> (f64, f64) {
        let mut sc = [0.0f64; 2];
        check(unsafe { sys::sdsp_nco_sincos(self.h, sc.as_mut_ptr()) });
        (sc[0], sc[1])
    }

    /// :119-122
    pub fn complex_exponential(&self) -> Complex<f64> {
        let (s, c) = self.sincos();
        Complex::new(c, s)
    }

    /// :124-132
    pub fn set_internal_pll_bandwidth(&mut self, bandwidth: f64) -> Result<(), Box<dyn Error>> {
        match unsafe { sys::sdsp_nco_set_internal_pll_bandwidth(self.h, bandwidth) } {
            0 => {
                self.alpha = bandwidth;
                self.beta = self.alpha.sqrt();
                Ok(())
            }
            sys::SDSP_E_NCO_BANDWIDTH_OUT_OF_RANGE => Err(Box::new(NCOError(NCOErrorCode::BandwidthOutOfRange))),
            rc => Err(Box::new(last_error(rc))),
        }
    }

    /// :135-138
    pub fn pll_step(&mut self, delta_phi: f64) {
        check(unsafe { sys::sdsp_nco_pll_step(self.h, delta_phi) })
    }

    /// :141-144
    pub fn mix_up(&self, input: Complex<f64>) -> Complex<f64> {
        let complex_phasor = self.complex_exponential();
        complex_phasor * input
    }

    /// :147-150
    pub fn mix_down(&self, input: Complex<f64>) -> Complex<f64> {
        let complex_phasor = self.complex_exponential().conj();
        complex_phasor * input
    }

    /// :153-161: out[i] = mix_up(input[i]), then step() -- on the device.  (The reference's
    /// loop writes into an empty `Vec` and panics for any non-empty input; this is the loop
    /// it spells out.)
    pub fn mix_up_block(&mut self, input: &[Complex<f64>]) -> Vec<Complex<f64>> {
        self.mix_block(input, 0)
    }

    /// :164-172
    pub fn mix_down_block(&mut self, input: &[Complex<f64>]) -> Vec<Complex<f64>> {
        self.mix_block(input, 1)
    }

    fn mix_block(&mut self, input: &[Complex<f64>], down: i32) -> Vec<Complex<f64>> {
        let mut out = vec![Complex::new(0.0, 0.0); input.len()];
        check(unsafe {
            sys::sdsp_nco_mix_block(self.h, down, 1, input.as_ptr() as _, input.len(), out.as_mut_ptr() as _)
        });
        out
    }
}

/// nco/mod.rs:175-187
pub fn constrain(theta: f64) -> u32 {
    unsafe { sys::sdsp_nco_constrain(theta) }
}

impl Default for NCO {
    fn default() -> Self {
        Self::new()
    }
}

impl Drop for NCO {
    fn drop(&mut self) {
        unsafe { sys::sdsp_nco_destroy(self.h) }
    }
}

impl fmt::Display for NCO {
    /// nco/mod.rs:195-203
    fn fmt(&self, f: &mut fmt::Formatter) -> fmt::Result {
        let (mut theta, mut delta_theta) = (0u32, 0u32);
        check(unsafe { sys::sdsp_nco_get_state(self.h, &mut theta, &mut delta_theta) });
        write!(f, "NCO [Theta={}] [ΔTheta={}] [Alpha={}] [Beta={}]", theta, delta_theta, self.alpha, self.beta)
    }
}
