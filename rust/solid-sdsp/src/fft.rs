//! `solid::fft` (src/fft/mod.rs:15-215): FFT::new / FFT::execute on the device
//! (every size the reference plans; unnormalised REVERSE like the reference).
use crate::{device, last_error, sys};

use std::error::Error;

use num::Complex;

#[derive(Debug, PartialEq, Eq, Clone, Copy)]
pub enum FFTDirection {
    FORWARD,
    REVERSE,
}

#[derive(Debug, PartialEq, Eq, Clone, Copy)]
pub enum FFTFlags {
    ESTIMATE,
    MEASURE,
}

pub struct FFT {
    h: *mut sys::sdsp_fft,
    nfft: usize,
}

impl FFT {
    /// FFT::new(nfft, direction, flags)  fft/mod.rs:175-186 (flags do not change the plan)
    pub fn new(nfft: usize, direction: FFTDirection, _flags: FFTFlags) -> Self {
        let mut h = std::ptr::null_mut();
        let d = if direction == FFTDirection::FORWARD { 0 } else { 1 };
        let rc = unsafe { sys::sdsp_fft_create(&mut h, nfft, d, 1, device()) };
        assert_eq!(rc, 0, "{}", last_error(rc));
        FFT { h, nfft }
    }

    /// FFT::execute(&input)  fft/mod.rs:188-215: nfft Complex<f64> in, nfft out
    pub fn execute(&self, input: &[Complex<f64>]) -> Result<Vec<Complex<f64>>, Box<dyn Error>> {
        if input.len() < self.nfft {
            return Err(Box::new(last_error(90)));
        }
        let mut out = vec![Complex::new(0.0, 0.0); self.nfft];
        match unsafe { sys::sdsp_fft_execute(self.h, input.as_ptr() as _, out.as_mut_ptr() as _, 1) } {
            0 => Ok(out),
            rc => Err(Box::new(last_error(rc))),
        }
    }
}

impl Drop for FFT {
    fn drop(&mut self) {
        unsafe { sys::sdsp_fft_destroy(self.h) }
    }
}
