//! `solid::fft` (src/fft/mod.rs:15-215): FFT::new / FFT::execute on the device
//! (every size the reference plans; unnormalised REVERSE like the reference).
//! The public enums and the error type are the reference's (mod.rs:16-55,
//! 145-161); the plan itself is the device's (include/sdsp.h sdsp_fft_*), so
//! `FFTMethod` records the reference planner's choice (mod.rs:123-143) for
//! callers that inspect it, not the kernel that runs.
use crate::{device, last_error, sys};

use std::error::Error;
use std::fmt;

use num::Complex;

#[derive(Debug, PartialEq, Eq, Clone, Copy)]
pub enum FFTDirection {
    FORWARD,
    REVERSE,
}

#[derive(Debug, PartialEq, Eq, Clone, Copy)]
pub enum FFTType {
    DEFAULT,
    FORWARD,
    REVERSE,
    REDFT00,
    REDFT01,
    REDFT10,
    REDFT11,
    RODFT00,
    RODFT01,
    RODFT10,
    RODFT11,
    MDCT,
    IMDCT,
}

#[derive(Debug, PartialEq, Eq, Clone, Copy)]
pub enum FFTMethod {
    DEFAULT,
    RADIX2,
    MIXEDRADIX,
    RADER,
    RADER2,
    DFT,
    UNKNOWN,
}

#[derive(Debug, PartialEq, Eq, Clone, Copy)]
pub enum FFTFlags {
    ESTIMATE,
    MEASURE,
}

/// mod.rs:145-150 (the reference's variants; the device plan reports only NotEnoughBuffer)
#[allow(dead_code)]
#[derive(Debug, PartialEq)]
enum FFTErrorCode {
    NotEnoughBuffer,
    RadixFFTNotMultipleOf2,
    BadExecuteMethod,
}

/// mod.rs:152-161
#[derive(Debug)]
pub struct FFTError(FFTErrorCode);

impl fmt::Display for FFTError {
    fn fmt(&self, f: &mut fmt::Formatter) -> fmt::Result {
        write!(f, "FFT Error: {:?}", self.0)
    }
}

impl Error for FFTError {}

fn is_radix2(n: usize) -> bool {
    n != 0 && n & (n - 1) == 0
}

fn is_prime(n: usize) -> bool {
    if n < 2 {
        return false;
    }
    let mut d = 2usize;
    while d * d <= n {
        if n % d == 0 {
            return false;
        }
        d += 1;
    }
    true
}

/// the reference planner's choice, mod.rs:123-143
fn estimate_method(nfft: usize) -> FFTMethod {
    if nfft == 0 {
        FFTMethod::UNKNOWN
    } else if nfft <= 8 || nfft == 11 || nfft == 13 || nfft == 16 || nfft == 17 {
        FFTMethod::DFT
    } else if is_radix2(nfft) {
        FFTMethod::MIXEDRADIX
    } else if is_prime(nfft) {
        if is_radix2(nfft - 1) {
            FFTMethod::RADER
        } else {
            FFTMethod::RADER2
        }
    } else {
        FFTMethod::MIXEDRADIX
    }
}

#[allow(dead_code)]
pub struct FFT {
    h: *mut sys::sdsp_fft,
    nfft: usize,
    fft_direction: FFTDirection,
    fft_type: FFTType,
    fft_method: FFTMethod,
    fft_flags: FFTFlags,
}

impl FFT {
    /// FFT::new(nfft, direction, flags)  fft/mod.rs:175-186 (flags do not change the plan)
    pub fn new(nfft: usize, direction: FFTDirection, flags: FFTFlags) -> Self {
        let mut h = std::ptr::null_mut();
        let d = if direction == FFTDirection::FORWARD { 0 } else { 1 };
        let rc = unsafe { sys::sdsp_fft_create(&mut h, nfft, d, 1, device()) };
        assert_eq!(rc, 0, "{}", last_error(rc));
        let fft_type = if direction == FFTDirection::FORWARD { FFTType::FORWARD } else { FFTType::REVERSE };
        FFT { h, nfft, fft_direction: direction, fft_type, fft_method: estimate_method(nfft), fft_flags: flags }
    }

    /// FFT::execute(&input)  fft/mod.rs:188-215: nfft Complex<f64> in, nfft out; a short
    /// input is the reference's NotEnoughBuffer (dft/mod.rs:139)
    pub fn execute(&self, input: &[Complex<f64>]) -> Result<Vec<Complex<f64>>, Box<dyn Error>> {
        if input.len() < self.nfft {
            return Err(Box::new(FFTError(FFTErrorCode::NotEnoughBuffer)));
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
