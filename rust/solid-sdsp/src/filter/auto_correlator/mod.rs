//! `solid::filter::auto_correlator` (src/filter/auto_correlator/mod.rs:26-215):
//! `AutoCorrelator<C>` on libsdsp.so (sdsp_acorr).  The two `Window`s and the
//! energy ring live in the handle; `execute_block` runs the push-then-execute loop
//! as the gfx950 `acorr_*` kernels, bit-identical to the reference order
//! (tests/test_gpu_rx.py), including the delayed window's unfilled tail.
use crate::{check, device, sys};

use std::error::Error;
use std::fmt;
use std::marker::PhantomData;

use num::complex::Complex;

/// The component types the handle runs: f32 (precision 0) and f64 (1).  The
/// reference's `push` needs `Complex<C>: Real<Output = f64>` (:99-102), i.e. C = f64;
/// the f32 handle runs the same operations at f32.
pub trait AcorrComponent: private::Sealed + Copy {
    const PRECISION: std::os::raw::c_int;
    fn zero() -> Self;
}
mod private {
    pub trait Sealed {}
}
impl private::Sealed for f32 {}
impl private::Sealed for f64 {}
impl AcorrComponent for f32 {
    const PRECISION: std::os::raw::c_int = 0;
    fn zero() -> Self {
        0.0
    }
}
impl AcorrComponent for f64 {
    const PRECISION: std::os::raw::c_int = 1;
    fn zero() -> Self {
        0.0
    }
}

/// auto_correlator/mod.rs:26-36
pub struct AutoCorrelator<C> {
    h: *mut sys::sdsp_acorr,
    _t: PhantomData<C>,
}

impl<C: AcorrComponent> AutoCorrelator<C> {
    /// :51-62 (the reference cannot fail; a device failure panics)
    pub fn new(window_size: usize, delay: usize) -> Self {
        let mut h = std::ptr::null_mut();
        check(unsafe { sys::sdsp_acorr_create(&mut h, window_size, delay, C::PRECISION, device()) });
        AutoCorrelator { h, _t: PhantomData }
    }

    /// :76-85
    pub fn reset(&mut self) {
        check(unsafe { sys::sdsp_acorr_reset(self.h) })
    }

    /// :99-111
    pub fn push(&mut self, sample: Complex<C>) {
        check(unsafe { sys::sdsp_acorr_push(self.h, &sample as *const Complex<C> as _) })
    }

    /// :128-137
    pub fn write(&mut self, samples: &[Complex<C>]) -> Result<(), Box<dyn Error>> {
        check(unsafe { sys::sdsp_acorr_write(self.h, samples.as_ptr() as _, samples.len()) });
        Ok(())
    }

    /// :156-163: sum over the windows, newest first, from zero
    pub fn execute(&self) -> Complex<C> {
        let mut out = Complex::new(C::zero(), C::zero());
        check(unsafe { sys::sdsp_acorr_execute(self.h, &mut out as *mut Complex<C> as _) });
        out
    }

    /// :181-191: push then execute per sample
    pub fn execute_block(&mut self, samples: &[Complex<C>]) -> Vec<Complex<C>> {
        let mut out = vec![Complex::new(C::zero(), C::zero()); samples.len()];
        check(unsafe {
            sys::sdsp_acorr_execute_block(self.h, samples.as_ptr() as _, samples.len(), out.as_mut_ptr() as _)
        });
        out
    }

    /// :212-214
    pub fn get_energy(&self) -> f64 {
        let mut e = 0.0f64;
        check(unsafe { sys::sdsp_acorr_get_energy(self.h, &mut e) });
        e
    }
}

impl<C> Drop for AutoCorrelator<C> {
    fn drop(&mut self) {
        unsafe { sys::sdsp_acorr_destroy(self.h) }
    }
}

/// :217-226
impl<C> fmt::Display for AutoCorrelator<C> {
    fn fmt(&self, f: &mut fmt::Formatter) -> fmt::Result {
        let typename = std::any::type_name::<C>();
        let mut e = 0.0f64;
        check(unsafe { sys::sdsp_acorr_get_energy(self.h, &mut e) });
        let (w, d) = unsafe { (sys::sdsp_acorr_window_size(self.h), sys::sdsp_acorr_delay(self.h)) };
        write!(f, "AutoCorrelator<{}> [Size={}] [Delay={}] [Energy={}]", typename, w, d, e)
    }
}
