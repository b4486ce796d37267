//! `solid::filter::fir` (src/filter/fir/mod.rs:58-304): FIRFilter on libsdsp.so.
//! Same constructor, accessors, error enum and `Filter` impl; the window and the
//! dot product live on the device (sdsp_fir handle, EXACT kernel by default:
//! bit-identical to the reference at the pair's precision).
pub mod decim;
pub mod interp;
pub mod pfb;

use super::{Filter, SdspPair};
use crate::{check, device, last_error, sys};

use std::error::Error;
use std::fmt;
use std::marker::PhantomData;

use num::{Complex, Zero};

#[derive(Debug)]
pub enum FIRErrorCode {
    CoefficientsLengthZero,
    DecimationLessThanOne,
    InterpolationLessThanOne,
    NotEnoughFilters,
}

#[derive(Debug)]
pub struct FIRError(pub FIRErrorCode);

impl fmt::Display for FIRError {
    fn fmt(&self, f: &mut fmt::Formatter) -> fmt::Result {
        write!(f, "FIR Filter Error {:?}", self.0)
    }
}

impl Error for FIRError {}

/// status code -> the reference's error (FIRErrorCode) or a device error
pub(crate) fn fir_status(rc: i32) -> Box<dyn Error> {
    match rc {
        sys::SDSP_E_COEFFICIENTS_LENGTH_ZERO => Box::new(FIRError(FIRErrorCode::CoefficientsLengthZero)),
        sys::SDSP_E_DECIMATION_LESS_THAN_ONE => Box::new(FIRError(FIRErrorCode::DecimationLessThanOne)),
        sys::SDSP_E_INTERPOLATION_LESS_THAN_ONE => Box::new(FIRError(FIRErrorCode::InterpolationLessThanOne)),
        sys::SDSP_E_NOT_ENOUGH_FILTERS => Box::new(FIRError(FIRErrorCode::NotEnoughFilters)),
        _ => Box::new(last_error(rc)),
    }
}

pub struct FIRFilter<Coef, In> {
    pub(crate) h: *mut sys::sdsp_fir,
    _t: PhantomData<(Coef, In)>,
}

impl<Coef: Copy + Zero, In: Copy> FIRFilter<Coef, In>
where
    (Coef, In): SdspPair,
{
    /// FIRFilter::new(&coefs, scale)  fir/mod.rs:79-96
    pub fn new(coefficents: &[Coef], scale: Coef) -> Result<Self, Box<dyn Error>> {
        let mut h = std::ptr::null_mut();
        let rc = unsafe {
            sys::sdsp_fir_create(&mut h, <(Coef, In)>::DTYPE, coefficents.as_ptr() as _, coefficents.len(),
                                 &scale as *const Coef as _, device())
        };
        if rc != 0 {
            return Err(fir_status(rc));
        }
        Ok(FIRFilter { h, _t: PhantomData })
    }

    pub fn set_scale(&mut self, scale: Coef) {
        check(unsafe { sys::sdsp_fir_set_scale(self.h, &scale as *const Coef as _) })
    }

    pub fn get_scale(&self) -> Coef {
        let mut s = Coef::zero();
        check(unsafe { sys::sdsp_fir_get_scale(self.h, &mut s as *mut Coef as _) });
        s
    }

    pub fn len(&self) -> usize {
        unsafe { sys::sdsp_fir_len(self.h) }
    }

    pub fn is_empty(&self) -> bool {
        self.len() == 0
    }

    /// coefficents(): the stored (reversed) taps, fir/mod.rs:124-127
    pub fn coefficents(&self) -> Vec<Coef> {
        let mut v = vec![Coef::zero(); self.len()];
        check(unsafe { sys::sdsp_fir_coefficients(self.h, v.as_mut_ptr() as _) });
        v
    }

    /// Opt into a fast kernel (sys::SDSP_ALGO_FMA / SDSP_ALGO_FFT); results then agree
    /// within the documented tolerance instead of bit for bit.
    pub fn set_algorithm(&mut self, algo: i32) -> Result<(), Box<dyn Error>> {
        match unsafe { sys::sdsp_fir_set_algo(self.h, algo) } {
            0 => Ok(()),
            rc => Err(Box::new(last_error(rc))),
        }
    }
}

impl<Coef, In> Clone for FIRFilter<Coef, In> {
    fn clone(&self) -> Self {
        let mut h = std::ptr::null_mut();
        check(unsafe { sys::sdsp_fir_clone(self.h, &mut h) });
        FIRFilter { h, _t: PhantomData }
    }
}

impl<Coef, In> Drop for FIRFilter<Coef, In> {
    fn drop(&mut self) {
        unsafe { sys::sdsp_fir_destroy(self.h) }
    }
}

pub(crate) fn run_block<Out: Zero + Clone>(h: *mut sys::sdsp_fir, input: *const std::os::raw::c_void, n: usize) -> Vec<Out> {
    let cap = unsafe { sys::sdsp_fir_output_count(h, n) };
    let mut out = vec![Out::zero(); cap];
    let mut got = 0usize;
    check(unsafe { sys::sdsp_fir_execute_block(h, input, n, out.as_mut_ptr() as _, &mut got) });
    out.truncate(got);
    out
}

pub(crate) fn response(h: *const sys::sdsp_fir, f: f64) -> Complex<f64> {
    let mut r = [0.0f64; 2];
    check(unsafe { sys::sdsp_fir_frequency_response(h, f, r.as_mut_ptr()) });
    Complex::new(r[0], r[1])
}

pub(crate) fn delay(h: *const sys::sdsp_fir, f: f64) -> f64 {
    let mut d = 0.0f64;
    check(unsafe { sys::sdsp_fir_group_delay(h, f, &mut d) });
    d
}

/// Out = Coef * In of the reference's Execute impls: In itself for every supported pair.
impl<Coef, In: Copy + Zero> Filter<In, In> for FIRFilter<Coef, In>
where
    (Coef, In): SdspPair,
{
    /// execute(sample): one output per input (fir/mod.rs:209-212) -- a device round trip
    fn execute(&mut self, sample: In) -> Vec<In> {
        run_block(self.h, &sample as *const In as _, 1)
    }
    fn execute_block(&mut self, samples: &[In]) -> Vec<In> {
        run_block(self.h, samples.as_ptr() as _, samples.len())
    }
    fn frequency_response(&self, frequency: f64) -> Complex<f64> {
        response(self.h, frequency)
    }
    fn group_delay(&self, frequency: f64) -> f64 {
        delay(self.h, frequency)
    }
}
