//! `solid::filter::fir` (src/filter/fir/mod.rs:35-318): `FIRFilter` on libsdsp.so.
//! Same constructor, accessors, error enum, `Clone`, `Display` and `Filter` impl.
//! The delay line lives in the handle (sdsp_fir): `execute(sample)` and short host
//! blocks run the reference arithmetic on the host against it, longer blocks the
//! gfx950 kernels (EXACT by default: bit-identical to the reference at the pair's
//! precision).  Device-only extras (algorithm choice, device-resident blocks) are
//! in `crate::sdsp::FirDevice`, so the inherent API is exactly the reference's.
pub mod decim;
pub mod interp;
pub mod pfb;

use super::{Filter, SdspPair};
use crate::{check, device, last_error, sys};

use std::error::Error;
use std::fmt;
use std::marker::PhantomData;

use num::{Complex, Zero};

/// fir/mod.rs:39-45
#[derive(Debug)]
pub enum FIRErrorCode {
    CoefficientsLengthZero,
    DecimationLessThanOne,
    InterpolationLessThanOne,
    NotEnoughFilters,
}

/// fir/mod.rs:47-56
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

/// fir/mod.rs:58-63
pub struct FIRFilter<Coef, In> {
    pub(crate) h: *mut sys::sdsp_fir,
    pub(crate) _t: PhantomData<(Coef, In)>,
}

impl<Coef: Copy + Zero, In: Copy> FIRFilter<Coef, In>
where
    (Coef, In): SdspPair,
{
    /// FIRFilter::new(&coefs, scale)  fir/mod.rs:79-88
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

    /// fir/mod.rs:106-108
    pub fn set_scale(&mut self, scale: Coef) {
        check(unsafe { sys::sdsp_fir_set_scale(self.h, &scale as *const Coef as _) })
    }

    /// fir/mod.rs:124-126
    pub fn get_scale(&self) -> Coef {
        get_scale(self.h)
    }

    /// fir/mod.rs:142-144
    pub fn len(&self) -> usize {
        unsafe { sys::sdsp_fir_len(self.h) }
    }

    /// fir/mod.rs:158-160
    pub fn is_empty(&self) -> bool {
        self.len() == 0
    }

    /// coefficients(): the stored (reversed) taps  fir/mod.rs:176-178
    pub fn coefficients(&self) -> Vec<Coef> {
        coefficients(self.h)
    }
}

pub(crate) fn get_scale<Coef: Zero>(h: *const sys::sdsp_fir) -> Coef {
    let mut s = Coef::zero();
    check(unsafe { sys::sdsp_fir_get_scale(h, &mut s as *mut Coef as _) });
    s
}

pub(crate) fn coefficients<Coef: Zero + Clone>(h: *const sys::sdsp_fir) -> Vec<Coef> {
    let mut v = vec![Coef::zero(); unsafe { sys::sdsp_fir_len(h) }];
    check(unsafe { sys::sdsp_fir_coefficients(h, v.as_mut_ptr() as _) });
    v
}

impl<Coef, In> Clone for FIRFilter<Coef, In> {
    /// derive(Clone) (fir/mod.rs:58): same taps, a snapshot of the delay line
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

impl<Coef, In> fmt::Debug for FIRFilter<Coef, In> {
    fn fmt(&self, f: &mut fmt::Formatter) -> fmt::Result {
        write!(f, "FIRFilter {{ len: {} }}", unsafe { sys::sdsp_fir_len(self.h) })
    }
}

/// "[c0, c1, ...]" of the stored taps, the DotProduct Display of the reference
/// prints only "DotProduct<T> [Size=n]" (dot_product/mod.rs:146-151)
pub(crate) fn dot_display<C>(len: usize) -> String {
    format!("DotProduct<{}> [Size={}]", std::any::type_name::<C>(), len)
}

impl<C: fmt::Display + Copy + Zero, T: fmt::Display + Copy> fmt::Display for FIRFilter<C, T>
where
    (C, T): SdspPair,
{
    /// fir/mod.rs:306-317
    fn fmt(&self, f: &mut fmt::Formatter) -> fmt::Result {
        write!(f, "FIR<{}> [Scale={:.5}] [Coefficients={}]", std::any::type_name::<C>(), self.get_scale(),
               dot_display::<C>(self.len()))
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

/// one input through the handle's step (host arithmetic against the handle's delay line)
pub(crate) fn run_one<Out: Zero + Clone>(h: *mut sys::sdsp_fir, input: *const std::os::raw::c_void) -> Vec<Out> {
    let mut out = vec![Out::zero(); 1];
    let mut got = 0usize;
    check(unsafe { sys::sdsp_fir_execute(h, input, out.as_mut_ptr() as _, &mut got) });
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
    /// execute(sample): one output per input (fir/mod.rs:209-212)
    fn execute(&mut self, sample: In) -> Vec<In> {
        run_one(self.h, &sample as *const In as _)
    }
    /// execute_block(&samples)  fir/mod.rs:235-241
    fn execute_block(&mut self, samples: &[In]) -> Vec<In> {
        run_block(self.h, samples.as_ptr() as _, samples.len())
    }
    /// scale * sum_i h[i] e^{+j 2 pi f i} over coefficients()  fir/mod.rs:263-273
    fn frequency_response(&self, frequency: f64) -> Complex<f64> {
        response(self.h, frequency)
    }
    /// fir_group_delay(coefficients(), f)  fir/mod.rs:293-303
    fn group_delay(&self, frequency: f64) -> f64 {
        delay(self.h, frequency)
    }
}
