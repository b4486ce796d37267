//! `solid::filter::iir` (src/filter/iir/mod.rs:17-420): `IIRFilter`, `IIRFilterType`,
//! the error enum, and the `sos` / `decim` / `interp` modules, on libsdsp.so (one
//! sdsp_iir handle per filter: the reference-order serial recurrence by default,
//! bit-identical; the block-parallel scans are opt-in through `crate::sdsp::IirDevice`).
pub mod decim;
pub mod interp;
pub mod sos;

use self::sos::SecondOrderFilter;
use super::{Filter, SdspIirPair};
use crate::{check, last_error, sys};

use std::cell::OnceCell;
use std::error::Error;
use std::fmt;
use std::marker::PhantomData;

use num::{Complex, Zero};

/// mod.rs:40-49
#[derive(Debug)]
pub enum IIRErrorCode {
    NumeratorLengthZero,
    DenominatorLengthZero,
    SecondOrderSectionSizeZero,
    SecondOrderSectionSizeMismatch,
    SecondOrderSectionSizeNotMultpleOf3,
    DecimationLessThanOne,
    InterpolationLessThanOne,
}

/// mod.rs:51-60
#[derive(Debug)]
pub struct IIRError(pub IIRErrorCode);

impl fmt::Display for IIRError {
    fn fmt(&self, f: &mut fmt::Formatter) -> fmt::Result {
        write!(f, "IIR Filter Error {:?}", self.0)
    }
}

impl Error for IIRError {}

/// mod.rs:62-66
#[derive(PartialEq, Eq, Debug, Clone, Copy)]
pub enum IIRFilterType {
    Normal,
    SecondOrder,
}

pub(crate) fn iir_status(rc: i32) -> Box<dyn Error> {
    let code = match rc {
        sys::SDSP_E_NUMERATOR_LENGTH_ZERO => IIRErrorCode::NumeratorLengthZero,
        sys::SDSP_E_DENOMINATOR_LENGTH_ZERO => IIRErrorCode::DenominatorLengthZero,
        sys::SDSP_E_SOS_SIZE_ZERO => IIRErrorCode::SecondOrderSectionSizeZero,
        sys::SDSP_E_SOS_SIZE_MISMATCH => IIRErrorCode::SecondOrderSectionSizeMismatch,
        sys::SDSP_E_SOS_SIZE_NOT_MULTIPLE_OF_3 => IIRErrorCode::SecondOrderSectionSizeNotMultpleOf3,
        sys::SDSP_E_IIR_DECIMATION_LESS_THAN_ONE => IIRErrorCode::DecimationLessThanOne,
        sys::SDSP_E_IIR_INTERPOLATION_LESS_THAN_ONE => IIRErrorCode::InterpolationLessThanOne,
        _ => return Box::new(last_error(rc)),
    };
    Box::new(IIRError(code))
}

pub(crate) fn kind(t: IIRFilterType) -> i32 {
    match t {
        IIRFilterType::Normal => 0,
        IIRFilterType::SecondOrder => 1,
    }
}

/// One device handle behind each reference IIR type, plus the host copies the
/// accessors return.  The sections of `second_order_filters()` are built on first
/// use from the stored coefficients (each its own handle, zero state: the cascade's
/// running state stays in the filter's handle).
pub(crate) struct IirCore<Coef, In> {
    pub(crate) h: *mut sys::sdsp_iir,
    pub(crate) iirtype: IIRFilterType,
    ff: Vec<Coef>,
    fb: Vec<Coef>,
    sections: OnceCell<Vec<SecondOrderFilter<Coef, In>>>,
    _t: PhantomData<In>,
}

impl<Coef: Copy + Zero, In: Copy + Zero> IirCore<Coef, In>
where
    (Coef, In): SdspIirPair<Coef = Coef>,
{
    pub(crate) fn new(h: *mut sys::sdsp_iir, iirtype: IIRFilterType, ff: &[Coef], fb: &[Coef]) -> Self {
        IirCore { h, iirtype, ff: ff.to_vec(), fb: fb.to_vec(), sections: OnceCell::new(), _t: PhantomData }
    }

    /// numerator_coefs(): Normal b/a0, SecondOrder the flat ff as given  mod.rs:182-184
    pub(crate) fn numerator_coefs(&self) -> Vec<Coef> {
        self.coefs(0)
    }

    /// denominator_coefs(): Normal a[1..]/a0, SecondOrder the flat fb as given  mod.rs:202-204
    pub(crate) fn denominator_coefs(&self) -> Vec<Coef> {
        self.coefs(1)
    }

    fn coefs(&self, which: i32) -> Vec<Coef> {
        let nn = unsafe { sys::sdsp_iir_num_coefs(self.h, 0) };
        let nd = unsafe { sys::sdsp_iir_num_coefs(self.h, 1) };
        let mut num = vec![0.0f64; nn];
        let mut den = vec![0.0f64; nd];
        check(unsafe { sys::sdsp_iir_coefficients(self.h, num.as_mut_ptr(), den.as_mut_ptr()) });
        let v = if which == 0 { num } else { den };
        v.into_iter().map(<(Coef, In)>::coef_from_f64).collect()
    }

    /// second_order_filters()  mod.rs:222-224
    pub(crate) fn second_order_filters(&self) -> &Vec<SecondOrderFilter<Coef, In>> {
        self.sections.get_or_init(|| {
            if self.iirtype != IIRFilterType::SecondOrder {
                return Vec::new();
            }
            (0..self.ff.len() / 3)
                .map(|i| {
                    SecondOrderFilter::new(&self.ff[3 * i..3 * i + 3], &self.fb[3 * i..3 * i + 3])
                        .expect("sections were validated when the filter was built")
                })
                .collect()
        })
    }

    pub(crate) fn run(&mut self, input: *const std::os::raw::c_void, n: usize) -> Vec<In> {
        let cap = unsafe { sys::sdsp_iir_output_count(self.h, n) };
        let mut out = vec![In::zero(); cap];
        let mut got = 0usize;
        check(unsafe { sys::sdsp_iir_execute_block(self.h, input, n, out.as_mut_ptr() as _, &mut got) });
        out.truncate(got);
        out
    }

    pub(crate) fn run_one(&mut self, input: *const std::os::raw::c_void) -> Vec<In> {
        let cap = unsafe { sys::sdsp_iir_output_count(self.h, 1) };
        let mut out = vec![In::zero(); cap.max(1)];
        let mut got = 0usize;
        check(unsafe { sys::sdsp_iir_execute(self.h, input, out.as_mut_ptr() as _, &mut got) });
        out.truncate(got);
        out
    }

    pub(crate) fn response(&self, f: f64) -> Complex<f64> {
        let mut r = [0.0f64; 2];
        check(unsafe { sys::sdsp_iir_frequency_response(self.h, f, r.as_mut_ptr()) });
        Complex::new(r[0], r[1])
    }

    pub(crate) fn delay(&self, f: f64) -> f64 {
        let mut d = 0.0f64;
        check(unsafe { sys::sdsp_iir_group_delay(self.h, f, &mut d) });
        d
    }

    pub(crate) fn try_clone(&self) -> Self {
        let mut h = std::ptr::null_mut();
        check(unsafe { sys::sdsp_iir_clone(self.h, &mut h) });
        IirCore { h, iirtype: self.iirtype, ff: self.ff.clone(), fb: self.fb.clone(), sections: OnceCell::new(),
                  _t: PhantomData }
    }
}

impl<Coef, In> Drop for IirCore<Coef, In> {
    fn drop(&mut self) {
        unsafe { sys::sdsp_iir_destroy(self.h) }
    }
}

/// mod.rs:68-75
pub struct IIRFilter<Coef, In> {
    pub(crate) core: IirCore<Coef, In>,
}

impl<Coef: Copy + Zero, In: Copy + Zero> IIRFilter<Coef, In>
where
    (Coef, In): SdspIirPair<Coef = Coef>,
{
    /// IIRFilter::new(&feed_forward, &feed_back, iirtype)  mod.rs:92-164
    pub fn new(feed_forward: &[Coef], feed_back: &[Coef], iirtype: IIRFilterType) -> Result<Self, Box<dyn Error>> {
        let mut h = std::ptr::null_mut();
        let rc = unsafe {
            sys::sdsp_iir_create(&mut h, <(Coef, In)>::DTYPE, feed_forward.as_ptr() as _, feed_forward.len(),
                                 feed_back.as_ptr() as _, feed_back.len(), kind(iirtype), crate::device())
        };
        if rc != 0 {
            return Err(iir_status(rc));
        }
        Ok(IIRFilter { core: IirCore::new(h, iirtype, feed_forward, feed_back) })
    }

    /// mod.rs:182-184
    pub fn numerator_coefs(&self) -> Vec<Coef> {
        self.core.numerator_coefs()
    }

    /// mod.rs:202-204
    pub fn denominator_coefs(&self) -> Vec<Coef> {
        self.core.denominator_coefs()
    }

    /// mod.rs:222-224
    pub fn second_order_filters(&self) -> &Vec<SecondOrderFilter<Coef, In>> {
        self.core.second_order_filters()
    }

    /// mod.rs:239-241
    pub fn iir_type(&self) -> &IIRFilterType {
        &self.core.iirtype
    }
}

impl<Coef: Copy + Zero, In: Copy + Zero> Clone for IIRFilter<Coef, In>
where
    (Coef, In): SdspIirPair<Coef = Coef>,
{
    /// derive(Clone) (mod.rs:68): coefficients and the running state
    fn clone(&self) -> Self {
        IIRFilter { core: self.core.try_clone() }
    }
}

impl<Coef, In> fmt::Debug for IIRFilter<Coef, In> {
    fn fmt(&self, f: &mut fmt::Formatter) -> fmt::Result {
        write!(f, "IIRFilter {{ iirtype: {:?} }}", self.core.iirtype)
    }
}

impl<C: fmt::Display, T: fmt::Display> fmt::Display for IIRFilter<C, T> {
    /// mod.rs:416-420
    fn fmt(&self, f: &mut fmt::Formatter) -> fmt::Result {
        write!(f, "IIR<{}>", std::any::type_name::<C>())
    }
}

impl<Coef: Copy + Zero, In: Copy + Zero> Filter<In, In> for IIRFilter<Coef, In>
where
    (Coef, In): SdspIirPair<Coef = Coef>,
{
    /// Normal DF-II or the section cascade  mod.rs:270-289
    fn execute(&mut self, input: In) -> Vec<In> {
        self.core.run_one(&input as *const In as _)
    }
    /// mod.rs:310-316
    fn execute_block(&mut self, samples: &[In]) -> Vec<In> {
        self.core.run(samples.as_ptr() as _, samples.len())
    }
    /// Normal: B/A over the stored vectors; SecondOrder: 0 (mod.rs:336-372)
    fn frequency_response(&self, frequency: f64) -> Complex<f64> {
        self.core.response(frequency)
    }
    /// mod.rs:392-413
    fn group_delay(&self, frequency: f64) -> f64 {
        self.core.delay(frequency)
    }
}
