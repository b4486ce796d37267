//! `solid::filter::iir` (src/filter/iir/mod.rs:62-414): IIRFilter, Decimating and
//! Interpolating forms, on libsdsp.so (sdsp_iir handle; EXACT serial recurrence by
//! default, bit-identical; the block-parallel scans are opt-in via set_algorithm).
use super::{Filter, SdspPair};
use crate::{check, device, last_error, sys};

use std::error::Error;
use std::fmt;
use std::marker::PhantomData;

use num::{Complex, Zero};

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

#[derive(Debug)]
pub struct IIRError(pub IIRErrorCode);

impl fmt::Display for IIRError {
    fn fmt(&self, f: &mut fmt::Formatter) -> fmt::Result {
        write!(f, "IIR Filter Error {:?}", self.0)
    }
}

impl Error for IIRError {}

#[derive(PartialEq, Eq, Debug, Clone, Copy)]
pub enum IIRFilterType {
    Normal,
    SecondOrder,
}

fn iir_status(rc: i32) -> Box<dyn Error> {
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

fn kind(t: IIRFilterType) -> i32 {
    match t {
        IIRFilterType::Normal => 0,
        IIRFilterType::SecondOrder => 1,
    }
}

/// One device handle behind all three reference types.
struct Handle(*mut sys::sdsp_iir);

impl Drop for Handle {
    fn drop(&mut self) {
        unsafe { sys::sdsp_iir_destroy(self.0) }
    }
}

impl Handle {
    fn run<Out: Zero + Clone>(&self, input: *const std::os::raw::c_void, n: usize) -> Vec<Out> {
        let cap = unsafe { sys::sdsp_iir_output_count(self.0, n) };
        let mut out = vec![Out::zero(); cap];
        let mut got = 0usize;
        check(unsafe { sys::sdsp_iir_execute_block(self.0, input, n, out.as_mut_ptr() as _, &mut got) });
        out.truncate(got);
        out
    }
    fn response(&self, f: f64) -> Complex<f64> {
        let mut r = [0.0f64; 2];
        check(unsafe { sys::sdsp_iir_frequency_response(self.0, f, r.as_mut_ptr()) });
        Complex::new(r[0], r[1])
    }
    fn delay(&self, f: f64) -> f64 {
        let mut d = 0.0f64;
        check(unsafe { sys::sdsp_iir_group_delay(self.0, f, &mut d) });
        d
    }
}

macro_rules! iir_type {
    ($name:ident, $ctor:ident $(, $extra:ident)?) => {
        pub struct $name<Coef, In> {
            h: Handle,
            iirtype: IIRFilterType,
            $($extra: usize,)?
            _t: PhantomData<(Coef, In)>,
        }

        impl<Coef, In> $name<Coef, In> {
            pub fn iir_type(&self) -> &IIRFilterType {
                &self.iirtype
            }
            pub fn reset(&mut self) {
                check(unsafe { sys::sdsp_iir_reset(self.h.0) })
            }
            /// Opt into the block-parallel scan (sys::SDSP_ALGO_FMA / SDSP_ALGO_AUTO).
            pub fn set_algorithm(&mut self, algo: i32) -> Result<(), Box<dyn Error>> {
                match unsafe { sys::sdsp_iir_set_algo(self.h.0, algo) } {
                    0 => Ok(()),
                    rc => Err(Box::new(last_error(rc))),
                }
            }
        }

        impl<Coef, In: Copy + Zero> Filter<In, In> for $name<Coef, In>
        where
            (Coef, In): SdspPair,
        {
            fn execute(&mut self, sample: In) -> Vec<In> {
                self.h.run(&sample as *const In as _, 1)
            }
            fn execute_block(&mut self, samples: &[In]) -> Vec<In> {
                self.h.run(samples.as_ptr() as _, samples.len())
            }
            fn frequency_response(&self, frequency: f64) -> Complex<f64> {
                self.h.response(frequency)
            }
            fn group_delay(&self, frequency: f64) -> f64 {
                self.h.delay(frequency)
            }
        }
    };
}

iir_type!(IIRFilter, sdsp_iir_create);
iir_type!(DecimatingIIRFilter, sdsp_iir_decim_create, decimation);
iir_type!(InterpolatingIIRFilter, sdsp_iir_interp_create, interpolation);

impl<Coef: Copy, In: Copy> IIRFilter<Coef, In>
where
    (Coef, In): SdspPair,
{
    /// IIRFilter::new(&ff, &fb, type)  iir/mod.rs:92-164
    pub fn new(feed_forward: &[Coef], feed_back: &[Coef], iirtype: IIRFilterType) -> Result<Self, Box<dyn Error>> {
        let mut h = std::ptr::null_mut();
        let rc = unsafe {
            sys::sdsp_iir_create(&mut h, <(Coef, In)>::DTYPE, feed_forward.as_ptr() as _, feed_forward.len(),
                                 feed_back.as_ptr() as _, feed_back.len(), kind(iirtype), device())
        };
        if rc != 0 {
            return Err(iir_status(rc));
        }
        Ok(IIRFilter { h: Handle(h), iirtype, _t: PhantomData })
    }
}

impl<Coef: Copy, In: Copy> DecimatingIIRFilter<Coef, In>
where
    (Coef, In): SdspPair,
{
    /// DecimatingIIRFilter::new(&ff, &fb, type, M)  iir/decim.rs:30-62
    pub fn new(feed_forward: &[Coef], feed_back: &[Coef], iirtype: IIRFilterType, decimation: usize)
               -> Result<Self, Box<dyn Error>> {
        let mut h = std::ptr::null_mut();
        let rc = unsafe {
            sys::sdsp_iir_decim_create(&mut h, <(Coef, In)>::DTYPE, feed_forward.as_ptr() as _, feed_forward.len(),
                                       feed_back.as_ptr() as _, feed_back.len(), kind(iirtype), decimation, device())
        };
        if rc != 0 {
            return Err(iir_status(rc));
        }
        Ok(DecimatingIIRFilter { h: Handle(h), iirtype, decimation, _t: PhantomData })
    }
    pub fn get_decimation(&self) -> usize {
        self.decimation
    }
}

impl<Coef: Copy, In: Copy> InterpolatingIIRFilter<Coef, In>
where
    (Coef, In): SdspPair,
{
    /// InterpolatingIIRFilter::new(&ff, &fb, type, M)  iir/interp.rs:29-60
    pub fn new(feed_forward: &[Coef], feed_back: &[Coef], iirtype: IIRFilterType, interpolation: usize)
               -> Result<Self, Box<dyn Error>> {
        let mut h = std::ptr::null_mut();
        let rc = unsafe {
            sys::sdsp_iir_interp_create(&mut h, <(Coef, In)>::DTYPE, feed_forward.as_ptr() as _, feed_forward.len(),
                                        feed_back.as_ptr() as _, feed_back.len(), kind(iirtype), interpolation,
                                        device())
        };
        if rc != 0 {
            return Err(iir_status(rc));
        }
        Ok(InterpolatingIIRFilter { h: Handle(h), iirtype, interpolation, _t: PhantomData })
    }
    pub fn get_interpolation(&self) -> usize {
        self.interpolation
    }
}
