//! `solid::filter::iir::interp` (src/filter/iir/interp.rs:1-278): InterpolatingIIRFilter —
//! per input, IIR(x) then IIR(0) M - 1 times (interp.rs:184-221).
use super::sos::SecondOrderFilter;
use super::{iir_status, kind, IIRFilterType, IirCore};
use crate::filter::{Filter, SdspIirPair};
use crate::sys;

use std::error::Error;
use std::fmt;

use num::{Complex, Zero};

/// interp.rs:5-9
pub struct InterpolatingIIRFilter<Coef, In> {
    core: IirCore<Coef, In>,
    interpolation: usize,
}

impl<Coef: Copy + Zero, In: Copy + Zero> InterpolatingIIRFilter<Coef, In>
where
    (Coef, In): SdspIirPair<Coef = Coef>,
{
    /// InterpolatingIIRFilter::new(&ff, &fb, iirtype, interpolation)  interp.rs:29-60
    pub fn new(feed_forward: &[Coef], feed_back: &[Coef], iirtype: IIRFilterType, interpolation: usize)
               -> Result<Self, Box<dyn Error>> {
        let mut h = std::ptr::null_mut();
        let rc = unsafe {
            sys::sdsp_iir_interp_create(&mut h, <(Coef, In)>::DTYPE, feed_forward.as_ptr() as _, feed_forward.len(),
                                       feed_back.as_ptr() as _, feed_back.len(), kind(iirtype), interpolation,
                                       crate::device())
        };
        if rc != 0 {
            return Err(iir_status(rc));
        }
        Ok(InterpolatingIIRFilter { core: IirCore::new(h, iirtype, feed_forward, feed_back), interpolation })
    }

    /// interp.rs:62-64
    pub fn get_interpolation(&self) -> usize {
        self.interpolation
    }

    /// interp.rs:86-88
    pub fn numerator_coefs(&self) -> Vec<Coef> {
        self.core.numerator_coefs()
    }

    /// interp.rs:110-112
    pub fn denominator_coefs(&self) -> Vec<Coef> {
        self.core.denominator_coefs()
    }

    /// interp.rs:132-134
    pub fn second_order_filters(&self) -> &Vec<SecondOrderFilter<Coef, In>> {
        self.core.second_order_filters()
    }

    /// interp.rs:152-154
    pub fn iir_type(&self) -> &IIRFilterType {
        &self.core.iirtype
    }
}

impl<Coef: Copy + Zero, In: Copy + Zero> Clone for InterpolatingIIRFilter<Coef, In>
where
    (Coef, In): SdspIirPair<Coef = Coef>,
{
    fn clone(&self) -> Self {
        InterpolatingIIRFilter { core: self.core.try_clone(), interpolation: self.interpolation }
    }
}

impl<Coef, In> fmt::Debug for InterpolatingIIRFilter<Coef, In> {
    fn fmt(&self, f: &mut fmt::Formatter) -> fmt::Result {
        write!(f, "InterpolatingIIRFilter {{ interpolation: {} }}", self.interpolation)
    }
}

impl<C: fmt::Display, T: fmt::Display> fmt::Display for InterpolatingIIRFilter<C, T> {
    /// interp.rs:270-278
    fn fmt(&self, f: &mut fmt::Formatter) -> fmt::Result {
        write!(f, "interpating IIR<{}: {}>", std::any::type_name::<C>(), self.interpolation)
    }
}

impl<Coef: Copy + Zero, In: Copy + Zero> Filter<In, In> for InterpolatingIIRFilter<Coef, In>
where
    (Coef, In): SdspIirPair<Coef = Coef>,
{
    /// interp.rs:184-190
    fn execute(&mut self, sample: In) -> Vec<In> {
        self.core.run_one(&sample as *const In as _)
    }
    /// interp.rs:215-221
    fn execute_block(&mut self, samples: &[In]) -> Vec<In> {
        self.core.run(samples.as_ptr() as _, samples.len())
    }
    /// the wrapped IIRFilter's  interp.rs:242-244
    fn frequency_response(&self, frequency: f64) -> Complex<f64> {
        self.core.response(frequency)
    }
    /// interp.rs:265-267
    fn group_delay(&self, frequency: f64) -> f64 {
        self.core.delay(frequency)
    }
}
