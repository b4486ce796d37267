//! `solid::filter::iir::decim` (src/filter/iir/decim.rs:1-290): DecimatingIIRFilter —
//! the IIR runs on every input, an output leaves when `(index + 1) % M == 0`
//! (decim.rs:190-233); the index lives in the handle.
use super::sos::SecondOrderFilter;
use super::{iir_status, kind, IIRFilterType, IirCore};
use crate::filter::{Filter, SdspIirPair};
use crate::sys;

use std::error::Error;
use std::fmt;

use num::{Complex, Zero};

/// decim.rs:5-10
pub struct DecimatingIIRFilter<Coef, In> {
    core: IirCore<Coef, In>,
    decimation: usize,
}

impl<Coef: Copy + Zero, In: Copy + Zero> DecimatingIIRFilter<Coef, In>
where
    (Coef, In): SdspIirPair<Coef = Coef>,
{
    /// DecimatingIIRFilter::new(&ff, &fb, iirtype, decimation)  decim.rs:30-62
    pub fn new(feed_forward: &[Coef], feed_back: &[Coef], iirtype: IIRFilterType, decimation: usize)
               -> Result<Self, Box<dyn Error>> {
        let mut h = std::ptr::null_mut();
        let rc = unsafe {
            sys::sdsp_iir_decim_create(&mut h, <(Coef, In)>::DTYPE, feed_forward.as_ptr() as _, feed_forward.len(),
                                       feed_back.as_ptr() as _, feed_back.len(), kind(iirtype), decimation,
                                       crate::device())
        };
        if rc != 0 {
            return Err(iir_status(rc));
        }
        Ok(DecimatingIIRFilter { core: IirCore::new(h, iirtype, feed_forward, feed_back), decimation })
    }

    /// decim.rs:64-66
    pub fn get_decimation(&self) -> usize {
        self.decimation
    }

    /// decim.rs:88-90
    pub fn numerator_coefs(&self) -> Vec<Coef> {
        self.core.numerator_coefs()
    }

    /// decim.rs:112-114
    pub fn denominator_coefs(&self) -> Vec<Coef> {
        self.core.denominator_coefs()
    }

    /// decim.rs:134-136
    pub fn second_order_filters(&self) -> &Vec<SecondOrderFilter<Coef, In>> {
        self.core.second_order_filters()
    }

    /// decim.rs:154-156
    pub fn iir_type(&self) -> &IIRFilterType {
        &self.core.iirtype
    }
}

impl<Coef: Copy + Zero, In: Copy + Zero> Clone for DecimatingIIRFilter<Coef, In>
where
    (Coef, In): SdspIirPair<Coef = Coef>,
{
    fn clone(&self) -> Self {
        DecimatingIIRFilter { core: self.core.try_clone(), decimation: self.decimation }
    }
}

impl<Coef, In> fmt::Debug for DecimatingIIRFilter<Coef, In> {
    fn fmt(&self, f: &mut fmt::Formatter) -> fmt::Result {
        write!(f, "DecimatingIIRFilter {{ decimation: {} }}", self.decimation)
    }
}

impl<C: fmt::Display, T: fmt::Display> fmt::Display for DecimatingIIRFilter<C, T> {
    /// decim.rs:282-290
    fn fmt(&self, f: &mut fmt::Formatter) -> fmt::Result {
        write!(f, "Decimating IIR<{}: {}>", std::any::type_name::<C>(), self.decimation)
    }
}

impl<Coef: Copy + Zero, In: Copy + Zero> Filter<In, In> for DecimatingIIRFilter<Coef, In>
where
    (Coef, In): SdspIirPair<Coef = Coef>,
{
    /// decim.rs:190-199
    fn execute(&mut self, sample: In) -> Vec<In> {
        self.core.run_one(&sample as *const In as _)
    }
    /// decim.rs:222-233
    fn execute_block(&mut self, samples: &[In]) -> Vec<In> {
        self.core.run(samples.as_ptr() as _, samples.len())
    }
    /// the wrapped IIRFilter's  decim.rs:254-256
    fn frequency_response(&self, frequency: f64) -> Complex<f64> {
        self.core.response(frequency)
    }
    /// decim.rs:277-279
    fn group_delay(&self, frequency: f64) -> f64 {
        self.core.delay(frequency)
    }
}
