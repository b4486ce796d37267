//! `solid::filter::fir::interp` (src/filter/fir/interp.rs:6-138): InterpolatingFIRFilter.
use super::fir_status;
use super::pfb::PolyPhaseFilterBank;
use crate::filter::{Filter, SdspPair};
use crate::{check, device, sys};

use std::error::Error;
use std::fmt;
use std::marker::PhantomData;

use num::{Complex, Zero};

pub struct InterpolatingFIRFilter<Coef, In> {
    filterbank: PolyPhaseFilterBank<Coef, In>,
    interpolation: usize,
}

impl<Coef: Copy + Zero, In: Copy + Zero> InterpolatingFIRFilter<Coef, In>
where
    (Coef, In): SdspPair,
{
    /// InterpolatingFIRFilter::new(&coefs, M)  interp.rs:27-54 (K = ceil_f32(L / M), zero-padded)
    pub fn new(coefficents: &[Coef], interpolation: usize) -> Result<Self, Box<dyn Error>> {
        let mut h = std::ptr::null_mut();
        let rc = unsafe {
            sys::sdsp_interp_create(&mut h, <(Coef, In)>::DTYPE, coefficents.as_ptr() as _, coefficents.len(),
                                    interpolation, device())
        };
        if rc != 0 {
            return Err(fir_status(rc));
        }
        Ok(InterpolatingFIRFilter { filterbank: PolyPhaseFilterBank { h, _t: PhantomData }, interpolation })
    }

    pub fn set_scale(&mut self, scale: Coef) {
        self.filterbank.set_scale(scale)
    }
    pub fn get_scale(&self) -> Coef {
        self.filterbank.get_scale()
    }
    pub fn len(&self) -> usize {
        self.filterbank.len()
    }
    pub fn is_empty(&self) -> bool {
        self.filterbank.is_empty()
    }
    pub fn coefficents(&self) -> Vec<Coef> {
        self.filterbank.coefficents().into_iter().flatten().collect()
    }
    pub fn interpolation(&self) -> usize {
        self.interpolation
    }
}

impl<Coef, In> Clone for InterpolatingFIRFilter<Coef, In> {
    /// derive(Clone) (interp.rs:6): the filterbank with its window
    fn clone(&self) -> Self {
        InterpolatingFIRFilter { filterbank: self.filterbank.clone(), interpolation: self.interpolation }
    }
}

impl<Coef, In> fmt::Debug for InterpolatingFIRFilter<Coef, In> {
    fn fmt(&self, f: &mut fmt::Formatter) -> fmt::Result {
        write!(f, "InterpolatingFIRFilter {{ interpolation: {} }}", self.interpolation)
    }
}

impl<Coef, In: Copy + Zero> Filter<In, In> for InterpolatingFIRFilter<Coef, In>
where
    (Coef, In): SdspPair,
{
    fn execute(&mut self, sample: In) -> Vec<In> {
        self.execute_block(&[sample])
    }
    /// push each input, then all M branch outputs (interp.rs:102-111)
    fn execute_block(&mut self, samples: &[In]) -> Vec<In> {
        let mut out = vec![In::zero(); samples.len() * self.interpolation];
        if !samples.is_empty() {
            check(unsafe {
                sys::sdsp_pfb_execute_block(self.filterbank.h, samples.as_ptr() as _, samples.len(),
                                            out.as_mut_ptr() as _)
            });
        }
        out
    }
    fn frequency_response(&self, frequency: f64) -> Complex<f64> {
        let mut r = [0.0f64; 2];
        check(unsafe { sys::sdsp_pfb_frequency_response(self.filterbank.h, frequency, r.as_mut_ptr()) });
        Complex::new(r[0], r[1])
    }
    fn group_delay(&self, frequency: f64) -> f64 {
        let mut d = 0.0f64;
        check(unsafe { sys::sdsp_pfb_group_delay(self.filterbank.h, frequency, &mut d) });
        d
    }
}
