//! `solid::filter::fir::decim` (src/filter/fir/decim.rs:5-281): DecimatingFIRFilter.
use super::{delay, fir_status, response, run_block};
use crate::filter::{Filter, SdspPair};
use crate::{check, device, sys};

use std::error::Error;
use std::marker::PhantomData;

use num::{Complex, Zero};

pub struct DecimatingFIRFilter<Coef, In> {
    h: *mut sys::sdsp_fir,
    _t: PhantomData<(Coef, In)>,
}

impl<Coef: Copy + Zero, In: Copy> DecimatingFIRFilter<Coef, In>
where
    (Coef, In): SdspPair,
{
    /// DecimatingFIRFilter::new(&coefs, scale, decimation)  decim.rs:27-50
    pub fn new(coefficents: &[Coef], scale: Coef, decimation: usize) -> Result<Self, Box<dyn Error>> {
        let mut h = std::ptr::null_mut();
        let rc = unsafe {
            sys::sdsp_decim_create(&mut h, <(Coef, In)>::DTYPE, coefficents.as_ptr() as _, coefficents.len(),
                                   &scale as *const Coef as _, decimation, device())
        };
        if rc != 0 {
            return Err(fir_status(rc));
        }
        Ok(DecimatingFIRFilter { h, _t: PhantomData })
    }

    pub fn decimation(&self) -> usize {
        unsafe { sys::sdsp_fir_decimation(self.h) }
    }

    /// push(sample): advance the window and the phase, no output (decim.rs:127-131)
    pub fn push(&mut self, sample: In) {
        check(unsafe { sys::sdsp_decim_push(self.h, &sample as *const In as _) })
    }

    /// write(&samples): push each sample (decim.rs:133-137)
    pub fn write(&mut self, samples: &[In]) {
        check(unsafe { sys::sdsp_decim_write(self.h, samples.as_ptr() as _, samples.len()) })
    }

    pub fn reset(&mut self) {
        check(unsafe { sys::sdsp_fir_reset(self.h) })
    }
}

impl<Coef, In> Drop for DecimatingFIRFilter<Coef, In> {
    fn drop(&mut self) {
        unsafe { sys::sdsp_fir_destroy(self.h) }
    }
}

impl<Coef, In: Copy + Zero> Filter<In, In> for DecimatingFIRFilter<Coef, In>
where
    (Coef, In): SdspPair,
{
    /// emits on inputs M-1, 2M-1, ... of the running phase (decim.rs:221-256)
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
