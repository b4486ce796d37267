//! `solid::filter::fir::decim` (src/filter/fir/decim.rs:5-296): DecimatingFIRFilter.
//! The phase counter `current_item` (decim.rs:7) lives in the handle; `push` /
//! `write` advance it without output, `execute` emits when it wraps to 0.
use super::{coefficients, delay, dot_display, fir_status, get_scale, response, run_block, run_one};
use crate::filter::{Filter, SdspPair};
use crate::{check, device, sys};

use std::error::Error;
use std::fmt;
use std::marker::PhantomData;

use num::{Complex, Zero};

/// decim.rs:5-10
pub struct DecimatingFIRFilter<Coef, In> {
    pub(crate) h: *mut sys::sdsp_fir,
    _t: PhantomData<(Coef, In)>,
}

impl<Coef: Copy + Zero, In: Copy> DecimatingFIRFilter<Coef, In>
where
    (Coef, In): SdspPair,
{
    /// DecimatingFIRFilter::new(&coefs, scale, decimation)  decim.rs:27-42
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

    /// decim.rs:60-62
    pub fn set_scale(&mut self, scale: Coef) {
        check(unsafe { sys::sdsp_fir_set_scale(self.h, &scale as *const Coef as _) })
    }

    /// decim.rs:78-80
    pub fn get_scale(&self) -> Coef {
        get_scale(self.h)
    }

    /// decim.rs:96-98
    pub fn get_decimation(&self) -> usize {
        unsafe { sys::sdsp_fir_decimation(self.h) }
    }

    /// push(sample): advance the phase and the window, no output  decim.rs:115-118
    pub fn push(&mut self, sample: In) {
        check(unsafe { sys::sdsp_decim_push(self.h, &sample as *const In as _) })
    }

    /// write(&samples): advance the phase by len and push each sample  decim.rs:136-139
    pub fn write(&mut self, samples: &[In]) {
        check(unsafe { sys::sdsp_decim_write(self.h, samples.as_ptr() as _, samples.len()) })
    }

    /// decim.rs:155-157
    pub fn len(&self) -> usize {
        unsafe { sys::sdsp_fir_len(self.h) }
    }

    /// decim.rs:171-173
    pub fn is_empty(&self) -> bool {
        self.len() == 0
    }

    /// the stored (reversed) taps  decim.rs:189-191
    pub fn coefficients(&self) -> Vec<Coef> {
        coefficients(self.h)
    }
}

impl<Coef, In> Clone for DecimatingFIRFilter<Coef, In> {
    /// derive(Clone) (decim.rs:5): taps, delay line and phase
    fn clone(&self) -> Self {
        let mut h = std::ptr::null_mut();
        check(unsafe { sys::sdsp_fir_clone(self.h, &mut h) });
        DecimatingFIRFilter { h, _t: PhantomData }
    }
}

impl<Coef, In> Drop for DecimatingFIRFilter<Coef, In> {
    fn drop(&mut self) {
        unsafe { sys::sdsp_fir_destroy(self.h) }
    }
}

impl<Coef, In> fmt::Debug for DecimatingFIRFilter<Coef, In> {
    fn fmt(&self, f: &mut fmt::Formatter) -> fmt::Result {
        write!(f, "DecimatingFIRFilter {{ len: {}, decimation: {} }}", unsafe { sys::sdsp_fir_len(self.h) },
               unsafe { sys::sdsp_fir_decimation(self.h) })
    }
}

impl<C: fmt::Display + Copy + Zero, T: fmt::Display + Copy> fmt::Display for DecimatingFIRFilter<C, T>
where
    (C, T): SdspPair,
{
    /// decim.rs:283-295
    fn fmt(&self, f: &mut fmt::Formatter) -> fmt::Result {
        let mut phase = 0usize;
        check(unsafe { sys::sdsp_fir_get_state(self.h, std::ptr::null_mut(), &mut phase) });
        write!(f, "FIR<{}> [Scale={:.5}] [Coefficients={}] [Decimation={}/{}]", std::any::type_name::<C>(),
               self.get_scale(), dot_display::<C>(self.len()), phase, self.get_decimation())
    }
}

impl<Coef, In: Copy + Zero> Filter<In, In> for DecimatingFIRFilter<Coef, In>
where
    (Coef, In): SdspPair,
{
    /// push, then emit when the phase wraps to 0  decim.rs:221-228
    fn execute(&mut self, sample: In) -> Vec<In> {
        run_one(self.h, &sample as *const In as _)
    }
    /// emits on inputs M-1, 2M-1, ... of the running phase  decim.rs:250-256
    fn execute_block(&mut self, samples: &[In]) -> Vec<In> {
        run_block(self.h, samples.as_ptr() as _, samples.len())
    }
    /// decim.rs:258-268
    fn frequency_response(&self, frequency: f64) -> Complex<f64> {
        response(self.h, frequency)
    }
    /// decim.rs:270-280
    fn group_delay(&self, frequency: f64) -> f64 {
        delay(self.h, frequency)
    }
}
