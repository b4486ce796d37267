//! `solid::filter::fir::pfb` (src/filter/fir/pfb.rs:3-91): PolyPhaseFilterBank.
use super::fir_status;
use crate::filter::SdspPair;
use crate::{check, device, sys};

use std::error::Error;
use std::fmt;
use std::marker::PhantomData;

use num::Zero;

pub struct PolyPhaseFilterBank<Coef, In> {
    pub(crate) h: *mut sys::sdsp_pfb,
    pub(crate) _t: PhantomData<(Coef, In)>,
}

impl<Coef: Copy + Zero, In: Copy + Zero> PolyPhaseFilterBank<Coef, In>
where
    (Coef, In): SdspPair,
{
    /// PolyPhaseFilterBank::new(&coefs, filters, scale)  pfb.rs:24-49 (K = len / filters, tail dropped)
    pub fn new(coefficients: &[Coef], filters: usize, scale: Coef) -> Result<Self, Box<dyn Error>> {
        let mut h = std::ptr::null_mut();
        let rc = unsafe {
            sys::sdsp_pfb_create(&mut h, <(Coef, In)>::DTYPE, coefficients.as_ptr() as _, coefficients.len(),
                                 filters, &scale as *const Coef as _, device())
        };
        if rc != 0 {
            return Err(fir_status(rc));
        }
        Ok(PolyPhaseFilterBank { h, _t: PhantomData })
    }

    pub fn set_scale(&mut self, scale: Coef) {
        check(unsafe { sys::sdsp_pfb_set_scale(self.h, &scale as *const Coef as _) })
    }

    pub fn get_scale(&self) -> Coef {
        let mut s = Coef::zero();
        check(unsafe { sys::sdsp_pfb_get_scale(self.h, &mut s as *mut Coef as _) });
        s
    }

    pub fn len(&self) -> usize {
        unsafe { sys::sdsp_pfb_len(self.h) }
    }

    pub fn is_empty(&self) -> bool {
        self.len() == 0
    }

    /// coefficents(): M branches of K stored (reversed) taps, pfb.rs:72-75
    pub fn coefficents(&self) -> Vec<Vec<Coef>> {
        let (m, k) = (self.len(), unsafe { sys::sdsp_pfb_subfilter_len(self.h) });
        let mut flat = vec![Coef::zero(); m * k];
        check(unsafe { sys::sdsp_pfb_coefficients(self.h, flat.as_mut_ptr() as _) });
        flat.chunks(k).map(|c| c.to_vec()).collect()
    }

    pub fn reset(&mut self) {
        check(unsafe { sys::sdsp_pfb_reset(self.h) })
    }

    pub fn push(&mut self, sample: In) {
        check(unsafe { sys::sdsp_pfb_push(self.h, &sample as *const In as _) })
    }

    /// execute(index): branch `index` over the current window (no scale, pfb.rs:85-90)
    pub fn execute<Out: Zero>(&mut self, index: usize) -> Out {
        assert!(index < self.len(), "index out of bounds");
        let mut o = Out::zero();
        check(unsafe { sys::sdsp_pfb_execute(self.h, index, &mut o as *mut Out as _) });
        o
    }
}

impl<Coef, In> Clone for PolyPhaseFilterBank<Coef, In> {
    fn clone(&self) -> Self {
        let mut h = std::ptr::null_mut();
        check(unsafe { sys::sdsp_pfb_clone(self.h, &mut h) });
        PolyPhaseFilterBank { h, _t: PhantomData }
    }
}

impl<Coef, In> fmt::Debug for PolyPhaseFilterBank<Coef, In> {
    fn fmt(&self, f: &mut fmt::Formatter) -> fmt::Result {
        write!(f, "PolyPhaseFilterBank {{ filters: {} }}", unsafe { sys::sdsp_pfb_len(self.h) })
    }
}

impl<Coef, In> Drop for PolyPhaseFilterBank<Coef, In> {
    fn drop(&mut self) {
        unsafe { sys::sdsp_pfb_destroy(self.h) }
    }
}
