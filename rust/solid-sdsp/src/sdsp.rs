//! Device-side extras that the reference types do not have, kept out of their
//! inherent API (which is exactly the reference's, tests/test_rust_shim_api.py):
//! the kernel choice, device-resident blocks on a caller's HIP stream, and the
//! reset/synchronise the C ABI offers.  `use solid::sdsp::*` to opt in.
use crate::filter::fir::decim::DecimatingFIRFilter;
use crate::filter::fir::FIRFilter;
use crate::filter::iir::IIRFilter;
use crate::{check, last_error, sys};

use std::error::Error;
use std::os::raw::c_void;

pub use crate::sys::{SDSP_ALGO_AUTO, SDSP_ALGO_EXACT, SDSP_ALGO_FFT, SDSP_ALGO_FMA};

/// The algorithm every FIR-type and IIR handle created afterwards starts on: SDSP_ALGO_EXACT
/// (the default, bit-identical to the reference), SDSP_ALGO_AUTO (long 32-bit blocks on the fast
/// kernels) or SDSP_ALGO_FMA.  The environment variable SDSP_DEFAULT_ALGO ("auto" / "exact" /
/// "fma") does the same for a whole process without a code change.
pub fn set_default_algorithm(algo: i32) -> Result<(), Box<dyn Error>> {
    match unsafe { sys::sdsp_set_default_algo(algo) } {
        0 => Ok(()),
        rc => Err(Box::new(last_error(rc))),
    }
}

/// The starting algorithm of new handles (set_default_algorithm / SDSP_DEFAULT_ALGO)
pub fn default_algorithm() -> i32 {
    unsafe { sys::sdsp_get_default_algo() }
}

/// FIRFilter / DecimatingFIRFilter on the device
pub trait FirDevice {
    /// SDSP_ALGO_EXACT (default, bit-identical), SDSP_ALGO_FMA, SDSP_ALGO_FFT (c32 FIR), SDSP_ALGO_AUTO
    fn set_algorithm(&mut self, algo: i32) -> Result<(), Box<dyn Error>>;
    /// per-sample calls and short host blocks on the host (true, default) or as device launches
    fn set_host_step(&mut self, on: bool);
    /// zero the delay line (and the phase)
    fn reset(&mut self);
    /// `n` device-resident samples -> `output_count(n)` device-resident outputs, asynchronous
    /// on `stream` (a hipStream_t; null = the handle's own).  Returns the output count.
    ///
    /// # Safety
    /// `d_in` / `d_out` must be device allocations of the handle's sample type and size.
    unsafe fn execute_block_device(&mut self, d_in: *const c_void, n: usize, d_out: *mut c_void,
                                   stream: *mut c_void) -> usize;
    fn synchronize(&mut self);
}

fn fir_handle_ops(h: *mut sys::sdsp_fir) -> FirOps {
    FirOps(h)
}
struct FirOps(*mut sys::sdsp_fir);
impl FirOps {
    fn set_algorithm(&self, algo: i32) -> Result<(), Box<dyn Error>> {
        match unsafe { sys::sdsp_fir_set_algo(self.0, algo) } {
            0 => Ok(()),
            rc => Err(Box::new(last_error(rc))),
        }
    }
    fn set_host_step(&self, on: bool) {
        check(unsafe { sys::sdsp_fir_set_tuning(self.0, sys::SDSP_TUNE_HOST_STEP, on as i32) })
    }
    fn reset(&self) {
        check(unsafe { sys::sdsp_fir_reset(self.0) })
    }
    unsafe fn block(&self, d_in: *const c_void, n: usize, d_out: *mut c_void, stream: *mut c_void) -> usize {
        let mut got = 0usize;
        check(sys::sdsp_fir_execute_block_device(self.0, d_in, n, d_out, &mut got, stream));
        got
    }
    fn synchronize(&self) {
        check(unsafe { sys::sdsp_fir_synchronize(self.0) })
    }
}

macro_rules! fir_device {
    ($t:ident) => {
        impl<Coef, In> FirDevice for $t<Coef, In> {
            fn set_algorithm(&mut self, algo: i32) -> Result<(), Box<dyn Error>> {
                fir_handle_ops(self.h).set_algorithm(algo)
            }
            fn set_host_step(&mut self, on: bool) {
                fir_handle_ops(self.h).set_host_step(on)
            }
            fn reset(&mut self) {
                fir_handle_ops(self.h).reset()
            }
            unsafe fn execute_block_device(&mut self, d_in: *const c_void, n: usize, d_out: *mut c_void,
                                           stream: *mut c_void) -> usize {
                fir_handle_ops(self.h).block(d_in, n, d_out, stream)
            }
            fn synchronize(&mut self) {
                fir_handle_ops(self.h).synchronize()
            }
        }
    };
}
fir_device!(FIRFilter);
fir_device!(DecimatingFIRFilter);

/// IIRFilter on the device
pub trait IirDevice {
    /// SDSP_ALGO_EXACT (default: the reference-order recurrence), SDSP_ALGO_FMA / SDSP_ALGO_AUTO
    /// (the block-parallel wave scan, ≤1e-5 f32 / ≤1e-12 f64 of the reference)
    fn set_algorithm(&mut self, algo: i32) -> Result<(), Box<dyn Error>>;
    fn reset(&mut self);
}

impl<Coef, In> IirDevice for IIRFilter<Coef, In> {
    fn set_algorithm(&mut self, algo: i32) -> Result<(), Box<dyn Error>> {
        match unsafe { sys::sdsp_iir_set_algo(self.core.h, algo) } {
            0 => Ok(()),
            rc => Err(Box::new(last_error(rc))),
        }
    }
    fn reset(&mut self) {
        check(unsafe { sys::sdsp_iir_reset(self.core.h) })
    }
}
