//! `solid::filter` (src/filter/mod.rs:1-22): the `Filter` trait, unchanged, and the
//! device-backed filter types.
pub mod auto_correlator;
pub mod fir;
pub mod firdes;
pub mod iir;
pub mod iirdes;

use num::Complex;

pub trait Filter<I, O> {
    /// Executes type `T` and returns the data type `O`
    fn execute(&mut self, sample: I) -> Vec<O>;
    /// Executes array of type `T` and returns an array of the data type `O`
    fn execute_block(&mut self, samples: &[I]) -> Vec<O>;
    /// Computes the Complex Frequency response of the filter
    fn frequency_response(&self, frequency: f64) -> Complex<f64>;
    /// Computes the Group Delay in samples
    fn group_delay(&self, frequency: f64) -> f64;
}

/// `(Coef, In)` -> the library's dtype code (include/sdsp.h sdsp_dtype).  Sealed:
/// exactly the six pairs the reference's `DotProduct<Coef>: Execute<In, Out>` impls cover.
pub trait SdspPair: private::Sealed {
    const DTYPE: std::os::raw::c_int;
}
/// The pairs of the IIR family: real coefficients (the reference's `Conj + Real` bounds,
/// src/filter/iir/mod.rs:244-262) over real or complex samples.
pub trait SdspIirPair: SdspPair {
    type Coef;
    /// one coefficient the library reports in f64, in the Coef type (exact for f32: the
    /// library divides f32 values in f64, and one rounding to f32 equals the f32 division)
    fn coef_from_f64(v: f64) -> Self::Coef;
}
mod private {
    pub trait Sealed {}
}
macro_rules! pair {
    ($c:ty, $i:ty, $d:ident) => {
        impl private::Sealed for ($c, $i) {}
        impl SdspPair for ($c, $i) {
            const DTYPE: std::os::raw::c_int = crate::sys::$d;
        }
    };
}
pair!(f32, f32, SDSP_RR32);
pair!(f32, Complex<f32>, SDSP_RC32);
pair!(Complex<f32>, Complex<f32>, SDSP_CC32);
pair!(f64, f64, SDSP_RR64);
pair!(f64, Complex<f64>, SDSP_RC64);
pair!(Complex<f64>, Complex<f64>, SDSP_CC64);

macro_rules! iir_pair {
    ($c:ty, $i:ty) => {
        impl SdspIirPair for ($c, $i) {
            type Coef = $c;
            fn coef_from_f64(v: f64) -> $c {
                v as $c
            }
        }
    };
}
iir_pair!(f32, f32);
iir_pair!(f32, Complex<f32>);
iir_pair!(f64, f64);
iir_pair!(f64, Complex<f64>);
