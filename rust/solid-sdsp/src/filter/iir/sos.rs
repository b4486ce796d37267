//! `solid::filter::iir::sos` (src/filter/iir/sos.rs:1-231): `SecondOrderFilter`.
//! One biquad as a one-section cascade handle of the library (the same DF-II
//! recurrence, sos.rs:92-114, bit-identical in the reference order); the
//! coefficient accessors and the host f64 response keep the reference's swapped
//! naming (numerator = a[1..]/a0, denominator = b/a0, sos.rs:72-73).
use super::super::SdspIirPair;
use super::iir_status;
use crate::{check, last_error, sys};

use std::error::Error;
use std::fmt;
use std::marker::PhantomData;

use either::Either;
use num::{Complex, Zero};

/// sos.rs:18-21
#[derive(Debug)]
pub enum SecondOrderErrorCode {
    CoefficientsNotInRange,
}

/// sos.rs:23-32
#[derive(Debug)]
pub struct SecondOrderError(pub SecondOrderErrorCode);

impl fmt::Display for SecondOrderError {
    fn fmt(&self, f: &mut fmt::Formatter) -> fmt::Result {
        write!(f, "Second Order Error {:?}", self.0)
    }
}

impl Error for SecondOrderError {}

/// Out = T for every pair the library serves (the reference's `DotProduct<C>: Execute<T, Out>`).
pub trait SameSample<T> {}
impl<T> SameSample<T> for T {}

/// sos.rs:34-39
pub struct SecondOrderFilter<C, T> {
    h: *mut sys::sdsp_iir,
    _t: PhantomData<(C, T)>,
}

impl<C: Copy + Zero, T: Copy + Zero> SecondOrderFilter<C, T>
where
    (C, T): SdspIirPair<Coef = C>,
{
    /// SecondOrderFilter::new(&feed_forward, &feed_back): the first three of each,
    /// divided by fb[0]  sos.rs:55-75
    pub fn new(feed_forward: &[C], feed_back: &[C]) -> Result<Self, Box<dyn Error>> {
        if feed_forward.len() < 3 || feed_back.len() < 3 {
            return Err(Box::new(SecondOrderError(SecondOrderErrorCode::CoefficientsNotInRange)));
        }
        let mut h = std::ptr::null_mut();
        let rc = unsafe {
            sys::sdsp_iir_create(&mut h, <(C, T)>::DTYPE, feed_forward.as_ptr() as _, 3, feed_back.as_ptr() as _, 3,
                                 1, crate::device())
        };
        if rc != 0 {
            return Err(iir_status(rc));
        }
        Ok(SecondOrderFilter { h, _t: PhantomData })
    }

    /// execute(Left(x) | Right(y)): w = in - (a1 w1 + a2 w2), out = b0 w + b1 w1 + b2 w2  sos.rs:92-114
    pub fn execute<Out>(&mut self, input: Either<T, Out>) -> Out
    where
        Out: Copy + Zero + SameSample<T>,
    {
        let p: *const std::os::raw::c_void = match &input {
            Either::Left(x) => x as *const T as _,
            Either::Right(y) => y as *const Out as _,
        };
        let mut o = Out::zero();
        let mut got = 0usize;
        check(unsafe { sys::sdsp_iir_execute(self.h, p, &mut o as *mut Out as _, &mut got) });
        o
    }

    /// numerator_coefs(): [a1, a2] / a0  sos.rs:132-134
    pub fn numerator_coefs(&self) -> Vec<C> {
        let (num, _) = self.section();
        num.iter().map(|&v| <(C, T)>::coef_from_f64(v)).collect()
    }

    /// denominator_coefs(): [b0, b1, b2] / a0  sos.rs:152-154
    pub fn denominator_coefs(&self) -> Vec<C> {
        let (_, den) = self.section();
        den.iter().map(|&v| <(C, T)>::coef_from_f64(v)).collect()
    }

    fn section(&self) -> ([f64; 2], [f64; 3]) {
        let mut num = [0.0f64; 2];
        let mut den = [0.0f64; 3];
        check(unsafe { sys::sdsp_sos_section_coefs(self.h, 0, num.as_mut_ptr(), den.as_mut_ptr()) });
        (num, den)
    }

    /// sum numerator_coefs * e^{+j2 pi f i} / sum denominator_coefs * e^{+j2 pi f i}  sos.rs:171-206
    pub fn frequency_response(&self, frequency: f64) -> Complex<f64> {
        let (num, den) = self.section();
        let poly = |c: &[f64]| {
            let mut o: Complex<f64> = Complex::zero();
            for (i, &v) in c.iter().enumerate() {
                o += Complex::from_polar(1.0, frequency * 2.0 * std::f64::consts::PI * (i as f64)) * v;
            }
            o
        };
        poly(&num) / poly(&den)
    }

    /// iir_group_delay(numerator_coefs, denominator_coefs, f) + 2  sos.rs:208-230
    pub fn group_delay(&self, frequency: f64) -> f64 {
        let (num, den) = self.section();
        let mut d = 0.0f64;
        match unsafe { sys::sdsp_iir_group_delay_taps(num.as_ptr(), 2, den.as_ptr(), 3, frequency, &mut d) } {
            0 => d + 2.0,
            rc => {
                if cfg!(debug_assertions) {
                    eprintln!("{}", last_error(rc));
                }
                0.0
            }
        }
    }
}

impl<C: Copy + Zero, T: Copy + Zero> Clone for SecondOrderFilter<C, T>
where
    (C, T): SdspIirPair<Coef = C>,
{
    /// derive(Clone) (sos.rs:34): coefficients and the two-sample state
    fn clone(&self) -> Self {
        let mut h = std::ptr::null_mut();
        check(unsafe { sys::sdsp_iir_clone(self.h, &mut h) });
        SecondOrderFilter { h, _t: PhantomData }
    }
}

impl<C, T> fmt::Debug for SecondOrderFilter<C, T> {
    fn fmt(&self, f: &mut fmt::Formatter) -> fmt::Result {
        write!(f, "SecondOrderFilter<{}, {}>", std::any::type_name::<C>(), std::any::type_name::<T>())
    }
}

impl<C, T> Drop for SecondOrderFilter<C, T> {
    fn drop(&mut self) {
        unsafe { sys::sdsp_iir_destroy(self.h) }
    }
}
