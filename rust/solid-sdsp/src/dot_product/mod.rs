//! `solid::dot_product` (src/dot_product/mod.rs:25-196): `DotProduct<T>` with the
//! reference's FORWARD / REVERSE copy (mod.rs:57-87) and sequential sum
//! (mod.rs:153-171), executed by `sdsp_dot_execute` (bit-identical, reference order).
pub mod execute;

use self::execute::Execute;
use crate::filter::SdspPair;
use crate::{check, sys};

use std::fmt;

use num::Zero;

/// mod.rs:31-34
pub enum Direction {
    FORWARD,
    REVERSE,
}

/// The taps are held in the stored order (REVERSE reversed at construction, as
/// `DotProduct::new` copies them, mod.rs:63-85); the library sums in that order.
#[derive(Debug)]
pub struct DotProduct<T> {
    stored: Vec<T>,
}

impl<T: Copy> DotProduct<T> {
    /// DotProduct::new(&coefficients, direction)  mod.rs:57-87
    pub fn new(coefficients: &[T], direction: Direction) -> Self {
        let mut stored = coefficients.to_vec();
        if let Direction::REVERSE = direction {
            stored.reverse();
        }
        DotProduct { stored }
    }

    /// coefficents() (sic): the stored order  mod.rs:102-109
    pub fn coefficents(&self) -> Vec<T> {
        self.stored.clone()
    }

    /// mod.rs:124-127
    pub fn len(&self) -> usize {
        self.stored.len()
    }

    /// mod.rs:141-144
    pub fn is_empty(&self) -> bool {
        self.stored.is_empty()
    }
}

impl<T: fmt::Display> fmt::Display for DotProduct<T> {
    /// mod.rs:146-151
    fn fmt(&self, f: &mut fmt::Formatter) -> fmt::Result {
        write!(f, "DotProduct<{}> [Size={}]", std::any::type_name::<T>(), self.stored.len())
    }
}

impl<T: Clone> Clone for DotProduct<T> {
    fn clone(&self) -> Self {
        DotProduct { stored: self.stored.clone() }
    }
}

/// `Execute<I, O>` for the six (T, I) pairs the library serves; O = I (mod.rs:153-171:
/// sum of the first min(n, len) products, from zero, in order).
impl<T: Copy, I: Copy + Zero> Execute<I, I> for DotProduct<T>
where
    (T, I): SdspPair,
{
    fn execute(&self, samples: &[I]) -> I {
        let mut o = I::zero();
        // FORWARD over the stored order: the library applies no further reversal
        check(unsafe {
            sys::sdsp_dot_execute(<(T, I)>::DTYPE, self.stored.as_ptr() as _, self.stored.len(), 0,
                                  samples.as_ptr() as _, samples.len(), &mut o as *mut I as _)
        });
        o
    }
}
