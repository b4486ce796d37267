//! `solid::dot_product` (src/dot_product/mod.rs:31-171, execute.rs:17): DotProduct
//! with the reference's FORWARD/REVERSE copy and sequential sum, executed by
//! sdsp_dot_execute (bit-identical).
use crate::filter::SdspPair;
use crate::{check, sys};

use num::Zero;

pub enum Direction {
    FORWARD,
    REVERSE,
}

pub mod execute {
    pub trait Execute<I, O> {
        fn execute(&self, samples: &[I]) -> O;
    }
}

pub struct DotProduct<T> {
    coefs: Vec<T>, // as given; the direction is applied by the library
    direction: i32,
}

impl<T: Copy> DotProduct<T> {
    pub fn new(coefficients: &[T], direction: Direction) -> Self {
        DotProduct {
            coefs: coefficients.to_vec(),
            direction: match direction {
                Direction::FORWARD => 0,
                Direction::REVERSE => 1,
            },
        }
    }
    /// stored order (REVERSE reverses the copy, mod.rs:73-81)
    pub fn coefficents(&self) -> Vec<T> {
        let mut v = self.coefs.clone();
        if self.direction == 1 {
            v.reverse();
        }
        v
    }
    pub fn len(&self) -> usize {
        self.coefs.len()
    }
    pub fn is_empty(&self) -> bool {
        self.coefs.is_empty()
    }
}

impl<T: Copy, I: Copy + Zero> execute::Execute<I, I> for DotProduct<T>
where
    (T, I): SdspPair,
{
    fn execute(&self, samples: &[I]) -> I {
        let mut o = I::zero();
        check(unsafe {
            sys::sdsp_dot_execute(<(T, I)>::DTYPE, self.coefs.as_ptr() as _, self.coefs.len(), self.direction,
                                  samples.as_ptr() as _, samples.len(), &mut o as *mut I as _)
        });
        o
    }
}
