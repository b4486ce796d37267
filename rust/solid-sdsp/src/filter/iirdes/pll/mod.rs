//! `solid::filter::iirdes::pll` (src/filter/iirdes/pll/mod.rs:24-99): active lag and
//! active proportional-integral loop filters, (feed_forward, feed_back) of 3 each,
//! computed by libsdsp's host code (design.cpp; equal to the reference's doctest values).
use super::{IirdesError, IirdesErrorCode};
use crate::sys;

use std::error::Error;

fn status(rc: i32) -> Result<(), Box<dyn Error>> {
    match rc {
        0 => Ok(()),
        1 => Err(Box::new(IirdesError(IirdesErrorCode::Bandwidth))),
        2 => Err(Box::new(IirdesError(IirdesErrorCode::DampingFactor))),
        _ => Err(Box::new(IirdesError(IirdesErrorCode::Gain))),
    }
}

/// pll/mod.rs:24-52
pub fn active_lag(
    bandwidth: f64,
    damping_factor: f64,
    loop_gain: f64,
) -> Result<(Vec<f64>, Vec<f64>), Box<dyn Error>> {
    let (mut b, mut a) = (vec![0.0f64; 3], vec![0.0f64; 3]);
    status(unsafe { sys::sdsp_active_lag(bandwidth, damping_factor, loop_gain, b.as_mut_ptr(), a.as_mut_ptr()) })?;
    Ok((b, a))
}

/// pll/mod.rs:71-99
pub fn active_proportional_integral(
    bandwidth: f64,
    damping_factor: f64,
    loop_gain: f64,
) -> Result<(Vec<f64>, Vec<f64>), Box<dyn Error>> {
    let (mut b, mut a) = (vec![0.0f64; 3], vec![0.0f64; 3]);
    status(unsafe {
        sys::sdsp_active_proportional_integral(bandwidth, damping_factor, loop_gain, b.as_mut_ptr(), a.as_mut_ptr())
    })?;
    Ok((b, a))
}
