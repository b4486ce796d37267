//! `solid` (juliantos/solid-dsp) streaming hot path on MI355X: the public types of
//! `src/filter/*`, `src/dot_product/*`, `src/fft/*`, `src/nco/*` and
//! `src/auto_gain_control/*` with the same names and
//! signatures (tests/test_rust_shim_api.py checks every `pub fn` against the
//! reference), executed by libsdsp.so (include/sdsp.h).  Device-only extras are
//! in `sdsp`.
pub mod auto_gain_control;
pub mod dot_product;
pub mod fft;
pub mod filter;
pub mod nco;
pub mod sdsp;
pub mod sys;

use std::error::Error;
use std::ffi::CStr;
use std::fmt;

/// A device-side failure the reference cannot produce (no GPU, out of memory,
/// a failed launch): `sdsp_last_error()` text plus the status code.
#[derive(Debug)]
pub struct SdspError {
    pub code: i32,
    pub message: String,
}

impl fmt::Display for SdspError {
    fn fmt(&self, f: &mut fmt::Formatter) -> fmt::Result {
        write!(f, "sdsp error {}: {}", self.code, self.message)
    }
}

impl Error for SdspError {}

pub(crate) fn last_error(code: i32) -> SdspError {
    let msg = unsafe { CStr::from_ptr(sys::sdsp_last_error()) };
    SdspError { code, message: msg.to_string_lossy().into_owned() }
}

/// Panics with the library's message: the reference's execute paths are infallible,
/// so a device failure there is a panic, as an out-of-bounds index is in the reference.
pub(crate) fn check(rc: i32) {
    if rc != 0 {
        panic!("{}", last_error(rc));
    }
}

/// The device a new handle binds to (SDSP_DEVICE, default 0): the reference types take no device argument.
pub(crate) fn device() -> i32 {
    std::env::var("SDSP_DEVICE").ok().and_then(|v| v.parse().ok()).unwrap_or(0)
}
