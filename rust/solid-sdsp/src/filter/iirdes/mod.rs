//! `solid::filter::iirdes` (src/filter/iirdes/mod.rs): the PLL loop-filter designs
//! the reference's IIR doctests build their filters from (`pll`).
pub mod pll;

use std::error::Error;
use std::fmt;

/// iirdes/mod.rs:22-29 (private in the reference)
#[derive(Debug)]
pub(crate) enum IirdesErrorCode {
    Bandwidth,
    DampingFactor,
    Gain,
}

#[derive(Debug)]
pub(crate) struct IirdesError(pub(crate) IirdesErrorCode);

impl fmt::Display for IirdesError {
    /// iirdes/mod.rs:34-38
    fn fmt(&self, f: &mut fmt::Formatter) -> fmt::Result {
        write!(f, "Iirdes Error: {:?}", self.0)
    }
}

impl Error for IirdesError {}
