//! `solid::dot_product::execute` (src/dot_product/execute.rs:1-18), unchanged.
pub trait Execute<I, O> {
    /// Computes the dot product of the stored coefficients and `samples`
    fn execute(&self, samples: &[I]) -> O;
}
