// Links libsdsp.so built by `make -C solid_dsp_amd/csrc` (hipcc --offload-arch=gfx950).
// SDSP_LIB_DIR overrides the default in-tree location (../../solid_dsp_amd/_build).
fn main() {
    let dir = std::env::var("SDSP_LIB_DIR").unwrap_or_else(|_| {
        let here = std::env::var("CARGO_MANIFEST_DIR").unwrap();
        format!("{}/../../solid_dsp_amd/_build", here)
    });
    println!("cargo:rustc-link-search=native={}", dir);
    println!("cargo:rustc-link-lib=dylib=sdsp");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", dir);
    println!("cargo:rerun-if-env-changed=SDSP_LIB_DIR");
}
