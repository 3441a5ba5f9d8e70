// Link against librtmi355x.so (make device -> build/librtmi355x.so of this repository) and, with
// the "rccl-gather" feature, librtgather.so (make gather).
// RT_MI355X_LIB_DIR overrides the default ../../build (relative to this crate); running the
// binary needs that directory and /opt/rocm/lib on LD_LIBRARY_PATH.
use std::env;
use std::path::PathBuf;

fn main() {
    println!("cargo:rerun-if-env-changed=RT_MI355X_LIB_DIR");
    let dir = match env::var("RT_MI355X_LIB_DIR") {
        Ok(d) => PathBuf::from(d),
        Err(_) => PathBuf::from(env::var("CARGO_MANIFEST_DIR").unwrap()).join("../../build"),
    };
    println!("cargo:rustc-link-search=native={}", dir.display());
    println!("cargo:rustc-link-search=native=/opt/rocm/lib");
    println!("cargo:rustc-link-lib=dylib=rtmi355x");
    if env::var_os("CARGO_FEATURE_RCCL_GATHER").is_some() {
        println!("cargo:rustc-link-lib=dylib=rtgather"); // and librccl.so through it
    }
}
