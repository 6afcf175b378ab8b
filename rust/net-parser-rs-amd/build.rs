// Links libnpr.so (net-parser-rs_amd/lib, built by `make -C net-parser-rs_amd` or
// `python -c 'import __graft_entry__ as g; g.build()'`).  NPR_LIB_DIR overrides the location.
use std::env;
use std::path::PathBuf;

fn main() {
    let dir = env::var("NPR_LIB_DIR").map(PathBuf::from).unwrap_or_else(|_| {
        PathBuf::from(env::var("CARGO_MANIFEST_DIR").unwrap()).join("../../net-parser-rs_amd/lib")
    });
    println!("cargo:rustc-link-search=native={}", dir.display());
    println!("cargo:rustc-link-lib=dylib=npr");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", dir.display());
    println!("cargo:rerun-if-env-changed=NPR_LIB_DIR");
}
