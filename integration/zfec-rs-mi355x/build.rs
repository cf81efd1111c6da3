// Link against the in-tree HIP library. STORB_RS_LIB_DIR overrides the
// default location (<repo>/storb_amd/lib, built by `make -C storb_amd`).
fn main() {
    let dir = std::env::var("STORB_RS_LIB_DIR").unwrap_or_else(|_| {
        let here = std::path::PathBuf::from(std::env::var("CARGO_MANIFEST_DIR").unwrap());
        here.join("../../storb_amd/lib").to_string_lossy().into_owned()
    });
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=storb_rs");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{dir}");
    println!("cargo:rerun-if-env-changed=STORB_RS_LIB_DIR");
}
