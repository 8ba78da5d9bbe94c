// Links libhbtc.so built by `make lib` (hbbft_amd/libhbtc.so).  HBTC_LIB_DIR overrides the path.
fn main() {
    let dir = std::env::var("HBTC_LIB_DIR").unwrap_or_else(|_| "../../hbbft_amd".to_string());
    println!("cargo:rustc-link-search=native={}", dir);
    println!("cargo:rustc-link-lib=dylib=hbtc");
    println!("cargo:rerun-if-env-changed=HBTC_LIB_DIR");
}
