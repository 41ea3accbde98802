// Links the engine: libnwv.so is built by `make lib` in the narwhal_amd checkout
// (hipcc --offload-arch=gfx950; include/nwv.h, include/nwv_types.h, include/nwv_service.h).
fn main() {
    let dir = std::env::var("NWV_LIB_DIR")
        .expect("set NWV_LIB_DIR to the directory holding libnwv.so (narwhal_amd/lib)");
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=nwv");
    // the engine is loaded next to the binary's own libraries at run time
    println!("cargo:rustc-link-arg=-Wl,-rpath,{dir}");
    println!("cargo:rerun-if-env-changed=NWV_LIB_DIR");
}
