// Links the in-tree engine library (make -C pa_amd) and the HIP runtime.
// STRAWBOAT_GPU_LIB_DIR overrides the directory of libstrawboat_gpu.so;
// ROCM_PATH that of libamdhip64.so (default /opt/rocm).
use std::env;
use std::path::PathBuf;

fn main() {
    let manifest = PathBuf::from(env::var("CARGO_MANIFEST_DIR").unwrap());
    let lib_dir = env::var("STRAWBOAT_GPU_LIB_DIR")
        .map(PathBuf::from)
        .unwrap_or_else(|_| manifest.join("../../pa_amd"));
    let rocm = env::var("ROCM_PATH").unwrap_or_else(|_| "/opt/rocm".to_string());
    println!("cargo:rustc-link-search=native={}", lib_dir.display());
    println!("cargo:rustc-link-search=native={}/lib", rocm);
    println!("cargo:rustc-link-lib=dylib=strawboat_gpu");
    println!("cargo:rustc-link-lib=dylib=amdhip64");
    println!("cargo:rerun-if-env-changed=STRAWBOAT_GPU_LIB_DIR");
    println!("cargo:rerun-if-env-changed=ROCM_PATH");
    println!("cargo:rerun-if-changed={}", manifest.join("../../include/strawboat_gpu.h").display());
}
