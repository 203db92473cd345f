//! Builds libcess_bls.so for gfx950 with hipcc (cess_amd/csrc/Makefile:
//! `hipcc --offload-arch=gfx950` for the HIP kernels and the host runtime,
//! linked against /opt/rocm's HIP runtime and RCCL) and links it.
//!
//! NOT COMPILED in this repository's image (no cargo); see Cargo.toml.
//! Environment:
//!   CESS_BLS_LIB_DIR  use a prebuilt library directory instead of running make
//!   HIPCC             hipcc to use (default /opt/rocm/bin/hipcc)
//!   CESS_BLS_JOBS     make -j (default 16)
use std::env;
use std::path::PathBuf;
use std::process::Command;

fn main() {
    let manifest = PathBuf::from(env::var("CARGO_MANIFEST_DIR").unwrap());
    let repo = manifest.join("..").join("..");
    let csrc = repo.join("cess_amd").join("csrc");
    println!("cargo:rerun-if-env-changed=CESS_BLS_LIB_DIR");
    println!("cargo:rerun-if-env-changed=HIPCC");
    let libdir = match env::var("CESS_BLS_LIB_DIR") {
        Ok(d) => PathBuf::from(d),
        Err(_) => {
            for entry in std::fs::read_dir(&csrc).expect("cess_amd/csrc") {
                let p = entry.unwrap().path();
                if let Some(ext) = p.extension() {
                    if ext == "hip" || ext == "cpp" || ext == "hpp" {
                        println!("cargo:rerun-if-changed={}", p.display());
                    }
                }
            }
            println!("cargo:rerun-if-changed={}", csrc.join("bls").display());
            println!("cargo:rerun-if-changed={}", repo.join("include").join("cess_bls.h").display());
            let jobs = env::var("CESS_BLS_JOBS").unwrap_or_else(|_| "16".into());
            let mut make = Command::new("make");
            make.arg("-C").arg(&csrc).arg(format!("-j{jobs}")).arg("ARCH=gfx950");
            if let Ok(h) = env::var("HIPCC") {
                make.arg(format!("HIPCC={h}"));
            }
            let st = make.status().expect("make (hipcc) failed to start");
            assert!(st.success(), "building libcess_bls.so with hipcc failed");
            repo.join("cess_amd").join("lib")
        }
    };
    println!("cargo:rustc-link-search=native={}", libdir.display());
    println!("cargo:rustc-link-lib=dylib=cess_bls");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", libdir.display());
    println!("cargo:include={}", repo.join("include").display());
}
