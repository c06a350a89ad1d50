//! Link the engine, and lift fastcdc 4.0.1's v2020 GEAR / MASKS out of the cargo registry
//! (the crate the reference already depends on, Cargo.lock:530-533): the engine refuses to
//! chunk with its placeholder table, and `available()` installs these arrays and runs the
//! reference fixture on the GPU before the first call.
use std::{env, fs, path::PathBuf};

fn main() {
    let dir = env::var("CHUNKER_AMD_LIB_DIR").expect("set CHUNKER_AMD_LIB_DIR to the directory of libchunker_amd.so");
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=chunker_amd");
    println!("cargo:rerun-if-env-changed=CHUNKER_AMD_LIB_DIR");

    let home = env::var("CARGO_HOME")
        .map(PathBuf::from)
        .unwrap_or_else(|_| PathBuf::from(env::var("HOME").unwrap()).join(".cargo"));
    let src = fs::read_dir(home.join("registry/src"))
        .expect("cargo registry")
        .filter_map(|e| e.ok())
        .map(|e| e.path().join("fastcdc-4.0.1/src/v2020/mod.rs"))
        .find(|p| p.exists())
        .expect("fastcdc 4.0.1 source in the cargo registry (cargo fetch)");
    let text = fs::read_to_string(&src).unwrap();
    let array = |name: &str, n: usize| -> String {
        let at = text.find(&format!("{name}:")).expect(name);
        let body = &text[at..];
        let (open, close) = (body.find("= [").unwrap() + 3, body.find("];").unwrap());
        let vals: Vec<&str> = body[open..close]
            .split(',')
            .map(|v| v.trim())
            .filter(|v| !v.is_empty() && !v.starts_with("//"))
            .collect();
        assert_eq!(vals.len(), n, "{name}");
        format!("pub const {name}: [u64; {n}] = [{}];\n", vals.join(", "))
    };
    let out = PathBuf::from(env::var("OUT_DIR").unwrap()).join("fastcdc_tables.rs");
    fs::write(out, array("GEAR", 256) + &array("MASKS", 26)).unwrap();
    println!("cargo:rerun-if-changed={}", src.display());
}
