"""The Rust drop-in crate (rust/narwhal-gpu-crypto) cannot be compiled here (no cargo), so its
FFI layer is checked mechanically against the C headers: every function declared in include/*.h
appears in src/ffi.rs with the same parameters (count, order and the Rust type each C type maps
to, constness included) and return type; every #[repr(C)] struct has the C struct's fields in the
same order with matching types; every NWV_* constant has the header's value.  The reference
binding this replaces: crypto/src/lib.rs:29-33 (scheme aliases), crypto/src/bls12377/mod.rs
:93-577 (a fastcrypto trait module)."""
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CRATE = os.path.join(ROOT, "rust", "narwhal-gpu-crypto")

STRUCTS = {"nwv_ctx": "NwvCtx", "nwv_staged": "NwvStaged", "nwv_service": "NwvService",
           "nwv_committee": "NwvCommittee", "nwv_header": "NwvHeader", "nwv_vote": "NwvVote",
           "nwv_certificate": "NwvCertificate", "nwv_bls_committee": "NwvBlsCommittee",
           "nwv_bls_header": "NwvBlsHeader", "nwv_bls_vote": "NwvBlsVote",
           "nwv_bls_certificate": "NwvBlsCertificate"}
SCALARS = {"size_t": "usize", "int": "c_int", "uint32_t": "u32", "uint64_t": "u64", "int64_t": "i64",
           "int32_t": "i32", "uint8_t": "u8", "char": "c_char", "double": "f64", "float": "f32", "void": "c_void",
           "nwv_done_fn": "NwvDoneFn"}


def _strip_c(text):
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return re.sub(r"//[^\n]*", "", text)


def c_headers():
    return _strip_c("".join(open(f).read() for f in sorted(glob.glob(os.path.join(ROOT, "include", "*.h")))))


def c_to_rust(decl):
    """'const uint8_t* const* sigs' -> ('sigs', '*const *const u8'); arrays decay to pointers"""
    decl = " ".join(decl.split())
    m = re.fullmatch(r"(const )?(\w+) ?((?:\* ?(?:const ?)?)*)(\w+)?(\[\d+\])?", decl)
    assert m, decl
    lead_const, base, stars, name, arr = m.groups()
    ptrs = re.findall(r"\*( ?const)?", stars)  # the const written after each '*'
    quals = []
    n = len(ptrs) + (1 if arr else 0)
    for i in range(n):
        if i == 0:
            quals.append("const" if lead_const else "mut")
        else:
            quals.append("const" if ptrs[i - 1].strip() == "const" else "mut")
    t = STRUCTS.get(base) or SCALARS[base]
    for q in quals:
        t = f"*{q} {t}"
    return name, t


def c_prototypes():
    out = {}
    for ret, name, params in re.findall(
            r"(?:^|\n)\s*((?:const\s+)?\w+\s*\**\s*)\b(nwv_\w+)\s*\(([^;{]*?)\)\s*;", c_headers()):
        ps = [] if params.strip() in ("", "void") else [p.strip() for p in params.split(",")]
        r = None if ret.strip() == "void" else c_to_rust(ret.strip() + " _r")[1]
        out[name] = ([c_to_rust(p) for p in ps], r)
    return out


def rust_externs():
    src = open(os.path.join(CRATE, "src", "ffi.rs")).read()
    block = src[src.index('extern "C" {'):]
    out = {}
    for name, params, ret in re.findall(r"pub fn (nwv_\w+)\(([^)]*)\)\s*(?:->\s*([^;]+))?;", block):
        ps = []
        for p in [x.strip() for x in params.split(",") if x.strip()]:
            a, t = p.split(":", 1)
            ps.append((a.strip(), " ".join(t.split())))
        out[name] = (ps, " ".join(ret.split()) if ret else None)
    return out


def test_every_c_function_is_bound_with_the_same_signature():
    c = c_prototypes()
    r = rust_externs()
    assert len(c) >= 50
    assert set(c) == set(r), (sorted(set(c) - set(r)), sorted(set(r) - set(c)))
    for name, (cps, cret) in c.items():
        rps, rret = r[name]
        assert [t for _, t in rps] == [t for _, t in cps], name
        assert [a for a, _ in rps] == [a for a, _ in cps], name
        assert rret == cret, name


def test_repr_c_structs_match_the_c_layout():
    hdr = c_headers()
    src = open(os.path.join(CRATE, "src", "ffi.rs")).read()
    for cname in ("nwv_committee", "nwv_header", "nwv_vote", "nwv_certificate", "nwv_bls_committee",
                  "nwv_bls_header", "nwv_bls_vote", "nwv_bls_certificate"):
        body = re.search(r"typedef struct \{([^}]*)\}\s*" + cname + r"\s*;", hdr).group(1)
        cfields = [c_to_rust(f.strip()) for f in body.split(";") if f.strip()]
        rbody = re.search(r"pub struct " + STRUCTS[cname] + r" \{([^}]*)\}", src).group(1)
        rfields = []
        for line in rbody.split(","):
            line = line.strip()
            if line.startswith("pub "):
                a, t = line[4:].split(":", 1)
                rfields.append((a.strip(), " ".join(t.split())))
        assert rfields == cfields, cname
        assert re.search(r"#\[repr\(C\)\]\s*#\[derive\(Clone, Copy\)\]\s*pub struct " + STRUCTS[cname], src)


def test_constants_match_the_headers():
    hdr = c_headers()
    src = open(os.path.join(CRATE, "src", "ffi.rs")).read()
    defines = {k: int(v) for k, v in re.findall(r"#define (NWV_[A-Z_]+) \(?(-?\d+)\)?", hdr)}
    consts = {k: int(v) for k, v in re.findall(r"pub const (NWV_[A-Z_]+): \w+ = (-?\d+);", src)}
    assert len(consts) >= 17
    for k, v in consts.items():
        assert defines[k] == v, k


def test_crate_links_the_engine_and_covers_the_trait_surface():
    """build.rs links libnwv; lib.rs implements the fastcrypto traits the reference's scheme
    modules implement (crypto/src/bls12377/mod.rs:244-291 Verifier / VerifyingKey, :485-577
    AggregateAuthenticator) by calling the engine, and maps errors like the reference"""
    build = open(os.path.join(CRATE, "build.rs")).read()
    assert "rustc-link-lib=dylib=nwv" in build and "NWV_LIB_DIR" in build
    lib = open(os.path.join(CRATE, "src", "lib.rs")).read()
    for needle in ("impl Verifier<GpuEd25519Signature> for GpuEd25519PublicKey",
                   "impl VerifyingKey for GpuEd25519PublicKey", "fn verify_batch_empty_fail",
                   "impl AggregateAuthenticator for GpuEd25519AggregateSignature", "fn batch_verify",
                   "nwv_ed25519_pubkey_verify", "nwv_ed25519_verify_batch_empty_fail",
                   "nwv_ed25519_aggregate_verify", "nwv_ed25519_aggregate_batch_verify",
                   "nwv_blake2b256_many", "nwv_batch_digest_serialized", "nwv_verify_mixed_many",
                   "nwv_validate_certificates", "nwv_service_verify_certificate",
                   "Critical Error! This behavious can signal something dangerous"):
        assert needle in lib, needle
    bls = open(os.path.join(CRATE, "src", "bls.rs")).read()  # the reference's default scheme
    for needle in ("impl Verifier<GpuBls12381Signature> for GpuBls12381PublicKey",
                   "impl VerifyingKey for GpuBls12381PublicKey",
                   "impl AggregateAuthenticator for GpuBls12381AggregateSignature", "fn batch_verify",
                   "nwv_bls_verify(", "nwv_bls_verify_batch_empty_fail(", "nwv_bls_aggregate_verify(",
                   "nwv_bls_aggregate_batch_verify(", "nwv_bls_verify_many(",
                   "Critical Error! This behavious can signal something dangerous"):
        assert needle in bls, needle
    drain = open(os.path.join(CRATE, "src", "core_drain.rs")).read()
    for needle in ("pub async fn drain", "try_recv", "timeout_at", "nwv_verify_mixed_many", "pub fn verify_items"):
        assert needle in drain, needle
    cargo = open(os.path.join(CRATE, "Cargo.toml")).read()
    assert 'fastcrypto = { version = "0.1.2"' in cargo  # the reference's pin (Cargo.lock:1534)
