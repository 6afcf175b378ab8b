"""INTEGRATION.md quotes the Rust crate's FFI binding byte for byte and lists its API files by hash, and every function
the crate's FFI module binds is declared in include/npr.h and exported by libnpr.so."""
import hashlib
import os
import re
import subprocess

from net_parser_rs import _abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CRATE = os.path.join(REPO, "rust", "net-parser-rs-amd")


def test_integration_md_quotes_the_committed_crate():
    doc = open(os.path.join(REPO, "INTEGRATION.md")).read()
    blocks = re.findall(r"### `rust/net-parser-rs-amd/([^`]+)`\n\n````[a-z]+\n(.*?)````\n", doc, re.S)
    assert {f for f, _ in blocks} == {"Cargo.toml", "build.rs", "src/ffi.rs"}
    for f, body in blocks:
        assert body == open(os.path.join(CRATE, f)).read(), f"INTEGRATION.md is stale for {f}: run scripts/gen_integration.py"
    listed = re.findall(r"\| `rust/net-parser-rs-amd/([^`]+)` \| (\d+) \| `([0-9a-f]{16})` \|", doc)
    assert {f for f, _, _ in listed} == {"src/lib.rs", "src/types.rs", "src/flow.rs", "src/layers.rs"}
    for f, _, h in listed:
        got = hashlib.sha256(open(os.path.join(CRATE, f), "rb").read()).hexdigest()[:16]
        assert got == h, f"INTEGRATION.md is stale for {f}: run scripts/gen_integration.py"


def test_ffi_rs_binds_only_declared_and_exported_symbols():
    ffi = open(os.path.join(CRATE, "src", "ffi.rs")).read()
    bound = set(re.findall(r"pub fn (npr_\w+)\(", ffi))
    header = open(os.path.join(REPO, "include", "npr.h")).read()
    declared = set(re.findall(r"\b(npr_[a-z0-9_]+)\s*\(", header))
    assert bound and bound <= declared
    out = subprocess.run(["nm", "-D", "--defined-only", _abi.LIB_PATH], capture_output=True, text=True).stdout
    assert bound <= set(re.findall(r" T (npr_\w+)", out))
    harness = open(os.path.join(REPO, "tests", "c_harness", "npr_harness.c")).read()
    called = set(re.findall(r"\b(npr_[a-z0-9_]+)\s*\(", harness))
    assert bound - {"npr_ctx_last_error", "npr_version"} <= called | {"npr_ctx_last_error"}, bound - called


def test_ffi_rs_struct_layouts_match_the_header():
    ffi = open(os.path.join(CRATE, "src", "ffi.rs")).read()
    # npr_flow field order and widths (32 B) and npr_record (24 B), as include/npr.h
    flow = re.search(r"pub struct npr_flow \{(.*?)\}", ffi, re.S).group(1)
    names = re.findall(r"pub (\w+):", flow)
    assert names == list(_abi.FLOW_DTYPE.names)
    rec = re.search(r"pub struct npr_record \{(.*?)\}", ffi, re.S).group(1)
    assert re.findall(r"pub (\w+):", rec) == list(_abi.RECORD_DTYPE.names)
