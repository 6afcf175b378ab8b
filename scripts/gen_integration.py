"""Regenerates INTEGRATION.md §2 from the committed crate files: the binding a maintainer adds
(Cargo.toml, build.rs, src/ffi.rs) quoted whole, the restated API files (src/lib.rs, types.rs,
flow.rs) listed with their sha256.  tests/test_integration_doc.py checks both against the files."""
import hashlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CRATE = "rust/net-parser-rs-amd"
QUOTED = [("Cargo.toml", "toml"), ("build.rs", "rust"), ("src/ffi.rs", "rust")]
LISTED = [("src/lib.rs", "the reference's record API (`src/lib.rs`, `record.rs`, `file.rs`, `global_header.rs`) over the C-ABI; `CaptureParser`"),
          ("src/types.rs", "the reference's public types, field for field (errors, header, ids, `Flow`, the flow error tree)"),
          ("src/flow.rs", "`FlowExtraction`, `convert_records` and the batched/pipelined additions; device rows to `Flow` / errors"),
          ("src/layers.rs", "the per-layer header objects (`Ethernet` ... `Vxlan`, `Layer2/3/4`) over the host layer parsers, and the layer-2/3/4 `FlowExtraction` impls")]
MARK = "## 2. The crate, file by file"
TAIL = "## 3. "


def sha(f):
    return hashlib.sha256(open(os.path.join(REPO, CRATE, f), "rb").read()).hexdigest()


def blocks():
    out = ["Generated from the committed files by `scripts/gen_integration.py`.  The FFI binding is\n"
           "quoted whole; the API files are listed (read them in the crate).\n",
           "| file | lines | sha256 | what |", "|---|---|---|---|"]
    for f, what in LISTED:
        n = open(os.path.join(REPO, CRATE, f)).read().count("\n")
        out.append(f"| `{CRATE}/{f}` | {n} | `{sha(f)[:16]}` | {what} |")
    out.append("")
    for f, lang in QUOTED:
        body = open(os.path.join(REPO, CRATE, f)).read()
        out.append(f"### `{CRATE}/{f}`\n\n````{lang}\n{body}````\n")
    return "\n".join(out)


def main():
    p = os.path.join(REPO, "INTEGRATION.md")
    doc = open(p).read()
    head, rest = doc.split(MARK, 1)
    tail = rest[rest.index("\n" + TAIL) + 1:]
    open(p, "w").write(head + MARK + "\n\n" + blocks() + "\n" + tail)


if __name__ == "__main__":
    sys.exit(main())
