"""Regenerates INTEGRATION.md §2 from the committed crate files (tests/test_integration_doc.py
checks that the quoted blocks are byte-identical to the files)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CRATE = "rust/net-parser-rs-amd"
FILES = [("Cargo.toml", "toml"), ("build.rs", "rust"), ("src/ffi.rs", "rust"), ("src/lib.rs", "rust"),
         ("src/types.rs", "rust"), ("src/flow.rs", "rust")]
MARK = "## 2. The crate, file by file"
TAIL = "## 3. "


def blocks():
    out = []
    for f, lang in FILES:
        body = open(os.path.join(REPO, CRATE, f)).read()
        out.append(f"### `{CRATE}/{f}`\n\n````{lang}\n{body}````\n")
    return "\n".join(out)


def main():
    p = os.path.join(REPO, "INTEGRATION.md")
    doc = open(p).read()
    head, rest = doc.split(MARK, 1)
    intro = rest.split("\n### ", 1)[0] if "\n### " in rest else rest.split(TAIL, 1)[0]
    tail = TAIL + rest.split("\n" + TAIL, 1)[1] if ("\n" + TAIL) in rest else ""
    new = head + MARK + intro.rstrip("\n") + "\n\n" + blocks() + ("\n" + tail if tail else "")
    open(p, "w").write(new)


if __name__ == "__main__":
    sys.exit(main())
