"""The plain-C caller (tests/c_harness/npr_harness.c) of every entry point the Rust crate binds:
built against include/npr.h + libnpr.so here; run on the GPU (`-m gpu`) over several captures,
each result checked against the oracle inside the harness."""
import os
import subprocess

import pytest

from net_parser_rs import synth

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS_DIR = os.path.join(REPO, "tests", "c_harness")
HARNESS = os.path.join(HARNESS_DIR, "build", "npr_harness")


def build():
    subprocess.run(["make", "-s", "-C", HARNESS_DIR], check=True)
    return HARNESS


def test_harness_builds_and_refuses_without_gpu():
    import torch
    exe = build()
    if torch.cuda.is_available():
        pytest.skip("GPU present: the gpu test runs it")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "no HIP device" in r.stderr


def test_harness_layer_traits_on_the_host(tmp_path):
    """The layer-2/3/4 FlowExtraction chain composed from libnpr's host layer parsers (what the Rust
    crate's trait impls do, rust/net-parser-rs-amd/src/layers.rs) gives the oracle's status leaf,
    error payload and flow on every record (the harness's host-only checks; no device needed)."""
    import torch
    exe = build()
    if torch.cuda.is_available():
        pytest.skip("GPU present: the gpu test runs the same checks")
    paths = []
    for name, blob in {"quirk": synth.quirk_corpus(5_000, seed=91), "quirk_be": synth.quirk_corpus(3_000, seed=92, big=True),
                       "adversarial": synth.quirk_corpus(2_000, seed=93, fake_every=3, zero_every=7, jumbo_every=150,
                                                         tail="truncated_payload"),
                       "flow_mix": synth.flow_mix(3_000)}.items():
        p = tmp_path / f"{name}.pcap"
        p.write_bytes(blob)
        paths.append(str(p))
    r = subprocess.run([exe] + paths, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "host-only checks: 0 failures" in r.stderr, r.stdout + r.stderr


@pytest.mark.gpu
def test_harness_on_device(tmp_path):
    exe = build()
    caps = {
        "c2.pcap": synth.fixed64(50_000),
        "c3.pcap": synth.variable_mix(5_000),
        "quirk.pcap": synth.quirk_corpus(5_000, seed=91),
        "quirk_be.pcap": synth.quirk_corpus(3_000, seed=92, big=True),
        "adversarial.pcap": synth.quirk_corpus(2_000, seed=93, fake_every=3, zero_every=7, jumbo_every=150,
                                               tail="truncated_payload"),
        "vxlan.pcap": synth.vxlan_corpus(4_000),
        "short.pcap": synth.global_header()[:20],
    }
    paths = []
    for name, blob in caps.items():
        p = tmp_path / name
        p.write_bytes(blob)
        paths.append(str(p))
    r = subprocess.run([exe] + paths, capture_output=True, text=True, timeout=300)
    print(r.stdout)
    print(r.stderr)
    assert r.returncode == 0 and "OK (0 failures)" in r.stdout
