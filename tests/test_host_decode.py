"""The device's general decoder (csrc/npr_decode.hpp decode<>, the source the kernels compile) built
for the host and checked against the oracle on the CPU: status, flow fields and error payload
(npr_flow_details) of every record of several corpora and of every truncation of each payload."""
import os
import subprocess

import pytest

from net_parser_rs import synth

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIR = os.path.join(REPO, "tests", "host_decode")


def corpora(tmp_path):
    caps = {
        "quirk.pcap": synth.quirk_corpus(4_000, seed=91),
        "quirk_be.pcap": synth.quirk_corpus(2_000, seed=92, big=True),
        "adversarial.pcap": synth.quirk_corpus(1_500, seed=93, fake_every=3, zero_every=7, jumbo_every=150),
        "vxlan.pcap": synth.vxlan_corpus(1_500),
        "flow_mix.pcap": synth.flow_mix(2_000),
        "c3.pcap": synth.variable_mix(1_000),
    }
    paths = []
    for name, blob in caps.items():
        p = tmp_path / name
        p.write_bytes(blob)
        paths.append(str(p))
    return paths


@pytest.mark.parametrize("exe", ["decode_check", "decode_check_san"])
def test_device_decoder_on_the_host_matches_oracle(tmp_path, exe):
    """decode_check_san: the same run under ASan + UBSan (any report aborts it: -fno-sanitize-recover),
    VERDICT r05 item 2's sanitizer pass over the quirk corpora."""
    subprocess.run(["make", "-s", "-C", DIR], check=True)
    r = subprocess.run([os.path.join(DIR, "build", exe)] + corpora(tmp_path), capture_output=True, text=True,
                       timeout=600, env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0"))
    assert r.returncode == 0 and " 0 mismatches" in r.stdout, r.stdout + r.stderr
