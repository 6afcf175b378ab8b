"""Seeded fuzzing of the HIP path against the oracle, bit-exact, through every launch shape.

Each case draws (from its seed) a base capture -- one of the synthetic corpora with random options,
or a splice of several -- then mutates it: random bytes overwritten, record headers' lengths set to
random / huge / zero values, header timestamps scrambled, payload spans replaced by fake header
chains, the tail cut at a random byte.  Every mutated capture is what the reference parses serially
(src/record.rs:30-49, src/flow/mod.rs:101-123): the chain may END early, records may turn into
errors, speculation may be fooled.  The case then runs one launch shape drawn from the seed (full
record table, resident single pass with default / few waves, the two-pass kernels, the sparse walk
at random lane spans and slot caps, chained links at a random chunk size) and compares everything
with the oracle via test_gpu_parity's checkers.  Parity is pinned by the oracle, which the
reference's own vectors pin (tests/test_oracle_kat.py); the mutations themselves have no reference
vectors ("parity unpinned" beyond the oracle).
"""
import struct

import numpy as np
import pytest

import _oracle
from net_parser_rs import synth
from test_gpu_parity import check_chunked, check_parity, sparse_forced

pytestmark = pytest.mark.gpu

N_CASES = 256


def base_capture(rng):
    kind = int(rng.integers(0, 6))
    seed = int(rng.integers(1, 1 << 30))
    n = int(rng.integers(200, 4000))
    if kind == 0:
        return synth.fixed64(n, seed=seed)
    if kind == 1:
        return synth.variable_mix(n, seed=seed)
    if kind == 2:
        return synth.quirk_corpus(n, seed=seed, big=bool(rng.integers(0, 2)),
                                  jumbo_every=int(rng.choice([0, 0, 50, 300])),
                                  fake_every=int(rng.choice([0, 0, 2, 5, 11])),
                                  zero_every=int(rng.choice([0, 0, 3, 9])),
                                  tail=rng.choice([None, None, "truncated_header", "truncated_payload", "huge_incl"]))
    if kind == 3:
        return synth.flow_mix(n, n_flows=int(rng.integers(1, 300)), seed=seed)
    if kind == 4:
        return synth.vxlan_corpus(min(n, 1500), seed=seed)
    # a splice: the record bodies of several corpora behind one (little-endian) header
    parts = [synth.global_header()]
    for _ in range(int(rng.integers(2, 5))):
        s2 = int(rng.integers(1, 1 << 30))
        m = int(rng.integers(50, 800))
        body = [synth.fixed64(m, seed=s2, with_header=False), synth.variable_mix(m, seed=s2, with_header=False),
                synth.quirk_corpus(m, seed=s2, with_header=False, fake_every=3)][int(rng.integers(0, 3))]
        parts.append(body)
    return b"".join(parts)


def record_offsets(blob):
    rc, hdr, recs, cons = _oracle.capture_file_parse(blob)
    return recs["offset"].astype(np.int64), hdr


def mutate(rng, blob):
    b = bytearray(blob)
    offs, hdr = record_offsets(bytes(b))
    big = hdr.endianness == 1
    e = ">" if big else "<"
    for _ in range(int(rng.integers(1, 6))):
        op = int(rng.integers(0, 6))
        if op == 0 and len(b) > 24:  # random bytes anywhere past the global header
            for _ in range(int(rng.integers(1, 40))):
                b[int(rng.integers(24, len(b)))] = int(rng.integers(0, 256))
        elif op == 1 and len(offs):  # a record's incl_len: random, huge, zero or off by a little
            o = int(offs[int(rng.integers(0, len(offs)))])
            (incl,) = struct.unpack_from(e + "I", b, o + 8)
            v = int(rng.choice([0, 1, 13, 0xFFFFFFFF, 1 << 18, (1 << 18) + 1, incl + 1, max(incl - 1, 0),
                                int(rng.integers(0, 4096))]))
            struct.pack_into(e + "I", b, o + 8, v & 0xFFFFFFFF)
        elif op == 2 and len(offs):  # timestamps scrambled (speculation's plausibility window)
            o = int(offs[int(rng.integers(0, len(offs)))])
            struct.pack_into(e + "II", b, o, int(rng.integers(0, 1 << 32)), int(rng.integers(0, 1 << 32)))
        elif op == 3 and len(offs) > 1:  # a payload span rewritten as a chain of fake headers
            k = int(rng.integers(0, len(offs) - 1))
            o, nxt = int(offs[k]) + 16, int(offs[k + 1])
            fake = b""
            while len(fake) < nxt - o:
                ln = int(rng.integers(0, 90))
                fake += struct.pack(e + "IIII", 1_600_000_000, 0, ln, ln) + bytes(rng.integers(0, 256, ln, dtype=np.uint8))
            b[o:nxt] = fake[: nxt - o]
        elif op == 4 and len(offs):  # orig_len below incl_len / random (no check in the reference)
            o = int(offs[int(rng.integers(0, len(offs)))])
            struct.pack_into(e + "I", b, o + 12, int(rng.integers(0, 1 << 32)))
        elif op == 5 and len(b) > 40:  # the capture cut at a random byte
            del b[int(rng.integers(24, len(b))):]
            offs, _ = record_offsets(bytes(b))
    return bytes(b)


SHAPES = ["full", "resident", "resident_w7", "resident_w48", "two_pass", "sparse", "sparse_span", "chunked"]


def run_shape(rng, blob, shape):
    if shape == "full":
        return check_parity(blob)
    if shape == "resident":
        return check_parity(blob, light=True)
    if shape == "resident_w7":
        return check_parity(blob, light=7)
    if shape == "resident_w48":
        return check_parity(blob, light=48)
    if shape == "two_pass":
        return check_parity(blob, light="decode")
    if shape == "sparse":
        return check_parity(blob, light="sparse")
    if shape == "sparse_span":
        span = int(rng.choice([64, 128, 256, 1000, 4096, 65536]))
        cap = int(rng.choice([0, 1, 2, 4, 33]))
        return check_parity(blob, light=f"sparse_s{span}" + (f"_c{cap}" if cap else ""))
    chunk = int(rng.choice([700, 4096, 9999, 65536, 333_333]))
    if rng.integers(0, 2):
        with sparse_forced(f"sparse_s{int(rng.choice([256, 2048]))}"):
            return check_chunked(blob, chunk)
    return check_chunked(blob, chunk)


@pytest.mark.parametrize("case", range(N_CASES))
def test_mutated_capture_matches_oracle(case):
    rng = np.random.default_rng(0xF022 + case)
    blob = mutate(rng, base_capture(rng))
    shape = SHAPES[case % len(SHAPES)]  # every shape sees N_CASES / 8 captures
    run_shape(rng, blob, shape)


@pytest.mark.parametrize("case", range(12))
def test_mutated_large_capture(case):
    """C2/C3-sized captures (all 256 workgroups of the resident pass, many sparse groups) with a few
    mutations deep inside, so contradictions land between workgroups far from the start."""
    rng = np.random.default_rng(0x1A26E + case)
    seed = int(rng.integers(1, 1 << 30))
    blob = synth.fixed64(int(rng.integers(200_000, 1_000_000)), seed=seed) if case % 2 == 0 else \
        synth.variable_mix(int(rng.integers(50_000, 150_000)), seed=seed)
    blob = mutate(rng, blob)
    run_shape(rng, blob, ["full", "resident", "sparse_span", "chunked", "resident_w48", "two_pass"][case % 6])


@pytest.mark.parametrize("case", range(32))
def test_unmutated_splice_every_shape(case):
    """Spliced corpora (record shapes change mid-capture) without mutations, all shapes in turn."""
    rng = np.random.default_rng(0x5B11CE + case)
    blob = base_capture(rng)
    for shape in SHAPES:
        run_shape(rng, blob, shape)


# ---- the other entry points over mutated captures ----------------------------------------------
@pytest.mark.parametrize("case", range(24))
def test_mutated_records_api(case):
    """npr_dev_extract_flows / npr_dev_convert_records over the parsed records of a mutated capture,
    some payloads shrunk to a prefix, the list permuted on odd cases."""
    from test_gpu_records_api import check_convert, check_dense, records_of
    rng = np.random.default_rng(0xA91 + case)
    blob = mutate(rng, base_capture(rng))
    recs = records_of(blob, shrink=float(rng.choice([0.0, 0.2, 0.7])), permute=bool(case & 1), seed=case)
    check_dense(blob, recs)
    check_convert(blob, recs, cap=None if case % 3 else max(1, len(recs) // 2))


@pytest.mark.parametrize("case", range(16))
def test_mutated_host_pipelined(case):
    """npr_parse_extract_pipelined (chunked H2D, chained links, per-link D2H) and, on odd cases, its
    bounded device window, over mutated captures at random chunk sizes."""
    from test_gpu_host_stream import check_pipelined, check_windowed
    rng = np.random.default_rng(0x91BE + case)
    blob = mutate(rng, base_capture(rng))
    chunk = int(rng.choice([65536, 100_000, 1 << 19]))
    if case & 1:
        check_windowed(blob, max(chunk, 1 << 16), int(rng.choice([3, 4, 7])))
    else:
        check_pipelined(blob, chunk, pinned=bool(case & 2))


@pytest.mark.parametrize("case", range(16))
def test_mutated_shards_in_process(case):
    """Record-range shards of a mutated capture (the multi-GPU path's per-rank launches and summary
    replay, in one process), merged and compared with the serial oracle."""
    import torch

    from net_parser_rs import _abi, device, parallel
    rng = np.random.default_rng(0x54A2D + case)
    blob = mutate(rng, base_capture(rng))
    rc, hdr, recs, cons = _oracle.capture_file_parse(blob)
    flows, v6 = _oracle.convert_records(blob, recs)
    t = torch.empty(len(blob), dtype=torch.uint8, device="cuda")
    t.copy_(torch.from_numpy(np.frombuffer(blob, dtype=np.uint8).copy()))
    ws = device.Workspace(len(recs) + 1, len(recs) + 1, records=False)
    local = parallel.device_local(ws, t, len(blob), endianness=hdr.endianness)
    world = int(rng.integers(2, 9))
    results, live, rounds = parallel.parse_sharded_inprocess(local, 24, len(blob), world)
    _, _, r_tot, f_tot = parallel.prefix_offsets(results, live)
    assert (r_tot, f_tot) == (len(recs), len(flows))
    merged, merged6 = parallel.merge_flows(results, live)
    assert merged.tobytes() == flows.tobytes()
    m = (flows["kind"] & _abi.KIND_IPV6) != 0
    if m.any():
        assert merged6[m].tobytes() == v6[m].tobytes()


@pytest.mark.parametrize("case", range(8))
def test_mutated_batches(case):
    """npr_dev_parse_extract_batch over 2-9 mutated captures of mixed shapes and byte orders."""
    from test_gpu_batch import run_batch
    rng = np.random.default_rng(0xBA7C + case)
    run_batch([mutate(rng, base_capture(rng)) for _ in range(int(rng.integers(2, 10)))])


@pytest.mark.parametrize("case", range(8))
def test_mutated_flow_table(case):
    """Row f4 (the distinct-flow table) over the flow table of a mutated capture, with random
    weights and, on odd cases, an output capacity below the distinct count."""
    import torch

    from test_gpu_flowtable import check, device_table
    rng = np.random.default_rng(0xF70 + case)
    blob = mutate(rng, base_capture(rng))
    fl, f6, n = device_table(blob)
    if n == 0:
        return
    w = torch.from_numpy(rng.integers(1, 1000, size=n, dtype=np.uint64).astype(np.int64)).cuda()
    check(fl, f6, n, weights=w, cap=max(1, n // 3) if case & 1 else None)


@pytest.mark.parametrize("case", range(8))
def test_mutated_vxlan(case):
    """Row f3: VXLAN inner flows over the records of a mutated VXLAN (or other) capture."""
    from test_vxlan import _check_device
    rng = np.random.default_rng(0x4789 + case)
    blob = mutate(rng, synth.vxlan_corpus(int(rng.integers(200, 3000)), seed=int(rng.integers(1, 1 << 30)))
                  if case % 4 else base_capture(rng))
    if len(_oracle.capture_file_parse(blob)[2]):
        _check_device(blob, int(rng.choice([0, 4789, 8472])), bool(case & 1))
