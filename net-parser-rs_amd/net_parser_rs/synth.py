"""Deterministic synthetic libpcap captures (BASELINE.json configs) and an adversarial corpus.

C2  `fixed64(n)`      n records, incl = orig = 64: Ethernet(0x0800) / IPv4 (IHL 5, total 50,
                      proto 6) / TCP (data offset 5, random 9-bit flags) / 10 payload bytes.
C3  `variable_mix(n)` frame length U[64, 1500], TCP or UDP with p = 1/2, IPv4 total = frame-14,
                      UDP length = frame-34, TCP data offset U[5, 15].
    `quirk_corpus(n)` every branch of the reference's parse tree (VLAN stacks, IHL != 5, trailers,
                      IPv6 extension chains, ARP, LLDP, 802.3 lengths, bad versions, wrong UDP
                      lengths, truncations, zero-length and jumbo records, fake record headers
                      inside payloads) — the inputs the reference's own tests never pin.

All generators are pure functions of (n, seed) via numpy PCG64.  Timestamps follow SURVEY §8d:
ts_sec = 1.6e9 + i // 1e6, ts_usec = i % 1e6.
"""
import struct

import numpy as np

MAGIC_LE = bytes.fromhex("d4c3b2a1")  # 0xA1B2C3D4 little-endian -> Endianness::Little
SEED = 0x4E50


def global_header(big=False, snaplen=65535, network=1, version=(2, 4)):
    if big:
        return bytes.fromhex("a1b2c3d4") + struct.pack(">HHiiII", version[0], version[1], 0, 0, snaplen, network)
    return MAGIC_LE + struct.pack("<HHiiII", version[0], version[1], 0, 0, snaplen, network)


def _ts(n, base=1_600_000_000):
    i = np.arange(n, dtype=np.int64)
    return (base + i // 1_000_000).astype(np.uint32), (i % 1_000_000).astype(np.uint32)


def fixed64(n, seed=SEED, with_header=True):
    """C2: n x 64-B Ethernet/IPv4/TCP records (80 B each with the record header)."""
    rng = np.random.default_rng(seed)
    rec = rng.integers(0, 256, size=(n, 80), dtype=np.uint8)
    sec, usec = _ts(n)
    hdr = np.empty((n, 4), dtype="<u4")
    hdr[:, 0] = sec
    hdr[:, 1] = usec
    hdr[:, 2] = 64
    hdr[:, 3] = 64
    rec[:, 0:16] = hdr.view(np.uint8).reshape(n, 16)
    f = rec[:, 16:]
    f[:, 12] = 0x08; f[:, 13] = 0x00                       # EtherType IPv4
    f[:, 14] = 0x45; f[:, 15] = 0x00                       # version 4, IHL 5, tos
    f[:, 16] = 0x00; f[:, 17] = 50                         # total length 50
    f[:, 20] = 0x00; f[:, 21] = 0x00                       # flags / fragment
    f[:, 22] = 64; f[:, 23] = 6                            # ttl, protocol TCP
    flags = rng.integers(0, 512, size=n, dtype=np.uint16)
    hv = (5 << 12) | flags
    f[:, 46] = (hv >> 8).astype(np.uint8); f[:, 47] = (hv & 0xff).astype(np.uint8)  # data offset 5
    body = rec.reshape(-1)
    return (global_header() + body.tobytes()) if with_header else body.tobytes()


BLOCK = 1 << 20  # records per independently seeded block (fixed64_range)


def _fixed64_block(k, seed):
    """Block k of the shard-independent C2-shape stream: records [k*BLOCK, (k+1)*BLOCK)."""
    rng = np.random.default_rng([seed, 4, k])
    n = BLOCK
    rec = rng.integers(0, 256, size=(n, 80), dtype=np.uint8)
    i = np.arange(k * BLOCK, (k + 1) * BLOCK, dtype=np.int64)
    hdr = np.empty((n, 4), dtype="<u4")
    hdr[:, 0] = (1_600_000_000 + i // 1_000_000).astype(np.uint32)
    hdr[:, 1] = (i % 1_000_000).astype(np.uint32)
    hdr[:, 2] = 64
    hdr[:, 3] = 64
    rec[:, 0:16] = hdr.view(np.uint8).reshape(n, 16)
    f = rec[:, 16:]
    f[:, 12] = 0x08; f[:, 13] = 0x00
    f[:, 14] = 0x45; f[:, 15] = 0x00
    f[:, 16] = 0x00; f[:, 17] = 50
    f[:, 20] = 0x00; f[:, 21] = 0x00
    f[:, 22] = 64; f[:, 23] = 6
    flags = rng.integers(0, 512, size=n, dtype=np.uint16)
    hv = (5 << 12) | flags
    f[:, 46] = (hv >> 8).astype(np.uint8); f[:, 47] = (hv & 0xff).astype(np.uint8)
    return rec


def fixed64_range(lo, hi, seed=SEED):
    """Records [lo, hi) of the C4 capture (64M x C2-shape records; shard-independent:
    record i's bytes depend only on i, through per-block seeding, so a rank generates exactly its
    own range).  Returns the bytes of file range [24 + 80*lo, 24 + 80*hi), preceded by the global
    header when lo == 0 (then the buffer starts at file byte 0), as a numpy uint8 array."""
    h = 24 if lo == 0 else 0
    out = np.empty(h + 80 * (hi - lo), dtype=np.uint8)
    if h:
        out[:24] = np.frombuffer(global_header(), dtype=np.uint8)
    for k in range(lo // BLOCK, (hi + BLOCK - 1) // BLOCK):
        b = _fixed64_block(k, seed)
        a, z = max(lo, k * BLOCK) - k * BLOCK, min(hi, (k + 1) * BLOCK) - k * BLOCK
        o = h + 80 * (k * BLOCK + a - lo)
        out[o: o + 80 * (z - a)] = b[a:z].reshape(-1)
    return out


def variable_mix(n, seed=SEED + 3, with_header=True):
    """C3: n records, frame length U[64, 1500], IPv4 + (TCP | UDP)."""
    rng = np.random.default_rng(seed)
    L = rng.integers(64, 1501, size=n).astype(np.int64)
    udp = rng.integers(0, 2, size=n).astype(bool)
    doff = rng.integers(5, 16, size=n).astype(np.int64)
    size = 16 + L
    off = np.zeros(n, dtype=np.int64)
    np.cumsum(size[:-1], out=off[1:])
    total = int(off[-1] + size[-1]) if n else 0
    buf = rng.integers(0, 256, size=total, dtype=np.uint8)
    sec, usec = _ts(n)

    def put32(col, v):
        vb = np.asarray(v, dtype="<u4").view(np.uint8).reshape(-1, 4)
        for k in range(4):
            buf[off + col + k] = vb[:, k]

    def put8(col, v):
        buf[off + col] = np.asarray(v, dtype=np.int64).astype(np.uint8)

    def put16be(col, v):
        v = np.asarray(v, dtype=np.int64)
        buf[off + col] = (v >> 8).astype(np.uint8)
        buf[off + col + 1] = (v & 0xff).astype(np.uint8)

    put32(0, sec); put32(4, usec); put32(8, L); put32(12, L)
    e = 16
    put16be(e + 12, 0x0800)
    put8(e + 14, 0x45); put8(e + 15, 0)
    put16be(e + 16, L - 14)
    put16be(e + 20, 0)
    put8(e + 22, 64)
    put8(e + 23, np.where(udp, 17, 6))
    l4 = e + 34
    hv = (doff << 12) | rng.integers(0, 512, size=n)
    tcp_hv = np.where(udp, (buf[off + l4 + 12].astype(np.int64) << 8) | buf[off + l4 + 13], hv)
    put16be(l4 + 12, tcp_hv)
    ulen = np.where(udp, L - 34, (buf[off + l4 + 4].astype(np.int64) << 8) | buf[off + l4 + 5])
    put16be(l4 + 4, ulen)
    body = buf.tobytes()
    return (global_header() + body) if with_header else body


# ---------------------------------------------------------------------------------------------
# quirk corpus
# ---------------------------------------------------------------------------------------------
_PROTOS = [6, 17, 1, 0, 43, 44, 50, 51, 59, 60, 58, 2, 255]
_ETYPES = [0x0800, 0x86DD, 0x0806, 0x88CC, 0x0000, 0x05DC, 0x05DD, 0x8100, 0x88A8, 0x9100, 0xFFFF, 0x0600]


def _l4(rng, proto, room):
    """A TCP / UDP / other header+payload with randomly right or wrong lengths."""
    if proto == 6:
        doff = int(rng.choice([5, 5, 5, 6, 8, 15, 4, 0, 1]))
        flags = int(rng.integers(0, 512))
        plen = int(rng.integers(0, 40))
        body = bytearray(rng.integers(0, 256, size=max(doff * 4, 20) + plen, dtype=np.uint8).tobytes())
        body[12:14] = struct.pack(">H", (doff << 12) | flags)
        return bytes(body)
    if proto == 17:
        plen = int(rng.integers(0, 40))
        body = bytearray(rng.integers(0, 256, size=8 + plen, dtype=np.uint8).tobytes())
        mode = rng.integers(0, 5)
        ulen = [8 + plen, 8 + plen, 8 + plen + 1, max(0, 8 + plen - 1), int(rng.integers(0, 8))][mode]
        body[4:6] = struct.pack(">H", ulen & 0xFFFF)
        return bytes(body)
    return rng.integers(0, 256, size=int(rng.integers(0, 30)), dtype=np.uint8).tobytes()


def _ipv4(rng):
    proto = int(rng.choice(_PROTOS))
    ihl = int(rng.choice([5, 5, 5, 5, 6, 7, 15, 4, 0]))
    ver = int(rng.choice([4, 4, 4, 4, 4, 6, 0]))
    l4 = _l4(rng, proto, 0)
    opts = rng.integers(0, 256, size=max(0, (ihl - 5) * 4), dtype=np.uint8).tobytes()
    hdr = bytearray(rng.integers(0, 256, size=20, dtype=np.uint8).tobytes())
    hdr[0] = (ver << 4) | ihl
    true_total = 20 + len(opts) + len(l4)
    mode = rng.integers(0, 6)
    total = [true_total, true_total, true_total - len(opts), true_total + 3, int(rng.integers(0, 24)),
             max(0, true_total - 5)][mode]
    hdr[2:4] = struct.pack(">H", total & 0xFFFF)
    hdr[9] = proto
    # quirk Q7: the reference reads the L4 header right after the fixed 20 bytes
    body = bytes(hdr) + (l4 + opts if rng.integers(0, 2) else opts + l4)
    trailer = rng.integers(0, 256, size=int(rng.choice([0, 0, 0, 2, 6])), dtype=np.uint8).tobytes()
    return body + trailer


def _ipv6(rng):
    nh_chain = [int(rng.choice([0, 43, 44, 50, 51, 60])) for _ in range(int(rng.choice([0, 0, 0, 1, 2, 3])))]
    final = int(rng.choice(_PROTOS))
    first = nh_chain[0] if nh_chain else final
    rest = nh_chain[1:] + [final] if nh_chain else []
    l4 = _l4(rng, final, 0)
    ver = int(rng.choice([6, 6, 6, 6, 4]))
    plen = len(l4) + int(rng.choice([0, 0, 0, 1, -1, 5]))
    hdr = bytearray(rng.integers(0, 256, size=8, dtype=np.uint8).tobytes())
    hdr[0] = (ver << 4) | (hdr[0] & 0x0F)
    hdr[4:6] = struct.pack(">H", max(0, plen) & 0xFFFF)
    hdr[6] = first
    # each "extension" the reference consumes is exactly one next-header byte (quirk Q11)
    ext = bytes(rest)
    addrs = rng.integers(0, 256, size=33, dtype=np.uint8).tobytes()  # hop limit + src + dst
    return bytes(hdr[:7]) + ext + addrs + l4 + rng.integers(0, 256, size=int(rng.choice([0, 0, 0, 3])),
                                                            dtype=np.uint8).tobytes()


def _frame(rng):
    macs = rng.integers(0, 256, size=12, dtype=np.uint8).tobytes()
    tags = b""
    for _ in range(int(rng.choice([0, 0, 0, 0, 1, 1, 2, 3]))):
        tags += struct.pack(">HH", int(rng.choice([0x8100, 0x88A8])), int(rng.integers(0, 65536)))
    et = int(rng.choice(_ETYPES + [0x0800] * 6 + [0x86DD] * 3))
    if et == 0x0800:
        l3 = _ipv4(rng)
    elif et == 0x86DD:
        l3 = _ipv6(rng)
    elif et == 0x0806:
        l3 = rng.integers(0, 256, size=int(rng.choice([28, 28, 46, 20])), dtype=np.uint8).tobytes()
    else:
        l3 = rng.integers(0, 256, size=int(rng.integers(0, 60)), dtype=np.uint8).tobytes()
    f = macs + tags + struct.pack(">H", et) + l3
    if rng.integers(0, 12) == 0:  # truncated capture (incl < frame)
        f = f[: int(rng.integers(0, len(f) + 1))]
    return f


def _fake_headers(rng, ts):
    """Payload bytes that look like a valid chain of pcap record headers (defeats speculation)."""
    out = b""
    for _ in range(int(rng.integers(1, 4))):
        ln = int(rng.integers(14, 80))
        out += struct.pack("<IIII", ts, int(rng.integers(0, 1_000_000)), ln, ln)
        out += rng.integers(0, 256, size=ln, dtype=np.uint8).tobytes()
    return out


def quirk_corpus(n, seed=SEED + 7, big=False, with_header=True, jumbo_every=0, fake_every=0,
                 zero_every=0, tail=None):
    """n records covering the reference's parse tree; options add adversarial record shapes.

    jumbo_every: every k-th record gets a 20-70 KB payload (larger than a device tile)
    fake_every:  every k-th record's payload is a chain of plausible fake record headers
    zero_every:  every k-th record has a zero-filled payload / zero-length record
    tail:        None | "truncated_header" | "truncated_payload" | "huge_incl"
    """
    rng = np.random.default_rng(seed)
    e = ">" if big else "<"
    parts = [global_header(big=big)] if with_header else []
    for i in range(n):
        ts = 1_600_000_000 + i // 1000
        if jumbo_every and i % jumbo_every == jumbo_every - 1:
            frame = _frame(rng) + rng.integers(0, 256, size=int(rng.integers(20_000, 70_000)), dtype=np.uint8).tobytes()
        elif fake_every and i % fake_every == fake_every - 1:
            frame = _frame(rng)[:14] + _fake_headers(rng, ts)
        elif zero_every and i % zero_every == zero_every - 1:
            frame = bytes(int(rng.choice([0, 0, 40, 200])))
        else:
            frame = _frame(rng)
        orig = len(frame) + int(rng.choice([0, 0, 0, 100]))
        parts.append(struct.pack(e + "IIII", ts, i % 1_000_000, len(frame), orig) + frame)
    if tail == "truncated_header":
        parts.append(struct.pack(e + "III", 1, 2, 3))
    elif tail == "truncated_payload":
        parts.append(struct.pack(e + "IIII", 1, 2, 500, 500) + bytes(100))
    elif tail == "huge_incl":
        parts.append(struct.pack(e + "IIII", 1, 2, 0xFFFFFF00, 0xFFFFFF00) + bytes(64))
    return b"".join(parts)


def _good_inner(rng):
    """A valid inner frame: Ethernet (0-1 VLAN tags) / IPv4 (IHL 5) or IPv6 / TCP or UDP."""
    macs = rng.integers(0, 256, size=12, dtype=np.uint8).tobytes()
    tags = struct.pack(">HH", 0x8100, int(rng.integers(0, 65536))) if rng.integers(0, 4) == 0 else b""
    proto = int(rng.choice([6, 17]))
    pay = rng.integers(0, 256, size=int(rng.integers(0, 60)), dtype=np.uint8).tobytes()
    ports = rng.integers(0, 256, size=4, dtype=np.uint8).tobytes()
    if proto == 6:
        l4 = bytearray(ports + rng.integers(0, 256, size=16, dtype=np.uint8).tobytes()) + pay
        l4[12:14] = struct.pack(">H", (5 << 12) | int(rng.integers(0, 512)))
    else:
        l4 = bytearray(ports + struct.pack(">HH", 8 + len(pay), 0)) + pay
    if rng.integers(0, 3):
        ip = bytearray(rng.integers(0, 256, size=20, dtype=np.uint8).tobytes())
        ip[0] = 0x45
        ip[2:4] = struct.pack(">H", 20 + len(l4))
        ip[9] = proto
        return macs + tags + b"\x08\x00" + bytes(ip) + bytes(l4)
    ip = bytearray(rng.integers(0, 256, size=40, dtype=np.uint8).tobytes())
    ip[0] = 0x60 | (ip[0] & 0x0F)
    ip[4:6] = struct.pack(">H", len(l4))
    ip[6] = proto
    return macs + tags + b"\x86\xdd" + bytes(ip) + bytes(l4)


def _outer_udp(rng, payload, dport, v6=False):
    """Ethernet / IPv4 (IHL 5) or IPv6 / UDP to `dport` carrying `payload` (all lengths exact)."""
    macs = rng.integers(0, 256, size=12, dtype=np.uint8).tobytes()
    udp = struct.pack(">HHHH", int(rng.integers(1024, 65536)), dport, 8 + len(payload), 0) + payload
    if not v6:
        ip = bytearray(rng.integers(0, 256, size=20, dtype=np.uint8).tobytes())
        ip[0] = 0x45
        ip[2:4] = struct.pack(">H", 20 + len(udp))
        ip[9] = 17
        return macs + b"\x08\x00" + bytes(ip) + udp
    ip = bytearray(rng.integers(0, 256, size=40, dtype=np.uint8).tobytes())
    ip[0] = 0x60
    ip[4:6] = struct.pack(">H", len(udp))
    ip[6] = 17
    return macs + b"\x86\xdd" + bytes(ip) + udp


def vxlan_corpus(n, seed=SEED + 11, with_header=True, port=4789):
    """Row f3 corpus: VXLAN-encapsulated frames (valid inner flows, inner failures from the quirk
    generator, truncated VXLAN headers, other UDP ports, IPv6 underlays) mixed with plain traffic."""
    rng = np.random.default_rng(seed)
    parts = [global_header()] if with_header else []
    for i in range(n):
        k = int(rng.integers(0, 10))
        if k <= 3:    # VXLAN, valid inner frame
            vx = struct.pack(">HHI", 0x0800, 0, int(rng.integers(0, 1 << 24)) << 8)
            frame = _outer_udp(rng, vx + _good_inner(rng), port, v6=bool(rng.integers(0, 4) == 0))
        elif k == 4:  # VXLAN, inner frame from the quirk generator (most fail somewhere)
            vx = struct.pack(">HHI", int(rng.integers(0, 65536)), int(rng.integers(0, 65536)),
                             int(rng.integers(0, 1 << 32)))
            frame = _outer_udp(rng, vx + _frame(rng), port)
        elif k == 5:  # UDP payload shorter than a VXLAN header
            frame = _outer_udp(rng, rng.integers(0, 256, size=int(rng.integers(0, 8)), dtype=np.uint8).tobytes(), port)
        elif k == 6:  # another UDP port
            frame = _outer_udp(rng, rng.integers(0, 256, size=int(rng.integers(0, 40)), dtype=np.uint8).tobytes(),
                               int(rng.choice([53, 5300, 4790])))
        else:         # plain traffic (TCP, broken outer frames, ...)
            frame = _frame(rng)
        parts.append(struct.pack("<IIII", 1_600_000_000 + i, i % 1_000_000, len(frame), len(frame)) + frame)
    return b"".join(parts)


def flow_mix(n, n_flows=500, seed=SEED + 13, with_header=True):
    """Row f4 corpus: n records drawn from a population of n_flows 5-tuples (IPv4 / IPv6, TCP / UDP,
    Zipf-like popularity), with per-record MACs, VLAN tags and payloads that are not part of the
    key, plus some frames that yield no flow."""
    rng = np.random.default_rng(seed)
    pop = []
    for _ in range(n_flows):
        v6 = bool(rng.integers(0, 4) == 0)
        pop.append((v6, int(rng.choice([6, 17])), rng.integers(0, 256, size=32 if v6 else 8, dtype=np.uint8).tobytes(),
                    int(rng.integers(0, 65536)), int(rng.integers(0, 65536))))
    weights = 1.0 / np.arange(1, n_flows + 1)
    picks = rng.choice(n_flows, size=n, p=weights / weights.sum())
    parts = [global_header()] if with_header else []
    for i in range(n):
        if rng.integers(0, 20) == 0:
            frame = _frame(rng)  # mostly no flow
        else:
            v6, proto, ips, sp, dp = pop[picks[i]]
            pay = rng.integers(0, 256, size=int(rng.integers(0, 30)), dtype=np.uint8).tobytes()
            if proto == 6:
                l4 = bytearray(struct.pack(">HH", sp, dp) + rng.integers(0, 256, size=16, dtype=np.uint8).tobytes())
                l4[12:14] = struct.pack(">H", 5 << 12)
                l4 = bytes(l4) + pay
            else:
                l4 = struct.pack(">HHHH", sp, dp, 8 + len(pay), 0) + pay
            macs = rng.integers(0, 256, size=12, dtype=np.uint8).tobytes()
            tag = struct.pack(">HH", 0x8100, int(rng.integers(0, 65536))) if rng.integers(0, 5) == 0 else b""
            if v6:
                ip = bytearray(rng.integers(0, 256, size=8, dtype=np.uint8).tobytes())
                ip[0] = 0x60
                ip[4:6] = struct.pack(">H", len(l4))
                ip[6] = proto
                frame = macs + tag + b"\x86\xdd" + bytes(ip) + ips + l4
            else:
                ip = bytearray(rng.integers(0, 256, size=12, dtype=np.uint8).tobytes())
                ip[0] = 0x45
                ip[2:4] = struct.pack(">H", 20 + len(l4))
                ip[9] = proto
                frame = macs + tag + b"\x08\x00" + bytes(ip) + ips + l4
        parts.append(struct.pack("<IIII", 1_600_000_000 + i, i % 1_000_000, len(frame), len(frame)) + frame)
    return b"".join(parts)


def corrupt_midfile(data, at_record, endianness_big=False):
    """Overwrite record `at_record`'s incl_len with a huge value (quirk Q3: the list stops there)."""
    buf = bytearray(data)
    e = ">" if endianness_big else "<"
    off = 24
    for _ in range(at_record):
        (incl,) = struct.unpack_from(e + "I", buf, off + 8)
        off += 16 + incl
    struct.pack_into(e + "I", buf, off + 8, 0x7FFFFFF0)
    return bytes(buf)
