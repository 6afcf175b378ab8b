// npr_layers.hip — host-side per-layer header objects (include/npr.h, "host-side per-layer header
// objects"): the reference's public layer parsers, each a nom 4 chain read step by step.
//   Ethernet::parse   src/layer2/ethernet.rs:143-216
//   IPv4::parse       src/layer3/ipv4.rs:76-160
//   IPv6::parse       src/layer3/ipv6.rs:51-99
//   Arp::parse        src/layer3/arp.rs:54-76
//   Tcp::parse        src/layer4/tcp.rs:54-101
//   Udp::parse        src/layer4/udp.rs:33-50
//   Vxlan::parse      src/layer4/vxlan.rs:31-48
// No device work: a frame's flow comes from the device decoder (npr_decode.hpp); these give callers
// the header objects themselves.  Errors are the reference's (src/errors.rs:16-55): nom's
// Needed::Size for Incomplete, the failing primitive's input range for a map_opt! / map_res! Failure.
#include <stdint.h>
#include <string.h>

#include "../../include/npr.h"

namespace {

// A nom 4 input cursor over input[0, n): each primitive either advances or records the error the
// reference's chain returns at that step.
struct Cursor {
  const uint8_t *b;
  size_t n;
  size_t i = 0;
  npr_status st = NPR_OK;
  uint64_t det = 0;

  bool need(uint64_t k) {
    if ((uint64_t)(n - i) < k) {
      st = NPR_INCOMPLETE;
      det = k;  // Needed::Size(k): what the primitive needs, not what is missing
      return false;
    }
    return true;
  }
  bool u8(uint8_t &v) {
    if (!need(1)) return false;
    v = b[i++];
    return true;
  }
  bool u16(uint16_t &v, bool big = true) {
    if (!need(2)) return false;
    v = big ? (uint16_t)(b[i] << 8 | b[i + 1]) : (uint16_t)(b[i] | b[i + 1] << 8);
    i += 2;
    return true;
  }
  bool u32(uint32_t &v, bool big = true) {
    if (!need(4)) return false;
    v = big ? (uint32_t)b[i] << 24 | (uint32_t)b[i + 1] << 16 | (uint32_t)b[i + 2] << 8 | b[i + 3]
            : (uint32_t)b[i] | (uint32_t)b[i + 1] << 8 | (uint32_t)b[i + 2] << 16 | (uint32_t)b[i + 3] << 24;
    i += 4;
    return true;
  }
  bool take(uint64_t k, uint64_t &off) {
    if (!need(k)) return false;
    off = i;
    i += (size_t)k;
    return true;
  }
  bool bytes(uint8_t *dst, size_t k) {
    if (!need(k)) return false;
    memcpy(dst, b + i, k);
    i += k;
    return true;
  }
  // map_opt! / map_res! over a primitive that started at `at`: nom's Code(input[at..], kind)
  bool fail(size_t at) {
    st = NPR_FAILURE;
    const uint64_t a = at < 0xffffffffu ? at : 0xffffffffu, e = n < 0xffffffffu ? n : 0xffffffffu;
    det = a | e << 32;
    return false;
  }
};

npr_status finish(const Cursor &c, size_t *consumed, uint64_t *detail) {
  if (consumed) *consumed = c.st == NPR_OK ? c.i : 0;
  if (detail) *detail = c.st == NPR_OK ? 0 : c.det;
  return c.st;
}

// InternetProtocolId::new (src/layer3/mod.rs:54-72)
bool protocol_known(uint8_t v) {
  switch (v) {
    case 0: case 1: case 6: case 17: case 43: case 44: case 50: case 51: case 59: case 60: return true;
    default: return false;
  }
}
// InternetProtocolId::has_next_option (src/layer3/mod.rs:74-84)
bool protocol_has_next(uint8_t v) {
  return v == 50 || v == 51 || v == 0 || v == 43 || v == 44 || v == 60;
}
// EthernetTypeId::new (src/layer2/ethernet.rs:57-73): 0 unknown, 1 VLAN tag type, 2 anything else known
int ether_type_kind(uint16_t v) {
  switch (v) {
    case 0x8100: case 0x88A8: return 1;
    case 0x88CC: case 0x0800: case 0x86DD: case 0x0806: return 2;
    default: return v <= 1500 ? 2 : 0;
  }
}

}  // namespace

extern "C" {

npr_status npr_ethernet_parse(const uint8_t *input, size_t len, npr_ethernet *out, npr_vlan_tag *vlans,
                              size_t vlan_cap, size_t *consumed, uint64_t *detail) {
  if (!out || (!input && len) || (!vlans && vlan_cap)) return NPR_ERR_ARG;
  memset(out, 0, sizeof(*out));
  Cursor c{input, len};
  // two MACs (mac_address: take!(6)), then parse_vlan_tag: EtherType / VLAN tags until a non-VLAN
  // type, whose rest is the payload (parse_not_vlan_tag)
  if (!c.bytes(out->dst_mac, 6) || !c.bytes(out->src_mac, 6)) return finish(c, consumed, detail);
  uint32_t nv = 0;
  for (;;) {
    const size_t at = c.i;
    uint16_t t;
    if (!c.u16(t)) return finish(c, consumed, detail);
    const int kind = ether_type_kind(t);
    if (kind == 0) {  // map_opt!(be_u16, EthernetTypeId::new) -> None
      c.fail(at);
      return finish(c, consumed, detail);
    }
    if (kind == 2) {
      out->ether_type = t;
      out->payload_offset = c.i;
      out->payload_length = len - c.i;
      c.i = len;
      break;
    }
    uint16_t total;
    if (!c.u16(total)) return finish(c, consumed, detail);
    if (nv < vlan_cap) {
      npr_vlan_tag &g = vlans[nv];
      g.vlan_type = t;
      g.vlan_value = total;
      g.prio = (uint8_t)(total & 0x7000);  // `as u8` of the masked value, as the reference writes it
      g.dei = (uint8_t)(total & 0x8000);
      g.id = total & 0x0FFF;
    }
    ++nv;
  }
  out->n_vlans = nv;
  const npr_status st = finish(c, consumed, detail);
  return st == NPR_OK && nv > vlan_cap ? NPR_ERR_CAPACITY : st;
}

npr_status npr_ipv4_parse(const uint8_t *input, size_t len, npr_ipv4 *out, size_t *consumed, uint64_t *detail) {
  if (!out || (!input && len)) return NPR_ERR_ARG;
  memset(out, 0, sizeof(*out));
  Cursor c{input, len};
  uint8_t vl;
  if (!c.u8(vl)) return finish(c, consumed, detail);
  if (vl >> 4 != 4) {  // Custom("Expected version 4, was {}")
    c.st = NPR_CUSTOM;
    c.det = vl >> 4;
    return finish(c, consumed, detail);
  }
  out->version_and_length = vl;
  const uint8_t words = vl & 0x0F;
  const uint8_t header_length = (uint8_t)(words * 4);
  const uint8_t additional = words > 5 ? (uint8_t)((words - 5) * 4) : 0;
  uint16_t raw;
  if (!c.u8(out->tos) || !c.u16(raw)) return finish(c, consumed, detail);
  out->raw_length = raw;
  const uint16_t length = (uint16_t)(raw - header_length);  // u16 subtraction, wrapping (:97-101)
  const uint64_t expected = (uint64_t)header_length + additional + length;
  if (!c.u16(out->id) || !c.u16(out->flags) || !c.u8(out->ttl)) return finish(c, consumed, detail);
  const size_t at = c.i;
  if (!c.u8(out->protocol)) return finish(c, consumed, detail);
  if (!protocol_known(out->protocol)) {
    c.fail(at);
    return finish(c, consumed, detail);
  }
  if (!c.u16(out->checksum) || !c.bytes(out->src_ip, 4) || !c.bytes(out->dst_ip, 4)) return finish(c, consumed, detail);
  if (!c.take(length, out->payload_offset)) return finish(c, consumed, detail);
  out->payload_length = length;
  if (additional > 0) {
    if (!c.take(additional, out->options_offset)) return finish(c, consumed, detail);
    out->options_length = additional;
  }
  if ((uint64_t)len > expected) {
    if (!c.take(len - expected, out->padding_offset)) return finish(c, consumed, detail);
    out->padding_length = len - expected;
  }
  return finish(c, consumed, detail);
}

npr_status npr_ipv6_parse(const uint8_t *input, size_t len, npr_ipv6 *out, size_t *consumed, uint64_t *detail) {
  if (!out || (!input && len)) return NPR_ERR_ARG;
  memset(out, 0, sizeof(*out));
  Cursor c{input, len};
  uint8_t first;
  if (!c.u8(first)) return finish(c, consumed, detail);
  if (first >> 4 != 6) {  // Custom("Expected version 6, version was {}")
    c.st = NPR_CUSTOM;
    c.det = first >> 4;
    return finish(c, consumed, detail);
  }
  // parse_ipv6: take!(3) (version and flow label), be_u16 payload length, map_opt!(be_u8) next header
  uint64_t skip;
  uint16_t payload_length;
  if (!c.take(3, skip) || !c.u16(payload_length)) return finish(c, consumed, detail);
  uint8_t h;
  size_t at = c.i;
  if (!c.u8(h)) return finish(c, consumed, detail);
  if (!protocol_known(h)) {
    c.fail(at);
    return finish(c, consumed, detail);
  }
  // parse_next_header: one map_opt!(be_u8) per header that has a next option (quirk Q11)
  while (protocol_has_next(h)) {
    at = c.i;
    if (!c.u8(h)) return finish(c, consumed, detail);
    if (!protocol_known(h)) {
      c.fail(at);
      return finish(c, consumed, detail);
    }
  }
  out->protocol = h;
  if (!c.take(1, skip) || !c.bytes(out->src_ip, 16) || !c.bytes(out->dst_ip, 16) ||
      !c.take(payload_length, out->payload_offset))
    return finish(c, consumed, detail);
  out->payload_length = payload_length;
  return finish(c, consumed, detail);
}

npr_status npr_arp_parse(const uint8_t *input, size_t len, npr_arp *out, size_t *consumed, uint64_t *detail) {
  if (!out || (!input && len)) return NPR_ERR_ARG;
  memset(out, 0, sizeof(*out));
  Cursor c{input, len};
  uint16_t hw_type, proto_type;
  uint8_t hw_len, proto_len;
  if (!c.u16(hw_type) || !c.u16(proto_type) || !c.u8(hw_len) || !c.u8(proto_len) || !c.u16(out->operation) ||
      !c.bytes(out->sender_mac, 6) || !c.bytes(out->sender_ip, 4) || !c.bytes(out->target_mac, 6) ||
      !c.bytes(out->target_ip, 4))
    return finish(c, consumed, detail);
  return finish(c, consumed, detail);
}

npr_status npr_tcp_parse(const uint8_t *input, size_t len, npr_tcp *out, size_t *consumed, uint64_t *detail) {
  if (!out || (!input && len)) return NPR_ERR_ARG;
  memset(out, 0, sizeof(*out));
  Cursor c{input, len};
  if (!c.u16(out->src_port) || !c.u16(out->dst_port) || !c.u32(out->sequence_number) ||
      !c.u32(out->acknowledgement_number))
    return finish(c, consumed, detail);
  const size_t at = c.i;
  uint16_t v;
  if (!c.u16(v)) return finish(c, consumed, detail);
  const uint32_t hl = (uint32_t)(v >> 12) * 4u;  // Tcp::extract_length
  if (hl < 20 || hl > 60) {  // map_res! -> Err
    c.fail(at);
    return finish(c, consumed, detail);
  }
  out->header_length_and_flags = v;
  out->header_length = hl;
  out->flags = v & 0x01FF;
  if (!c.u16(out->window) || !c.u16(out->check) || !c.u16(out->urgent) || !c.take(hl - 20, out->options_offset))
    return finish(c, consumed, detail);
  out->options_length = hl - 20;
  out->payload_offset = c.i;  // rest
  out->payload_length = len - c.i;
  c.i = len;
  return finish(c, consumed, detail);
}

npr_status npr_udp_parse(const uint8_t *input, size_t len, npr_udp *out, size_t *consumed, uint64_t *detail) {
  if (!out || (!input && len)) return NPR_ERR_ARG;
  memset(out, 0, sizeof(*out));
  Cursor c{input, len};
  uint16_t length;
  if (!c.u16(out->src_port) || !c.u16(out->dst_port) || !c.u16(length) || !c.u16(out->checksum))
    return finish(c, consumed, detail);
  const uint64_t payload = (uint64_t)length - 8u;  // (s as usize) - HEADER_LENGTH, wrapping below 8
  if (!c.take(payload, out->payload_offset)) return finish(c, consumed, detail);
  out->payload_length = payload;
  return finish(c, consumed, detail);
}

npr_status npr_vxlan_parse(const uint8_t *input, size_t len, npr_endianness endianness, npr_vxlan *out,
                           size_t *consumed, uint64_t *detail) {
  if (!out || (!input && len)) return NPR_ERR_ARG;
  memset(out, 0, sizeof(*out));
  Cursor c{input, len};
  const bool big = endianness == NPR_BIG;
  if (!c.u16(out->flags, big) || !c.u16(out->group_policy_id, big) || !c.u32(out->raw_network_identifier, big))
    return finish(c, consumed, detail);
  out->network_identifier = out->raw_network_identifier >> 8;
  out->payload_offset = c.i;  // rest
  out->payload_length = len - c.i;
  c.i = len;
  return finish(c, consumed, detail);
}

}  // extern "C"
