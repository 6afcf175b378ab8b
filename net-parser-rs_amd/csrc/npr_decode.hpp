// npr_decode.hpp — the general per-record decode tree, FlowExtraction::extract_flow
// (src/flow/mod.rs:23-41) as one straight-line function, compiled for the device (the kernels in
// npr_kernels.hip) and for the host (tests/host_decode: the same code checked against the oracle on
// the CPU).  Only the decoder's byte reader differs between the two.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/npr.h"

namespace npr {

#define NPR_HD __host__ __device__ __forceinline__

NPR_HD uint32_t be16_of(uint32_t w) { return ((w & 0xffu) << 8) | ((w >> 8) & 0xffu); }

// ---------------------------------------------------------------------------------------------
// per-record decode: FlowExtraction::extract_flow (src/flow/mod.rs:23-41) as one straight-line
// function.  Returns an npr_flow_status; with FIELDS it also fills the 32-B npr_flow words
// (d[0..6]; the record offset goes in by the caller) and the IPv6 addresses.
// Length checks are ordered exactly like the reference's do_parse! steps so the FIRST failing
// step decides between Incomplete / Failure / Custom.
// ---------------------------------------------------------------------------------------------
struct FlowWords {
  uint32_t d[8];  // d[7] unused: keeps put_flow's 16-B row halves inside d (else the widened load spans into v6 and pins both in scratch)
  uint32_t v6[8];
  uint32_t v6off;  // payload offset of the IPv6 address block (the resident kernel re-reads it)
  uint32_t l4off;  // payload offset of the L4 header (decode<> only; the VXLAN path reads past it)
};

// InternetProtocolId::new (src/layer3/mod.rs:54-72)
NPR_HD bool proto_known(uint32_t v) {
  return v == 0 || v == 1 || v == 6 || v == 17 || v == 43 || v == 44 || v == 50 || v == 51 ||
         v == 59 || v == 60;
}
// InternetProtocolId::has_next_option (src/layer3/mod.rs:74-84)
NPR_HD bool proto_has_next(uint32_t v) {
  return v == 0 || v == 43 || v == 44 || v == 50 || v == 51 || v == 60;
}

// DETAIL (the error-payload kernel only; compiled out everywhere else): *det = the payload the
// reference's error variant carries for the returned status (include/npr.h npr_flow_detail):
//   Incomplete of a nom primitive -> its Needed::Size (nom 4: the primitive's full size, take!(k) -> k)
//   a remainder left after a layer  -> rem.len()        (src/flow/layer2/ethernet.rs:67-76 ...)
//   map_opt! / map_res! failures    -> the frame offsets [start, end) of the failing primitive's input
//                                      (nom's error position and its parser's input end): start | end << 32
//   version != 4 / 6                -> the version nibble (the Custom message's value)
//   LLDP / 802.3 length             -> the EtherType;  IP protocol not TCP/UDP -> the protocol id
// Primitive sizes of the fixed headers, in parse order (the first one that does not fit is the
// Incomplete one):
// (template arguments, not tables: no array has to live in device memory)
template <unsigned... S>
NPR_HD uint64_t first_short(uint64_t avail) {
  uint64_t end = 0, r = 0;
  bool found = false;
  ((end += S, (!found && end > avail) ? (r = S, found = true) : false), ...);
  return r;
}
#define NPR_NEED_IPV4 1, 1, 2, 2, 2, 1, 1, 2, 4, 4  // src/layer3/ipv4.rs:96-122
#define NPR_NEED_IPV6 1, 3, 2, 1                    // src/layer3/ipv6.rs:58-66, :90
#define NPR_NEED_IPV6_TAIL 1, 16, 16                // src/layer3/ipv6.rs:41-43
#define NPR_NEED_ARP 2, 2, 1, 1, 2, 6, 4, 6, 4      // src/layer3/arp.rs:55-64
#define NPR_NEED_TCP 2, 2, 4, 4, 2, 2, 2, 2         // src/layer4/tcp.rs:64-86
#define NPR_NEED_UDP 2, 2, 2, 2                     // src/layer4/udp.rs:38-41
// det is volatile: every fail() site stores its own value.  (With a plain pointer the gfx950 build
// merged the payload into one 64-bit value across the decoder's divergent returns and stored wrong
// payloads, while the host build of the same source matched the oracle -- tests/host_decode.)
template <bool DETAIL>
NPR_HD uint32_t fail(volatile uint64_t *det, uint32_t code, uint64_t v) {
  if (DETAIL) *det = v;
  return code;
}

template <bool FIELDS, class R, bool DETAIL = false>
NPR_HD uint32_t decode(const R &r, uint32_t n, FlowWords &f, volatile uint64_t *det = nullptr) {
  if (DETAIL) *det = 0;
  // ---- Ethernet::parse (src/layer2/ethernet.rs:204-216): two mac_address (take!(6))
  if (n < 12) return fail<DETAIL>(det, NPR_FLOW_ETH_INCOMPLETE, 6);
  uint32_t m0 = 0, m1 = 0, m2 = 0;
  if (FIELDS) {
    m0 = r.le32(0);  // dst[0..3]
    m1 = r.le32(4);  // dst[4..5] src[0..1]
    m2 = r.le32(8);  // src[2..5]
  }
  // parse_vlan_tag recursion (:163-202): map_opt!(be_u16, EthernetTypeId::new), 802.1Q/ad tags
  uint32_t pos = 12, vlan = 0, etype;
  bool tagged = false;
  for (;;) {
    if (n - pos < 2) return fail<DETAIL>(det, NPR_FLOW_ETH_INCOMPLETE, 2);
    const uint32_t w = r.le32(pos);
    const uint32_t t = be16_of(w);
    if (t != 0x8100u && t != 0x88a8u) {
      // EthernetTypeId::new (:57-73): LLDP / IPv4 / IPv6 / ARP / <=1500 (length), else None
      if (!(t == 0x88ccu || t == 0x0800u || t == 0x86ddu || t == 0x0806u || t <= 1500u))
        return fail<DETAIL>(det, NPR_FLOW_ETH_FAILURE, pos | ((uint64_t)n << 32));
      etype = t;
      pos += 2;
      break;
    }
    if (n - pos - 2 < 2) return fail<DETAIL>(det, NPR_FLOW_ETH_INCOMPLETE, 2);  // TCI: be_u16 (:176)
    if (!tagged) vlan = be16_of(w >> 16) & 0x0FFFu;                             // vlans_to_vlan: first tag (:134-137)
    tagged = true;
    pos += 4;
  }
  // ---- layer-3 dispatch (src/flow/layer2/ethernet.rs:55-131); payload = rest
  const uint32_t l3 = pos, n3 = n - pos;
  uint32_t l4, n4, proto;
  bool v6;
  if (etype == 0x0800u) {
    // IPv4::parse (src/layer3/ipv4.rs:148-160) -> parse_ipv4 (:76-146)
    if (n3 < 1) return fail<DETAIL>(det, NPR_FLOW_L2_IPV4_INCOMPLETE, 1);
    const uint32_t w0 = r.le32(l3);
    const uint32_t b0 = w0 & 0xffu;
    if ((b0 >> 4) != 4u) return fail<DETAIL>(det, NPR_FLOW_L2_IPV4_CUSTOM, b0 >> 4);
    const uint32_t hw = b0 & 0x0Fu, hl = hw * 4u, add = hw > 5u ? (hw - 5u) * 4u : 0u;
    if (n3 < 4) return fail<DETAIL>(det, NPR_FLOW_L2_IPV4_INCOMPLETE, DETAIL ? first_short<NPR_NEED_IPV4>(n3) : 0);  // tos, length
    const uint32_t length = (be16_of(w0 >> 16) - hl) & 0xffffu;  // u16 wrapping (:100)
    const uint64_t expected = (uint64_t)hl + add + length;        // (:107)
    if (n3 < 10) return fail<DETAIL>(det, NPR_FLOW_L2_IPV4_INCOMPLETE, DETAIL ? first_short<NPR_NEED_IPV4>(n3) : 0);
    proto = (r.le32(l3 + 8) >> 8) & 0xffu;
    if (!proto_known(proto)) return fail<DETAIL>(det, NPR_FLOW_L2_IPV4_FAILURE, (l3 + 9u) | ((uint64_t)n << 32));  // map_opt! (:119)
    if (n3 < 20) return fail<DETAIL>(det, NPR_FLOW_L2_IPV4_INCOMPLETE, DETAIL ? first_short<NPR_NEED_IPV4>(n3) : 0);
    if (n3 - 20u < length) return fail<DETAIL>(det, NPR_FLOW_L2_IPV4_INCOMPLETE, length);  // payload: take!(length)
    uint64_t p4 = 20ull + length;
    if (add) {                                                // options (:124)
      if ((uint64_t)n3 - p4 < add) return fail<DETAIL>(det, NPR_FLOW_L2_IPV4_INCOMPLETE, add);
      p4 += add;
    }
    if ((uint64_t)n3 > expected) {                            // padding (:125-129)
      const uint64_t pad = (uint64_t)n3 - expected;
      if ((uint64_t)n3 - p4 < pad) return fail<DETAIL>(det, NPR_FLOW_L2_IPV4_INCOMPLETE, pad);
      p4 += pad;
    }
    if (p4 != n3) return fail<DETAIL>(det, NPR_FLOW_L2_IPV4_REMAINDER, (uint64_t)n3 - p4);  // rem.is_empty() (:67-76)
    if (FIELDS) {
      f.d[0] = r.le32(l3 + 12);
      f.d[1] = r.le32(l3 + 16);
    }
    l4 = l3 + 20u;  // the L4 parse starts right after the fixed header (quirk Q7)
    n4 = length;
    v6 = false;
  } else if (etype == 0x86ddu) {
    // IPv6::parse (src/layer3/ipv6.rs:87-99) -> parse_ipv6 (:58-71) -> parse_next_header (:29-56)
    if (n3 < 1) return fail<DETAIL>(det, NPR_FLOW_L2_IPV6_INCOMPLETE, 1);
    if ((r.u8(l3) >> 4) != 6u) return fail<DETAIL>(det, NPR_FLOW_L2_IPV6_CUSTOM, r.u8(l3) >> 4);
    if (n3 < 7) return fail<DETAIL>(det, NPR_FLOW_L2_IPV6_INCOMPLETE, DETAIL ? first_short<NPR_NEED_IPV6>(n3) : 0);  // take!(3), be_u16, be_u8
    const uint32_t w1 = r.le32(l3 + 4);
    const uint32_t plen = be16_of(w1);
    uint32_t nh = (w1 >> 16) & 0xffu;
    if (!proto_known(nh)) return fail<DETAIL>(det, NPR_FLOW_L2_IPV6_FAILURE, (l3 + 6u) | ((uint64_t)n << 32));
    uint32_t p = 7;
    while (proto_has_next(nh)) {                              // one byte per extension (quirk Q11)
      if (n3 - p < 1) return fail<DETAIL>(det, NPR_FLOW_L2_IPV6_INCOMPLETE, 1);
      nh = r.u8(l3 + p);
      if (!proto_known(nh)) return fail<DETAIL>(det, NPR_FLOW_L2_IPV6_FAILURE, (l3 + p) | ((uint64_t)n << 32));
      ++p;
    }
    if (n3 - p < 33u)                                          // hop limit, src, dst
      return fail<DETAIL>(det, NPR_FLOW_L2_IPV6_INCOMPLETE, DETAIL ? first_short<NPR_NEED_IPV6_TAIL>(n3 - p) : 0);
    const uint32_t sa = l3 + p + 1u;
    p += 33u;
    if (n3 - p < plen) return fail<DETAIL>(det, NPR_FLOW_L2_IPV6_INCOMPLETE, plen);  // payload: take!(p)
    if (n3 - p != plen) return fail<DETAIL>(det, NPR_FLOW_L2_IPV6_REMAINDER, n3 - p - plen);
    if (FIELDS) {
#pragma unroll
      for (int k = 0; k < 8; ++k) f.v6[k] = r.le32(sa + 4u * (uint32_t)k);
      f.v6off = sa;
      f.d[0] = 0;
      f.d[1] = 0;
    }
    l4 = l3 + p;
    n4 = plen;
    proto = nh;
    v6 = true;
  } else if (etype == 0x0806u) {
    // Arp::parse: 28 fixed bytes (src/layer3/arp.rs:54-76); the flow is always Err
    if (n3 < 28) return fail<DETAIL>(det, NPR_FLOW_L2_ARP_INCOMPLETE, DETAIL ? first_short<NPR_NEED_ARP>(n3) : 0);
    if (n3 != 28) return fail<DETAIL>(det, NPR_FLOW_L2_ARP_REMAINDER, n3 - 28u);
    return NPR_FLOW_L3_ARP;
  } else {
    return fail<DETAIL>(det, NPR_FLOW_L2_ETHERTYPE, etype);  // LLDP / PayloadLength (:125-130)
  }
  // ---- layer-4 dispatch (src/flow/layer3/ipv4.rs:49-101, ipv6.rs:49-100)
  bool udp;
  if (proto == 6u) {
    // Tcp::parse (src/layer4/tcp.rs:59-101)
    const uint32_t inc = v6 ? NPR_FLOW_L3_IPV6_TCP_INCOMPLETE : NPR_FLOW_L3_IPV4_TCP_INCOMPLETE;
    if (n4 < 14) return fail<DETAIL>(det, inc, DETAIL ? first_short<NPR_NEED_TCP>(n4) : 0);
    const uint32_t thl = (be16_of(r.le32(l4 + 12)) >> 12) * 4u;  // extract_length (:54-57)
    if (thl < 20u || thl > 60u)  // map_res! (:68): the error's position is the be_u16's input
      return fail<DETAIL>(det, v6 ? NPR_FLOW_L3_IPV6_TCP_FAILURE : NPR_FLOW_L3_IPV4_TCP_FAILURE,
                         (l4 + 12u) | ((uint64_t)(l4 + n4) << 32));
    if (n4 < thl) return fail<DETAIL>(det, inc, DETAIL ? (n4 < 20u ? first_short<NPR_NEED_TCP>(n4) : thl - 20u) : 0);
    udp = false;  // payload: rest -> never a remainder
  } else if (proto == 17u) {
    // Udp::parse (src/layer4/udp.rs:33-50): take!(length - 8) with usize wrapping
    const uint32_t inc = v6 ? NPR_FLOW_L3_IPV6_UDP_INCOMPLETE : NPR_FLOW_L3_IPV4_UDP_INCOMPLETE;
    if (n4 < 8) return fail<DETAIL>(det, inc, DETAIL ? first_short<NPR_NEED_UDP>(n4) : 0);
    const uint32_t L = be16_of(r.le32(l4 + 4));
    if (L < 8u || n4 - 8u < L - 8u) return fail<DETAIL>(det, inc, (uint64_t)L - 8ull);  // (usize wrap below 8)
    if (n4 != L)
      return fail<DETAIL>(det, v6 ? NPR_FLOW_L3_IPV6_UDP_REMAINDER : NPR_FLOW_L3_IPV4_UDP_REMAINDER, n4 - L);
    udp = true;
  } else {
    return fail<DETAIL>(det, v6 ? NPR_FLOW_L3_IPV6_PROTOCOL : NPR_FLOW_L3_IPV4_PROTOCOL, proto);
  }
  if (FIELDS) {  // Flow::new (src/flow/mod.rs:64-86)
    f.l4off = l4;
    const uint32_t wp = r.le32(l4);
    f.d[2] = be16_of(wp) | (be16_of(wp >> 16) << 16);
    f.d[3] = vlan | (m1 & 0xffff0000u);
    f.d[4] = m2;
    f.d[5] = m0;
    f.d[6] = (m1 & 0xffffu) | (((v6 ? NPR_FLOW_KIND_IPV6 : 0u) | (udp ? NPR_FLOW_KIND_UDP : 0u)) << 16);
  }
  return NPR_FLOW_OK;
}


#undef NPR_HD
#undef NPR_NEED_IPV4
#undef NPR_NEED_IPV6
#undef NPR_NEED_IPV6_TAIL
#undef NPR_NEED_ARP
#undef NPR_NEED_TCP
#undef NPR_NEED_UDP

}  // namespace npr
