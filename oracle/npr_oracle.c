/*
 * npr_oracle.c — PARITY ORACLE, TEST INFRASTRUCTURE ONLY (see npr_oracle.h for pinning).
 *
 * Every parser below is written as the reference's nom do_parse! chain, one step per line,
 * in the same order, so "which error comes first" matches the reference.  Cursor convention:
 * `pos` bytes consumed out of `n`; NEED(k) is the Incomplete check of a k-byte primitive.
 */
#include "npr_oracle.h"

#include <string.h>

/* The error payload of the last failing step (npr.h "npr_flow_details"): g_need = the failing
 * primitive's Needed::Size (nom 4.2 primitives report their full size: be_u16 -> 2, take!(k) -> k),
 * g_fail = the input position (in the failing parser's own input) of a map_opt! / map_res! failure.
 * Thread-local: the bench leg runs the parsers on several threads. */
static _Thread_local uint64_t g_need, g_fail;

#define NEED(k)                                                                                    \
  do {                                                                                             \
    if ((size_t)(n - pos) < (size_t)(k)) {                                                         \
      g_need = (uint64_t)(size_t)(k);                                                              \
      return OR_INCOMPLETE;                                                                        \
    }                                                                                              \
  } while (0)

static uint16_t rd_be16(const uint8_t *p) { return (uint16_t)((p[0] << 8) | p[1]); }
static uint32_t rd_be32(const uint8_t *p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
static uint32_t rd_le32(const uint8_t *p) {
  return ((uint32_t)p[3] << 24) | ((uint32_t)p[2] << 16) | ((uint32_t)p[1] << 8) | p[0];
}
static uint32_t rd_u32(const uint8_t *p, int big) { return big ? rd_be32(p) : rd_le32(p); }
static uint16_t rd_u16(const uint8_t *p, int big) {
  return big ? rd_be16(p) : (uint16_t)(p[0] | (p[1] << 8));
}

/* ---- src/global_header.rs:40-70 ---------------------------------------------------------- */
int or_global_header_parse(const uint8_t *in, size_t n, npr_global_header *out, size_t *consumed) {
  size_t pos = 0;
  /* u32!(NATIVE_ENDIAN) on a little-endian host; == MAGIC (0xA1B2C3D4) => native (Little),
   * anything else => Big (global_header.rs:43-53). */
  NEED(4);
  uint32_t e = rd_le32(in);
  int big = (e == 0xA1B2C3D4u) ? 0 : 1;
  pos += 4;
  NEED(2); uint16_t vmaj = rd_u16(in + pos, big); pos += 2;   /* version_major :54 */
  NEED(2); uint16_t vmin = rd_u16(in + pos, big); pos += 2;   /* version_minor :55 */
  NEED(4); int32_t zone = (int32_t)rd_u32(in + pos, big); pos += 4; /* zone :56 */
  NEED(4); int32_t sig = (int32_t)rd_u32(in + pos, big); pos += 4;  /* sig_figs :57 */
  NEED(4); uint32_t snap = rd_u32(in + pos, big); pos += 4;   /* snap_length :58 */
  NEED(4); uint32_t net = rd_u32(in + pos, big); pos += 4;    /* network :59 */
  out->endianness = big ? NPR_BIG : NPR_LITTLE;
  out->version_major = vmaj;
  out->version_minor = vmin;
  out->zone = zone;
  out->sig_figs = sig;
  out->snap_length = snap;
  out->network = net;
  if (consumed) *consumed = pos;
  return OR_OK;
}

/* ---- src/record.rs:102-121 --------------------------------------------------------------- */
int or_record_parse(const uint8_t *in, size_t n, int big, npr_record *out, size_t *consumed) {
  size_t pos = 0;
  NEED(4); uint32_t ts_s = rd_u32(in + pos, big); pos += 4;   /* ts_seconds :107 */
  NEED(4); uint32_t ts_u = rd_u32(in + pos, big); pos += 4;   /* ts_microseconds :108 */
  NEED(4); uint32_t incl = rd_u32(in + pos, big); pos += 4;   /* actual_length :109 */
  NEED(4); uint32_t orig = rd_u32(in + pos, big); pos += 4;   /* original_length :110 */
  NEED(incl); pos += incl;                                      /* payload: take!(actual_length) :111 */
  out->offset = 0;
  out->ts_sec = ts_s;
  out->ts_usec = ts_u;
  out->actual_length = incl;
  out->original_length = orig;
  if (consumed) *consumed = pos;
  return OR_OK;
}

/* ---- src/record.rs:21-54: loop until the first Incomplete (no other error is possible) --- */
size_t or_records_parse(const uint8_t *in, size_t len, int big, npr_record *out, size_t cap,
                        size_t *consumed) {
  size_t cur = 0, count = 0;
  for (;;) {
    npr_record r;
    size_t used = 0;
    if (or_record_parse(in + cur, len - cur, big, &r, &used) != OR_OK) break; /* :37-45 */
    r.offset = cur;
    if (count < cap) out[count] = r;
    count++;
    cur += used; /* current = rem :33 */
  }
  if (consumed) *consumed = cur;
  return count;
}

/* ---- src/file.rs:14-35 -------------------------------------------------------------------- */
int or_capture_file_parse(const uint8_t *in, size_t len, npr_global_header *hdr, npr_record *out,
                          size_t cap, size_t *n_out, size_t *consumed) {
  size_t used = 0;
  int rc = or_global_header_parse(in, len, hdr, &used); /* :18 */
  if (rc != OR_OK) return rc;
  size_t cons = 0;
  size_t n = or_records_parse(in + used, len - used, hdr->endianness == NPR_BIG, out,
                              cap, &cons); /* :27 */
  for (size_t i = 0; i < n && i < cap; ++i) out[i].offset += used;
  if (n_out) *n_out = n;
  if (consumed) *consumed = used + cons;
  return OR_OK;
}

/* ---- L2: src/layer2/ethernet.rs ----------------------------------------------------------- */
/* EthernetTypeId::new (:57-73): 0 = unknown, 1 = vlan, 2 = L3/payload-length */
static int eth_type_class(uint16_t t) {
  switch (t) {
  case 0x8100: case 0x88a8: return 1;
  case 0x88cc: case 0x0800: case 0x86dd: case 0x0806: return 2;
  default: return t <= 1500 ? 2 : 0;
  }
}

int or_eth_parse(const uint8_t *in, size_t n, or_eth *v) {
  size_t pos = 0;
  NEED(6); v->dst_mac = in + pos; pos += 6; /* mac_address :114, :209 */
  NEED(6); v->src_mac = in + pos; pos += 6; /* :209 */
  v->vlan = 0;
  v->n_vlans = 0;
  for (;;) { /* parse_vlan_tag recursion (:163-202) */
    NEED(2);
    uint16_t t = rd_be16(in + pos); pos += 2;   /* map_opt!(be_u16, EthernetTypeId::new) :170 */
    int cls = eth_type_class(t);
    if (cls == 0) { g_fail = pos - 2; return OR_FAILURE; } /* map_opt!'s input: the type field */
    if (cls == 1) {
      NEED(2);
      uint16_t tci = rd_be16(in + pos); pos += 2; /* total: be_u16 :176 */
      if (v->n_vlans == 0) v->vlan = tci & 0x0FFF; /* id :181, first tag :135 */
      v->n_vlans++;
      continue;
    }
    v->ether_type = t;
    v->payload_off = pos; /* parse_not_vlan_tag: payload = rest (:150) */
    return OR_OK;
  }
}

/* ---- L3 ids: src/layer3/mod.rs:54-84 ------------------------------------------------------ */
static int ip_proto_known(uint8_t v) {
  switch (v) {
  case 0: case 1: case 6: case 17: case 43: case 44: case 50: case 51: case 59: case 60: return 1;
  default: return 0;
  }
}
static int ip_proto_has_next(uint8_t v) {
  return v == 50 || v == 51 || v == 0 || v == 43 || v == 44 || v == 60;
}

/* ---- src/layer3/ipv4.rs:76-160 ------------------------------------------------------------ */
int or_ipv4_parse(const uint8_t *in, size_t n, or_ip *v) {
  size_t pos = 0;
  NEED(1);
  uint8_t val = in[0]; pos = 1;                               /* be_u8 :151 */
  if ((val >> 4) != 4) return OR_CUSTOM;                      /* :153-157 */
  const size_t input_length = n;                              /* :149 */
  uint8_t header_words = val & 0x0F;                          /* :81 */
  uint8_t header_length = (uint8_t)(header_words * 4);        /* :82 */
  uint8_t additional_length = header_words > 5 ? (uint8_t)((header_words - 5) * 4) : 0; /* :83-87 */
  NEED(1); pos += 1;                                          /* tos :98 */
  NEED(2);
  uint16_t raw_length = rd_be16(in + pos); pos += 2;          /* :99 */
  uint16_t length = (uint16_t)(raw_length - (uint16_t)header_length); /* wrapping :100 */
  size_t expected_length = (size_t)header_length + additional_length + length; /* :107 */
  NEED(2); pos += 2;                                          /* id :116 */
  NEED(2); pos += 2;                                          /* flags :117 */
  NEED(1); pos += 1;                                          /* ttl :118 */
  NEED(1);
  uint8_t protocol = in[pos]; pos += 1;                       /* map_opt! :119 */
  if (!ip_proto_known(protocol)) { g_fail = pos - 1; return OR_FAILURE; }
  NEED(2); pos += 2;                                          /* checksum :120 */
  NEED(4); v->src = in + pos; pos += 4;                       /* src_ip :121 */
  NEED(4); v->dst = in + pos; pos += 4;                       /* dst_ip :122 */
  NEED(length); v->payload_off = pos; v->payload_len = length; pos += length; /* :123 */
  if (additional_length > 0) { NEED(additional_length); pos += additional_length; } /* :124 */
  if (input_length > expected_length) {                       /* :125-129 */
    size_t pad = input_length - expected_length;
    NEED(pad); pos += pad;
  }
  v->protocol = protocol;
  v->rem = n - pos;
  return OR_OK;
}

/* ---- src/layer3/ipv6.rs:29-99 ------------------------------------------------------------- */
int or_ipv6_parse(const uint8_t *in, size_t n, or_ip *v) {
  size_t pos = 0;
  NEED(1);
  uint8_t b0 = in[0]; pos = 1;                                /* be_u8 :90 */
  if ((b0 >> 4) != 6) return OR_CUSTOM;                       /* :92-97 */
  NEED(3); pos += 3;                                          /* _f: take!(3) :61 */
  NEED(2); uint16_t payload_length = rd_be16(in + pos); pos += 2; /* p: be_u16 :62 */
  NEED(1); uint8_t nh = in[pos]; pos += 1;                    /* h: map_opt! :63 */
  if (!ip_proto_known(nh)) { g_fail = pos - 1; return OR_FAILURE; }
  while (ip_proto_has_next(nh)) {                             /* parse_next_header :34-37 */
    NEED(1); nh = in[pos]; pos += 1;                          /* map_opt!(be_u8, ..) :35 */
    if (!ip_proto_known(nh)) { g_fail = pos - 1; return OR_FAILURE; }
  }
  NEED(1); pos += 1;                                          /* _h: take!(1) hop limit :41 */
  NEED(16); v->src = in + pos; pos += 16;                     /* :42 */
  NEED(16); v->dst = in + pos; pos += 16;                     /* :43 */
  NEED(payload_length);
  v->payload_off = pos; v->payload_len = payload_length; pos += payload_length; /* :44 */
  v->protocol = nh;
  v->rem = n - pos;
  return OR_OK;
}

/* ---- src/layer3/arp.rs:54-76 ------------------------------------------------------------- */
int or_arp_parse(const uint8_t *in, size_t n, or_arp *v) {
  size_t pos = 0;
  NEED(2); pos += 2; NEED(2); pos += 2;                       /* hardware / protocol type :56-57 */
  NEED(1); pos += 1; NEED(1); pos += 1;                       /* address lengths :58-59 */
  NEED(2); v->operation = rd_be16(in + pos); pos += 2;        /* operation :60 */
  NEED(6); v->sender_mac = in + pos; pos += 6;                /* :61 */
  NEED(4); v->sender_ip = in + pos; pos += 4;                 /* :62 */
  NEED(6); v->target_mac = in + pos; pos += 6;                /* :63 */
  NEED(4); v->target_ip = in + pos; pos += 4;                 /* :64 */
  v->rem = n - pos;
  return OR_OK;
}

/* ---- src/layer4/tcp.rs:59-101 ------------------------------------------------------------- */
size_t or_tcp_extract_length(uint16_t value) { return (size_t)((value >> 12) * 4); } /* :54-57 */

int or_tcp_parse(const uint8_t *in, size_t n, or_l4 *v) {
  size_t pos = 0;
  NEED(2); v->src_port = rd_be16(in + pos); pos += 2;         /* src_port :64 */
  NEED(2); v->dst_port = rd_be16(in + pos); pos += 2;         /* dst_port :65 */
  NEED(4); pos += 4; NEED(4); pos += 4;                       /* seq / ack :66-67 */
  NEED(2);
  uint16_t hv = rd_be16(in + pos); pos += 2;                  /* map_res!(be_u16, ..) :68 */
  size_t hl = or_tcp_extract_length(hv);                      /* extract_length :54-57 */
  if (!(hl >= 20 && hl <= 60)) { g_fail = pos - 2; return OR_FAILURE; } /* map_res! :71-82 */
  NEED(2); pos += 2; NEED(2); pos += 2; NEED(2); pos += 2;    /* window/check/urgent :84-86 */
  NEED(hl - 20); pos += hl - 20;                              /* options :87 */
  v->header_length = hl;
  v->payload_off = pos; v->payload_len = n - pos;             /* payload: rest :88 */
  v->rem = 0;
  return OR_OK;
}

/* ---- src/layer4/udp.rs:33-50 -------------------------------------------------------------- */
int or_udp_parse(const uint8_t *in, size_t n, or_l4 *v) {
  size_t pos = 0;
  NEED(2); v->src_port = rd_be16(in + pos); pos += 2;         /* :38 */
  NEED(2); v->dst_port = rd_be16(in + pos); pos += 2;         /* :39 */
  NEED(2);
  size_t length = (size_t)rd_be16(in + pos) - 8;              /* wrapping usize :40 */
  pos += 2;
  NEED(2); pos += 2;                                          /* checksum :41 */
  NEED(length); v->payload_off = pos; v->payload_len = length; pos += length; /* take! :42 */
  v->header_length = 8;
  v->rem = n - pos;
  return OR_OK;
}

static void put_offset(npr_flow *f, uint64_t off) {
  for (int i = 0; i < 5; ++i) f->record_offset[i] = (uint8_t)(off >> (8 * i));
}

/* ---- src/flow/mod.rs:23-41 + src/flow/layer{2,3,4}/ (per-layer impls) ---------------------------------- */
/* l4 / l4n (optional): the L4 header's start and length (the IP payload) of an Ok flow */
static int extract_flow_l4(const uint8_t *p, size_t n, uint64_t record_offset, npr_flow *f, npr_flow_v6 *v6,
                           const uint8_t **l4_out, size_t *l4n_out, uint64_t *det) {
  uint64_t dummy;
  if (!det) det = &dummy;
  *det = 0;
  or_eth e;
  int rc = or_eth_parse(p, n, &e); /* Ethernet::parse, mod.rs:28-31 */
  if (rc == OR_INCOMPLETE) { *det = g_need; return NPR_FLOW_ETH_INCOMPLETE; }
  if (rc != OR_OK) { *det = g_fail | ((uint64_t)n << 32); return NPR_FLOW_ETH_FAILURE; }
  /* rem is always empty (payload = rest), so mod.rs:33-40 never fails. */
  const uint8_t *l3 = p + e.payload_off;
  size_t l3n = n - e.payload_off;
  or_ip ip;
  int v6flag;
  switch (e.ether_type) { /* flow/layer2/ethernet.rs:55-131 */
  case 0x0800:
    rc = or_ipv4_parse(l3, l3n, &ip);
    if (rc == OR_INCOMPLETE) { *det = g_need; return NPR_FLOW_L2_IPV4_INCOMPLETE; }
    if (rc == OR_FAILURE) { *det = (e.payload_off + g_fail) | ((uint64_t)n << 32); return NPR_FLOW_L2_IPV4_FAILURE; }
    if (rc == OR_CUSTOM) { *det = l3[0] >> 4; return NPR_FLOW_L2_IPV4_CUSTOM; }
    if (ip.rem != 0) { *det = ip.rem; return NPR_FLOW_L2_IPV4_REMAINDER; } /* :67-76 */
    v6flag = 0;
    break;
  case 0x86dd:
    rc = or_ipv6_parse(l3, l3n, &ip);
    if (rc == OR_INCOMPLETE) { *det = g_need; return NPR_FLOW_L2_IPV6_INCOMPLETE; }
    if (rc == OR_FAILURE) { *det = (e.payload_off + g_fail) | ((uint64_t)n << 32); return NPR_FLOW_L2_IPV6_FAILURE; }
    if (rc == OR_CUSTOM) { *det = l3[0] >> 4; return NPR_FLOW_L2_IPV6_CUSTOM; }
    if (ip.rem != 0) { *det = ip.rem; return NPR_FLOW_L2_IPV6_REMAINDER; } /* :91-100 */
    v6flag = 1;
    break;
  case 0x0806: {
    or_arp a;
    if (or_arp_parse(l3, l3n, &a) != OR_OK) { *det = g_need; return NPR_FLOW_L2_ARP_INCOMPLETE; } /* :104-111 */
    if (a.rem != 0) { *det = a.rem; return NPR_FLOW_L2_ARP_REMAINDER; }                           /* :112-122 */
    return NPR_FLOW_L3_ARP;                                               /* layer3/arp.rs:24-26 */
  }
  default:
    *det = e.ether_type;
    return NPR_FLOW_L2_ETHERTYPE; /* LLDP / PayloadLength :125-130 */
  }
  /* flow/layer3/ipv4.rs:49-101 and flow/layer3/ipv6.rs:49-100 */
  const uint8_t *l4 = l3 + ip.payload_off;
  size_t l4n = ip.payload_len;
  or_l4 t;
  int udp;
  if (ip.protocol == 6) {
    rc = or_tcp_parse(l4, l4n, &t);
    if (rc == OR_INCOMPLETE) { *det = g_need; return v6flag ? NPR_FLOW_L3_IPV6_TCP_INCOMPLETE : NPR_FLOW_L3_IPV4_TCP_INCOMPLETE; }
    if (rc != OR_OK) {
      *det = ((uint64_t)(l4 - p) + g_fail) | ((uint64_t)(l4 - p + l4n) << 32); /* the TCP input is the IP payload */
      return v6flag ? NPR_FLOW_L3_IPV6_TCP_FAILURE : NPR_FLOW_L3_IPV4_TCP_FAILURE;
    }
    udp = 0;
  } else if (ip.protocol == 17) {
    rc = or_udp_parse(l4, l4n, &t);
    if (rc != OR_OK) { *det = g_need; return v6flag ? NPR_FLOW_L3_IPV6_UDP_INCOMPLETE : NPR_FLOW_L3_IPV4_UDP_INCOMPLETE; }
    if (t.rem != 0) { *det = t.rem; return v6flag ? NPR_FLOW_L3_IPV6_UDP_REMAINDER : NPR_FLOW_L3_IPV4_UDP_REMAINDER; }
    udp = 1;
  } else {
    *det = ip.protocol;
    return v6flag ? NPR_FLOW_L3_IPV6_PROTOCOL : NPR_FLOW_L3_IPV4_PROTOCOL;
  }
  /* Flow::new (flow/mod.rs:64-86) */
  memset(f, 0, sizeof(*f));
  if (!v6flag) {
    memcpy(f->src_ip, ip.src, 4);
    memcpy(f->dst_ip, ip.dst, 4);
  } else if (v6) {
    memcpy(v6->src_ip, ip.src, 16);
    memcpy(v6->dst_ip, ip.dst, 16);
  }
  f->src_port = t.src_port;
  f->dst_port = t.dst_port;
  f->vlan = e.vlan;
  memcpy(f->src_mac, e.src_mac, 6);
  memcpy(f->dst_mac, e.dst_mac, 6);
  f->kind = (uint8_t)((v6flag ? NPR_FLOW_KIND_IPV6 : 0) | (udp ? NPR_FLOW_KIND_UDP : 0));
  put_offset(f, record_offset);
  if (l4_out) *l4_out = l4;
  if (l4n_out) *l4n_out = l4n;
  return NPR_FLOW_OK;
}

int or_extract_flow(const uint8_t *p, size_t n, uint64_t record_offset, npr_flow *f, npr_flow_v6 *v6) {
  return extract_flow_l4(p, n, record_offset, f, v6, NULL, NULL, NULL);
}

int or_extract_flow_detail(const uint8_t *p, size_t n, uint64_t record_offset, npr_flow *f, npr_flow_v6 *v6,
                           uint64_t *detail) {
  return extract_flow_l4(p, n, record_offset, f, v6, NULL, NULL, detail);
}

/* ---- row f3: src/layer4/vxlan.rs:31-48 (Vxlan::parse) + src/flow/layer4/vxlan.rs:32-50 ----- */
int or_vxlan_parse(const uint8_t *in, size_t n, int big, or_vxlan *v) {
  size_t pos = 0;
  NEED(2); v->flags = rd_u16(in + pos, big); pos += 2;                   /* u16!(endianness) :38 */
  NEED(2); v->group_policy_id = rd_u16(in + pos, big); pos += 2;         /* :39 */
  NEED(4); v->raw_network_identifier = rd_u32(in + pos, big); pos += 4;  /* u32! :40 */
  v->network_identifier = v->raw_network_identifier >> 8;                /* :45 */
  v->payload_off = pos;                                                  /* rest :42 */
  return OR_OK;
}

/* One record: the outer frame's flow must be Ok and UDP (to dst_port unless 0); its UDP payload
 * is a VXLAN header + an inner Ethernet frame, whose flow is the result. */
int or_vxlan_flow(const uint8_t *p, size_t n, uint64_t record_offset, uint32_t dst_port, int big, npr_flow *f,
                  npr_flow_v6 *v6, uint32_t *vni) {
  npr_flow outer;
  const uint8_t *l4 = NULL;
  size_t l4n = 0;
  *vni = 0;
  int st = extract_flow_l4(p, n, record_offset, &outer, NULL, &l4, &l4n, NULL);
  if (st != NPR_FLOW_OK) return st;
  if (!(outer.kind & NPR_FLOW_KIND_UDP)) return NPR_VXLAN_NOT_UDP;
  if (dst_port && outer.dst_port != dst_port) return NPR_VXLAN_PORT;
  or_l4 u;
  if (or_udp_parse(l4, l4n, &u) != OR_OK) return NPR_VXLAN_INNER; /* (an Ok UDP flow re-parses) */
  or_vxlan x;
  if (or_vxlan_parse(l4 + u.payload_off, u.payload_len, big, &x) != OR_OK) return NPR_VXLAN_INCOMPLETE;
  *vni = x.network_identifier;
  /* Ethernet::parse(payload) then l2.extract_flow(); the remainder is always empty (:35-47) */
  const uint8_t *inner = l4 + u.payload_off + x.payload_off;
  st = or_extract_flow(inner, u.payload_len - x.payload_off, record_offset, f, v6);
  return st == NPR_FLOW_OK ? NPR_FLOW_OK : NPR_VXLAN_INNER + st;
}

void or_vxlan_flows(const uint8_t *buf, size_t len, const npr_record *recs, size_t n, uint32_t dst_port, int big,
                    npr_flow *flows, npr_flow_v6 *flows_v6, uint8_t *status, uint32_t *vni) {
  for (size_t i = 0; i < n; ++i) {
    npr_flow f;
    npr_flow_v6 v6;
    uint32_t id = 0;
    memset(&f, 0, sizeof f);
    memset(&v6, 0, sizeof v6);
    const size_t off = (size_t)recs[i].offset + 16, plen = recs[i].actual_length;
    int st = (off > len || len - off < plen) ? -1
                                             : or_vxlan_flow(buf + off, plen, recs[i].offset, dst_port, big, &f, &v6, &id);
    if (st != NPR_FLOW_OK) {
      memset(&f, 0, sizeof f);
      memset(&v6, 0, sizeof v6);
    }
    if (flows) flows[i] = f;
    if (flows_v6) flows_v6[i] = v6;
    if (status) status[i] = (uint8_t)st;
    if (vni) vni[i] = id;
  }
}

static int record_flow(const uint8_t *buf, size_t len, const npr_record *r, npr_flow *f,
                       npr_flow_v6 *v6) {
  size_t off = (size_t)r->offset + 16;
  size_t plen = r->actual_length;
  if (off > len || len - off < plen) return -1; /* not a record of this buffer */
  return or_extract_flow(buf + off, plen, r->offset, f, v6); /* payload() :44-48 */
}

void or_extract_flows(const uint8_t *buf, size_t len, const npr_record *recs, size_t n,
                      npr_flow *flows, npr_flow_v6 *flows_v6, uint8_t *status) {
  for (size_t i = 0; i < n; ++i) {
    npr_flow f;
    npr_flow_v6 v6;
    memset(&f, 0, sizeof f);
    memset(&v6, 0, sizeof v6);
    int st = record_flow(buf, len, &recs[i], &f, &v6);
    if (st != NPR_FLOW_OK) {
      memset(&f, 0, sizeof f);
      memset(&v6, 0, sizeof v6);
    }
    if (flows) flows[i] = f;
    if (flows_v6) flows_v6[i] = v6;
    if (status) status[i] = (uint8_t)st;
  }
}

/* The error payload of each record's extract_flow (npr.h npr_flow_details). */
void or_flow_details(const uint8_t *buf, size_t len, const npr_record *recs, size_t n, uint8_t *status,
                     uint64_t *detail) {
  for (size_t i = 0; i < n; ++i) {
    npr_flow f;
    npr_flow_v6 v6;
    uint64_t d = 0;
    const size_t off = (size_t)recs[i].offset + 16, plen = recs[i].actual_length;
    int st = -1;
    if (!(off > len || len - off < plen)) st = extract_flow_l4(buf + off, plen, recs[i].offset, &f, &v6, NULL, NULL, &d);
    if (status) status[i] = (uint8_t)st;
    if (detail) detail[i] = d;
  }
}

/* ---- src/flow/mod.rs:101-123: pop from the END, keep Ok ----------------------------------- */
size_t or_convert_records(const uint8_t *buf, size_t len, const npr_record *recs, size_t n,
                          npr_flow *out, npr_flow_v6 *out_v6, size_t cap) {
  size_t k = 0;
  for (size_t i = n; i-- > 0;) { /* records.pop() :107 */
    npr_flow f;
    npr_flow_v6 v6;
    memset(&v6, 0, sizeof v6);
    if (record_flow(buf, len, &recs[i], &f, &v6) == NPR_FLOW_OK) { /* :109-111 */
      if (k < cap) {
        out[k] = f;
        if (out_v6) out_v6[k] = v6;
      }
      k++;
    }
  }
  return k;
}

size_t or_bench_extract(const uint8_t *in, size_t len, npr_record *rec_scratch, size_t rec_cap,
                        npr_flow *flow_scratch, npr_flow_v6 *v6_scratch, size_t flow_cap,
                        size_t *n_records) {
  npr_global_header h;
  size_t n = 0, cons = 0;
  if (or_capture_file_parse(in, len, &h, rec_scratch, rec_cap, &n, &cons) != OR_OK) {
    if (n_records) *n_records = 0;
    return 0;
  }
  if (n_records) *n_records = n;
  if (n > rec_cap) n = rec_cap;
  return or_convert_records(in, len, rec_scratch, n, flow_scratch, v6_scratch, flow_cap);
}

/* ---- bench leg on T host threads: the same CaptureFile::parse + convert_records result ------
 * The record chain is walked serially (it IS serial: src/record.rs:30-49, and cheap); the
 * extract_flow tree, which is ~85 % of the reference's `extract` time (benches/benches.rs:80-81),
 * runs on T threads over contiguous record ranges; every thread then writes its Ok flows to
 * their reverse-order rows from a prefix of the per-thread counts (src/flow/mod.rs:101-123). */
#include <pthread.h>

typedef struct {
  _Alignas(128) const uint8_t *in;
  size_t len;
  const npr_record *recs;
  size_t lo, hi, ok, base, cap;
  npr_flow *dense, *out;
  npr_flow_v6 *dense6, *out6;
  uint8_t *st;
  int phase;
} or_mt_job;

static void *or_mt_run(void *arg) {
  or_mt_job *j = (or_mt_job *)arg;
  if (j->phase == 0) {
    size_t ok = 0; /* a local count: the jobs share cache lines */
    for (size_t i = j->lo; i < j->hi; ++i) {
      const int st = record_flow(j->in, j->len, &j->recs[i], &j->dense[i], &j->dense6[i]);
      j->st[i] = (uint8_t)st;
      ok += st == NPR_FLOW_OK;
    }
    j->ok = ok;
  } else {
    size_t k = j->base; /* Ok flows of the records after this range come first */
    for (size_t i = j->hi; i-- > j->lo;) {
      if (j->st[i] != NPR_FLOW_OK) continue;
      if (k < j->cap) {
        j->out[k] = j->dense[i];
        if (j->out6) j->out6[k] = j->dense6[i];
      }
      k++;
    }
  }
  return NULL;
}

size_t or_bench_extract_mt(const uint8_t *in, size_t len, npr_record *rec_scratch, size_t rec_cap,
                           npr_flow *dense, npr_flow_v6 *dense6, uint8_t *status, npr_flow *out,
                           npr_flow_v6 *out6, size_t flow_cap, size_t *n_records, int nthreads) {
  npr_global_header h;
  size_t n = 0, cons = 0;
  if (or_capture_file_parse(in, len, &h, rec_scratch, rec_cap, &n, &cons) != OR_OK) {
    if (n_records) *n_records = 0;
    return 0;
  }
  if (n_records) *n_records = n;
  if (n > rec_cap) n = rec_cap;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  or_mt_job jobs[256];
  pthread_t th[256];
  for (int t = 0; t < nthreads; ++t) {
    or_mt_job *j = &jobs[t];
    j->in = in, j->len = len, j->recs = rec_scratch;
    j->lo = n * (size_t)t / (size_t)nthreads, j->hi = n * (size_t)(t + 1) / (size_t)nthreads;
    j->dense = dense, j->dense6 = dense6, j->st = status, j->out = out, j->out6 = out6, j->cap = flow_cap;
    j->phase = 0;
  }
  for (int ph = 0; ph < 2; ++ph) {
    if (ph == 1) { /* exclusive prefix from the END: the last range's flows are rows 0.. */
      size_t acc = 0;
      for (int t = nthreads; t-- > 0;) {
        jobs[t].base = acc;
        acc += jobs[t].ok;
        jobs[t].phase = 1;
      }
    }
    for (int t = 1; t < nthreads; ++t) pthread_create(&th[t], NULL, or_mt_run, &jobs[t]);
    or_mt_run(&jobs[0]);
    for (int t = 1; t < nthreads; ++t) pthread_join(th[t], NULL);
  }
  size_t total = 0;
  for (int t = 0; t < nthreads; ++t) total += jobs[t].ok;
  return total;
}
