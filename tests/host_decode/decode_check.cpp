// The device's general decoder (net-parser-rs_amd/csrc/npr_decode.hpp: decode<>, the same source
// the kernels compile) built for the HOST and checked against the oracle on the CPU: status, flow
// fields and the error payload (npr_flow_details) of every record of each capture given, and of
// every truncation of each record's payload (every prefix length: each Incomplete step of the
// reference's nom chains).  Test infrastructure (tests/test_host_decode.py runs it).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../net-parser-rs_amd/csrc/npr_decode.hpp"

extern "C" {
#include "npr_oracle.h"
}

namespace {

struct HostReader {  // the byte reader of the device's GlobalReader, over host memory
  const uint8_t *g;
  uint64_t gavail;
  uint32_t u8(uint32_t q) const { return (uint64_t)q < gavail ? g[q] : 0u; }
  uint32_t le32(uint32_t q) const { return u8(q) | (u8(q + 1) << 8) | (u8(q + 2) << 16) | (u8(q + 3) << 24); }
};

// the npr_flow row the kernels build from FlowWords (put_flow) for an Ok record
void row_of(const npr::FlowWords &f, uint64_t off, npr_flow *row) {
  uint32_t w[8] = {f.d[0], f.d[1], f.d[2], f.d[3], f.d[4], f.d[5], f.d[6] | ((uint32_t)(off & 0xffu) << 24),
                   (uint32_t)(off >> 8)};
  memcpy(row, w, 32);
}

long failures = 0;
long checked = 0;

void check_one(const uint8_t *p, uint32_t n, uint64_t off, const char *what) {
  npr_flow of{};
  npr_flow_v6 o6{};
  uint64_t odet = 0;
  const int ost = or_extract_flow_detail(p, n, off, &of, &o6, &odet);
  npr::FlowWords f{};
  volatile uint64_t det = 0;
  const uint32_t st = npr::decode<true, HostReader, true>(HostReader{p, n}, n, f, &det);
  ++checked;
  const uint64_t dv = det;
  bool ok = (int)st == ost && dv == odet;
  if (ok && st == NPR_FLOW_OK) {
    npr_flow row;
    row_of(f, off, &row);
    if (f.d[6] & (NPR_FLOW_KIND_IPV6 << 16)) {  // IPv4 address words are 0; the side row holds IPv6
      ok = !memcmp(f.v6, &o6, 32);
    }
    ok = ok && !memcmp(&row, &of, 32);
  }
  if (!ok && failures++ < 20)
    fprintf(stderr, "MISMATCH %s offset %llu len %u: status %u vs %d, detail %llu vs %llu\n", what,
            (unsigned long long)off, n, st, ost, (unsigned long long)dv, (unsigned long long)odet);
}

}  // namespace

int main(int argc, char **argv) {
  for (int a = 1; a < argc; ++a) {
    FILE *fp = fopen(argv[a], "rb");
    if (!fp) {
      fprintf(stderr, "cannot read %s\n", argv[a]);
      return 2;
    }
    std::vector<uint8_t> buf;
    uint8_t tmp[1 << 16];
    size_t k;
    while ((k = fread(tmp, 1, sizeof tmp, fp)) > 0) buf.insert(buf.end(), tmp, tmp + k);
    fclose(fp);
    npr_global_header h;
    size_t n = 0, cons = 0;
    std::vector<npr_record> recs(buf.size() / 16 + 1);
    if (or_capture_file_parse(buf.data(), buf.size(), &h, recs.data(), recs.size(), &n, &cons) != OR_OK) continue;
    for (size_t i = 0; i < n; ++i) {
      const uint8_t *p = buf.data() + recs[i].offset + 16;
      const uint32_t len = recs[i].actual_length;
      check_one(p, len, recs[i].offset, "record");
      for (uint32_t m = 0; m < len && m < 160; ++m) check_one(p, m, recs[i].offset, "prefix");
    }
    printf("%s: %zu records\n", argv[a], n);
  }
  printf("%ld decodes, %ld mismatches\n", checked, failures);
  return failures ? 1 : 0;
}
