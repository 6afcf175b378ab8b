"""CPU checker for row f4 (the distinct-flow table; test infrastructure).  The table is not in the
reference: its parity is derived from the per-record flows the oracle produces, as SURVEY.md §8
row f4 prescribes: key = {kind (family | protocol), src ip, dst ip, src port, dst port}; per key the
first-seen row (lowest record offset), the sum of weights, output in input order of first-seen rows."""
import numpy as np

from net_parser_rs import _abi


def keys(flows, flows_v6):
    kind = flows["kind"].astype(np.uint64)
    out = []
    for i in range(len(flows)):
        f = flows[i]
        if kind[i] & _abi.KIND_IPV6:
            ips = bytes(flows_v6[i]["src_ip"]) + bytes(flows_v6[i]["dst_ip"])
        else:
            ips = bytes(f["src_ip"]) + bytes(f["dst_ip"])
        out.append((int(kind[i]), int(f["src_port"]), int(f["dst_port"]), ips))
    return out


def offsets(flows):
    return np.array([int.from_bytes(bytes(r), "little") for r in flows["record_offset"]], dtype=np.uint64)


def aggregate(flows, flows_v6, weights=None):
    """-> (rows: indices of first-seen input rows in input order, counts per row)."""
    ks = keys(flows, flows_v6)
    off = offsets(flows)
    w = np.ones(len(flows), dtype=np.uint64) if weights is None else np.asarray(weights, dtype=np.uint64)
    first, total = {}, {}
    for i, k in enumerate(ks):
        if k not in first or off[i] < off[first[k]]:
            first[k] = i
        total[k] = total.get(k, 0) + int(w[i])
    rows = sorted(first.values())
    return np.array(rows, dtype=np.int64), np.array([total[ks[i]] for i in rows], dtype=np.uint64)
