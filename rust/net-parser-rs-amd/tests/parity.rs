//! `cargo test` on a machine with an MI355X: this crate against the reference crate (net-parser-rs
//! 0.3, a dev-dependency: the checker only, never linked into the library) on the same capture
//! bytes.  The types are separate restatements, so results are compared through their `Debug` and
//! `Display` forms, which the restatement keeps identical.
use net_parser_rs_amd as amd;

/// A little-endian capture: Eth/IPv4/TCP and Eth/IPv4/UDP records, ARP records (never a flow),
/// VLAN-tagged records, frames cut short, wrong UDP lengths, unknown protocols, and a truncated
/// tail (the chain stops before it, Q3).
fn capture() -> Vec<u8> {
    let mut v = vec![0xd4, 0xc3, 0xb2, 0xa1, 2, 0, 4, 0];
    v.extend_from_slice(&[0u8; 8]);
    v.extend_from_slice(&65535u32.to_le_bytes());
    v.extend_from_slice(&1u32.to_le_bytes());
    for i in 0..5000u32 {
        let mut f: Vec<u8> = (0..12).map(|k| (i as u8).wrapping_mul(7).wrapping_add(k)).collect();
        if i % 7 == 3 {
            f.extend_from_slice(&[0x81, 0x00, 0x00, (i % 4000) as u8]);
        }
        if i % 11 == 5 {
            f.extend_from_slice(&[0x08, 0x06]);
            f.extend_from_slice(&[1u8; 28]);
        } else {
            let udp = i % 2 == 1;
            let proto = if i % 13 == 6 { 47 } else if udp { 17 } else { 6 };
            f.extend_from_slice(&[0x08, 0x00, 0x45, 0x00]);
            let l4len: u16 = if udp { 8 + 12 } else { 20 + 10 };
            f.extend_from_slice(&(20 + l4len).to_be_bytes());
            f.extend_from_slice(&[0, 0, 0, 0, 64, proto, 0, 0]);
            f.extend_from_slice(&[10, 0, (i >> 8) as u8, i as u8, 192, 168, 1, (i % 250) as u8]);
            f.extend_from_slice(&((1000 + i) as u16).to_be_bytes());
            f.extend_from_slice(&80u16.to_be_bytes());
            if udp {
                let ul = if i % 17 == 9 { l4len - 3 } else { l4len };
                f.extend_from_slice(&ul.to_be_bytes());
                f.extend_from_slice(&[0u8; 2]);
                f.extend_from_slice(&[9u8; 12]);
            } else {
                f.extend_from_slice(&[0u8; 8]);
                f.extend_from_slice(&[if i % 19 == 4 { 0x20 } else { 0x50 }, 0x18]);
                f.extend_from_slice(&[0u8; 6]);
                f.extend_from_slice(&[7u8; 10]);
            }
        }
        if i % 23 == 8 {
            f.truncate(f.len() * (i as usize % 5) / 5); // a frame cut short: every Incomplete step
        }
        v.extend_from_slice(&(1_600_000_000 + i / 1000).to_le_bytes());
        v.extend_from_slice(&(i % 1_000_000).to_le_bytes());
        v.extend_from_slice(&(f.len() as u32).to_le_bytes());
        v.extend_from_slice(&(f.len() as u32).to_le_bytes());
        v.extend_from_slice(&f);
    }
    v.extend_from_slice(&[1, 2, 3]); // truncated record header
    v
}

fn same_record(a: &amd::PcapRecord, b: &net_parser_rs::PcapRecord) -> bool {
    a.timestamp == b.timestamp
        && a.actual_length == b.actual_length
        && a.original_length == b.original_length
        && a.payload.as_ptr() == b.payload.as_ptr()
        && a.payload.len() == b.payload.len()
        && format!("{}", a) == format!("{}", b)
}

#[test]
fn capture_file_parse_matches_reference() {
    let data = capture();
    let (rem_a, fa) = amd::parse(&data).expect("device parse");
    let (rem_r, fr) = net_parser_rs::parse(&data).expect("reference parse");
    assert_eq!(rem_a.len(), rem_r.len());
    assert_eq!(format!("{:?}", fa.global_header), format!("{:?}", fr.global_header));
    assert_eq!(fa.records.len(), fr.records.len());
    let (ra, rr) = (fa.records.into_inner(), fr.records.into_inner());
    assert!(ra.iter().zip(rr.iter()).all(|(a, b)| same_record(a, b)));
}

#[test]
fn single_object_parsers_match_reference_on_every_prefix() {
    // GlobalHeader::parse / PcapRecord::parse over truncated inputs: the same Ok values, the same
    // Incomplete { size } (npr_global_header_parse / npr_record_parse + nom's Needed sizes)
    let data = capture();
    for k in 0..=40 {
        let a = amd::GlobalHeader::parse(&data[..k]);
        let r = net_parser_rs::GlobalHeader::parse(&data[..k]);
        assert_eq!(format!("{:?}", a), format!("{:?}", r), "header prefix {}", k);
    }
    for big in [false, true].iter() {
        let e = if *big { nom::Endianness::Big } else { nom::Endianness::Little };
        for k in 0..=120 {
            let s = &data[24..24 + k];
            let a = amd::PcapRecord::parse(s, e).map(|(rem, r)| (rem.len(), format!("{} {:?}", r, r.payload)));
            let r = net_parser_rs::PcapRecord::parse(s, e).map(|(rem, r)| (rem.len(), format!("{} {:?}", r, r.payload)));
            assert_eq!(format!("{:?}", a), format!("{:?}", r), "record prefix {} big {}", k, big);
        }
    }
}

#[test]
fn convert_records_matches_reference() {
    let data = capture();
    let (_, fa) = amd::parse(&data).unwrap();
    let (_, fr) = net_parser_rs::parse(&data).unwrap();
    let a = amd::flow::convert_records(fa.records.into_inner());
    let r = net_parser_rs::flow::convert_records(fr.records.into_inner());
    assert_eq!(a.len(), r.len());
    for ((ra, fa), (rr, fr)) in a.iter().zip(r.iter()) {
        assert!(same_record(ra, rr));
        assert_eq!(format!("{:?}", fa), format!("{:?}", fr));
        assert_eq!(format!("{}", fa), format!("{}", fr));
    }
    let (_, fa2) = amd::parse(&data).unwrap();
    let b = amd::flow::convert_records_in(&data, fa2.records.into_inner());
    assert!(b.iter().zip(a.iter()).all(|(x, y)| x.1 == y.1 && x.0.payload.as_ptr() == y.0.payload.as_ptr()));
    let (rem, c) = amd::flow::parse_and_convert(&data).unwrap();
    assert_eq!(rem.len(), 3);
    assert!(c.iter().zip(a.iter()).all(|(x, y)| x.1 == y.1 && x.0.payload.as_ptr() == y.0.payload.as_ptr()));
}

#[test]
fn extract_flow_results_and_errors_equal_the_reference() {
    // every record: Ok flows equal, errors equal in variant, payload (sizes, ids, positions) and
    // message, through Debug and Display
    use amd::flow::FlowExtraction as _;
    use net_parser_rs::flow::FlowExtraction as _;
    let data = capture();
    let (_, fa) = amd::parse(&data).unwrap();
    let (_, fr) = net_parser_rs::parse(&data).unwrap();
    let ra = fa.records.into_inner();
    let rr = fr.records.into_inner();
    let batch = amd::flow::extract_flows(&ra);
    for (i, (a, r)) in ra.iter().zip(rr.iter()).enumerate().take(1500) {
        let x = a.extract_flow();
        let y = r.extract_flow();
        assert_eq!(format!("{:?}", x), format!("{:?}", y), "record {}", i);
        if let (Err(x), Err(y)) = (&x, &y) {
            assert_eq!(format!("{}", x), format!("{}", y), "record {}", i);
        }
        assert_eq!(format!("{:?}", batch[i]), format!("{:?}", y), "record {} (batch)", i);
    }
}

#[test]
fn readme_facade() {
    let data = capture();
    let recs = amd::CaptureParser::parse_file(&data).expect("Could not parse");
    assert_eq!(recs.len(), 5000);
    let packet = amd::CaptureParser::parse_record(&data[24..]).expect("Could not parse");
    use amd::flow::*;
    let flow = packet.extract_flow().expect("Could not extract flow");
    assert_eq!(flow.destination.port, 80);
}

#[test]
fn concurrent_threads() {
    // reentrant like the reference: several threads parse and convert at once (each its own context)
    let data = std::sync::Arc::new(capture());
    let want = {
        let (_, f) = net_parser_rs::parse(&data).unwrap();
        net_parser_rs::flow::convert_records(f.records.into_inner()).len()
    };
    let hs: Vec<_> = (0..4)
        .map(|_| {
            let d = data.clone();
            std::thread::spawn(move || {
                (0..20)
                    .map(|_| {
                        let (_, f) = amd::parse(&d).unwrap();
                        amd::flow::convert_records(f.records.into_inner()).len()
                    })
                    .collect::<Vec<_>>()
            })
        })
        .collect();
    for h in hs {
        assert!(h.join().unwrap().iter().all(|&k| k == want));
    }
}

/// Eth/IPv4/UDP to 4789 carrying VXLAN + an inner Eth/IPv4/TCP frame, every 3rd record a
/// VXLAN payload cut short of its 8-byte header, every 5th one sent to another port.
fn vxlan_capture() -> Vec<u8> {
    let mut v = vec![0xd4, 0xc3, 0xb2, 0xa1, 2, 0, 4, 0];
    v.extend_from_slice(&[0u8; 8]);
    v.extend_from_slice(&65535u32.to_le_bytes());
    v.extend_from_slice(&1u32.to_le_bytes());
    for i in 0..600u32 {
        let mut inner: Vec<u8> = (0..12).map(|k| (i as u8).wrapping_add(k)).collect();
        inner.extend_from_slice(&[0x08, 0x00, 0x45, 0x00, 0, 40, 0, 0, 0, 0, 64, 6, 0, 0]);
        inner.extend_from_slice(&[172, 16, (i >> 8) as u8, i as u8, 10, 1, 2, 3]);
        inner.extend_from_slice(&((2000 + i) as u16).to_be_bytes());
        inner.extend_from_slice(&443u16.to_be_bytes());
        inner.extend_from_slice(&[0u8; 8]);
        inner.extend_from_slice(&[0x50, 0x10, 0, 0, 0, 0, 0, 0]);
        let mut vx = vec![0x08, 0x00, 0x00, 0x00];
        vx.extend_from_slice(&((i * 977) << 8).to_be_bytes());
        vx.extend_from_slice(&inner);
        if i % 3 == 2 {
            vx.truncate(5);
        }
        let port: u16 = if i % 5 == 4 { 4790 } else { 4789 };
        let udp_len = 8 + vx.len() as u16;
        let mut f: Vec<u8> = (0..12).map(|k| (i as u8).wrapping_mul(3).wrapping_add(k)).collect();
        f.extend_from_slice(&[0x08, 0x00, 0x45, 0x00]);
        f.extend_from_slice(&(20 + udp_len).to_be_bytes());
        f.extend_from_slice(&[0, 0, 0, 0, 64, 17, 0, 0, 10, 0, 0, 1, 10, 0, 0, 2]);
        f.extend_from_slice(&((40000 + i) as u16).to_be_bytes());
        f.extend_from_slice(&port.to_be_bytes());
        f.extend_from_slice(&udp_len.to_be_bytes());
        f.extend_from_slice(&[0, 0]);
        f.extend_from_slice(&vx);
        v.extend_from_slice(&1_600_000_000u32.to_le_bytes());
        v.extend_from_slice(&i.to_le_bytes());
        v.extend_from_slice(&(f.len() as u32).to_le_bytes());
        v.extend_from_slice(&(f.len() as u32).to_le_bytes());
        v.extend_from_slice(&f);
    }
    v
}

#[test]
fn vxlan_inner_flows_match_reference() {
    use net_parser_rs::flow::layer2::FlowExtraction as _;
    let data = vxlan_capture();
    let (_, fa) = amd::parse(&data).unwrap();
    let recs = fa.records.into_inner();
    let got = amd::flow::vxlan_flows(Some(&data), &recs, 4789, nom::Endianness::Big);
    assert_eq!(got.len(), 600);
    for (i, (r, (res, vni))) in recs.iter().zip(got.iter()).enumerate() {
        let udp_payload = &r.payload[14 + 20 + 8..];
        if i % 5 == 4 {
            assert!(res.is_err(), "record {}: other port", i);
            continue;
        }
        match net_parser_rs::layer4::Vxlan::parse(udp_payload, nom::Endianness::Big) {
            Err(_) => assert!(res.is_err(), "record {}: short VXLAN header", i),
            Ok((_, vx)) => {
                assert_eq!(*vni, vx.network_identifier, "record {}", i);
                let (_, l2) = net_parser_rs::layer2::ethernet::Ethernet::parse(vx.payload).unwrap();
                let want = l2.extract_flow().unwrap();
                assert_eq!(format!("{:?}", res.as_ref().unwrap()), format!("{:?}", want), "record {}", i);
            }
        }
    }
}

#[test]
fn layer_objects_match_reference() {
    // Ethernet / IPv4 / IPv6 / Arp / Tcp / Udp / Vxlan ::parse over every frame of the capture and
    // over every prefix of a few: the same objects (Debug), the same errors, the same as_bytes
    let data = capture();
    let (_, fa) = net_parser_rs::CaptureFile::parse(&data).unwrap();
    let recs = fa.records.into_inner();
    let mut frames: Vec<&[u8]> = recs.iter().map(|r| r.payload).collect();
    for f in recs.iter().take(40).map(|r| r.payload) {
        for k in 0..f.len() {
            frames.push(&f[..k]);
        }
    }
    for (i, f) in frames.iter().enumerate() {
        let a = amd::layer2::ethernet::Ethernet::parse(f);
        let r = net_parser_rs::layer2::ethernet::Ethernet::parse(f);
        assert_eq!(format!("{:?}", a), format!("{:?}", r), "ethernet {}", i);
        let (pa, pr) = match (a, r) {
            (Ok((_, a)), Ok((_, r))) => {
                assert_eq!(a.as_bytes(), r.as_bytes(), "ethernet as_bytes {}", i);
                (a.payload, r.payload)
            }
            _ => continue,
        };
        let a4 = amd::layer3::ipv4::IPv4::parse(pa);
        let r4 = net_parser_rs::layer3::ipv4::IPv4::parse(pr);
        assert_eq!(format!("{:?}", a4), format!("{:?}", r4), "ipv4 {}", i);
        assert_eq!(format!("{:?}", amd::layer3::ipv6::IPv6::parse(pa)), format!("{:?}", net_parser_rs::layer3::ipv6::IPv6::parse(pr)), "ipv6 {}", i);
        assert_eq!(format!("{:?}", amd::layer3::arp::Arp::parse(pa)), format!("{:?}", net_parser_rs::layer3::arp::Arp::parse(pr)), "arp {}", i);
        if let (Ok((_, a4)), Ok((_, r4))) = (a4, r4) {
            assert_eq!(a4.as_bytes(), r4.as_bytes(), "ipv4 as_bytes {}", i);
            let (at, rt) = (amd::layer4::tcp::Tcp::parse(a4.payload), net_parser_rs::layer4::tcp::Tcp::parse(r4.payload));
            assert_eq!(format!("{:?}", at), format!("{:?}", rt), "tcp {}", i);
            let (au, ru) = (amd::layer4::udp::Udp::parse(a4.payload), net_parser_rs::layer4::udp::Udp::parse(r4.payload));
            assert_eq!(format!("{:?}", au), format!("{:?}", ru), "udp {}", i);
            for e in [nom::Endianness::Big, nom::Endianness::Little].iter() {
                assert_eq!(
                    format!("{:?}", amd::layer4::vxlan::Vxlan::parse(a4.payload, *e)),
                    format!("{:?}", net_parser_rs::layer4::vxlan::Vxlan::parse(r4.payload, *e)),
                    "vxlan {}",
                    i
                );
            }
        }
    }
}

#[test]
fn ethernet_flow_extraction_matches_reference() {
    use amd::flow::layer2::FlowExtraction as _;
    let data = capture();
    let (_, fa) = net_parser_rs::CaptureFile::parse(&data).unwrap();
    for r in fa.records.into_inner().iter().take(500) {
        if let (Ok((_, a)), Ok((_, b))) =
            (amd::layer2::ethernet::Ethernet::parse(r.payload), net_parser_rs::layer2::ethernet::Ethernet::parse(r.payload))
        {
            use net_parser_rs::flow::layer2::FlowExtraction as RefL2;
            assert_eq!(format!("{:?}", a.extract_flow()), format!("{:?}", RefL2::extract_flow(&b)));
        }
    }
}

#[test]
fn layer3_and_layer4_flow_extraction_match_reference() {
    // <IPv4 | IPv6 | Arp as flow::layer3::FlowExtraction>::extract_flow(l2) over every Ethernet
    // payload of the capture (and every prefix of a few), and <Tcp | Udp as
    // flow::layer4::FlowExtraction>::extract_flow(l2, l3) on the parsed L4 objects: the same Flow or
    // the same error (Debug), src/flow/layer3/{ipv4,ipv6,arp}.rs, src/flow/layer4/{tcp,udp}.rs
    use amd::flow::layer3::FlowExtraction as _;
    use amd::flow::layer4::FlowExtraction as _;
    use net_parser_rs::flow::layer3::FlowExtraction as RefL3;
    use net_parser_rs::flow::layer4::FlowExtraction as RefL4;
    let data = capture();
    let (_, fa) = net_parser_rs::CaptureFile::parse(&data).unwrap();
    let recs = fa.records.into_inner();
    let mut frames: Vec<&[u8]> = recs.iter().map(|r| r.payload).collect();
    for f in recs.iter().take(40).map(|r| r.payload) {
        for k in 0..f.len() {
            frames.push(&f[..k]);
        }
    }
    let mut compared = 0usize;
    for (i, f) in frames.iter().enumerate() {
        let (a, r) = match (amd::layer2::ethernet::Ethernet::parse(f), net_parser_rs::layer2::ethernet::Ethernet::parse(f)) {
            (Ok((_, a)), Ok((_, r))) => (a, r),
            _ => continue,
        };
        let al2 = amd::flow::info::layer2::Info {
            id: amd::flow::info::layer2::Id::Ethernet,
            src_mac: a.src_mac,
            dst_mac: a.dst_mac,
            vlan: a.vlan(),
        };
        let rl2 = net_parser_rs::flow::info::layer2::Info {
            id: net_parser_rs::flow::info::layer2::Id::Ethernet,
            src_mac: r.src_mac.clone(),
            dst_mac: r.dst_mac.clone(),
            vlan: r.vlan(),
        };
        if let (Ok((_, a4)), Ok((_, r4))) = (amd::layer3::ipv4::IPv4::parse(a.payload), net_parser_rs::layer3::ipv4::IPv4::parse(r.payload)) {
            assert_eq!(format!("{:?}", a4.extract_flow(al2)), format!("{:?}", RefL3::extract_flow(&r4, rl2.clone())), "ipv4 flow {}", i);
            let al3 = amd::flow::info::layer3::Info { id: amd::flow::info::layer3::Id::IPv4, src_ip: a4.src_ip, dst_ip: a4.dst_ip };
            let rl3 = net_parser_rs::flow::info::layer3::Info { id: net_parser_rs::flow::info::layer3::Id::IPv4, src_ip: r4.src_ip, dst_ip: r4.dst_ip };
            if let (Ok((_, at)), Ok((_, rt))) = (amd::layer4::tcp::Tcp::parse(a4.payload), net_parser_rs::layer4::tcp::Tcp::parse(r4.payload)) {
                assert_eq!(format!("{:?}", at.extract_flow(al2, al3)), format!("{:?}", RefL4::extract_flow(&rt, rl2.clone(), rl3.clone())), "tcp flow {}", i);
            }
            if let (Ok((_, au)), Ok((_, ru))) = (amd::layer4::udp::Udp::parse(a4.payload), net_parser_rs::layer4::udp::Udp::parse(r4.payload)) {
                assert_eq!(format!("{:?}", au.extract_flow(al2, al3)), format!("{:?}", RefL4::extract_flow(&ru, rl2.clone(), rl3.clone())), "udp flow {}", i);
            }
            compared += 1;
        }
        if let (Ok((_, a6)), Ok((_, r6))) = (amd::layer3::ipv6::IPv6::parse(a.payload), net_parser_rs::layer3::ipv6::IPv6::parse(r.payload)) {
            assert_eq!(format!("{:?}", a6.extract_flow(al2)), format!("{:?}", RefL3::extract_flow(&r6, rl2.clone())), "ipv6 flow {}", i);
        }
        if let (Ok((_, aa)), Ok((_, ra))) = (amd::layer3::arp::Arp::parse(a.payload), net_parser_rs::layer3::arp::Arp::parse(r.payload)) {
            assert_eq!(format!("{:?}", aa.extract_flow(al2)), format!("{:?}", RefL3::extract_flow(&ra, rl2.clone())), "arp flow {}", i);
        }
    }
    assert!(compared > 1000, "{} IPv4 frames compared", compared);
}
