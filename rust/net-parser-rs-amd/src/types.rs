//! The public data types of net-parser-rs 0.3, restated field for field (same names, derives,
//! `Display` strings and error messages) so that this crate replaces the reference crate outright:
//! nothing of the reference is linked or executed.  Only the types that the drop-in's functions
//! take or return are here; the parsers that produce them run in libnpr (include/npr.h).
//!
//! | module here                  | reference                                                       |
//! |------------------------------|-----------------------------------------------------------------|
//! | `common`                     | src/common.rs:3-26                                              |
//! | `errors`                     | src/errors.rs:3-55                                              |
//! | `global_header`              | src/global_header.rs:4-37 (parse: crate root, over the C-ABI)   |
//! | `layer2::ethernet`           | src/layer2/ethernet.rs:16-98 (the EtherType ids; the structs: layers.rs) |
//! | `layer3`                     | src/layer3/mod.rs:25-84 (InternetProtocolId; the structs: layers.rs) |
//! | `layer4`                     | src/layer4 (the structs: layers.rs)                             |
//! | `flow_types::{device, info}` | src/flow/device.rs:7-27, src/flow/info.rs:1-95                  |
//! | `flow_types::errors` + tree  | src/flow/errors.rs:5-19 and the per-layer `errors` modules      |

/// src/common.rs
pub mod common {
    pub const MAC_LENGTH: usize = 6;

    #[derive(Clone, Copy, Debug, Default, PartialEq, Eq, Hash)]
    pub struct MacAddress(pub [u8; MAC_LENGTH]);

    pub type Vlan = u16;
    pub type Port = u16;

    impl std::fmt::Display for MacAddress {
        /// lowercase `xx:xx:xx:xx:xx:xx` (src/common.rs:18-26)
        fn fmt(&self, f: &mut std::fmt::Formatter) -> std::fmt::Result {
            for (i, b) in self.0.iter().enumerate() {
                if i > 0 {
                    f.write_str(":")?;
                }
                write!(f, "{:02x}", b)?;
            }
            Ok(())
        }
    }
}

/// src/errors.rs: the parse error of every nom-level parser
pub mod errors {
    #[derive(Clone, Debug)]
    pub enum Error {
        Incomplete { size: Option<usize> },
        Failure { msg: String },
        Custom { msg: String },
    }

    impl std::fmt::Display for Error {
        fn fmt(&self, f: &mut std::fmt::Formatter) -> std::fmt::Result {
            match self {
                Error::Incomplete { size } => write!(f, "Incomplete: {:?}", size),
                Error::Failure { msg } | Error::Custom { msg } => f.write_str(msg),
            }
        }
    }

    impl std::error::Error for Error {}

    /// nom errors convert as the reference's do (src/errors.rs:16-55): Needed sizes carried,
    /// Error / Failure contexts formatted into the message.
    impl<I: std::fmt::Debug, E: std::fmt::Debug> From<nom::Err<I, E>> for Error {
        fn from(err: nom::Err<I, E>) -> Self {
            Error::from(&err)
        }
    }

    impl<I: std::fmt::Debug, E: std::fmt::Debug> From<&nom::Err<I, E>> for Error {
        fn from(err: &nom::Err<I, E>) -> Self {
            match err {
                nom::Err::Incomplete(nom::Needed::Unknown) => Error::Incomplete { size: None },
                nom::Err::Incomplete(nom::Needed::Size(n)) => Error::Incomplete { size: Some(*n) },
                nom::Err::Error(c) => Error::Failure { msg: format!("Error: {:?}", c) },
                nom::Err::Failure(c) => Error::Failure { msg: format!("Failure: {:?}", c) },
            }
        }
    }
}

/// src/global_header.rs: the 24-byte libpcap file header (GlobalHeader::parse is in the crate root)
pub mod global_header {
    use nom::Endianness;

    #[cfg(target_endian = "little")]
    pub const NATIVE_ENDIAN: Endianness = Endianness::Little;
    #[cfg(target_endian = "big")]
    pub const NATIVE_ENDIAN: Endianness = Endianness::Big;

    #[allow(unused)]
    #[derive(Clone, Copy, Debug)]
    pub struct GlobalHeader {
        pub endianness: Endianness,
        pub version_major: u16,
        pub version_minor: u16,
        pub zone: i32,
        pub sig_figs: i32,
        pub snap_length: u32,
        pub network: u32,
    }

    impl Default for GlobalHeader {
        /// a v2.4 Ethernet capture in native order, snap length 1500 (src/global_header.rs:25-37)
        fn default() -> Self {
            GlobalHeader {
                endianness: NATIVE_ENDIAN,
                version_major: 2,
                version_minor: 4,
                zone: 0,
                sig_figs: 0,
                snap_length: 1500,
                network: 1,
            }
        }
    }
}

/// src/layer2: the EtherType ids that appear in the flow error tree
pub mod layer2 {
    pub mod ethernet {
        /// EtherTypes of a layer-3 payload (src/layer2/ethernet.rs:16-33)
        #[derive(Clone, Copy, Debug, PartialEq)]
        pub enum Layer3Id {
            Lldp,
            IPv4,
            IPv6,
            Arp,
        }

        impl Layer3Id {
            pub fn value(&self) -> u16 {
                match self {
                    Layer3Id::Lldp => 0x88cc,
                    Layer3Id::IPv4 => 0x0800,
                    Layer3Id::IPv6 => 0x86dd,
                    Layer3Id::Arp => 0x0806,
                }
            }
        }

        /// 802.1Q / 802.1ad tag EtherTypes (src/layer2/ethernet.rs:35-48)
        #[derive(Clone, Copy, Debug, PartialEq)]
        pub enum VlanTypeId {
            VlanTagId,
            ProviderBridging,
        }

        impl VlanTypeId {
            pub fn value(&self) -> u16 {
                match self {
                    VlanTypeId::VlanTagId => 0x8100,
                    VlanTypeId::ProviderBridging => 0x88a8,
                }
            }
        }

        /// src/layer2/ethernet.rs:50-82
        #[derive(Clone, Copy, Debug, PartialEq)]
        pub enum EthernetTypeId {
            PayloadLength(u16),
            Vlan(VlanTypeId),
            L3(Layer3Id),
        }

        impl EthernetTypeId {
            /// EthernetTypeId::new (src/layer2/ethernet.rs:57-73): None for an unknown EtherType
            pub(crate) fn from_value(v: u16) -> Option<EthernetTypeId> {
                Some(match v {
                    0x8100 => EthernetTypeId::Vlan(VlanTypeId::VlanTagId),
                    0x88a8 => EthernetTypeId::Vlan(VlanTypeId::ProviderBridging),
                    0x88cc => EthernetTypeId::L3(Layer3Id::Lldp),
                    0x0800 => EthernetTypeId::L3(Layer3Id::IPv4),
                    0x86dd => EthernetTypeId::L3(Layer3Id::IPv6),
                    0x0806 => EthernetTypeId::L3(Layer3Id::Arp),
                    x if x <= 1500 => EthernetTypeId::PayloadLength(x),
                    _ => return None,
                })
            }

            /// EthernetTypeId::value (src/layer2/ethernet.rs:75-81)
            pub(crate) fn value(&self) -> u16 {
                match self {
                    EthernetTypeId::PayloadLength(v) => *v,
                    EthernetTypeId::Vlan(v) => v.value(),
                    EthernetTypeId::L3(v) => v.value(),
                }
            }
        }

        /// src/layer2/ethernet.rs:84-217 (parse over npr_ethernet_parse: crate::layers)
        pub use crate::layers::{Ethernet, VlanTag};
    }

    pub use crate::layers::Layer2;
    pub use ethernet::Ethernet;
}

/// src/layer3/mod.rs: IP protocol numbers
pub mod layer3 {
    #[derive(Clone, Copy, Debug, PartialEq, Eq)]
    pub enum InternetProtocolId {
        AuthenticationHeader,
        HopByHop,
        EncapsulatingSecurityPayload,
        ICMP,
        IPv6Route,
        IPv6Fragment,
        IPv6NoNext,
        IPv6Options,
        Tcp,
        Udp,
    }

    // (id, protocol number): the ten protocols the reference knows (src/layer3/mod.rs:39-72)
    const TABLE: [(InternetProtocolId, u8); 10] = [
        (InternetProtocolId::HopByHop, 0),
        (InternetProtocolId::ICMP, 1),
        (InternetProtocolId::Tcp, 6),
        (InternetProtocolId::Udp, 17),
        (InternetProtocolId::IPv6Route, 43),
        (InternetProtocolId::IPv6Fragment, 44),
        (InternetProtocolId::AuthenticationHeader, 50),
        (InternetProtocolId::EncapsulatingSecurityPayload, 51),
        (InternetProtocolId::IPv6NoNext, 59),
        (InternetProtocolId::IPv6Options, 60),
    ];

    impl InternetProtocolId {
        pub fn value(&self) -> u8 {
            TABLE.iter().find(|(id, _)| id == self).map(|(_, v)| *v).unwrap_or(0)
        }

        pub fn new(value: u8) -> Option<InternetProtocolId> {
            TABLE.iter().find(|(_, v)| *v == value).map(|(id, _)| *id)
        }

        /// the extension-header ids whose next byte is another header id (src/layer3/mod.rs:74-84)
        pub fn has_next_option(v: InternetProtocolId) -> bool {
            matches!(
                v,
                InternetProtocolId::AuthenticationHeader
                    | InternetProtocolId::EncapsulatingSecurityPayload
                    | InternetProtocolId::HopByHop
                    | InternetProtocolId::IPv6Route
                    | InternetProtocolId::IPv6Fragment
                    | InternetProtocolId::IPv6Options
            )
        }
    }

    /// src/layer3/{arp,ipv4,ipv6}.rs (parse over npr_arp_parse / npr_ipv4_parse / npr_ipv6_parse)
    pub mod arp {
        pub use crate::layers::Arp;
    }
    pub mod ipv4 {
        pub use crate::layers::IPv4;
    }
    pub mod ipv6 {
        pub use crate::layers::IPv6;
    }
    pub use crate::layers::{Arp, IPv4, IPv6, Layer3};
}

/// src/layer4/{tcp,udp,vxlan}.rs (parse over npr_tcp_parse / npr_udp_parse / npr_vxlan_parse)
pub mod layer4 {
    pub mod tcp {
        pub use crate::layers::{HeaderLengthAndFlags, Tcp};
    }
    pub mod udp {
        pub use crate::layers::Udp;
    }
    pub mod vxlan {
        pub use crate::layers::Vxlan;
    }
    pub use crate::layers::{Layer4, Tcp, Udp, Vxlan};
}

/// src/flow/{device,info,errors}.rs and the per-layer `errors` modules of src/flow/layer{2,3,4}
pub mod flow_types {
    /// src/flow/device.rs
    pub mod device {
        use crate::common::MacAddress;
        use std::net::{IpAddr, Ipv4Addr};

        /// the mac, ip and port of one end of a flow
        #[derive(Clone, Copy, Debug, PartialEq, Eq, Hash)]
        pub struct Device {
            pub mac: MacAddress,
            pub ip: IpAddr,
            pub port: u16,
        }

        impl Default for Device {
            fn default() -> Self {
                Device { mac: MacAddress::default(), ip: IpAddr::V4(Ipv4Addr::UNSPECIFIED), port: 0 }
            }
        }

        impl std::fmt::Display for Device {
            fn fmt(&self, f: &mut std::fmt::Formatter) -> std::fmt::Result {
                write!(f, "Mac={}   Ip={}   Port={}", self.mac, self.ip, self.port)
            }
        }
    }

    /// src/flow/info.rs
    pub mod info {
        pub mod layer2 {
            use crate::common::{MacAddress, Vlan};

            #[derive(Clone, Copy, Debug, PartialEq, Eq, Hash)]
            pub enum Id {
                Ethernet,
            }

            impl Default for Id {
                fn default() -> Self {
                    Id::Ethernet
                }
            }

            #[derive(Clone, Copy, Debug, Default)]
            pub struct Info {
                pub id: Id,
                pub src_mac: MacAddress,
                pub dst_mac: MacAddress,
                pub vlan: Vlan,
            }
        }

        pub mod layer3 {
            use std::net::{IpAddr, Ipv4Addr};

            #[derive(Clone, Copy, Debug, PartialEq, Eq, Hash)]
            pub enum Id {
                Arp,
                IPv4,
                IPv6,
            }

            impl Default for Id {
                fn default() -> Self {
                    Id::IPv4
                }
            }

            #[derive(Clone, Copy, Debug)]
            pub struct Info {
                pub id: Id,
                pub dst_ip: IpAddr,
                pub src_ip: IpAddr,
            }

            impl Default for Info {
                fn default() -> Self {
                    let any = IpAddr::V4(Ipv4Addr::UNSPECIFIED);
                    Info { id: Id::default(), dst_ip: any, src_ip: any }
                }
            }
        }

        pub mod layer4 {
            #[derive(Clone, Copy, Debug, PartialEq, Eq, Hash)]
            pub enum Id {
                Tcp,
                Udp,
                Vxlan,
            }

            impl Default for Id {
                fn default() -> Self {
                    Id::Udp
                }
            }

            #[derive(Clone, Copy, Debug, Default)]
            pub struct Info {
                pub id: Id,
                pub dst_port: u16,
                pub src_port: u16,
            }
        }
    }

    /// src/flow/errors.rs: the error of FlowExtraction::extract_flow
    pub mod errors {
        use super::{layer2, layer3, layer4};
        use crate::errors::Error as NetParserError;

        #[derive(Debug)]
        pub enum Error {
            NetParser(NetParserError),
            L2(layer2::errors::Error),
            L3(layer3::errors::Error),
            L4(layer4::errors::Error),
            Incomplete { size: usize },
        }

        impl std::fmt::Display for Error {
            fn fmt(&self, f: &mut std::fmt::Formatter) -> std::fmt::Result {
                match self {
                    Error::NetParser(_) => f.write_str("NetParserError error while parsing layer2"),
                    Error::L2(_) => f.write_str("Layer2 error while parsing"),
                    Error::L3(_) => f.write_str("Layer3 error while parsing"),
                    Error::L4(_) => f.write_str("Layer4 error while parsing"),
                    Error::Incomplete { size } => write!(f, "Parse was incomplete: {}", size),
                }
            }
        }

        impl std::error::Error for Error {
            fn source(&self) -> Option<&(dyn std::error::Error + 'static)> {
                match self {
                    Error::NetParser(e) => Some(e),
                    Error::L2(e) => Some(e),
                    Error::L3(e) => Some(e),
                    Error::L4(e) => Some(e),
                    Error::Incomplete { .. } => None,
                }
            }
        }

        impl From<NetParserError> for Error {
            fn from(e: NetParserError) -> Self {
                Error::NetParser(e)
            }
        }
        impl From<layer2::errors::Error> for Error {
            fn from(e: layer2::errors::Error) -> Self {
                Error::L2(e)
            }
        }
        impl From<layer3::errors::Error> for Error {
            fn from(e: layer3::errors::Error) -> Self {
                Error::L3(e)
            }
        }
        impl From<layer4::errors::Error> for Error {
            fn from(e: layer4::errors::Error) -> Self {
                Error::L4(e)
            }
        }
    }

    // One error enum per level of the reference's flow dispatch.  `wrap!` writes the enum whose
    // variants each wrap one inner error (Display = a fixed text, or the text with the inner error's
    // Debug form), with From conversions and source().
    macro_rules! wrap {
        ($(#[$m:meta])* $name:ident { $($var:ident($inner:ty) => $text:literal $($dbg:ident)?),* $(,)? }) => {
            $(#[$m])*
            #[derive(Debug)]
            pub enum $name {
                $($var($inner)),*
            }
            impl std::fmt::Display for $name {
                fn fmt(&self, f: &mut std::fmt::Formatter) -> std::fmt::Result {
                    match self {
                        $($name::$var(_e) => wrap!(@text f, _e, $text $(, $dbg)?)),*
                    }
                }
            }
            impl std::error::Error for $name {
                fn source(&self) -> Option<&(dyn std::error::Error + 'static)> {
                    match self {
                        $($name::$var(e) => Some(e)),*
                    }
                }
            }
            $(impl From<$inner> for $name {
                fn from(e: $inner) -> Self {
                    $name::$var(e)
                }
            })*
        };
        (@text $f:ident, $e:ident, $text:literal) => { $f.write_str($text) };
        (@text $f:ident, $e:ident, $text:literal, $dbg:ident) => { write!($f, "{}{:?}", $text, $e) };
    }

    /// src/flow/layer2/{mod,ethernet}.rs
    pub mod layer2 {
        /// src/flow/layer2/mod.rs:6-8 (implemented for layer2::Ethernet in crate::layers)
        pub trait FlowExtraction {
            fn extract_flow(&self) -> Result<crate::flow::Flow, crate::flow::errors::Error>;
        }

        pub mod errors {
            wrap!(Error { Ethernet(super::ethernet::errors::Error) => "Ethernet Error" });
        }
        pub mod ethernet {
            pub mod errors {
                use crate::errors::Error as NetParserError;
                use crate::layer2::ethernet::EthernetTypeId;

                #[derive(Debug)]
                pub enum Error {
                    NetParser { l3: EthernetTypeId, err: NetParserError },
                    Incomplete { l3: EthernetTypeId, size: usize },
                    EthernetType { etype: EthernetTypeId },
                }

                impl std::fmt::Display for Error {
                    fn fmt(&self, f: &mut std::fmt::Formatter) -> std::fmt::Result {
                        match self {
                            Error::NetParser { l3, err } => write!(f, "Failed parse of {:?}: {}", l3, err),
                            Error::Incomplete { l3, size } => write!(f, "Incomplete parse of {:?}: {}", l3, size),
                            Error::EthernetType { etype } => write!(f, "Unknown Ethernet Type: {:?}", etype),
                        }
                    }
                }

                impl std::error::Error for Error {}
            }
        }
    }

    /// src/flow/layer3/{mod,arp,ipv4,ipv6}.rs
    pub mod layer3 {
        /// src/flow/layer3/mod.rs:9-11 (implemented for layer3::{IPv4, IPv6, Arp} in crate::layers)
        pub trait FlowExtraction {
            fn extract_flow(&self, l2: super::info::layer2::Info) -> Result<crate::flow::Flow, crate::flow::errors::Error>;
        }

        pub mod errors {
            wrap!(Error {
                Arp(super::arp::errors::Error) => "ARP Error: " debug,
                IPv4(super::ipv4::errors::Error) => "IPv4 Error: " debug,
                IPv6(super::ipv6::errors::Error) => "IPv6 Error: " debug,
            });
        }
        pub mod arp {
            pub mod errors {
                use crate::errors::Error as NetParserError;

                #[derive(Debug)]
                pub enum Error {
                    NetParser(NetParserError),
                    Flow,
                }

                impl std::fmt::Display for Error {
                    fn fmt(&self, f: &mut std::fmt::Formatter) -> std::fmt::Result {
                        f.write_str(match self {
                            Error::NetParser(_) => "Error parsing ARP",
                            Error::Flow => "ARP cannot be converted to a flow",
                        })
                    }
                }

                impl std::error::Error for Error {}

                impl From<NetParserError> for Error {
                    fn from(e: NetParserError) -> Self {
                        Error::NetParser(e)
                    }
                }
            }
        }

        // IPv4 and IPv6 share one error shape (and, in the reference, one "IPv4" message)
        macro_rules! ip_errors {
            () => {
                pub mod errors {
                    use crate::errors::Error as NetParserError;
                    use crate::layer3::InternetProtocolId;

                    #[derive(Debug)]
                    pub enum Error {
                        NetParser { l4: InternetProtocolId, err: NetParserError },
                        Incomplete { l4: InternetProtocolId, size: usize },
                        InternetProtocolId { id: InternetProtocolId },
                    }

                    impl std::fmt::Display for Error {
                        fn fmt(&self, f: &mut std::fmt::Formatter) -> std::fmt::Result {
                            match self {
                                Error::NetParser { l4, err } => write!(f, "Failed parse of {:?}: {}", l4, err),
                                Error::Incomplete { l4, size } => write!(f, "Incomplete parse of {:?}: {}", l4, size),
                                Error::InternetProtocolId { id } => {
                                    write!(f, "Unknown type while parsing IPv4: {:?}", id)
                                }
                            }
                        }
                    }

                    impl std::error::Error for Error {}
                }
            };
        }
        pub mod ipv4 {
            ip_errors!();
        }
        pub mod ipv6 {
            ip_errors!();
        }
    }

    /// src/flow/layer4/{mod,tcp,udp,vxlan}.rs
    pub mod layer4 {
        /// src/flow/layer4/mod.rs:10-12 (implemented for layer4::{Tcp, Udp} in crate::layers)
        pub trait FlowExtraction {
            fn extract_flow(
                &self,
                l2: super::info::layer2::Info,
                l3: super::info::layer3::Info,
            ) -> Result<crate::flow::Flow, crate::flow::errors::Error>;
        }

        pub mod errors {
            wrap!(Error {
                Tcp(super::tcp::errors::Error) => "Tcp Error: " debug,
                Udp(super::udp::errors::Error) => "Udp Error: " debug,
                Vxlan(super::vxlan::errors::Error) => "Vxlan Error: " debug,
            });
        }
        pub mod tcp {
            pub mod errors {
                wrap!(Error { NetParser(crate::errors::Error) => "Error Parsing TCP: " debug });
            }
        }
        pub mod udp {
            pub mod errors {
                wrap!(Error { NetParser(crate::errors::Error) => "Error parsing UDP: " debug });
            }
        }
        pub mod vxlan {
            pub mod errors {
                use crate::errors::Error as NetParserError;
                use crate::layer2::ethernet::EthernetTypeId;

                #[derive(Debug)]
                pub enum Error {
                    NetParser(NetParserError),
                    Incomplete { l3: EthernetTypeId, size: usize },
                }

                impl std::fmt::Display for Error {
                    fn fmt(&self, f: &mut std::fmt::Formatter) -> std::fmt::Result {
                        match self {
                            Error::NetParser(e) => write!(f, "Error parsing Vxlan: {:?}", e),
                            Error::Incomplete { l3, size } => write!(f, "Incomplete parse of {:?}: {}", l3, size),
                        }
                    }
                }

                impl std::error::Error for Error {}

                impl From<NetParserError> for Error {
                    fn from(e: NetParserError) -> Self {
                        Error::NetParser(e)
                    }
                }
            }
        }
    }
}
