"""Host-side argument handling of libpnet_amd.packet (no GPU calls)."""
import ipaddress

import pytest

from libpnet_amd import packet


def test_address_forms():
    assert packet._addr("10.0.0.1", 4) == bytes([10, 0, 0, 1])
    assert packet._addr(ipaddress.IPv6Address("::1"), 16) == bytes(15) + b"\x01"
    assert packet._addr(bytes([1, 2, 3, 4]), 4) == bytes([1, 2, 3, 4])
    with pytest.raises(ValueError):
        packet._addr("10.0.0.1", 16)


def test_ipv4_checksum_rejects_short_packet_like_new():
    # Ipv4Packet::new returns None below 20 bytes (ipv4.rs, decorator.rs:593-600)
    with pytest.raises(ValueError):
        packet.ipv4.checksum(b"\x45" * 19)


def test_reference_names_present():
    for mod, names in ((packet.util, ("checksum", "ipv4_checksum", "ipv6_checksum")),
                       (packet.ipv4, ("checksum",)), (packet.icmp, ("checksum",)), (packet.icmpv6, ("checksum",)),
                       (packet.udp, ("ipv4_checksum", "ipv6_checksum", "ipv4_checksum_adv", "ipv6_checksum_adv")),
                       (packet.tcp, ("ipv4_checksum", "ipv6_checksum", "ipv4_checksum_adv", "ipv6_checksum_adv"))):
        for n in names:
            assert callable(getattr(mod, n))
