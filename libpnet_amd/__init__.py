"""libpnet_amd — MI355X-native engine for libpnet's per-packet receive hot path.

Ethernet/IPv4/IPv6 header extraction + ones-complement Internet checksums
(UDP/TCP/ICMP/ICMPv6) over device-resident frame batches, bit-exact with
pnet_packet. The product is libpnetgpu.so (HIP kernels behind the C-ABI in
include/pnetgpu.h); this package is its Python host binding.
"""
from ._lib import DEFS, LIB_PATH, PnetGpuError, lib  # noqa: F401  (fails loudly if the .so is absent)
from . import packet, synth  # noqa: F401  (packet: pnet_packet's function names)
from .ring import HostRegistration, Ring, batch_pack, host_threads, pcap_frames, pcap_index, pcap_info  # noqa: F401
from .afpacket import AfPacket, tpacket3_walk  # noqa: F401
from .views import frame_view  # noqa: F401
from .engine import (ALL_COLUMNS, COUNTER_NAMES, DESC_COMPACT, DESC_HINT_JUMBO, DESC_HINT_LARGE, desc_size_hint, FIELD_COLUMNS, IPV4_COLUMNS, RECORD_COLUMNS,  # noqa: F401
                     Context, RxResult,
                     checksum_adv_slices, checksum_slices, checksum_slices_compact, checksum_slices_strided, column_bytes, context, ipv4_checksum_slices,
                     ipv6_checksum_slices, last_rx_kernel, rx_process, slice_descriptors, tx_fill_checksums)

__version__ = "0.1.0"
