"""Size-independent properties of the sender side at every workload's full
per-GPU size (the bench's batches): after tx_fill_checksums every frame whose
checksums the receive path computes verifies (no bad IPv4 header or L4
checksum left), a second fill changes no byte (idempotence), and the patched
bytes differ from the input only inside the two checksum fields of each frame
(the 1 % of corrupted frames keep their corruption, now covered by a correct
checksum). The bit-exact comparison with the oracle's fill is in
test_gpu_tx.py (smaller batches) and test_gpu_deferred.py."""
import numpy as np
import pytest
import torch

import libpnet_amd as lp
from tests.test_gpu_parity import FULL, to_dev

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", list(FULL))
def test_tx_fill_full_size_properties(name):
    n = FULL[name]
    w = lp.synth.make(name, n, seed=21, corrupt_ppm=10000)
    d = to_dev(w.buf)
    if w.stride:
        kw = dict(stride=w.stride, frame_len=w.frame_len, n_frames=n)
    else:
        kw = dict(offsets=to_dev(w.offsets.astype(np.int64)), lengths=to_dev(w.lengths.astype(np.int32)))
    before = d.clone()
    first = lp.tx_fill_checksums(d, columns=("status",), counters=True, **kw)
    once = d.clone()
    lp.tx_fill_checksums(d, columns=("status",), counters=True, **kw)
    assert torch.equal(d, once), "a second fill changed bytes"
    res = lp.rx_process(d, columns=lp.IPV4_COLUMNS, **kw)
    torch.cuda.synchronize()
    c = res.counter_dict()
    assert c["frames"] == n and c["ip_csum_bad"] == 0 and c["l4_csum_bad"] == 0, c
    # every changed byte lies inside a checksum field the receive path located:
    # the IPv4 header checksum (frame bytes 24-25) or the L4 one (UDP +6, TCP +16,
    # ICMP / ICMPv6 +2 from the L4 offset)
    changed = torch.nonzero(once != before).flatten().cpu().numpy().astype(np.int64)
    rec = res.numpy()
    offs = (np.arange(n, dtype=np.int64) * w.stride) if w.stride else w.offsets.astype(np.int64)
    i = np.searchsorted(offs, changed, side="right") - 1
    rel = changed - offs[i]
    lut = np.full(256, -100, np.int64)
    lut[[17, 6, 1, 58]] = [6, 16, 2, 2]
    l4rel = rel - rec["l4_offset"][i].astype(np.int64) - lut[rec["ip_proto"][i]]
    ok = (((rel == 24) | (rel == 25)) & (rec["ethertype"][i] == 0x0800)) | (l4rel == 0) | (l4rel == 1)
    assert ok.all(), f"{int((~ok).sum())} bytes changed outside the checksum fields"
    assert first.counter_dict()["frames"] == n
