"""CPU checks of the synthetic workload producer against the oracle."""
import numpy as np
import pytest

import libpnet_amd as lp
from oracle import coracle, pyoracle


def oracle_counts(r):
    st = r["status"].astype(np.int64)
    v4 = (st & 3) == 1
    return {"ip_bad": int((v4 & ((st & pyoracle.ST_L3_MALFORMED) == 0) & ((st & pyoracle.ST_IP_CSUM_OK) == 0)).sum()),
            "l4_bad": int((((st & pyoracle.ST_L4_CSUM_DONE) != 0) & ((st & pyoracle.ST_L4_CSUM_OK) == 0)).sum())}


def run_oracle(w, nthreads=4):
    if w.stride:
        return coracle.rx_batch(w.buf, w.n, stride=w.stride, frame_len=w.frame_len, nthreads=nthreads)
    return coracle.rx_batch(w.buf, w.n, offsets=w.offsets, lengths=w.lengths, nthreads=nthreads)


@pytest.mark.parametrize("name,n", [("rs_sender", 64), ("udp64", 50000), ("tcp1500", 3000), ("udp1500", 3000), ("imix", 20000),
                                    ("udp6_jumbo", 300)])
def test_workload_verifies_and_counts(name, n):
    w = lp.synth.make(name, n, seed=5, corrupt_ppm=10000)
    r = run_oracle(w)
    c = oracle_counts(r)
    assert c["ip_bad"] == w.expect["ip_bad"] and c["l4_bad"] == w.expect["l4_bad"]
    assert (r["status"] & (pyoracle.ST_L4_CSUM_DONE)).all()
    assert w.expect["bytes"] == (n * w.stride if w.stride else int(w.lengths.sum()))


def test_rs_sender_frame_is_the_reference_frame():
    w = lp.synth.make("rs_sender", 4, corrupt_ppm=0)
    r = run_oracle(w)
    assert (r["ip_csum"] == 0xB8CA).all() and (r["l4_csum"] == 0xB94C).all()
    assert bytes(w.buf[34 + 8:34 + 13]) == b"rmesg"


def test_deterministic_across_threads():
    a = lp.synth.make("imix", 30000, seed=9, nthreads=1)
    b = lp.synth.make("imix", 30000, seed=9, nthreads=7)
    assert (a.buf == b.buf).all() and (a.offsets == b.offsets).all()


@pytest.mark.parametrize("name", ["udp64", "imix", "tcp1500", "udp1500"])
def test_range_is_a_slice_of_the_whole_batch(name):
    """pnetgpu_synth_fill_range: frames [first, first + n) equal those frames of the
    whole batch byte for byte (a rank's shard of the bench's global batch), and
    pnetgpu_synth_lengths gives their lengths without building them."""
    whole = lp.synth.make(name, 700, seed=9)
    part = lp.synth.make(name, 250, seed=9, first=333)
    if whole.stride:
        s = whole.stride
        assert np.array_equal(part.buf[:250 * s], whole.buf[333 * s:583 * s])
    else:
        lo = int(whole.offsets[333])
        hi = int(whole.offsets[582] + whole.lengths[582])
        assert np.array_equal(part.buf[:hi - lo], whole.buf[lo:hi])
        assert np.array_equal(part.lengths, whole.lengths[333:583])
    assert np.array_equal(lp.synth.lengths(name, 250, seed=9, first=333),
                          whole.lengths[333:583] if not whole.stride else np.full(250, whole.stride, np.uint32))
