"""CPU checks of the sender-side restatement (oracle_tx_fill): building the
rs_sender frame with zeroed checksum fields and filling them reproduces the
reference frame (benches/rs_sender.rs:25-101), and every patched frame verifies."""
import numpy as np

import libpnet_amd as lp
from oracle import coracle, pyoracle
from tests import kats


def test_rs_sender_fill_reproduces_reference_frame():
    (v,) = [k for k in kats.by_kind("rx_frame") if k["name"] == "rs_sender_frame"]
    ref = np.frombuffer(v["data"], np.uint8)
    blank = ref.copy()
    blank[24:26] = 0          # IPv4 checksum field
    blank[40:42] = 0          # UDP checksum field
    patched, rec = coracle.tx_fill(np.concatenate([blank, np.zeros(16, np.uint8)]), 1, stride=64, frame_len=64)
    assert bytes(patched[:64]) == v["data"]
    assert rec["ip_csum"][0] == 0xB8CA and rec["l4_csum"][0] == 0xB94C


def test_fill_then_verify_all_ok():
    w = lp.synth.make("imix", 5000, seed=8, corrupt_ppm=400000)
    patched, before = coracle.tx_fill(w.buf, w.n, offsets=w.offsets, lengths=w.lengths)
    after = coracle.rx_batch(patched, w.n, offsets=w.offsets, lengths=w.lengths)
    st = after["status"]
    assert ((st & pyoracle.ST_L4_CSUM_OK) != 0).all() and ((st & pyoracle.ST_IP_CSUM_OK) != 0).all()
    # the computed values do not depend on the stored fields (skipped words)
    assert (after["l4_csum"] == before["l4_csum"]).all() and (after["ip_csum"] == before["ip_csum"]).all()
