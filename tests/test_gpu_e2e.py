"""GPU: the bench's PCIe-inclusive pipeline (bench.e2e_rate) computes the right
records, for a fixed-stride batch and for a compact-descriptor IMIX batch
(each chunk's frame span + rebased u32/u16 descriptors shipped with its size
hint): the last two chunks' device results equal the oracle's records on the
same frames. The rates it reports are the bench's e2e lines."""
import numpy as np
import pytest
import torch

import bench
from oracle import coracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,n", [("udp64", 1 << 16), ("imix", 1 << 16), ("udp6_jumbo", 1 << 10)])
def test_e2e_pipeline_records_equal_oracle(name, n):
    lp = bench.load_library()
    dev = torch.device("cuda", 0)
    sh = bench.Shard(name, n, 7, dev)
    w = sh.w
    checked = []

    def verify(first, m, res):
        torch.cuda.synchronize()
        got = res.numpy()
        if w.stride:
            rec = coracle.rx_batch(w.buf, m, stride=w.stride, frame_len=w.frame_len, first=first * w.stride)
        else:
            rec = coracle.rx_batch(w.buf, m, offsets=w.offsets[first:first + m], lengths=w.lengths[first:first + m])
        for c in lp.IPV4_COLUMNS:
            assert np.array_equal(got[c], rec[c]), (name, first, c)
        checked.append(first)

    out = bench.e2e_rate(sh, dev, chunks=4, reps=1, verify=verify, seconds=0)
    assert out is not None and out["mpkts_s"] > 0 and out["stages"]["h2d_s"] > 0
    assert checked == [2 * (n // 4), 3 * (n // 4)]
    up = out["link_bytes_per_frame"]["up"]
    assert up == pytest.approx(sh.frame_bytes / n + (0 if w.stride else 6), rel=0.02)
