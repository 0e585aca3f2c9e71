"""GPU parity of the opt-in dispatch extensions (PNETGPU_RX_VLAN,
PNETGPU_RX_IPV6_EXT) vs the oracle: descriptor mode at arbitrary alignment
(L4 headers beyond the LDS window included), fixed-stride mode, and TX fill."""
import numpy as np
import pytest
import torch

import libpnet_amd as lp
from libpnet_amd.engine import ALL_COLUMNS
from oracle import coracle
from tests import framegen
from tests.test_gpu_parity import compare, to_dev

pytestmark = pytest.mark.gpu
FLAGS = [0, 1, 2, 3]


@pytest.mark.parametrize("flags", FLAGS)
def test_extension_frames_desc(flags):
    rng = np.random.default_rng(40 + flags)
    frames = framegen.extension_frames(rng) + framegen.random_frames(rng, 800)
    buf, offs, lens = framegen.pack(frames, gap=13, rng=rng)
    rec = coracle.rx_batch(buf, len(frames), offsets=offs, lengths=lens, flags=flags)
    for data_offset in (0, 3):
        d = to_dev(np.concatenate([np.zeros(16, np.uint8), buf]))[data_offset:]
        res = lp.rx_process(d, offsets=to_dev((offs + 16 - data_offset).astype(np.int64)),
                            lengths=to_dev(lens.astype(np.int32)), columns=ALL_COLUMNS, flags=flags)
        torch.cuda.synchronize()
        compare(res, rec)


@pytest.mark.parametrize("flags", [1, 3])
def test_vlan_stride_mode(flags):
    rng = np.random.default_rng(7)
    frames = [framegen.add_vlan(framegen.build_frame(rng, "udp", 22), [(0x8100, i)]) for i in range(1000)]
    stride = 64
    buf = np.zeros(stride * len(frames) + 32, np.uint8)
    for i, f in enumerate(frames):
        buf[i * stride:i * stride + len(f)] = np.frombuffer(f, np.uint8)
    rec = coracle.rx_batch(buf, len(frames), stride=stride, frame_len=len(frames[0]), flags=flags)
    res = lp.rx_process(to_dev(buf), stride=stride, frame_len=len(frames[0]), n_frames=len(frames),
                        columns=ALL_COLUMNS, flags=flags)
    torch.cuda.synchronize()
    compare(res, rec)
    assert (res.numpy()["l3_offset"] == 18).all()


@pytest.mark.parametrize("flags", [3])
def test_tx_fill_with_extensions(flags):
    rng = np.random.default_rng(77)
    frames = framegen.extension_frames(rng)
    buf, offs, lens = framegen.pack(frames, gap=7, rng=rng)
    d = to_dev(buf.copy())
    res = lp.tx_fill_checksums(d, offsets=to_dev(offs.astype(np.int64)), lengths=to_dev(lens.astype(np.int32)),
                               columns=ALL_COLUMNS, flags=flags)
    want_buf, want_rec = coracle.tx_fill(buf, len(frames), offsets=offs, lengths=lens, flags=flags)
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy(), want_buf)
    compare(res, want_rec)
