"""GPU parity of the MTU shape with several runs per wave: the record stores and
the TX fill's in-place writes of the last three runs are held back in
registers (rx_generic.h; kDeferRuns / kTxDeferRuns in rx_config.h) and stored when a newer run
needs the place or at the wave's end. The full-size tests run 4 runs per wave;
here the grid is cut to one block per CU (the blocks_per_cu tuning) so waves
hold 4, 8 (the claimed-run schedule then joins in) or a ragged number of runs,
receive and TX, against the oracle (records, counters, patched bytes)."""
import numpy as np
import pytest
import torch

import libpnet_amd as lp
from oracle import coracle
from tests.test_gpu_parity import NTHREADS, compare, oracle_counters, to_dev

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["tcp1500", "udp1500"])
@pytest.mark.parametrize("n,per_cu", [(1 << 18, 1), ((1 << 18) + 37, 1), (1 << 19, 1), (1 << 19, 2)])
@pytest.mark.parametrize("tx", [False, True])
def test_mtu_runs_per_wave(name, n, per_cu, tx, tune):
    w = lp.synth.make(name, n, seed=n + per_cu, corrupt_ppm=30000)
    lens = np.full(n, w.frame_len, np.uint32)
    tune("blocks_per_cu", per_cu)
    d = to_dev(w.buf)
    # no IPv6 address columns: those make the kernel store each run at once
    cols = lp.IPV4_COLUMNS + (("vlan_tci", "l3_offset") if not tx else ())
    kw = dict(stride=w.stride, frame_len=w.frame_len, n_frames=n)
    if tx:
        res = lp.tx_fill_checksums(d, columns=cols, counters=True, **kw)
        want_buf, rec = coracle.tx_fill(w.buf, n, stride=w.stride, frame_len=w.frame_len)
    else:
        res = lp.rx_process(d, columns=cols, **kw)
        rec = coracle.rx_batch(w.buf, n, stride=w.stride, frame_len=w.frame_len, nthreads=NTHREADS)
    torch.cuda.synchronize()
    assert lp.engine.last_rx_kernel().startswith("rx_kernel<8, 8, 4"), lp.engine.last_rx_kernel()
    compare(res, rec)
    assert res.counter_dict() == oracle_counters(rec, lens)
    if tx:
        got = d.cpu().numpy()
        assert np.array_equal(got, want_buf), f"{int((got != want_buf).sum())} bytes differ"
