"""The host build of the traffic generator (ingot_amd.hostgen, used for
bench.py's CPU baseline before the process touches the GPU): the same bytes
as the device generator, and (CPU) the workload shape the oracle sees."""
import numpy as np
import pytest

import oracle
from ingot_amd import Chain, GenProfile
from ingot_amd.hostgen import gen_frames_host

PROFILES = [(p, None) for p in GenProfile] + [(GenProfile.V4UDP64, 64),
                                             (GenProfile.MIXED, 2048)]


def test_host_generator_shapes():
    """C2: every 64-B slot parses as UdpParser, Ok; C3 lengths in [64, 1500]
    (raised to fit the chain) with a mix of v4/v6 and TCP/UDP; deterministic."""
    a, o, ln = gen_frames_host(GenProfile.V4UDP64, 4096, stride=64)
    assert o is None and ln is None and a.nbytes == 4096 * 64 + 256
    rec = oracle.parse_batch(a, None, None, Chain.UdpParser, stride=64, n=4096)
    assert (rec["status"] == 0).all() and (rec["payload_off"] == 42).all()
    a, o, ln = gen_frames_host(GenProfile.MIXED, 20_000)
    assert ln.min() >= 64 and ln.max() <= 1500 + 200
    rec = oracle.parse_batch(a, o, ln, Chain.GenericUlp)
    assert (rec["status"] == 0).all()
    assert set(np.unique(rec["l3_kind"])) == {1, 2} and set(np.unique(rec["l4_kind"])) == {1, 2}
    a2, o2, ln2 = gen_frames_host(GenProfile.MIXED, 20_000, threads=3)
    assert a2.tobytes() == a.tobytes() and (o2 == o).all() and (ln2 == ln).all()
    # a later shard starts where the first one's frames continue
    _, _, l_first = gen_frames_host(GenProfile.MIXED, 1000, first=19_000)
    assert (l_first == ln[19_000:]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("profile,stride", PROFILES)
def test_host_generator_equals_device(profile, stride):
    import torch

    import ingot_amd

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    n = 100_003
    da, do, dl = ingot_amd.gen_frames(profile, n, stride=stride, first=5)
    torch.cuda.synchronize()
    ha, ho, hl = gen_frames_host(profile, n, stride=stride, first=5)
    if dl is not None:
        assert (dl.cpu().numpy() == hl).all()
    if do is not None:
        assert (do.cpu().numpy().view(np.uint64) == ho).all()
    d = da.cpu().numpy()
    assert d.shape == ha.shape
    bad = np.nonzero(d != ha)[0]
    assert bad.size == 0, (profile.name, bad[:10])
