"""k_fast's whole-plane NMS fallback (taken when a wave finds more corners than its corner list
holds, 256 by default; csrc/orb_hip.hip k_fast) is bit-exact with the oracle: the list capacity
is lowered through orb_debug_set_fast_corner_list so that the fallback runs in every workgroup
with a corner (cap 0) or in most of them (cap 8), on scene, low-texture and noise frames, and
through the batched device path as well as the host entry point."""
import numpy as np
import pytest

import orbslam_jpminipc_amd as orb
from oracle_lib import Oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cap", [0, 8])
def test_corner_list_fallback_parity(cap):
    ext = orb.ORBextractor(1000, 1.2, 8, orb.FAST_SCORE, 20, device=0)
    ora = Oracle(1000, 1.2, 8, 1, 20)
    assert orb.hip_lib().orb_debug_set_fast_corner_list(ext._h, cap) == 0
    frames = list(orb.synth_stream(640, 480, stream=3, first=0, count=2))
    frames += [orb.synth_special(k, 640, 480, seed=5) for k in (orb.SYN_LOWTEX, orb.SYN_NOISE)]
    for img in frames:
        kg, dg = ext(img)
        ko, do = ora.extract(img)
        assert len(kg) == len(ko) and kg.tobytes() == ko.tobytes()
        assert (dg is None and len(ko) == 0) or dg.tobytes() == do.tobytes()


def test_corner_list_fallback_batch_device():
    import torch

    B = 4
    frames = orb.synth_stream(1241, 376, stream=1, first=0, count=B)
    ext = orb.ORBextractor(2000, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=B)
    d = torch.from_numpy(frames).cuda()
    ref = [t.clone() for t in ext.extract_batch_device(d)]
    assert orb.hip_lib().orb_debug_set_fast_corner_list(ext._h, 4) == 0
    out = ext.extract_batch_device(d)
    torch.cuda.synchronize()
    for a, b in zip(ref, out):
        assert torch.equal(a, b)
    ora = Oracle(2000, 1.2, 8, 1, 20)
    n = out[2].cpu().numpy()
    ko, do = ora.extract(frames[0])
    assert n[0] == len(ko)
    assert out[0][0, : n[0]].cpu().numpy().tobytes() == ko.tobytes()
    assert out[1][0, : n[0]].cpu().numpy().tobytes() == do.tobytes()
    assert orb.hip_lib().orb_debug_set_fast_corner_list(ext._h, 257) < 0
