"""GPU parity for Scene::find3d2dMatches: the hash-join
kernels (through the C ABI) against the oracle's literal loops, exact."""
import numpy as np
import pytest
import torch

from sfmx import scene
import scene_cases

pytestmark = pytest.mark.gpu


def test_edge_case_exact():
    from oracle import oracle
    kps, pairs, m, off, oo, osh, oxy = scene_cases.edge_case()
    for shot in range(4):
        ek, ep = oracle.find_3d2d_matches(kps, pairs, m, off, oo, osh, oxy, shot)
        gk, gp, gxy = scene.find_3d2d_matches(kps, pairs, m, off, oo, osh, oxy, shot)
        assert np.array_equal(gk, ek) and np.array_equal(gp, ep), (shot, gk, ek)
        hit = gk >= 0
        assert np.array_equal(gxy[hit], kps[shot][gk[hit]]) and np.all(np.isnan(gxy[~hit]))


@pytest.mark.parametrize("seed", [3, 7])
def test_scene_exact_every_shot(seed):
    from oracle import oracle
    kps, pairs, m, off, oo, osh, oxy = scene_cases.scene_case(8, 1500, seed=seed)
    for shot in range(8):
        ek, ep = oracle.find_3d2d_matches(kps, pairs, m, off, oo, osh, oxy, shot)
        gk, gp, _ = scene.find_3d2d_matches(kps, pairs, m, off, oo, osh, oxy, shot)
        assert np.array_equal(gk, ek) and np.array_equal(gp, ep)
        assert (gk >= 0).sum() > 0


def test_device_inputs():
    kps, pairs, m, off, oo, osh, oxy = scene_cases.scene_case(6, 1200, seed=5)
    hk, hp, hxy = scene.find_3d2d_matches(kps, pairs, m, off, oo, osh, oxy, 2)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    dk = [d(k) for k in kps]
    dm, doff, doo, dsh, dxy = d(m.view(np.uint8)), d(off), d(oo), d(osh), d(oxy)
    n = len(osh)
    ok, op, oxy_out = (torch.zeros(n, dtype=torch.int32, device="cuda"), torch.zeros(n, dtype=torch.int32, device="cuda"),
                       torch.zeros(2 * n, dtype=torch.float32, device="cuda"))
    scene.find_3d2d_matches_device([t.data_ptr() for t in dk], [len(k) for k in kps], pairs, dm.data_ptr(),
                                   doff.data_ptr(), doo.data_ptr(), len(oo) - 1, dsh.data_ptr(), dxy.data_ptr(), 2,
                                   ok.data_ptr(), op.data_ptr(), oxy_out.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(ok.cpu().numpy(), hk) and np.array_equal(op.cpu().numpy(), hp)
    assert np.array_equal(oxy_out.cpu().numpy().reshape(-1, 2), hxy, equal_nan=True)
