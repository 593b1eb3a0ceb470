"""CPU tests of the host-side boundary around the render: ImageRaySampler.reconstruct
(reference scenedino/common/ray_sampler.py:515-607, incl. the dino_artifacts branch
:599-605) against shapes the reference itself produced (tests/golden/reconstruct_shapes.json,
made by tests/golden/make_golden.py fx_reconstruct), and the debug NaN guard of
NeRFRenderer.composite (reference scenedino/renderer/nerf.py:428-432)."""
import importlib.util
import json
import os

import pytest
import torch

from scenedino_amd.common.ray_sampler import ImageRaySampler
from scenedino_amd.renderer.nerf import NeRFRenderer

HERE = os.path.dirname(__file__)


def _make_golden():
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(HERE, "golden", "make_golden.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)  # module level only defines helpers; the reference is imported lazily
    return mod


@pytest.mark.parametrize("mode", ["patch", "upscaled"])
def test_reconstruct_matches_reference_shapes(mode):
    with open(os.path.join(HERE, "golden", "reconstruct_shapes.json")) as f:
        want = json.load(f)[mode]
    mg = _make_golden()
    upscaled = mode == "upscaled"
    inp = mg._reconstruct_input(upscaled=upscaled)
    flat = {k: v.clone() for k, v in inp["coarse"].items()}
    flat.update({k: v.clone() for k, v in inp.items() if torch.is_tensor(v)})
    s = ImageRaySampler(z_near=3, z_far=80, height=8, width=16, channels=3, dino_upscaled=upscaled)
    out = s.reconstruct(inp)
    got = {k: list(v.shape) for k, v in out.items() if torch.is_tensor(v)}
    got.update({"coarse." + k: list(v.shape) for k, v in out["coarse"].items()})
    assert got == want
    # reconstruct only re-views: every element stays where it was in row-major order
    for k, v in out["coarse"].items():
        assert torch.equal(v.reshape(-1), flat[k].reshape(-1)), k
    for k in ("rgb_gt", "dino_gt", "dino_artifacts"):
        assert torch.equal(out[k].reshape(-1), flat[k].reshape(-1)), k


def test_reconstruct_without_artifacts_leaves_dict_alone():
    mg = _make_golden()
    inp = mg._reconstruct_input()
    del inp["dino_artifacts"]
    out = ImageRaySampler(z_near=3, z_far=80, height=8, width=16).reconstruct(inp)
    assert "dino_artifacts" not in out
    assert list(out["dino_gt"].shape) == [2, 1, 2, 4, 6]


def _composite_outputs(R=4, K=5):
    w = torch.rand(1, R, K)
    return [w, torch.rand(1, R, 3), torch.rand(1, R), torch.rand(1, R, K),
            torch.zeros(1, R, K, 1, dtype=torch.bool), torch.rand(1, R, K)]


def test_nan_guard_silent_without_nan(capsys):
    NeRFRenderer._nan_guard(*_composite_outputs())
    NeRFRenderer._nan_guard(None, None, torch.rand(3), None, None, None)
    assert capsys.readouterr().out == ""


@pytest.mark.parametrize("slot", [0, 2, 3, 5])
def test_nan_guard_exits_on_nan(capsys, slot):
    outs = _composite_outputs()
    outs[slot].view(-1)[1] = float("nan")
    with pytest.raises(SystemExit):
        NeRFRenderer._nan_guard(*outs)
    names = ["weights", "rgb_final", "depth_final", "alphas", "invalid", "z_samp"]
    assert f"Detected NaN in {names[slot]}" in capsys.readouterr().out


def test_nan_check_flag_from_env(monkeypatch):
    monkeypatch.setenv("SCENEDINO_AMD_NAN_CHECK", "1")
    assert NeRFRenderer().check_nan
    monkeypatch.setenv("SCENEDINO_AMD_NAN_CHECK", "0")
    assert not NeRFRenderer().check_nan
