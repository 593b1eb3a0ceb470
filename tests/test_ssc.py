"""SSCBench scoring: the FOV mask and the per-frame counts of
sscbench/evaluate_model_sscbench.py.

Fixture tests/golden/ssc_scoring.json holds what the reference's own functions produced
(tests/golden/make_golden.py, fx_ssc_scoring) on the seeded frames of tests/_ssc_inputs.py.
Integer work: every count must be bit-exact.  The final tables (IoU / mIoU / Hungarian) are
checked against oracle/ssc_oracle.py's restatement of :532-609 (parity unpinned there:
the reference computes them inside main())."""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

from _ssc_inputs import make_frame
from conftest import GOLDEN
from oracle import ssc_oracle as so
from scenedino_amd import sscbench as sb

G = json.load(open(os.path.join(GOLDEN, "ssc_scoring.json")))
KEYS = ["tp", "fp", "tn", "fn", "tp_seg", "fp_seg", "tn_seg", "fn_seg", "confusion_seg",
        "tp_recall_seg", "sum_recall_seg"]


def _eq_counts(c, ref):
    for k in KEYS:
        assert np.array_equal(np.asarray(c[k]).astype(np.int64), np.asarray(ref[k])), k


@pytest.fixture(scope="module")
def fov_cpu():
    return so.fov_mask(sb.read_calib()["Tr"], sb.get_cam_k())


# ---------------------------------------------------------------- CPU: oracle + host logic
def test_label_maps_match_reference_yaml():
    lm = G["label_maps"]
    assert {int(k): v for k, v in lm["sscbench_to_label"].items()} == sb.SSCBENCH_TO_LABEL
    assert {int(k): v for k, v in lm["cityscapes_to_label"].items()} == sb.CITYSCAPES_TO_LABEL
    assert {int(k): v for k, v in lm["labels"].items()} == sb.LABELS
    assert {int(k): v for k, v in lm["weights"].items()} == sb.WEIGHTS
    assert so.SSCBENCH_TO_LABEL == sb.SSCBENCH_TO_LABEL


def test_oracle_fov_matches_reference(fov_cpu):
    assert hashlib.sha256(fov_cpu.astype(np.uint8).tobytes()).hexdigest() == G["fov_sha256"]


@pytest.mark.parametrize("fi", [0, 1])
def test_oracle_counts_match_reference(fov_cpu, fi):
    fr = G["frames"][fi]
    sig, segs, gt = make_frame(fr["seed"])
    C = so.frame_confusions(sig, segs, gt, fov_cpu)
    for i, size in enumerate(so.SIZES):
        _eq_counts(so.counts_from_confusion(C[i]), fr["sizes"][str(size)])


def test_crop_bounds_reference_floor_division():
    # int(12.8 // 0.2) etc. as the reference evaluates them
    assert [sb.crop_bounds(s) for s in sb.SIZES] == [(64, 96, 160), (128, 64, 192), (256, 0, 256)]


def test_host_counts_and_tables_from_golden_confusions():
    """counts_from_confusion + tables() (host side of SSCBenchScores) on the reference's
    confusion matrices of the two frames summed, vs the oracle restatement."""
    conf = {}
    for size in sb.SIZES:
        conf[size] = sum(np.asarray(fr["sizes"][str(size)]["confusion_seg"], np.int64)
                         for fr in G["frames"])
        ref = {k: sum(np.asarray(fr["sizes"][str(size)][k], np.int64) for fr in G["frames"])
               for k in KEYS}
        _eq_counts(sb.counts_from_confusion(conf[size]), ref)
    scores = sb.SSCBenchScores(device="cpu")
    acc = np.concatenate([conf[s].reshape(-1) for s in sb.SIZES] + [np.zeros(1, np.int64)])
    scores._acc = torch.from_numpy(acc)
    got, want = scores.tables(), so.results_tables(conf)
    for mode in ("direct", "hungarian"):
        np.testing.assert_array_equal(got[mode]["table"], want[mode]["table"])
        assert got[mode]["miou"] == want[mode]["miou"]
        assert got[mode]["weighted_miou"] == want[mode]["weighted_miou"]
    np.testing.assert_array_equal(got["hungarian"]["reassignment"],
                                  want["hungarian"]["reassignment"])
    rep = scores.report()
    assert "Mode: hungarian" in rep and rep.count("| mIoU") == 2


def test_unmapped_label_raises_on_host():
    scores = sb.SSCBenchScores(device="cpu")
    scores._acc[-1] = 3
    with pytest.raises(KeyError):
        scores.results()


# ---------------------------------------------------------------- GPU: sd_voxel_fov / sd_ssc_confusion
@pytest.mark.gpu
def test_fov_kernel_matches_reference():
    m = sb.get_fov_mask("cuda").cpu().numpy()
    assert hashlib.sha256(m.astype(np.uint8).tobytes()).hexdigest() == G["fov_sha256"]
    assert int(m.sum()) == G["fov_count"]


@pytest.mark.gpu
def test_confusion_kernel_matches_reference_counts():
    fov = sb.get_fov_mask("cuda")
    scores = sb.SSCBenchScores(device="cuda", check_each_frame=True)
    for fr in G["frames"]:
        sig, segs, gt = make_frame(fr["seed"])
        one = sb.SSCBenchScores(device="cuda", check_each_frame=True)
        args = [torch.from_numpy(sig).cuda(), torch.from_numpy(segs).cuda(),
                torch.from_numpy(gt).cuda(), fov]
        one.add_frame(*args)
        scores.add_frame(*args)
        res = one.results()
        for size in sb.SIZES:
            _eq_counts(res[size], fr["sizes"][str(size)])
    conf = {size: sum(np.asarray(fr["sizes"][str(size)]["confusion_seg"], np.int64)
                      for fr in G["frames"]) for size in sb.SIZES}
    got = scores.confusions()
    for size in sb.SIZES:
        np.testing.assert_array_equal(got[size], conf[size])
    want = so.results_tables(conf)
    tabs = scores.tables()
    for mode in ("direct", "hungarian"):
        np.testing.assert_array_equal(tabs[mode]["table"], want[mode]["table"])


@pytest.mark.gpu
@pytest.mark.parametrize("dims,additional", [((40, 200, 16), True), ((64, 256, 48), False)])
def test_confusion_kernel_ragged_shapes_vs_oracle(dims, additional):
    """Shapes other than 256 x 256 x 32 (crop windows partly or wholly outside the grid,
    nz = 16 / 48), with and without the additional invalids; host numpy inputs and float64
    class ids as downsample_and_predict returns them."""
    sig, segs, gt = make_frame(7, dims)
    rng = np.random.default_rng(5)
    fov = rng.random(dims) < 0.7
    sig[rng.random(dims) < 0.01] = np.nan  # NaN densities keep their class (numpy compare)
    scores = sb.SSCBenchScores(device="cuda", additional_invalids=additional)
    scores.add_frame(sig, segs.astype(np.float64), gt.astype(np.int64), fov)
    got = scores.confusions()
    want = so.frame_confusions(sig, segs, gt, fov, additional_invalids=additional)
    for i, size in enumerate(sb.SIZES):
        np.testing.assert_array_equal(got[size], want[i])


@pytest.mark.gpu
def test_confusion_kernel_flags_unmapped_labels():
    sig, segs, gt = make_frame(3, (16, 16, 16))
    fov = np.ones((16, 16, 16), bool)
    gt[0, 0, 0] = 42       # no key in sscbench_to_label
    scores = sb.SSCBenchScores(device="cuda", check_each_frame=True)
    with pytest.raises(KeyError):
        scores.add_frame(sig, segs, gt, fov)
    segs2 = segs.copy()
    segs2[1, 1, 1] = 19    # no cityscapes class 19
    scores = sb.SSCBenchScores(device="cuda")
    scores.add_frame(sig, segs2, make_frame(3, (16, 16, 16))[2], fov)
    with pytest.raises(KeyError):
        scores.results()
