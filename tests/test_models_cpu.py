"""CPU checks of the PyTorch oracles (shapes, weight round trips) and of host-side weight re-packing
used by the native engines (transposed conv -> parity-class 3x3 conv)."""
import pytest
import torch
import torch.nn.functional as F


def test_deconv_as_conv_identity_2d_3d():
    from stereoalgorithms_amd.ops import deconv_as_conv_weight
    torch.manual_seed(0)
    x = torch.randn(1, 6, 5, 7)
    wt = torch.randn(6, 3, 4, 4)
    ref = F.conv_transpose2d(x, wt, None, 2, 1)
    eq = F.conv2d(x, deconv_as_conv_weight(wt), None, 1, 1)
    for p in range(4):
        pb, pa = p & 1, p >> 1
        torch.testing.assert_close(eq[:, 3 * p:3 * p + 3], ref[:, :, pa::2, pb::2], rtol=1e-5, atol=1e-5)
    x3 = torch.randn(1, 4, 3, 4, 5)
    wt3 = torch.randn(4, 2, 4, 4, 4)
    ref3 = F.conv_transpose3d(x3, wt3, None, 2, 1)
    eq3 = F.conv3d(x3, deconv_as_conv_weight(wt3), None, 1, 1)
    for p in range(8):
        pb, pa, pc = p & 1, (p >> 1) & 1, p >> 2
        torch.testing.assert_close(eq3[:, 2 * p:2 * p + 2], ref3[:, :, pc::2, pa::2, pb::2], rtol=1e-5, atol=1e-5)


def test_fast_acvnet_oracle_shapes_and_save(tmp_path):
    from stereoalgorithms_amd.models import fast_acvnet as FA
    from stereoalgorithms_amd.utils.weights import save_model
    m = FA.build("fastacvnet-plus", seed=0)
    torch.manual_seed(1)
    l, r = torch.randn(1, 3, 64, 96), torch.randn(1, 3, 64, 96)
    with torch.no_grad():
        d = m(l, r)
    assert d.shape == (1, 64, 96) and torch.isfinite(d).all()
    assert d.min() >= 0 and d.max() <= 4 * 47 + 1e-3  # convex mix of sampled disparities, x4
    path = save_model(m, tmp_path / "f.safetensors", "fastacvnet-plus")
    from safetensors import safe_open
    with safe_open(str(path), "pt") as f:
        keys = set(f.keys())
        meta = f.metadata()
    assert "feature.block0.0.0.conv_dw.weight" in keys and "spx.0.bias" in keys
    assert "hourglass_att.conv2_up.conv.weight" in keys and meta.get("model") == "fastacvnet-plus"


@pytest.mark.parametrize("preset", ["crestereo-iter2"])
def test_crestereo_oracle_shape(preset):
    from stereoalgorithms_amd.models import crestereo as CR
    m = CR.build(preset, seed=0)
    with torch.no_grad():
        d = m(torch.rand(1, 3, 64, 64) * 255, torch.rand(1, 3, 64, 64) * 255)
    assert d.shape[0] == 1 and d.shape[-2:] == (64, 64) and torch.isfinite(d).all()


@pytest.mark.parametrize("preset", ["hitnet-d400", "hitnet-xl"])
def test_hitnet_oracle_shapes_and_names(preset, tmp_path):
    """HITNet v2 oracle: both presets run, produce non-negative full-resolution disparity, and the
    state_dict holds the names the native engine loads (csrc/models/hitnet.cpp)."""
    from stereoalgorithms_amd.models import hitnet as HN
    m = HN.build(preset, seed=0)
    with torch.no_grad():
        d = m(torch.rand(1, 6, 64, 96))
    assert d.shape == (1, 64, 96) and (d >= 0).all()
    sd = m.state_dict()
    for k in ("prop.3.inp.weight", "prop.0.inp.weight", "prop.0.out.weight", "refine.0.inp.weight",
              "refine.1.out.weight", "prop.0.res.0.conv1.weight", "init.3.tile.weight", "feature.up.0.deconv.weight"):
        assert k in sd, k
    cfg = HN.PRESETS[preset]
    # coarsest level: one candidate (64 inputs); finer levels: two candidates jointly (128 -> 2 x 17 outputs)
    assert sd["prop.3.inp.weight"].shape[1] == 64 and sd["prop.0.inp.weight"].shape[1] == 128
    assert sd["prop.0.out.weight"].shape[0] == 34 and sd["refine.1.out.weight"].shape[0] == 16
    assert len([k for k in sd if k.startswith("prop.0.res.") and k.endswith("conv1.weight")]) == len(cfg["dils"])


def test_hitnet_plane_split_consistency():
    """Splitting a tile hypothesis evaluates the same slanted plane at every pixel."""
    from stereoalgorithms_amd.models import hitnet as HN
    torch.manual_seed(0)
    h = torch.randn(2, 16, 3, 5)
    for t in (4, 2):
        a = HN.plane_pixels(h, t)
        b = HN.plane_pixels(HN.split_hyp(h, t), t // 2)
        assert torch.allclose(a, b, atol=1e-5)
