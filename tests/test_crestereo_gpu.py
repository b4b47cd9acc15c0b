"""CREStereo: kernel numerics vs the PyTorch fp32 oracle pieces (models/crestereo.py) and the native
engine end to end vs the oracle with the same seeded weights."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def ops():
    from stereoalgorithms_amd import ops as O
    return O


def nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def rel_err(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("small_patch", [False, True])
@pytest.mark.parametrize("mode", ["offset", "iter", "window"])
@pytest.mark.parametrize("kernel", ["8", "w", "t"])
def test_agcl_vs_oracle(small_patch, mode, kernel, monkeypatch):
    """AGCL kernel vs the oracle: learned-offset mode, iter mode (per-tap warped windows), and the plain window mode
    (no offsets: the wave kernel shares the taps' bilinear corners); every kernel (SA_AGCL_KERNEL 8 / w; "t" = the
    default dispatch, whose iter mode is the tiled warp-once kernel -- run on ragged 4 x 32 tiles)."""
    from stereoalgorithms_amd.models.crestereo import AGCL
    monkeypatch.setenv("SA_AGCL_KERNEL", kernel)
    monkeypatch.setenv("SA_AGCL_TILE", "1" if kernel == "t" else "0")
    O = ops()
    torch.manual_seed(0)
    n, c, h, w = (2, 256, 13, 70) if kernel == "t" else (2, 256, 12, 20)
    iter_mode = mode == "iter"
    f1 = torch.randn(n, c, h, w, device=DEV).half().float()
    f2 = torch.randn(n, c, h, w, device=DEV).half().float()
    flow = torch.randn(n, 2, h, w, device=DEV) * 3
    offset = (torch.rand(n, 18, h, w, device=DEV) * 2 - 1).half().float()
    if mode == "window":
        offset.zero_()
    agcl = AGCL(f1, f2)
    with torch.no_grad():
        ref = agcl.corr_iter(flow, small_patch) if iter_mode else agcl.corr_offset(flow, offset, small_patch)
    out = O.agcl_corr(nhwc(f1).half(), nhwc(f2).half(), nhwc(flow), None if mode != "offset" else nhwc(offset).half(),
                      small_patch=small_patch, iter_mode=iter_mode)
    torch.cuda.synchronize()
    assert out.shape == (n, h, w, 40) and out[..., 36:].abs().max().item() == 0
    assert rel_err(out[..., :36].permute(0, 3, 1, 2), ref) < 5e-3


@pytest.mark.parametrize("small_patch", [False, True])
@pytest.mark.parametrize("shape", [(2, 13, 70), (1, 120, 160)])
def test_agcl_conv1x1_vs_oracle(small_patch, shape):
    """Fused iter-mode AGCL + convc1 (1x1 36 -> 256, bias, relu) vs the oracle's corr_iter -> conv2d -> relu, on
    ragged 2 x 32 tiles and at the 1/4-scale b1 size; the correlation is rounded to fp16 like the unfused path."""
    from stereoalgorithms_amd.models.crestereo import AGCL
    O = ops()
    torch.manual_seed(3)
    n, h, w = shape
    c = 256
    f1 = torch.randn(n, c, h, w, device=DEV).half().float()
    f2 = torch.randn(n, c, h, w, device=DEV).half().float()
    flow = torch.randn(n, 2, h, w, device=DEV) * 3
    wt = torch.randn(256, 36, 1, 1, device=DEV) / 6
    b = torch.randn(256, device=DEV) * 0.1
    with torch.no_grad():
        corr = AGCL(f1, f2).corr_iter(flow, small_patch)
        ref = F.relu(F.conv2d(corr.half().float(), wt.half().float(), b))
    out = O.agcl_conv1x1(nhwc(f1).half(), nhwc(f2).half(), nhwc(flow), wt, b, small_patch=small_patch)
    torch.cuda.synchronize()
    assert out.shape == (n, h, w, 256)
    assert torch.isfinite(out.float()).all()
    assert rel_err(out.permute(0, 3, 1, 2), ref) < 5e-3


@pytest.mark.parametrize("small_patch", [False, True])
@pytest.mark.parametrize("shape", [(2, 13, 70), (1, 120, 160)])
def test_cre_motion_head_vs_oracle(small_patch, shape):
    """One-launch motion-encoder head: relu(convc1(AGCL iter)) as above, relu(convf1(flow)) (7x7, pad 3, on the
    fp16-rounded flow like the unfused path's flow features) and the fp16 flow copy."""
    from stereoalgorithms_amd.models.crestereo import AGCL
    O = ops()
    torch.manual_seed(4)
    n, h, w = shape
    f1 = torch.randn(n, 256, h, w, device=DEV).half().float()
    f2 = torch.randn(n, 256, h, w, device=DEV).half().float()
    flow = torch.randn(n, 2, h, w, device=DEV) * 3
    wc = torch.randn(256, 36, 1, 1, device=DEV) / 6
    bc = torch.randn(256, device=DEV) * 0.1
    wf = torch.randn(128, 2, 7, 7, device=DEV) / 10
    bf = torch.randn(128, device=DEV) * 0.1
    with torch.no_grad():
        corr = AGCL(f1, f2).corr_iter(flow, small_patch)
        ref_c = F.relu(F.conv2d(corr.half().float(), wc.half().float(), bc))
        ref_f = F.relu(F.conv2d(flow.half().float(), wf.half().float(), bf, padding=3))
    cor, flo, fcopy = O.cre_motion_head(nhwc(f1).half(), nhwc(f2).half(), nhwc(flow), wc, bc, wf, bf,
                                        small_patch=small_patch)
    torch.cuda.synchronize()
    assert rel_err(cor.permute(0, 3, 1, 2), ref_c) < 5e-3
    assert rel_err(flo.permute(0, 3, 1, 2), ref_f) < 2e-3
    assert torch.equal(fcopy, nhwc(flow).half())


@pytest.mark.parametrize("shape", [(2, 13, 70), (1, 30, 40), (1, 60, 80)])
def test_cre_motion_head_pre_vs_oracle(shape):
    """The coarse levels' head: AGCL in offset mode (learned offsets) by agcl_corr, then convc1 + convf1 + flow copy
    from that correlation in one launch, vs the oracle."""
    from stereoalgorithms_amd.models.crestereo import AGCL
    O = ops()
    torch.manual_seed(5)
    n, h, w = shape
    f1 = torch.randn(n, 256, h, w, device=DEV).half().float()
    f2 = torch.randn(n, 256, h, w, device=DEV).half().float()
    flow = torch.randn(n, 2, h, w, device=DEV) * 3
    offset = (torch.rand(n, 18, h, w, device=DEV) * 2 - 1).half().float()
    wc = torch.randn(256, 36, 1, 1, device=DEV) / 6
    bc = torch.randn(256, device=DEV) * 0.1
    wf = torch.randn(128, 2, 7, 7, device=DEV) / 10
    bf = torch.randn(128, device=DEV) * 0.1
    corr = O.agcl_corr(nhwc(f1).half(), nhwc(f2).half(), nhwc(flow), nhwc(offset).half(), small_patch=False,
                       iter_mode=False)
    cor, flo, fcopy = O.cre_motion_head_pre(corr, nhwc(flow), wc, bc, wf, bf)
    torch.cuda.synchronize()
    with torch.no_grad():
        ref_corr = AGCL(f1, f2).corr_offset(flow, offset, False)
        ref_c = F.relu(F.conv2d(ref_corr.half().float(), wc.half().float(), bc))
        ref_f = F.relu(F.conv2d(flow.half().float(), wf.half().float(), bf, padding=3))
        # the arithmetic of the head alone, on the kernel's own fp16 correlation
        own_c = F.relu(F.conv2d(corr[..., :36].permute(0, 3, 1, 2).float(), wc.half().float(), bc))
    assert rel_err(cor.permute(0, 3, 1, 2), own_c) < 2e-3
    assert rel_err(cor.permute(0, 3, 1, 2), ref_c) < 5e-3
    assert rel_err(flo.permute(0, 3, 1, 2), ref_f) < 2e-3
    assert torch.equal(fcopy, nhwc(flow).half())


@pytest.mark.parametrize("n,L,S", [(2, 77, 90), (2, 1200, 1200), (1, 1200, 1200)])
def test_linear_attention_layer_pieces(n, L, S):
    """Chunked linear attention (partial KV / Ksum per 64 tokens, ordered reduction) vs the oracle, at the
    CREStereo 1/16 token count (30 x 40) and at ragged chunk edges; repeated calls are bitwise equal."""
    from stereoalgorithms_amd.models.crestereo import LinearAttention
    O = ops()
    torch.manual_seed(1)
    hds, d = 8, 32
    q = torch.randn(n, L, hds * d, device=DEV).half()
    kv = torch.randn(n, S, 2 * hds * d, device=DEV).half()
    k, v = kv[..., :256], kv[..., 256:]
    ref = LinearAttention()(q.float().view(n, L, hds, d), k.float().reshape(n, S, hds, d),
                            v.float().reshape(n, S, hds, d)).reshape(n, L, hds * d)
    out = O.linear_attention(q, k, v, heads=hds)
    out2 = O.linear_attention(q, k, v, heads=hds)
    torch.cuda.synchronize()
    assert rel_err(out, ref) < 3e-3
    assert torch.equal(out, out2)
    x = torch.randn(n, L, 256, device=DEV).half()
    res = torch.randn(n, L, 256, device=DEV).half()
    g, b = torch.rand(256, device=DEV) + 0.5, torch.randn(256, device=DEV) * 0.1
    ln = O.layernorm(x, g, b, res=res)
    ref = F.layer_norm(x.float(), (256,), g, b) + res.float()
    assert rel_err(ln, ref) < 2e-3


def test_convex_and_interp_flow():
    from stereoalgorithms_amd.models.crestereo import CREStereo
    O = ops()
    torch.manual_seed(2)
    n, h, w = 2, 7, 9
    flow = torch.randn(n, 2, h, w, device=DEV)
    mask = torch.randn(n, 144, h, w, device=DEV).half().float()
    ref = CREStereo.convex_upsample(flow, mask, 4)
    out = O.convex_upsample_c(nhwc(mask).half(), nhwc(flow), 4, 1.0, 2)
    assert rel_err(out.permute(0, 3, 1, 2), ref) < 2e-3
    ref2 = -0.5 * F.interpolate(flow, size=(5, 6), mode="bilinear", align_corners=True)
    out2 = O.interp_flow(nhwc(flow), 5, 6, -0.5)
    assert rel_err(out2.permute(0, 3, 1, 2), ref2) < 1e-5


def _pairs(b, h, w, seed=3):
    from stereoalgorithms_amd.utils.synthetic import batch_pairs
    l, r = batch_pairs(b, h, w, seed=seed)
    return torch.from_numpy(l).cuda(), torch.from_numpy(r).cuda()


@pytest.mark.parametrize("preset,hw", [("crestereo-iter2", (64, 96)), ("crestereo-iter5", (96, 128))])
def test_engine_matches_oracle(tmp_path, preset, hw):
    from stereoalgorithms_amd.models import crestereo as CR
    from stereoalgorithms_amd.models.engine import NativeStereoEngine
    from stereoalgorithms_amd.utils.weights import save_model
    h, w = hw
    m = CR.build(preset, seed=0)
    path = save_model(m, tmp_path / "cre.safetensors", preset)
    left, right = _pairs(2, h, w)
    eng = NativeStereoEngine("", str(path), h, w, batch=2)
    disp = eng.run(left, right)
    disp2 = eng.run(left, right)
    torch.cuda.synchronize()
    m = m.cuda()
    with torch.no_grad():
        rgb = lambda t: t.flip(-1).permute(0, 3, 1, 2).float()
        ref = m(rgb(left), rgb(right))[:, 0]
    rel = rel_err(disp, ref)
    print(f"{preset}: |ref| {ref.abs().mean().item():.4f} rel {rel:.3e}")
    assert torch.equal(disp, disp2)
    assert torch.isfinite(disp).all()
    assert rel < 3e-2
