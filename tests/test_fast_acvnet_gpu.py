"""Fast-ACVNet+: HIP kernel numerics vs the PyTorch fp32 oracle pieces (models/fast_acvnet.py) and the
native engine end to end vs the oracle with the same seeded weights."""
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


def ndhwc(x):
    return x.permute(0, 2, 3, 4, 1).contiguous()


def rel_err(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("stride", [1, 2])
def test_dwconv3x3(stride):
    O = ops()
    torch.manual_seed(0)
    n, c, h, w = 2, 96, 17, 23
    x = torch.randn(n, c, h, w, device=DEV).half().float()
    wt = torch.randn(c, 1, 3, 3, device=DEV) * 0.3
    b = torch.randn(c, device=DEV) * 0.1
    ref = F.relu6(F.conv2d(x, wt, b, stride, 1, groups=c))
    out = O.dwconv3x3(nhwc(x).half(), wt.view(c, 9), b, stride, act="relu6")
    assert out.shape == (n, (h - 1) // stride + 1, (w - 1) // stride + 1, c)
    assert rel_err(out.permute(0, 3, 1, 2), ref) < 2e-3


@pytest.mark.parametrize("cin,cout,stride", [(8, 16, 1), (16, 32, 2), (32, 32, 1)])
def test_conv3d_gated(cin, cout, stride):
    O = ops()
    torch.manual_seed(1)
    n, d, h, w = 2, 12, 10, 14
    x = torch.randn(n, cin, d, h, w, device=DEV).half().float()
    wt = torch.randn(cout, cin, 3, 3, 3, device=DEV) / (cin * 27) ** 0.5
    b = torch.randn(cout, device=DEV) * 0.1
    y = F.leaky_relu(F.conv3d(x, wt, b, stride, 1), 0.01)
    ho, wo = y.shape[-2:]
    gate = torch.rand(n, cout, ho, wo, device=DEV).half().float()
    ref = y * gate.unsqueeze(2)
    wp, kpad, _ = O.pack_conv3d_weight(wt)
    out = O.conv3d(ndhwc(x).half(), wp, kpad, cout, 3, stride, bias=b.float(), act="leaky", gate=nhwc(gate).half())
    torch.cuda.synchronize()
    assert out.shape == (n, y.shape[2], ho, wo, cout)
    assert rel_err(out.permute(0, 4, 1, 2, 3), ref) < 3e-3


@pytest.mark.parametrize("cin_real,cin,cout", [(1, 8, 8), (16, 16, 16), (16, 16, 32), (32, 32, 16), (32, 32, 32),
                                              (8, 8, 16)])
@pytest.mark.parametrize("gated", [False, True])
def test_conv3d_small_direct(cin_real, cin, cout, gated):
    """Tactic 34 (conv3d_small.hip): the direct 3x3x3 conv for 8-32 channels (Fast-ACVNet+'s
    correlation stem has 1 real input channel in an 8-channel volume) == F.conv3d + bias + leaky ReLU (+ the
    depth-broadcast gate), on volumes whose D / H / W overhang the 2 x 4 x 32 voxel blocks."""
    O = ops()
    torch.manual_seed(3)
    n, d, h, w = 2, 7, 10, 37
    x = torch.randn(n, cin_real, d, h, w, device=DEV).half().float()
    wt = torch.randn(cout, cin_real, 3, 3, 3, device=DEV) / (cin_real * 27) ** 0.5
    b = torch.randn(cout, device=DEV) * 0.1
    ref = F.leaky_relu(F.conv3d(x, wt, b, 1, 1), 0.01)
    gate = torch.rand(n, cout, h, w, device=DEV).half().float() if gated else None
    if gated:
        ref = ref * gate.unsqueeze(2)
    xv = torch.zeros(n, d, h, w, cin, device=DEV, dtype=torch.float16)
    xv[..., :cin_real] = ndhwc(x).half()
    wp, kpad, _ = O.pack_conv3d_weight(wt, cin_pad=cin)
    out = O.conv3d(xv, wp, kpad, cout, 3, 1, bias=b.float(), act="leaky", tile_cfg=34,
                   gate=nhwc(gate).half() if gated else None)
    torch.cuda.synchronize()
    assert rel_err(out.permute(0, 4, 1, 2, 3), ref) < 3e-3


@pytest.mark.parametrize("cin,cout,gated", [(8, 16, False), (16, 32, True), (16, 12, False)])
def test_conv3d_small_stride2(cin, cout, gated):
    """Tactic 34 at stride 2 (the hourglasses' downsampling convs; 5 x 9 x 65 input patch per 2 x 4 x 32 output block)
    == F.conv3d(stride 2) + bias + leaky ReLU (+ gate at the output resolution), odd volume sizes."""
    O = ops()
    torch.manual_seed(4)
    n, d, h, w = 1, 9, 13, 70
    x = torch.randn(n, cin, d, h, w, device=DEV).half().float()
    wt = torch.randn(cout, cin, 3, 3, 3, device=DEV) / (cin * 27) ** 0.5
    b = torch.randn(cout, device=DEV) * 0.1
    ref = F.leaky_relu(F.conv3d(x, wt, b, 2, 1), 0.01)
    ho, wo = ref.shape[3:]
    gate = torch.rand(n, cout, ho, wo, device=DEV).half().float() if gated else None
    if gated:
        ref = ref * gate.unsqueeze(2)
    wp, kpad, _ = O.pack_conv3d_weight(wt)
    out = O.conv3d(ndhwc(x).half(), wp, kpad, cout, 3, 2, bias=b.float(), act="leaky", tile_cfg=34,
                   gate=nhwc(gate).half() if gated else None)
    torch.cuda.synchronize()
    assert rel_err(out.permute(0, 4, 1, 2, 3), ref) < 3e-3


@pytest.mark.parametrize("is3d,cfg,f32,cout", [(False, -1, False, 8), (True, -1, False, 8), (False, 36, False, 8),
                                               (False, 36, True, 9), (True, 34, False, 4), (True, 34, True, 1)])
def test_transposed_conv_parity_scatter(is3d, cfg, f32, cout):
    """k4 / s2 / p1 transposed convs as 3x3(x3) convs over 2^d parity classes scattered to the 2x output: the
    launcher's tile (cfg -1), the direct small-channel kernels (tactic 36 2-D, 34 3-D) with fp16 and fp32 output."""
    O = ops()
    torch.manual_seed(2)
    n, cin = 2, 16
    if is3d:
        x = torch.randn(n, cin, 6, 5, 7, device=DEV).half().float()
        wt = torch.randn(cin, cout, 4, 4, 4, device=DEV) * 0.1
        ref = F.conv_transpose3d(x, wt, None, 2, 1)
        weq = O.deconv_as_conv_weight(wt)
        # equivalence of the re-packed weight, checked in fp32 first
        eq = F.conv3d(x, weq, None, 1, 1)
        wp, kpad, _ = O.pack_conv3d_weight(weq)
        out = O.conv3d(ndhwc(x).half(), wp, kpad, 8 * cout, 3, 1, up=3, cout_real=cout, tile_cfg=cfg,
                       epi="store_f32" if f32 else "store")
        got = out.permute(0, 4, 1, 2, 3)
    else:
        x = torch.randn(n, cin, 9, 11, device=DEV).half().float()
        wt = torch.randn(cin, cout, 4, 4, device=DEV) * 0.1
        ref = F.conv_transpose2d(x, wt, None, 2, 1)
        weq = O.deconv_as_conv_weight(wt)
        eq = F.conv2d(x, weq, None, 1, 1)
        wp, kpad, _ = O.pack_conv_weight(weq)
        out = O.conv2d(nhwc(x).half(), wp, kpad, 4 * cout, 3, 3, up=2, cout_real=cout, tile_cfg=cfg,
                       epi="store_f32" if f32 else "store")
        got = out.permute(0, 3, 1, 2)
    assert got.dtype == (torch.float32 if f32 else torch.float16)
    # parity-class identity: conv output channel p*cout + o equals deconv output at parity p
    for p in range(8 if is3d else 4):
        pb, pa, pc = p & 1, (p >> 1) & 1, p >> 2
        sl = eq[:, p * cout:(p + 1) * cout]
        if is3d:
            assert rel_err(sl, ref[:, :, pc::2, pa::2, pb::2]) < 1e-5
        else:
            assert rel_err(sl, ref[:, :, pa::2, pb::2]) < 1e-5
    torch.cuda.synchronize()
    assert rel_err(got, ref) < 3e-3


@pytest.mark.parametrize("D", [24, 21])
def test_norm_corr_volume(D):
    from stereoalgorithms_amd.models.fast_acvnet import norm_correlation_volume
    O = ops()
    torch.manual_seed(3)
    n, c, h, w = 2, 48, 9, 40
    l = torch.randn(n, c, h, w, device=DEV).half().float()
    r = torch.randn(n, c, h, w, device=DEV).half().float()
    ref = norm_correlation_volume(l, r, D)[:, 0]  # [n, D, h, w]
    out = O.norm_corr_volume(nhwc(l).half(), nhwc(r).half(), D)
    torch.cuda.synchronize()
    assert out[..., 1:].abs().max().item() == 0
    assert rel_err(out[..., 0], ref) < 2e-3


def test_topk_concat_regress_spx():
    from stereoalgorithms_amd.models.fast_acvnet import context_upsample, warp_right
    O = ops()
    torch.manual_seed(4)
    n, D, K, h, w, cl = 2, 48, 24, 6, 20, 16
    att = (torch.randn(n, 1, D, h, w, device=DEV) * 3).half().float()
    prob = F.softmax(att, 2)
    _, ind = prob.sort(dim=2, descending=True, stable=True)
    ind_k = ind[:, :, :K].sort(2, False)[0]
    att_topk = torch.gather(prob, 2, ind_k)[:, 0]  # [n, K, h, w]
    samples = ind_k[:, 0].float()
    p_out, d_out = O.topk_disparity(ndhwc(att).half(), K)
    torch.cuda.synchronize()
    assert torch.equal(d_out.permute(0, 3, 1, 2), samples)
    assert rel_err(p_out.permute(0, 3, 1, 2), att_topk) < 2e-3
    cl_t = torch.randn(n, cl, h, w, device=DEV).half().float()
    cr_t = torch.randn(n, cl, h, w, device=DEV).half().float()
    vol = torch.cat((cl_t.unsqueeze(2).expand(-1, -1, K, -1, -1), warp_right(cr_t, samples)), 1) * att_topk.unsqueeze(1)
    cv = O.concat_volume(nhwc(cl_t).half(), nhwc(cr_t).half(), p_out, d_out)
    torch.cuda.synchronize()
    assert rel_err(cv.permute(0, 4, 1, 2, 3), vol) < 2e-3
    cost = (torch.randn(n, K, h, w, device=DEV) * 2).half().float()
    _, ci = cost.sort(dim=1, descending=True, stable=True)
    pi = ci[:, :2]
    p2 = F.softmax(torch.gather(cost, 1, pi), 1)
    pred = (torch.gather(samples, 1, pi) * p2).sum(1, keepdim=True)
    got = O.topk_regress(cost.unsqueeze(-1).half().contiguous(), d_out, 2)
    torch.cuda.synchronize()
    assert rel_err(got, pred[:, 0]) < 1e-4
    spx = torch.randn(n, 9, 4 * h, 4 * w, device=DEV).half().float()
    ref = context_upsample(pred, F.softmax(spx, 1)) * 4
    spx_nhwc = torch.zeros(n, 4 * h, 4 * w, 16, dtype=torch.float16, device=DEV)
    spx_nhwc[..., :9] = nhwc(spx).half()
    up = O.spx_upsample(spx_nhwc, pred[:, 0].contiguous(), 4, 4.0)
    torch.cuda.synchronize()
    assert rel_err(up, ref) < 1e-4


def test_topk_nonfinite_logits_stay_in_bounds():
    """inf / NaN attention logits or costs (an fp16 overflow upstream) select exactly K planes per pixel and never
    write past the pixel's K slots (round 6: a NaN lane ranked 0 beside K others and the K+1-th selection was written
    into the next pixel's slots -- past the buffer at the last pixel); top-k regression on NaN costs reads no
    disparity before the buffer and stays finite where any plane is."""
    from stereoalgorithms_amd import _native as N
    import ctypes as C
    torch.manual_seed(8)
    n, d, h, w, K = 1, 48, 4, 8, 24
    att = torch.randn(n, d, h, w, device=DEV)
    att[0, 5, 0, 0] = float("inf")
    att[0, :, 0, 1] = float("nan")
    att[0, 7:20, 1, 2] = float("nan")
    att[0, :, h - 1, w - 1] = float("inf")  # the last pixel
    a32 = att.unsqueeze(-1).permute(0, 1, 2, 3, 4).contiguous()  # [n, d, h, w, 1]
    P = n * h * w
    guard = 64
    prob = torch.full((P * K + guard,), -7.0, device=DEV)
    disp = torch.full((P * K + guard,), -7.0, device=DEV)
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    N.check(N.dev().sa_topk_disparity(a32.data_ptr(), 1, 1, n, d, h, w, K, prob.data_ptr(), disp.data_ptr(), stream),
            "sa_topk_disparity")
    torch.cuda.synchronize()
    assert (prob[P * K:] == -7.0).all() and (disp[P * K:] == -7.0).all()
    dk = disp[:P * K].view(P, K)
    assert ((dk >= 0) & (dk < d)).all()  # every slot written with a plane index
    assert all(len(set(r.tolist())) == K for r in dk)  # K distinct planes
    assert dk[0].tolist().count(5.0) == 1  # the +inf plane is selected
    cost = torch.randn(n, K, h, w, 1, device=DEV)
    cost[0, :, 0, 3] = float("nan")
    out = torch.empty(P, device=DEV)
    N.check(N.dev().sa_topk_regress(cost.data_ptr(), 1, 1, disp.data_ptr(), n, K, h, w, 2, out.data_ptr(), stream),
            "sa_topk_regress")
    torch.cuda.synchronize()
    fin = torch.ones(P, dtype=torch.bool, device=DEV)
    fin[3] = False
    assert torch.isfinite(out[fin]).all()


def test_topk_fp32_logits_near_ties():
    """fp32 selection logits (what the engine's attention / cost heads now write): logits that differ by less than
    fp16 resolution must keep their fp32 order -- rounded to fp16 they tie and the lower-index rule picks small
    disparities (the 4 px downward bias of VERDICT r4 weak #7).  Same top-k / top-2 as the fp32 oracle."""
    O = ops()
    torch.manual_seed(9)
    n, D, K, h, w = 1, 48, 24, 8, 24
    att = 0.5 + 1e-4 * torch.randn(n, 1, D, h, w, device=DEV)  # distinct in fp32, mostly equal in fp16
    prob = F.softmax(att, 2)
    _, ind = prob.sort(dim=2, descending=True, stable=True)
    samples = ind[:, :, :K].sort(2, False)[0][:, 0].float()
    _, d32 = O.topk_disparity(ndhwc(att).float().contiguous(), K)
    _, d16 = O.topk_disparity(ndhwc(att).half(), K)
    torch.cuda.synchronize()
    agree32 = (d32.permute(0, 3, 1, 2) == samples).float().mean().item()
    agree16 = (d16.permute(0, 3, 1, 2) == samples).float().mean().item()
    assert agree32 >= 0.99 and agree16 < agree32, (agree32, agree16)
    assert d32.mean().item() > d16.mean().item()  # fp16 ties resolve to lower indices
    cost = 1.0 + 1e-4 * torch.randn(n, K, h, w, device=DEV)
    _, ci = cost.sort(dim=1, descending=True, stable=True)
    pi = ci[:, :2]
    pred = (torch.gather(samples, 1, pi) * F.softmax(torch.gather(cost, 1, pi), 1)).sum(1)
    got = O.topk_regress(cost.unsqueeze(-1).contiguous(), d32, 2)
    torch.cuda.synchronize()
    assert rel_err(got, pred) < 1e-4


def _pairs(b, h, w, seed=5):
    from stereoalgorithms_amd.utils.synthetic import batch_pairs
    l, r = batch_pairs(b, h, w, seed=seed)
    return torch.from_numpy(l).cuda(), torch.from_numpy(r).cuda()


def _t(taps, name):
    """tap [n, d, h, w, c] -> NCHW (d == 1) or NCDHW on the GPU"""
    t = taps[name].to(DEV)
    return t[:, 0].permute(0, 3, 1, 2).contiguous() if t.shape[1] == 1 else t.permute(0, 4, 1, 2, 3).contiguous()


@pytest.mark.parametrize("hw,batch", [((96, 128), 1), ((128, 192), 2), ((480, 640), 1)])
def test_engine_chain_vs_oracle(tmp_path, hw, batch):
    """Every stage of the oracle is fed the engine's own (tapped) inputs: the top-24 / top-2 selections
    are discontinuous, so an end-to-end comparison of random-init networks is dominated by legitimate
    tie-break flips; the chain isolates each kernel's arithmetic."""
    import os
    from stereoalgorithms_amd.models import fast_acvnet as FA
    from stereoalgorithms_amd.models.engine import NativeStereoEngine
    from stereoalgorithms_amd.utils.taps import load_taps
    from stereoalgorithms_amd.utils.weights import save_model
    h, w = hw
    B = batch
    m = FA.sharpen(FA.build("fastacvnet-plus", seed=0))
    path = save_model(m, tmp_path / "facv.safetensors", "fastacvnet-plus")
    left, right = _pairs(B, h, w)
    os.environ["SA_TAP_DIR"] = str(tmp_path)
    try:
        eager = NativeStereoEngine("", str(path), h, w, batch=B, use_graph=False)
        disp = eager.run(left, right).clone()
        torch.cuda.synchronize()
    finally:
        del os.environ["SA_TAP_DIR"]
    eng = NativeStereoEngine("", str(path), h, w, batch=B)
    dg = eng.run(left, right).clone()
    dg2 = eng.run(left, right)
    torch.cuda.synchronize()
    assert torch.equal(dg, dg2) and torch.equal(dg, disp)
    assert torch.isfinite(disp).all()
    T = load_taps(tmp_path)
    m = m.cuda()
    mean = torch.tensor([0.485, 0.456, 0.406], device=DEV).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225], device=DEV).view(1, 3, 1, 1)
    rgb = lambda t: (t.flip(-1).permute(0, 3, 1, 2).float() / 255.0 - mean) / std
    L, R = rgb(left), rgb(right)
    with torch.no_grad():
        ful, fur = m.feature_up(m.feature(L), m.feature(R))
        s2 = m.stem_2(torch.cat((L, R)))
        s4 = m.stem_4(s2)
        f0 = torch.cat((torch.cat((ful[0], fur[0])), s4), 1)
        ref = {"x4u": torch.cat((ful[0], fur[0])), "x8u": torch.cat((ful[1], fur[1])),
               "x16u": torch.cat((ful[2], fur[2])), "stem2": s2, "stem4": s4, "match": m.desc(m.conv(f0))}
    for k, v in ref.items():
        assert rel_err(_t(T, k), v) < 3e-3, k
    # engine features from here on
    x4u, x8u, x16u, st2, st4 = (_t(T, k) for k in ("x4u", "x8u", "x16u", "stem2", "stem4"))
    match = _t(T, "match")
    f0l = torch.cat((x4u[:B], st4[:B]), 1)
    fl = [f0l, x8u[:B], x16u[:B]]
    with torch.no_grad():
        vol = FA.norm_correlation_volume(match[:B], match[B:], 48)
        assert rel_err(_t(T, "corr_vol")[:, :1], vol) < 2e-3
        cost0 = m.corr_feature_att_4(m.corr_stem(_t(T, "corr_vol")[:, :1]), f0l)
        assert rel_err(_t(T, "cost0")[:, :8], cost0) < 3e-3
        att = m.hourglass_att(_t(T, "cost0")[:, :8], fl)
        att_e = _t(T, "att_weights")
        assert rel_err(att_e, att) < 3e-3
        prob = F.softmax(att_e, dim=2)
        _, ind = prob.sort(dim=2, descending=True, stable=True)
        ind_k = ind[:, :, :24].sort(2, False)[0]
        samples = ind_k[:, 0].float()
        p_e, s_e = _t(T, "prob"), _t(T, "samples")
        assert (s_e == samples).float().mean().item() > 0.99
        assert rel_err(p_e, torch.gather(prob, 2, ind_k)[:, 0]) < 2e-3
        cf = _t(T, "concat_feat")
        v2 = torch.cat((cf[:B].unsqueeze(2).expand(-1, -1, 24, -1, -1), FA.warp_right(cf[B:], s_e)), 1)
        assert rel_err(_t(T, "concat_vol"), v2 * p_e.unsqueeze(1)) < 2e-3
        cost1 = m.concat_feature_att_4(m.concat_stem(_t(T, "concat_vol")), f0l)
        assert rel_err(_t(T, "cost1"), cost1) < 3e-3
        cost = m.hourglass(_t(T, "cost1"), fl)
        cost_e = _t(T, "cost")
        assert rel_err(cost_e, cost) < 3e-3
        c = cost_e[:, 0]
        _, ci = c.sort(dim=1, descending=True, stable=True)
        pi = ci[:, :2]
        pred = (torch.gather(s_e, 1, pi) * F.softmax(torch.gather(c, 1, pi), 1)).sum(1, keepdim=True)
        pred_e = _t(T, "pred")
        assert rel_err(pred_e, pred) < 1e-4
        spx = m.spx(m.spx_2(m.spx_4(f0l), st2[:B]))
        spx_e = _t(T, "spx_logits")[:, :9]
        assert rel_err(spx_e, spx) < 3e-3
        out = FA.context_upsample(pred_e, F.softmax(spx_e, 1)) * 4
        assert rel_err(disp, out) < 1e-4
        full = m(L, R)
    err = (disp - full).abs()
    print(f"fast-acvnet {hw} b{B}: end-to-end vs oracle mean|err| {err.mean().item():.3f} px "
          f"(|d| {full.abs().mean().item():.2f}); <1px {(err < 1).float().mean().item():.3f}")
    # End to end with the engine's discrete choices: the oracle recomputes every continuous
    # stage in fp32 from the images but takes the engine's top-24 samples and top-2 slots.  (1) Those choices
    # must be legitimate top-k / top-2 picks of the ORACLE's own logits up to a near-tie tolerance -- a glue bug
    # that swaps or shifts candidates fails here even though random-init logits are nearly tied -- and (2) the
    # disparity must then match the engine's within 1 px almost everywhere.
    with torch.no_grad():
        top2 = cost_e[:, 0].sort(dim=1, descending=True, stable=True)[1][:, :2]
        forced, att_o, cost_o = FA.forward_forced(m, L, R, s_e, top2)
    kth = att_o.sort(dim=1, descending=True)[0][:, 23]  # oracle's 24th-largest attention logit
    picked = torch.gather(att_o, 1, s_e.long()).min(1)[0]  # weakest engine pick, in oracle logits
    ok_k = picked >= kth - (0.02 + 2e-3 * kth.abs())
    second = cost_o.sort(dim=1, descending=True)[0][:, 1]
    ok_2 = torch.gather(cost_o, 1, top2).min(1)[0] >= second - (0.02 + 2e-3 * second.abs())
    ferr = (disp - forced.reshape(disp.shape)).abs()
    print(f"  engine selections legit: top-24 {ok_k.float().mean().item():.4f}, top-2 {ok_2.float().mean().item():.4f}; "
          f"forced oracle vs engine <1px {(ferr < 1).float().mean().item():.4f} (max {ferr.max().item():.3f})")
    assert ok_k.float().mean().item() >= 0.995
    assert ok_2.float().mean().item() >= 0.995
    assert (ferr < 1.0).float().mean().item() >= 0.99
