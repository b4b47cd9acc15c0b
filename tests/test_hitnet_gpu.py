"""HITNet native engine vs the PyTorch fp32 oracle (models/hitnet.py), stage by stage.

Argmin / argmax decisions (tile init, candidate selection) are discontinuous, so the engine is checked as
a chain: every stage of the oracle is fed the engine's own (tapped) inputs and must reproduce the
engine's outputs; only the continuous feature extractor is compared end to end."""
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel_err(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def nchw(t):  # tap [n, 1, h, w, c] -> [n, c, h, w] on the GPU
    return t[:, 0].permute(0, 3, 1, 2).contiguous().to(DEV)


# (preset, batch, H, W, scaled init): the small shapes at the default init, and the benchmarked 480x640 graphs
# (HitNet/test/main.cpp:9 middlebury_d400 saved_model_480x640; README_en.md:171,192 flyingthings_finalpass_xl)
# with the variance-preserving init (models/hitnet.py scale_init) so their features are in fp16's normal range
CONFIGS = [("hitnet-d400", 2, 128, 192, False), ("hitnet-xl", 2, 128, 192, False),
           ("hitnet-d400", 1, 480, 640, True), ("hitnet-xl", 1, 480, 640, True)]


@pytest.fixture(scope="module", params=CONFIGS, ids=lambda c: f"{c[0]}-{c[2]}x{c[3]}")
def run(request, tmp_path_factory):
    from stereoalgorithms_amd.models import hitnet as HN
    from stereoalgorithms_amd.models.engine import NativeStereoEngine
    from stereoalgorithms_amd.utils.synthetic import batch_pairs
    from stereoalgorithms_amd.utils.taps import load_taps
    from stereoalgorithms_amd.utils.weights import save_model
    preset, B, H, W, scaled = request.param
    d = tmp_path_factory.mktemp(preset)
    m = HN.build(preset, seed=0)
    if scaled:
        m = HN.scale_init(m)
    path = save_model(m, d / "hitnet.safetensors", preset)
    l, r = batch_pairs(B, H, W, seed=7)
    left, right = torch.from_numpy(l).to(DEV), torch.from_numpy(r).to(DEV)
    os.environ["SA_TAP_DIR"] = str(d)
    try:
        eng = NativeStereoEngine("", str(path), H, W, batch=B, use_graph=False)
        disp = eng.run(left, right).clone()
        torch.cuda.synchronize()
    finally:
        del os.environ["SA_TAP_DIR"]
    taps = load_taps(d)
    graph = NativeStereoEngine("", str(path), H, W, batch=B)
    disp_g = graph.run(left, right)
    torch.cuda.synchronize()
    x6 = torch.cat([t.flip(-1).permute(0, 3, 1, 2).float() / 255.0 for t in (left, right)], 1)
    return dict(m=m.to(DEV), taps=taps, disp=disp, disp_graph=disp_g, x6=x6, B=B, preset=preset, full=scaled)


def test_features(run):
    m, taps, B = run["m"], run["taps"], run["B"]
    with torch.no_grad():
        e = m.feature(torch.cat((run["x6"][:, :3], run["x6"][:, 3:]), 0))
    for l in range(5):
        assert rel_err(nchw(taps[f"e{l}"]), e[l]) < 3e-3, l


def _cand_blocks(x, ncand, cin, cpad):
    """[B, ncand*cpad, h, w] joint layout -> list over candidates of (cost [B, cin-16], h [B, 16])."""
    out = []
    for k in range(ncand):
        blk = x[:, k * cpad:k * cpad + cin]
        out.append((blk[:, :cin - 16], blk[:, cin - 16:]))
    return out


def test_levels_chain(run):
    from stereoalgorithms_amd.models import hitnet as HN
    m, taps, B = run["m"], run["taps"], run["B"]
    for l in range(HN.HYP_LEVELS - 1, -1, -1):
        e = nchw(taps[f"e{l}"])
        el, er = e[:B], e[B:]
        cand = nchw(taps[f"cand{l}"])  # [ncand*B, 16, th, tw]
        ncand = cand.shape[0] // B
        cands = [cand[k * B:(k + 1) * B] for k in range(ncand)]
        tl_e, tr_e = nchw(taps[f"tl{l}"]), nchw(taps[f"tr{l}"])
        with torch.no_grad():
            tl, tr = m.init[l].tiles(el, er)
            assert rel_err(tl_e, tl) < 3e-3 and rel_err(tr_e, tr) < 3e-3
            hi = m.init[l].hypothesis(tl_e, tr_e, m.maxdisp >> l)  # argmin on the engine's tile features
        init_e = cands[-1]
        same = (init_e[:, 0] == hi[:, 0])
        # fp32 sums of the same fp16 operands in a different order: only exact near-ties may differ
        assert same.float().mean().item() > 0.98, f"level {l}: d_init agreement {same.float().mean().item():.3f}"
        msk = same.unsqueeze(1).expand_as(hi)
        assert rel_err(init_e[msk], hi[msk]) < 5e-3
        if ncand > 1:  # slot 0 = slanted-plane upsampling of the coarser selected hypothesis
            up = HN.upsample_hyp(nchw(taps[f"hyp{l + 1}"]))
            assert rel_err(cands[0], up) < 1e-6
        net = m.prop[l]
        blocks = _cand_blocks(nchw(taps[f"cost{l}"]), ncand, net.cin, (net.cin + 7) // 8 * 8)
        with torch.no_grad():
            for k, (cst, hc) in enumerate(blocks):
                assert rel_err(cst, HN.warp_cost(el, er, cands[k])) < 3e-3
                assert rel_err(hc, cands[k]) < 2e-3
            outs, confs = net([c.float() for c, _ in blocks], cands)
        delta = nchw(taps[f"delta{l}"])  # [B, ncand*17 (+pad), th, tw] raw update output
        for k in range(ncand):
            dk = delta[:, k * 17:(k + 1) * 17]
            assert rel_err(dk[:, 16:17], confs[k]) < 5e-3
            # outs clamp d at 0: compare slopes / descriptor directly and d via the clamp
            assert rel_err(dk[:, 1:16], (outs[k] - cands[k])[:, 1:16]) < 5e-3
            assert rel_err((cands[k][:, :1] + dk[:, :1]).clamp_min(0), outs[k][:, :1]) < 5e-3
        # selection from the engine's own deltas
        hyp = nchw(taps[f"hyp{l}"])
        best, bc = None, None
        for k in range(ncand):
            dk = delta[:, k * 17:(k + 1) * 17]
            h = cands[k] + dk[:, :16]
            h = torch.cat((h[:, :1].clamp_min(0), h[:, 1:]), 1)
            c = dk[:, 16:17]
            if best is None:
                best, bc = h, c
            else:
                t = c > bc
                best, bc = torch.where(t, h, best), torch.where(t, c, bc)
        assert rel_err(hyp, best) < 1e-6


def test_refinement_chain(run):
    """Final refinement: split of the previous winner into 2x2 / 1x1 tiles, warped cost on e_0, update."""
    from stereoalgorithms_amd.models import hitnet as HN
    m, taps, B = run["m"], run["taps"], run["B"]
    e = nchw(taps["e0"])
    el, er = e[:B], e[B:]
    prev, pt = nchw(taps["hyp0"]), 4
    for j, t in enumerate((2, 1)):
        cand = nchw(taps[f"rcand{j}"])
        assert rel_err(cand, HN.split_hyp(prev, pt)) < 1e-6
        net = m.refine[j]
        ((cst, hc),) = _cand_blocks(nchw(taps[f"rcost{j}"]), 1, net.cin, (net.cin + 7) // 8 * 8)
        with torch.no_grad():
            assert rel_err(cst, HN.warp_cost(el, er, cand, t)) < 3e-3
            assert rel_err(hc, cand) < 2e-3
            (out,), _ = net([cst.float()], [cand])
        delta = nchw(taps[f"rdelta{j}"])[:, :16]
        assert rel_err(delta[:, 1:16], (out - cand)[:, 1:16]) < 5e-3
        hyp = nchw(taps[f"rhyp{j}"])
        ref = cand + delta
        ref = torch.cat((ref[:, :1].clamp_min(0), ref[:, 1:]), 1)
        assert rel_err(hyp, ref) < 1e-6
        prev, pt = hyp, t


def test_final_expand_and_graph(run):
    from stereoalgorithms_amd.models import hitnet as HN
    ref = HN.expand_final(nchw(run["taps"]["rhyp1"]), 1)
    assert rel_err(run["disp"], ref) < 1e-6
    assert torch.equal(run["disp"], run["disp_graph"])
    assert torch.isfinite(run["disp"]).all() and run["disp"].min().item() >= 0


def test_end_to_end_away_from_ties(run):
    """The engine's disparity vs the fp32 oracle's own forward pass, end to end.  HITNet's tile-init argmin and
    candidate argmax are discontinuous, so pixels whose result hangs on a near-tie decision (best two tile
    costs or the two candidates' confidences within 1 %, models/hitnet.py near_tie_mask) may go either way;
    everywhere else >= 98 % of the pixels must agree within 1 px.  At 480x640 the oracle must be
    non-degenerate (mean disparity >= 5 px) and the near-tie share small enough for the check to mean
    something.  Only the scaled-init graphs: at PyTorch's default init the coarse features are ~1e-7, in fp16's
    subnormal range, so an fp16 implementation cannot track the fp32 oracle there (an fp16-rounded copy of the
    oracle itself agrees on 39 % / 87 % of the pixels; those configurations are pinned by the chain tests)."""
    from stereoalgorithms_amd.models import hitnet as HN
    if not run["full"]:
        pytest.skip("default init: features in fp16's subnormal range (chain tests cover this configuration)")
    with torch.no_grad():
        ref, tie = HN.near_tie_mask(run["m"], run["x6"])
    disp = run["disp_graph"]
    err = (disp - ref).abs()
    keep = ~tie
    within = (err[keep] < 1.0).float().mean().item()
    print(f"{run['preset']} {tuple(disp.shape)}: oracle mean {ref.mean().item():.2f} px (std {ref.std().item():.2f}), "
          f"near-tie share {tie.float().mean().item():.3f}, <1px away from ties {within:.4f}, "
          f"<1px overall {(err < 1.0).float().mean().item():.4f}")
    if run["full"]:
        assert ref.mean().item() >= 5.0, "degenerate oracle output"
        assert tie.float().mean().item() < 0.15
    assert within >= 0.98
