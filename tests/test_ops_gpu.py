"""Numerics of every hand-written HIP kernel vs. a plain PyTorch fp32 reference of the same op."""
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


def nchw(x):
    return x.permute(0, 3, 1, 2).float()


def rel_err(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("cin,cout,k,stride,hw,cfg", [
    (64, 64, 3, 1, (24, 40), -1),
    (64, 96, 3, 2, (30, 41), -1),
    (128, 256, 3, 1, (20, 32), 0),
    (128, 256, 3, 1, (20, 32), 1),
    (256, 2, 3, 1, (12, 16), 2),
    (256, 144, 1, 1, (12, 16), 3),
    (8, 64, 7, 2, (33, 47), -1),
    (96, 128, 1, 2, (21, 19), -1),
])
def test_conv2d_vs_torch(cin, cout, k, stride, hw, cfg):
    O = ops()
    torch.manual_seed(0)
    n = 2
    x = torch.randn(n, cin, *hw, device=DEV)
    w = torch.randn(cout, cin, k, k, device=DEV) / math.sqrt(cin * k * k)
    b = torch.randn(cout, device=DEV) * 0.1
    ref = F.relu(F.conv2d(x.half().float(), w.half().float(), b, stride=stride, padding=k // 2))
    wp, kpad, _ = O.pack_conv_weight(w)
    out = O.conv2d(nhwc(x).half(), wp, kpad, cout, k, k, bias=b.float().contiguous(), stride=stride, act="relu",
                   tile_cfg=cfg)
    torch.cuda.synchronize()
    assert out.shape == (n, ref.shape[2], ref.shape[3], cout)
    assert rel_err(nchw(out), ref) < 2e-3


@pytest.mark.parametrize("cfg,splitk", [(1, 4), (0, 3), (2, 8), (3, 0)])
def test_conv2d_splitk(cfg, splitk):
    """Split-K partial slabs + last-arriver reduction equal the unsplit conv (run twice: the
    arrival counters must be reset by the reducers)."""
    O = ops()
    torch.manual_seed(5)
    n, cin, cout, h, w = 1, 256, 128 if cfg != 2 else 2, 15, 20
    x = torch.randn(n, cin, h, w, device=DEV)
    wt = torch.randn(cout, cin, 3, 3, device=DEV) / math.sqrt(cin * 9)
    b = torch.randn(cout, device=DEV) * 0.1
    ref = torch.tanh(F.conv2d(x.half().float(), wt.half().float(), b, padding=1))
    wp, kpad, _ = O.pack_conv_weight(wt)
    ws = O.splitk_workspace()
    for _ in range(2):
        out = O.conv2d(nhwc(x).half(), wp, kpad, cout, 3, 3, bias=b.contiguous(), act="tanh", tile_cfg=cfg,
                       splitk=splitk, workspace=ws)
        torch.cuda.synchronize()
        assert rel_err(nchw(out), ref) < 2e-3
    assert ws[1].abs().sum().item() == 0


def test_conv2d_splitk_gru_epilogue():
    O = ops()
    torch.manual_seed(6)
    n, hd, h, w = 1, 128, 6, 10
    net = torch.randn(n, hd, h, w, device=DEV).tanh()
    x = torch.randn(n, 128, h, w, device=DEV)
    cz, cr = (torch.randn(n, hd, h, w, device=DEV) * 0.5 for _ in range(2))
    wz, wr = (torch.randn(hd, 2 * hd, 3, 3, device=DEV) / math.sqrt(2 * hd * 9) for _ in range(2))
    hx = torch.cat([net, x], 1).half().float()
    z = torch.sigmoid(F.conv2d(hx, wz.half().float(), padding=1) + cz.half().float())
    r = torch.sigmoid(F.conv2d(hx, wr.half().float(), padding=1) + cr.half().float())
    net_h = nhwc(net).half()
    ctx = nhwc(torch.cat([cz, cr], 1)).half()
    wzr, kpad, _ = O.pack_conv_weight(torch.cat([wz, wr], 0))
    zb = torch.empty(n, h, w, hd, device=DEV, dtype=torch.float16)
    rhb = torch.empty_like(zb)
    O.conv2d([net_h, nhwc(x).half()], wzr, kpad, 2 * hd, 3, 3, out=zb, epi="gru_zr", ctx=ctx, aux=zb,
             hbuf=net_h, rh=rhb, splitk=0, workspace=O.splitk_workspace())
    torch.cuda.synchronize()
    assert rel_err(nchw(zb), z) < 3e-3
    assert rel_err(nchw(rhb), r * net.half().float()) < 3e-3


@pytest.mark.parametrize("cfg", [0, 1, 3])
def test_conv2d_register_bk32_vs_bk64(cfg):
    """K padded to 32 only (odd multiple) forces the register-staged BK=32 loop; 64-padded weights take the
    BK=64 loop.  Both must equal the torch reference."""
    O = ops()
    torch.manual_seed(7)
    n, cin, cout, h, w = 2, 24, 128 if cfg == 0 else 64, 13, 21
    x = torch.randn(n, cin, h, w, device=DEV)
    wt = torch.randn(cout, cin, 3, 3, device=DEV) / math.sqrt(cin * 9)
    ref = F.conv2d(x.half().float(), wt.half().float(), padding=1)
    wp, kpad, _ = O.pack_conv_weight(wt)
    assert kpad % 64 == 0
    out = O.conv2d(nhwc(x).half(), wp, kpad, cout, 3, 3, tile_cfg=cfg)
    # K = 9 * 24 = 216 -> 256 (64-aligned) vs 224 (32- but not 64-aligned)
    k = 9 * cin
    k32 = (k + 31) // 32 * 32
    assert k32 % 64 != 0
    wp32 = torch.zeros(wp.shape[0], k32, dtype=wp.dtype, device=DEV)
    wp32[:, :k] = wp[:, :k]
    out32 = O.conv2d(nhwc(x).half(), wp32.contiguous(), k32, cout, 3, 3, tile_cfg=cfg)
    torch.cuda.synchronize()
    assert rel_err(nchw(out), ref) < 2e-3
    assert rel_err(nchw(out32), ref) < 2e-3


def test_conv2d_multisource_concat_and_residual():
    O = ops()
    torch.manual_seed(1)
    n, h, w = 2, 17, 23
    a = torch.randn(n, 128, h, w, device=DEV)
    big = torch.randn(n, h, w, 256, device=DEV).half()  # second source is a channel slice of a wider buffer
    bsl = big[..., 64:192]
    wt = torch.randn(96, 256, 3, 3, device=DEV) / math.sqrt(256 * 9)
    res = torch.randn(n, h, w, 96, device=DEV).half()
    ref = F.conv2d(torch.cat([a.half().float(), nchw(bsl)], 1), wt.half().float(), padding=1)
    ref = F.relu(ref + nchw(res))
    wp, kpad, _ = O.pack_conv_weight(wt)
    out = O.conv2d([nhwc(a).half(), bsl], wp, kpad, 96, 3, 3, res=res, act="none", act2="relu")
    torch.cuda.synchronize()
    assert rel_err(nchw(out), ref) < 2e-3


@pytest.mark.parametrize("srcs,cout,k,stride,hw,n,splitk", [
    ((128, 256), 256, 3, 1, (20, 33), 2, 1),   # GRU z/r shape: two sources, 2 n-tiles
    ((64,), 64, 3, 1, (17, 23), 1, 1),          # Cout < BN (padded weight rows)
    ((128,), 128, 3, 2, (31, 40), 2, 1),        # stride 2
    ((192, 64), 96, 1, 1, (9, 30), 3, 1),       # 1x1, M tail, tiles spanning images
    ((128, 128, 128), 128, 3, 1, (24, 32), 1, 3),  # three sources + forced split-K
    ((64,), 128, 7, 1, (12, 12), 1, 1),         # 49 taps
])
@pytest.mark.parametrize("cfg", [4, 10, 11, 14, 15, 16, 17, 18, 19])
def test_conv2d_glds3_vs_torch(srcs, cout, k, stride, hw, n, splitk, cfg):
    """8-wave global->LDS DMA kernels: 256x128 (cfg 4: 3-deep LDS ring, counted vmcnt, XCD-ordered
    tiles), the wide tiles 256x256 / 512x128 (cfg 10 / 11: BK 32 4-deep ring, 32x32x16 MFMA,
    two-band epilogue; never split), the deep rings (cfg 14-17: 4-8 stages, up to 7 in flight) and the 8-wave
    ping-pong tiles (cfg 18 / 19: 256x256 / 256x128, wave groups offset by one barrier; 20 / 21 with the DMA
    issued inside the MFMA slot; never split)."""
    if 10 <= cfg <= 13 and splitk != 1:
        pytest.skip("wide tiles are never split")
    if cfg >= 18 and splitk > 1:
        splitk = 0  # ping-pong tiles: automatic K split of the last round's tiles (here: every tile)
    O = ops()
    torch.manual_seed(11)
    xs = [torch.randn(n, c, *hw, device=DEV) for c in srcs]
    cin = sum(srcs)
    w = torch.randn(cout, cin, k, k, device=DEV) / math.sqrt(cin * k * k)
    b = torch.randn(cout, device=DEV) * 0.1
    ref = F.conv2d(torch.cat([x.half().float() for x in xs], 1), w.half().float(), b, stride=stride,
                   padding=k // 2)
    ref = F.leaky_relu(ref, 0.1)
    wp, kpad, _ = O.pack_conv_weight(w)
    ws = O.splitk_workspace() if splitk != 1 else None
    for _ in range(2):
        out = O.conv2d([nhwc(x).half() for x in xs], wp, kpad, cout, k, k, bias=b.contiguous(), stride=stride,
                       act="leaky", alpha=0.1, tile_cfg=cfg, splitk=splitk, workspace=ws)
        torch.cuda.synchronize()
        assert rel_err(nchw(out), ref) < 2e-3


@pytest.mark.parametrize("srcs,cout,k,hw,n", [
    ((128, 128, 128), 256, 3, (120, 160), 1),  # RAFT-SF 1/4 GRU z/r at batch 1 (150 tiles of 256x128 < 256 CUs)
    ((128, 256), 256, 3, (60, 80), 2),         # multi-tile stream-K ranges, tiles spanning images
    ((64,), 128, 3, (17, 23), 1),              # fewer k-steps than blocks (G capped), M tail
    ((192, 64), 96, 1, (9, 30), 3),            # 1x1, Cout < BN
])
@pytest.mark.parametrize("cfg", [4, 5, 7, 8])
def test_conv2d_streamk_vs_torch(srcs, cout, k, hw, n, cfg):
    """Stream-K (splitk = -1): G resident blocks share the T x nk k-steps equally, partial tiles are finished
    by the last contributor.  Repeated launches must be bitwise identical (fixed-order reduction, counters
    reset by the last arriver) and match torch."""
    O = ops()
    torch.manual_seed(13)
    xs = [torch.randn(n, c, *hw, device=DEV) for c in srcs]
    cin = sum(srcs)
    w = torch.randn(cout, cin, k, k, device=DEV) / math.sqrt(cin * k * k)
    b = torch.randn(cout, device=DEV) * 0.1
    ref = F.conv2d(torch.cat([x.half().float() for x in xs], 1), w.half().float(), b, padding=k // 2)
    ref = F.leaky_relu(ref, 0.1)
    wp, kpad, _ = O.pack_conv_weight(w)
    ws = O.splitk_workspace(1 << 25, 8192)
    outs = []
    for _ in range(3):
        out = O.conv2d([nhwc(x).half() for x in xs], wp, kpad, cout, k, k, bias=b.contiguous(), act="leaky",
                       alpha=0.1, tile_cfg=cfg, splitk=-1, workspace=ws)
        torch.cuda.synchronize()
        outs.append(out.clone())
        assert rel_err(nchw(out), ref) < 2e-3
    assert all(torch.equal(o, outs[0]) for o in outs)
    assert int(ws[1].abs().sum()) == 0, "tile counters not reset"


@pytest.mark.parametrize("cfg,splitk", [(18, 1), (19, 1), (18, 0), (19, 0)])
def test_conv2d_ping_pong_full_size_race_screen(cfg, splitk):
    """Ping-pong tiles at the RAFT-SF batch-8 GRU z/r shape (600 / 1200 tiles, 108 ring stages per tile):
    matches torch and repeated launches are bitwise identical (a misplaced vmcnt / barrier shows up as rare
    wrong tiles that differ between launches).  splitk 0: the 88 tiles of cfg 18's partial last round are
    K-split in two (fixed-order slab reduction)."""
    O = ops()
    torch.manual_seed(17)
    n, h, w = 8, 120, 160
    xs = [torch.randn(n, 128, h, w, device=DEV) for _ in range(3)]
    w3 = torch.randn(256, 384, 3, 3, device=DEV) / math.sqrt(384 * 9)
    ref = F.conv2d(torch.cat([x.half().float() for x in xs], 1), w3.half().float(), padding=1)
    wp, kpad, _ = O.pack_conv_weight(w3)
    xh = [nhwc(x).half() for x in xs]
    ws = O.splitk_workspace(1 << 25, 8192) if splitk == 0 else None
    outs = []
    for _ in range(4):
        outs.append(O.conv2d(xh, wp, kpad, 256, 3, 3, tile_cfg=cfg, splitk=splitk, workspace=ws).clone())
    torch.cuda.synchronize()
    assert rel_err(nchw(outs[0]), ref) < 2e-3
    assert all(torch.equal(o, outs[0]) for o in outs[1:])


def test_conv2d_streamk_gru_zr_epilogue():
    """Stream-K with the fused ConvGRU z / r*h epilogue (the RAFT b1 hot conv)."""
    O = ops()
    torch.manual_seed(14)
    n, hd, h, w = 1, 128, 60, 80
    net = torch.randn(n, hd, h, w, device=DEV).tanh()
    x = torch.randn(n, 256, h, w, device=DEV)
    cz, cr = (torch.randn(n, hd, h, w, device=DEV) * 0.5 for _ in range(2))
    wz, wr = (torch.randn(hd, hd + 256, 3, 3, device=DEV) / math.sqrt((hd + 256) * 9) for _ in range(2))
    hx = torch.cat([net, x], 1).half().float()
    z = torch.sigmoid(F.conv2d(hx, wz.half().float(), padding=1) + cz.half().float())
    r = torch.sigmoid(F.conv2d(hx, wr.half().float(), padding=1) + cr.half().float())
    net_h = nhwc(net).half()
    ctx = nhwc(torch.cat([cz, cr], 1)).half()
    wzr, kpad, _ = O.pack_conv_weight(torch.cat([wz, wr], 0))
    zb = torch.empty(n, h, w, hd, device=DEV, dtype=torch.float16)
    rhb = torch.empty_like(zb)
    ws = O.splitk_workspace(1 << 25, 8192)
    O.conv2d([net_h, nhwc(x).half()], wzr, kpad, 2 * hd, 3, 3, out=zb, epi="gru_zr", ctx=ctx, aux=zb,
             hbuf=net_h, rh=rhb, tile_cfg=4, splitk=-1, workspace=ws)
    torch.cuda.synchronize()
    assert rel_err(nchw(zb), z) < 3e-3
    assert rel_err(nchw(rhb), r * net.half().float()) < 3e-3


@pytest.mark.parametrize("cfg", [4, 10, 11, 18, 19])
def test_conv2d_glds3_gru_and_stats_epilogues(cfg):
    O = ops()
    torch.manual_seed(12)
    n, hd, h, w = 2, 128, 21, 26
    net = torch.randn(n, hd, h, w, device=DEV).tanh()
    x = torch.randn(n, 256, h, w, device=DEV)
    cz, cr = (torch.randn(n, hd, h, w, device=DEV) * 0.5 for _ in range(2))
    wz, wr = (torch.randn(hd, hd + 256, 3, 3, device=DEV) / math.sqrt((hd + 256) * 9) for _ in range(2))
    hx = torch.cat([net, x], 1).half().float()
    z = torch.sigmoid(F.conv2d(hx, wz.half().float(), padding=1) + cz.half().float())
    r = torch.sigmoid(F.conv2d(hx, wr.half().float(), padding=1) + cr.half().float())
    net_h = nhwc(net).half()
    ctx = nhwc(torch.cat([cz, cr], 1)).half()
    wzr, kpad, _ = O.pack_conv_weight(torch.cat([wz, wr], 0))
    zb = torch.empty(n, h, w, hd, device=DEV, dtype=torch.float16)
    rhb = torch.empty_like(zb)
    O.conv2d([net_h, nhwc(x).half()], wzr, kpad, 2 * hd, 3, 3, out=zb, epi="gru_zr", ctx=ctx, aux=zb,
             hbuf=net_h, rh=rhb, tile_cfg=cfg)
    torch.cuda.synchronize()
    assert rel_err(nchw(zb), z) < 3e-3
    assert rel_err(nchw(rhb), r * net.half().float()) < 3e-3
    w2 = torch.randn(128, 256, 3, 3, device=DEV) / 48
    wp2, kp2, _ = O.pack_conv_weight(w2)
    stats = torch.zeros(n, 128, 2, dtype=torch.int64, device=DEV)
    y = O.conv2d(nhwc(x).half(), wp2, kp2, 128, 3, 3, stats=stats, tile_cfg=cfg)
    torch.cuda.synchronize()
    yr = F.conv2d(x.half().float(), w2.half().float(), padding=1)
    assert rel_err(nchw(y), yr) < 2e-3
    assert rel_err(stats[..., 0].double() / 2 ** 24, yr.sum((2, 3))) < 1e-2
    assert rel_err(stats[..., 1].double() / 2 ** 24, (yr * yr).sum((2, 3))) < 1e-2


@pytest.mark.parametrize("n,hw", [(1, (120, 160)), (8, (120, 160)), (2, (37, 70)), (1, (5, 3))])
def test_flow_head_tail(n, hw):
    """Fused tap projection + stencil (one launch, halo-tiled; both tile shapes) == F.conv2d 256 -> 1 in fp32
    on the same fp16 operands, accumulated into the flow."""
    O = ops()
    torch.manual_seed(47)
    base = torch.randn(n, *hw, 320, device=DEV).half()
    y = base[..., :256]
    w2 = torch.randn(1, 256, 3, 3, device=DEV) / 48
    b2 = torch.randn(1, device=DEV) * 0.1
    flow0 = torch.randn(n, *hw, device=DEV)
    flow = flow0.clone()
    O.flow_head_tail(y, w2[0].permute(1, 2, 0).reshape(9, 256), b2.contiguous(), flow)
    torch.cuda.synchronize()
    ref = F.conv2d(y.float().permute(0, 3, 1, 2), w2.half().float(), b2, padding=1)[:, 0]
    assert rel_err(flow - flow0, ref) < 2e-3


@pytest.mark.parametrize("n,hw", [(1, (120, 160)), (1, (30, 40)), (2, (37, 70))])
def test_flow_head_tail_two_channels(n, hw):
    """CREStereo's flow-head conv2 (256 -> 2, 3x3) as one halo-tiled launch == F.conv2d in fp32 on the same fp16
    operands, accumulated into the interleaved (x, y) flow."""
    O = ops()
    torch.manual_seed(48)
    y = torch.randn(n, *hw, 256, device=DEV).half()
    w2 = torch.randn(2, 256, 3, 3, device=DEV) / 48
    b2 = torch.randn(2, device=DEV) * 0.1
    flow0 = torch.randn(n, *hw, 2, device=DEV)
    flow = flow0.clone()
    O.flow_head_tail2(y, w2, b2.contiguous(), flow)
    torch.cuda.synchronize()
    ref = F.conv2d(y.float().permute(0, 3, 1, 2), w2.half().float(), b2, padding=1).permute(0, 2, 3, 1)
    assert rel_err(flow - flow0, ref) < 2e-3


@pytest.mark.parametrize("n,hw,act,stats", [(2, (17, 70), "relu", False), (1, (48, 128), "none", True),
                                             (3, (5, 9), "leaky", True), (2, (33, 190), "none", True)])
def test_conv3x3_c64_direct(n, hw, act, stats):
    """Direct 3x3 64 -> 64 conv (tile_cfg 23: two waves per SIMD, buffer-store epilogue): tails in both dims,
    several images per block, slotted statistics folded to the unsplit sums."""
    O = ops()
    torch.manual_seed(31)
    x = torch.randn(n, 64, *hw, device=DEV)
    w = torch.randn(64, 64, 3, 3, device=DEV) / 24
    b = torch.randn(64, device=DEV) * 0.1
    ref = F.conv2d(x.half().float(), w.half().float(), b, padding=1)
    ref = {"relu": F.relu, "none": lambda t: t, "leaky": lambda t: F.leaky_relu(t, 0.1)}[act](ref)
    wp, kpad, _ = O.pack_conv_weight(w)
    kw = {}
    if stats:
        st = torch.zeros(16, n, 64, 2, dtype=torch.int64, device=DEV)
        kw = dict(stats=st, stats_slots=16)
    out = O.conv2d(nhwc(x).half(), wp, kpad, 64, 3, 3, bias=b.contiguous(), act=act, alpha=0.1, tile_cfg=23, **kw)
    torch.cuda.synchronize()
    assert rel_err(nchw(out), ref) < 2e-3
    if stats:
        O.stats_reduce(st, 16)
        torch.cuda.synchronize()
        y = nchw(out)
        assert rel_err(st[0, ..., 0].double() / 2 ** 24, y.sum((2, 3))) < 1e-3
        assert rel_err(st[0, ..., 1].double() / 2 ** 24, (y * y).sum((2, 3))) < 1e-3


@pytest.mark.parametrize("n,hw,stride,act,stats", [(2, (37, 70), 1, "relu", False), (1, (48, 128), 1, "none", True),
                                                    (3, (9, 5), 1, "leaky", True), (2, (33, 47), 2, "relu", False),
                                                    (1, (64, 130), 2, "none", True)])
def test_conv7x7_stem(n, hw, stride, act, stats):
    """7x7 stem conv (tile_cfg 22) on the encoders' 3-real-of-8-channel input: tails in both dims, several
    images per block, junk in the padding channels ignored, slotted statistics folded to the unsplit sums."""
    O = ops()
    torch.manual_seed(37)
    x = torch.rand(n, 3, *hw, device=DEV) * 2 - 1
    xp = torch.zeros(n, *hw, 8, device=DEV, dtype=torch.float16)
    xp[..., :3] = nhwc(x).half()
    xp[..., 3:] = 7.0  # never read: only the real channels are staged
    w = torch.randn(64, 3, 7, 7, device=DEV) / 12
    b = torch.randn(64, device=DEV) * 0.1
    ref = F.conv2d(x.half().float(), w.half().float(), b, stride=stride, padding=3)
    ref = {"relu": F.relu, "none": lambda t: t, "leaky": lambda t: F.leaky_relu(t, 0.1)}[act](ref)
    wp, kpad, cin_pad = O.pack_conv_weight(w, [(3, 8)])
    assert cin_pad == 8
    kw = {}
    if stats:
        st = torch.zeros(16, n, 64, 2, dtype=torch.int64, device=DEV)
        kw = dict(stats=st, stats_slots=16)
    out = O.conv2d(xp, wp, kpad, 64, 7, 7, bias=b.contiguous(), stride=stride, act=act, alpha=0.1, tile_cfg=22,
                   cin_real=3, **kw)
    torch.cuda.synchronize()
    assert out.shape[1:3] == ref.shape[2:]
    assert rel_err(nchw(out), ref) < 2e-3
    # the generic implicit GEMM on the same args agrees (the tuner's first candidate)
    gen = O.conv2d(xp, wp, kpad, 64, 7, 7, bias=b.contiguous(), stride=stride, act=act, alpha=0.1, tile_cfg=1,
                   cin_real=3)
    xp[..., 3:] = 0
    gen0 = O.conv2d(xp, wp, kpad, 64, 7, 7, bias=b.contiguous(), stride=stride, act=act, alpha=0.1, tile_cfg=1)
    torch.cuda.synchronize()
    assert rel_err(nchw(gen0), ref) < 2e-3 and torch.isfinite(gen).all()
    if stats:
        O.stats_reduce(st, 16)
        torch.cuda.synchronize()
        y = nchw(out)
        assert rel_err(st[0, ..., 0].double() / 2 ** 24, y.sum((2, 3))) < 1e-3
        assert rel_err(st[0, ..., 1].double() / 2 ** 24, (y * y).sum((2, 3))) < 1e-3


@pytest.mark.parametrize("n,hw,act,mode", [(2, (17, 70), "relu", "plain"), (1, (48, 128), "none", "stats"),
                                           (3, (5, 9), "leaky", "stats"), (2, (33, 97), "relu", "res"),
                                           (1, (30, 66), "none", "res_none")])
@pytest.mark.parametrize("cin,stride", [(96, 1), (64, 2)])
def test_conv3x3_c96_direct(n, hw, act, mode, cin, stride):
    """Direct 3x3 -> 96 conv (tile_cfg 24; 96 -> 96 stride 1, 64 -> 96 stride 2): tails in both dims, several
    images per workgroup, slotted statistics folded to the unsplit sums, residual epilogue from a channel slice
    of a wider tensor."""
    O = ops()
    torch.manual_seed(41)
    x = torch.randn(n, cin, *hw, device=DEV)
    w = torch.randn(96, cin, 3, 3, device=DEV) / math.sqrt(cin * 9)
    b = torch.randn(96, device=DEV) * 0.1
    ref = F.conv2d(x.half().float(), w.half().float(), b, stride=stride, padding=1)
    hw = tuple(ref.shape[2:])
    ref = {"relu": F.relu, "none": lambda t: t, "leaky": lambda t: F.leaky_relu(t, 0.1)}[act](ref)
    wp, kpad, _ = O.pack_conv_weight(w)
    kw = {}
    if mode == "stats":
        st = torch.zeros(16, n, 96, 2, dtype=torch.int64, device=DEV)
        kw = dict(stats=st, stats_slots=16)
    if mode.startswith("res"):
        big = torch.randn(n, *hw, 192, device=DEV).half()
        res = big[..., 96:]
        kw = dict(res=res, act2="relu" if mode == "res" else "none")
        ref = ref + nchw(res)
        ref = F.relu(ref) if mode == "res" else ref
    out = O.conv2d(nhwc(x).half(), wp, kpad, 96, 3, 3, bias=b.contiguous(), stride=stride, act=act, alpha=0.1,
                   tile_cfg=24, **kw)
    torch.cuda.synchronize()
    assert rel_err(nchw(out), ref) < 2e-3
    if mode == "stats":
        O.stats_reduce(st, 16)
        torch.cuda.synchronize()
        y = nchw(out)
        assert rel_err(st[0, ..., 0].double() / 2 ** 24, y.sum((2, 3))) < 1e-3
        assert rel_err(st[0, ..., 1].double() / 2 ** 24, (y * y).sum((2, 3))) < 1e-3


@pytest.mark.parametrize("cin,cout,n,hw,act,stats", [(64, 96, 2, (31, 63), "relu", False),
                                                     (64, 96, 3, (32, 64), "none", True),
                                                     (96, 128, 2, (17, 9), "leaky", False),
                                                     (96, 128, 1, (64, 32), "none", True)])
def test_conv1x1_point(cin, cout, n, hw, act, stats):
    """Strided 1x1 conv (tile_cfg 25, the encoders' downsample): odd sizes, images spanning waves, slotted
    statistics folded to the unsplit sums."""
    O = ops()
    torch.manual_seed(43)
    x = torch.randn(n, cin, *hw, device=DEV)
    w = torch.randn(cout, cin, 1, 1, device=DEV) / math.sqrt(cin)
    b = torch.randn(cout, device=DEV) * 0.1
    ref = F.conv2d(x.half().float(), w.half().float(), b, stride=2)
    ref = {"relu": F.relu, "none": lambda t: t, "leaky": lambda t: F.leaky_relu(t, 0.1)}[act](ref)
    wp, kpad, _ = O.pack_conv_weight(w)
    kw = {}
    if stats:
        st = torch.zeros(16, n, cout, 2, dtype=torch.int64, device=DEV)
        kw = dict(stats=st, stats_slots=16)
    out = O.conv2d(nhwc(x).half(), wp, kpad, cout, 1, 1, bias=b.contiguous(), stride=2, pad=0, act=act, alpha=0.1,
                   tile_cfg=25, **kw)
    torch.cuda.synchronize()
    assert rel_err(nchw(out), ref) < 2e-3
    if stats:
        O.stats_reduce(st, 16)
        torch.cuda.synchronize()
        y = nchw(out)
        assert rel_err(st[0, ..., 0].double() / 2 ** 24, y.sum((2, 3))) < 1e-3
        assert rel_err(st[0, ..., 1].double() / 2 ** 24, (y * y).sum((2, 3))) < 1e-3


@pytest.mark.parametrize("n,hw,act2", [(2, (17, 70), "relu"), (1, (33, 190), "none")])
def test_conv3x3_c64_direct2_residual(n, hw, act2):
    """Direct conv v2 (tile_cfg 23) residual epilogue y = act2(relu(conv + b) + res) (the batch-norm
    ResidualBlock's second conv), residual read from a channel slice of a wider tensor."""
    O = ops()
    torch.manual_seed(33)
    x = torch.randn(n, 64, *hw, device=DEV)
    w = torch.randn(64, 64, 3, 3, device=DEV) / 24
    b = torch.randn(64, device=DEV) * 0.1
    big = torch.randn(n, *hw, 128, device=DEV).half()
    res = big[..., 64:]
    ref = F.relu(F.conv2d(x.half().float(), w.half().float(), b, padding=1)) + nchw(res)
    ref = F.relu(ref) if act2 == "relu" else ref
    wp, kpad, _ = O.pack_conv_weight(w)
    out = O.conv2d(nhwc(x).half(), wp, kpad, 64, 3, 3, bias=b.contiguous(), act="relu", res=res, act2=act2,
                   tile_cfg=23)
    torch.cuda.synchronize()
    assert rel_err(nchw(out), ref) < 2e-3


@pytest.mark.parametrize("n,hw,stats,act", [(2, (17, 70), True, "none"), (1, (48, 128), False, "relu"),
                                            (3, (5, 9), True, "none"), (2, (33, 190), True, "leaky"),
                                            (300, (2, 64), True, "none"), (4, (64, 640), True, "none")])
def test_conv3x3_c64_direct2_folded_input_norm(n, hw, stats, act):
    """Direct conv v2 (tile_cfg 23) with the input instance norm folded in (SaConvArgs.in_stats): the conv reads a
    raw conv output and normalises its DMA'd pieces in LDS one tile ahead (-65504 padding -> relu(IN) = 0) --
    BITWISE the conv of instnorm_apply's relu(IN(x)) (same arithmetic), output statistics included; many images per
    workgroup (the per-image mean / rstd slots), tails in both dims.  Other tactics refuse in_stats."""
    O = ops()
    torch.manual_seed(35)
    raw = (torch.randn(n, *hw, 64, device=DEV) * 3 + torch.randn(1, 1, 1, 64, device=DEV) * 5).half()
    st_in = torch.zeros(16, n, 64, 2, dtype=torch.int64, device=DEV)
    for r in range(16):  # spread like the conv epilogues' slotted atomics
        part = raw.float()[:, r::16]
        st_in[r, ..., 0] = torch.round(part.sum((1, 2)).double() * 2 ** 24).long()
        st_in[r, ..., 1] = torch.round((part * part).sum((1, 2)).double() * 2 ** 24).long()
    w = torch.randn(64, 64, 3, 3, device=DEV) / 24
    b = torch.randn(64, device=DEV) * 0.1
    wp, kpad, _ = O.pack_conv_weight(w)
    a1 = O.instnorm_apply(raw, st_in, act="relu", slots=16)
    kw_ref, kw_fold = {}, {}
    if stats:
        st_ref = torch.zeros(16, n, 64, 2, dtype=torch.int64, device=DEV)
        st_fold = torch.zeros_like(st_ref)
        kw_ref, kw_fold = dict(stats=st_ref, stats_slots=16), dict(stats=st_fold, stats_slots=16)
    ref = O.conv2d(a1, wp, kpad, 64, 3, 3, bias=b.contiguous(), act=act, alpha=0.1, tile_cfg=23, **kw_ref)
    out = O.conv2d(raw, wp, kpad, 64, 3, 3, bias=b.contiguous(), act=act, alpha=0.1, tile_cfg=23,
                   in_stats=st_in, in_slots=16, **kw_fold)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    if stats:
        assert torch.equal(st_fold, st_ref)
    # and against fp32 torch: relu(instance_norm(raw)) -> conv
    xn = F.relu(F.instance_norm(raw.float().permute(0, 3, 1, 2), eps=1e-5)).half().float()
    r32 = F.conv2d(xn, w.half().float(), b, padding=1)
    r32 = {"relu": F.relu, "none": lambda t: t, "leaky": lambda t: F.leaky_relu(t, 0.1)}[act](r32)
    assert rel_err(nchw(out), r32) < 3e-3
    with pytest.raises(RuntimeError):
        O.conv2d(raw, wp, kpad, 64, 3, 3, bias=b.contiguous(), tile_cfg=1, in_stats=st_in, in_slots=16)


@pytest.mark.parametrize("n,hw,cin,cout,act,res", [(2, (60, 80), 16, 96, "relu6", False),
                                                    (2, (30, 40), 24, 144, "relu6", False),
                                                    (1, (30, 40), 144, 24, "none", True),
                                                    (3, (7, 9), 8, 20, "leaky", False),
                                                    (1, (15, 20), 256, 192, "relu", True),
                                                    (2, (5, 13), 32, 192, "none", False),
                                                    (1, (30, 40), 128, 256, "relu", False),
                                                    (1, (9, 11), 96, 232, "none", True)])
def test_conv_pointwise_narrow(n, hw, cin, cout, act, res):
    """Pointwise 1x1 conv (tile_cfg 35: one wave per 16 pixels x all <= 192 columns, transposed MFMA product):
    odd pixel counts (partial last tile), K and N not multiples of 32 / 16, residual from a channel slice of a wider
    tensor, output into a channel slice."""
    O = ops()
    torch.manual_seed(51)
    x = torch.randn(n, cin, *hw, device=DEV)
    w = torch.randn(cout, cin, 1, 1, device=DEV) / math.sqrt(cin)
    b = torch.randn(cout, device=DEV) * 0.1
    ref = F.conv2d(x.half().float(), w.half().float(), b)
    acts = {"relu": F.relu, "none": lambda t: t, "leaky": lambda t: F.leaky_relu(t, 0.1),
            "relu6": lambda t: t.clamp(0, 6)}
    ref = acts[act](ref)
    wp, kpad, _ = O.pack_conv_weight(w)
    kw = {}
    if res:
        big = torch.randn(n, *hw, cout + 8, device=DEV).half()
        r = big[..., 8:]
        kw = dict(res=r, act2="none")
        ref = ref + nchw(r)
    outbuf = torch.zeros(n, *hw, cout + 4, device=DEV, dtype=torch.float16)
    out = outbuf[..., 4:]
    O.conv2d(nhwc(x).half(), wp, kpad, cout, 1, 1, bias=b.contiguous(), act=act, alpha=0.1, tile_cfg=35, out=out,
             pad=0, **kw)
    torch.cuda.synchronize()
    assert rel_err(nchw(out), ref) < 2e-3
    assert (outbuf[..., :4] == 0).all()


@pytest.mark.parametrize("n,hw,cin,cout", [(2, (30, 40), 16, 16), (1, (15, 21), 32, 12), (1, (7, 9), 24, 48)])
def test_conv_pointwise_transposed_k2s2(n, hw, cin, cout):
    """ConvTranspose2d(k=2, s=2) as tactic 35's 1x1 conv over 4 parity classes scattered to the 2x output (HITNet's
    upsampling) == F.conv_transpose2d in fp32 on the same fp16 operands; two channel-concatenated sources too."""
    O = ops()
    torch.manual_seed(55)
    x = torch.randn(n, cin, *hw, device=DEV)
    wt = torch.randn(cin, cout, 2, 2, device=DEV) / math.sqrt(cin)
    b = torch.randn(cout, device=DEV) * 0.1
    ref = F.leaky_relu(F.conv_transpose2d(x.half().float(), wt.half().float(), b, stride=2), 0.1)
    w1 = torch.zeros(4 * cout, cin, 1, 1, device=DEV)
    for p in range(4):
        w1[p * cout:(p + 1) * cout, :, 0, 0] = wt[:, :, p >> 1, p & 1].t()
    wp, kpad, _ = O.pack_conv_weight(w1)
    out = torch.full((n, 2 * hw[0], 2 * hw[1], cout), 7.0, device=DEV, dtype=torch.float16)
    xh = nhwc(x).half()
    srcs = [xh] if cin % 16 else [xh[..., :cin // 2].contiguous(), xh[..., cin // 2:].contiguous()]
    O.conv2d(srcs, wp, kpad, 4 * cout, 1, 1, bias=b.repeat(4).contiguous(), act="leaky", alpha=0.1, tile_cfg=35,
             out=out, pad=0, up=2, cout_real=cout)
    torch.cuda.synchronize()
    assert rel_err(nchw(out), ref) < 2e-3


@pytest.mark.parametrize("n,hw,cins,cout,act,res,dil,f32", [(2, (60, 80), (32,), 32, "leaky", False, 1, False),
                                                             (2, (30, 40), (24, 24), 48, "relu", False, 1, False),
                                                             (1, (17, 70), (8,), 20, "none", False, 1, False),
                                                             (1, (20, 50), (64,), 64, "relu", True, 1, False),
                                                             (2, (9, 33), (48,), 36, "none", False, 1, False),
                                                             (1, (24, 40), (32, 32), 64, "leaky", False, 1, False),
                                                             (3, (5, 7), (16,), 16, "relu", True, 1, False),
                                                             (1, (30, 40), (32,), 32, "leaky", True, 2, False),
                                                             (2, (19, 45), (64,), 32, "none", False, 4, False),
                                                             (1, (33, 70), (32,), 34, "none", False, 1, True),
                                                             (1, (15, 20), (16,), 17, "leaky", False, 2, True),
                                                             (1, (12, 40), (48, 48), 32, "relu", False, 1, False),
                                                             (2, (9, 20), (96,), 64, "none", True, 2, False)])
def test_conv2d_small_direct(n, hw, cins, cout, act, res, dil, f32):
    """Direct 3x3 conv for small channel counts (tile_cfg 36: 8 x 32 blocks, the (8 + 2d) x (32 + 2d) patch in LDS once
    for all 9 taps, transposed MFMA): one or two channel-concatenated sources, dilation 1 / 2 / 4, tails in both dims,
    Cout not a multiple of 16, residual from a channel slice, fp16 output into a channel slice or fp32 output."""
    O = ops()
    torch.manual_seed(53)
    cin = sum(cins)
    xs = [torch.randn(n, c, *hw, device=DEV) for c in cins]
    x = torch.cat(xs, 1)
    w = torch.randn(cout, cin, 3, 3, device=DEV) / math.sqrt(cin * 9)
    b = torch.randn(cout, device=DEV) * 0.1
    ref = F.conv2d(x.half().float(), w.half().float(), b, padding=dil, dilation=dil)
    ref = {"relu": F.relu, "none": lambda t: t, "leaky": lambda t: F.leaky_relu(t, 0.1)}[act](ref)
    wp, kpad, _ = O.pack_conv_weight(w)
    kw = {}
    if res:
        big = torch.randn(n, *hw, cout + 8, device=DEV).half()
        r = big[..., 8:]
        kw = dict(res=r, act2="none")
        ref = ref + nchw(r)
    if f32:  # an even row width that is not a multiple of 4 (HITNet's 34-wide fp32 tiles)
        outbuf = torch.zeros(n, *hw, cout + cout % 2 + 2, device=DEV, dtype=torch.float32)
        out = outbuf[..., 2:2 + cout]
        kw["epi"] = "store_f32"
    else:
        outbuf = torch.zeros(n, *hw, cout + 4, device=DEV, dtype=torch.float16)
        out = outbuf[..., 4:]
    O.conv2d([nhwc(t).half() for t in xs], wp, kpad, cout, 3, 3, bias=b.contiguous(), act=act, alpha=0.1,
             tile_cfg=36, out=out, dil=dil, **kw)
    torch.cuda.synchronize()
    assert rel_err(nchw(out), ref) < 2e-3
    assert (outbuf[..., :2] == 0).all()


@pytest.mark.parametrize("n,hw,cin,cout,res", [(2, (48, 64), 8, 32, False), (1, (33, 71), 32, 48, True),
                                                (1, (20, 40), 16, 64, False), (2, (9, 17), 32, 20, False)])
def test_conv2d_small_direct_stride2(n, hw, cin, cout, res):
    """Tactic 36 at stride 2 (the 17 x 65 input patch in LDS, Cin <= 32): odd input sizes, residual."""
    O = ops()
    torch.manual_seed(57)
    x = torch.randn(n, cin, *hw, device=DEV)
    w = torch.randn(cout, cin, 3, 3, device=DEV) / math.sqrt(cin * 9)
    b = torch.randn(cout, device=DEV) * 0.1
    ref = F.relu(F.conv2d(x.half().float(), w.half().float(), b, stride=2, padding=1))
    ho, wo = ref.shape[2:]
    kw = {}
    if res:
        r = torch.randn(n, ho, wo, cout, device=DEV).half()
        kw = dict(res=r, act2="none")
        ref = ref + nchw(r)
    wp, kpad, _ = O.pack_conv_weight(w)
    out = O.conv2d(nhwc(x).half(), wp, kpad, cout, 3, 3, bias=b.contiguous(), act="relu", stride=2, tile_cfg=36, **kw)
    torch.cuda.synchronize()
    assert out.shape[1:3] == (ho, wo)
    assert rel_err(nchw(out), ref) < 2e-3


def test_instnorm_apply_residual_activation():
    """instnorm_apply's res_act: y = act2(res_act(IN(res)) + act(IN(x))) -- the folded stem's layer1.0 residual."""
    O = ops()
    torch.manual_seed(36)
    n, hw, c = 2, (13, 40), 64
    x = (torch.randn(n, *hw, c, device=DEV) * 2).half()
    r = (torch.randn(n, *hw, c, device=DEV) + 0.5).half()

    def stats(t):
        st = torch.zeros(1, n, c, 2, dtype=torch.int64, device=DEV)
        st[0, ..., 0] = torch.round(t.float().sum((1, 2)).double() * 2 ** 24).long()
        st[0, ..., 1] = torch.round((t.float() ** 2).sum((1, 2)).double() * 2 ** 24).long()
        return st
    out = O.instnorm_apply(x, stats(x), act="relu", res=r, res_stats=stats(r), act2="relu", res_act="relu")
    torch.cuda.synchronize()
    inn = lambda t: F.instance_norm(t.float().permute(0, 3, 1, 2), eps=1e-5)
    ref = F.relu(F.relu(inn(r)) + F.relu(inn(x)))
    assert rel_err(nchw(out), ref) < 2e-3


def test_conv2d_padded_channels_and_output_slice():
    O = ops()
    torch.manual_seed(2)
    n, h, w = 1, 15, 20
    x = torch.randn(n, 36, h, w, device=DEV)
    wt = torch.randn(64, 36, 1, 1, device=DEV) / 6
    xp = torch.zeros(n, h, w, 40, device=DEV, dtype=torch.float16)
    xp[..., :36] = nhwc(x).half()
    wp, kpad, cin_pad = O.pack_conv_weight(wt, [(36, 40)])
    assert cin_pad == 40
    buf = torch.zeros(n, h, w, 128, device=DEV, dtype=torch.float16)
    O.conv2d(xp, wp, kpad, 64, 1, 1, out=buf[..., 64:128], act="relu")
    torch.cuda.synchronize()
    ref = F.relu(F.conv2d(x.half().float(), wt.half().float()))
    assert rel_err(nchw(buf[..., 64:]), ref) < 2e-3
    assert buf[..., :64].abs().max().item() == 0


def test_conv2d_gru_epilogues():
    O = ops()
    torch.manual_seed(3)
    n, hd, h, w = 2, 128, 12, 16
    net = torch.randn(n, hd, h, w, device=DEV).tanh()
    x = torch.randn(n, 256, h, w, device=DEV)
    cz, cr, cq = (torch.randn(n, hd, h, w, device=DEV) * 0.5 for _ in range(3))
    wz, wr, wq = (torch.randn(hd, hd + 256, 3, 3, device=DEV) / math.sqrt((hd + 256) * 9) for _ in range(3))
    bz, br, bq = (torch.randn(hd, device=DEV) * 0.1 for _ in range(3))
    hx = torch.cat([net, x], 1).half().float()
    z = torch.sigmoid(F.conv2d(hx, wz.half().float(), bz, padding=1) + cz.half().float())
    r = torch.sigmoid(F.conv2d(hx, wr.half().float(), br, padding=1) + cr.half().float())
    rh = (r * net.half().float()).half().float()
    q = torch.tanh(F.conv2d(torch.cat([rh, x.half().float()], 1), wq.half().float(), bq, padding=1) + cq.half().float())
    ref = (1 - z) * net.half().float() + z * q

    net_h = nhwc(net).half()
    ctx = nhwc(torch.cat([cz, cr, cq], 1)).half()
    xh = nhwc(x).half()
    wzr, kpad, _ = O.pack_conv_weight(torch.cat([wz, wr], 0))
    wqp, kpq, _ = O.pack_conv_weight(wq)
    zb = torch.empty(n, h, w, hd, device=DEV, dtype=torch.float16)
    rhb = torch.empty_like(zb)
    O.conv2d([net_h, xh], wzr, kpad, 2 * hd, 3, 3, bias=torch.cat([bz, br]).contiguous(), out=zb, epi="gru_zr",
             ctx=ctx, aux=zb, hbuf=net_h, rh=rhb)
    O.conv2d([rhb, xh], wqp, kpq, hd, 3, 3, bias=bq.contiguous(), out=net_h, epi="gru_q", ctx=ctx[..., 2 * hd:],
             aux=zb, hbuf=net_h)
    torch.cuda.synchronize()
    assert rel_err(nchw(zb), z) < 3e-3
    assert rel_err(nchw(net_h), ref) < 3e-3


@pytest.mark.parametrize("cfg,splitk", [(-1, 1), (5, 1), (4, 1), (16, 2), (7, 3), (37, 1), (38, 1)])
def test_conv2d_gru_zrq_split(cfg, splitk):
    """ConvGRU with q's x-input half hoisted into the z/r conv (SA_EPI_GRU_ZRQ, Cout = 3 hd, q's h-input weights
    zeroed there) and the q conv over r*h alone adding it back (SA_EPI_GRU_Q + res), against the fp32 GRU."""
    O = ops()
    torch.manual_seed(5)
    n, hd, h, w = 1, 128, 30, 40
    net = torch.randn(n, hd, h, w, device=DEV).tanh()
    x = torch.randn(n, 256, h, w, device=DEV)
    cz, cr, cq = (torch.randn(n, hd, h, w, device=DEV) * 0.5 for _ in range(3))
    wz, wr, wq = (torch.randn(hd, hd + 256, 3, 3, device=DEV) / math.sqrt((hd + 256) * 9) for _ in range(3))
    bz, br, bq = (torch.randn(hd, device=DEV) * 0.1 for _ in range(3))
    hx = torch.cat([net, x], 1).half().float()
    z = torch.sigmoid(F.conv2d(hx, wz.half().float(), bz, padding=1) + cz.half().float())
    r = torch.sigmoid(F.conv2d(hx, wr.half().float(), br, padding=1) + cr.half().float())
    rh = (r * net.half().float()).half().float()
    q = torch.tanh(F.conv2d(torch.cat([rh, x.half().float()], 1), wq.half().float(), bq, padding=1) + cq.half().float())
    ref = (1 - z) * net.half().float() + z * q

    net_h = nhwc(net).half()
    ctx = nhwc(torch.cat([cz, cr, cq], 1)).half()
    xh = nhwc(x).half()
    wqx = wq.clone()
    wqx[:, :hd] = 0
    wzrq, kpad, _ = O.pack_conv_weight(torch.cat([wz, wr, wqx], 0))
    wqh, kph, _ = O.pack_conv_weight(wq[:, :hd].contiguous())
    zb = torch.empty(n, h, w, hd, device=DEV, dtype=torch.float16)
    rhb = torch.empty_like(zb)
    qx = torch.empty_like(zb)
    wsplit = cfg in (37, 38)  # workgroup split-K: partials in the workspace, reduce + gate epilogue launch
    ws = O.splitk_workspace(1 << 22, 4096) if splitk != 1 or wsplit else None
    O.conv2d([net_h, xh], wzrq, kpad, 3 * hd, 3, 3, bias=torch.cat([bz, br, bq]).contiguous(), out=qx,
             epi="gru_zrq", ctx=ctx, aux=zb, hbuf=net_h, rh=rhb, tile_cfg=cfg, splitk=splitk, workspace=ws)
    O.conv2d([rhb], wqh, kph, hd, 3, 3, out=net_h, epi="gru_q", res=qx, aux=zb, hbuf=net_h, tile_cfg=cfg,
             workspace=ws if wsplit else None)
    torch.cuda.synchronize()
    assert rel_err(nchw(zb), z) < 3e-3
    assert rel_err(nchw(net_h), ref) < 4e-3


@pytest.mark.parametrize("srcs,cout,k,stride,dil,hw,n,res", [
    ((32,), 32, 3, 1, 1, (60, 80), 1, False),      # HITNet tile-update conv (K = 288 -> Kpad 320)
    ((24, 8), 64, 3, 1, 2, (30, 40), 2, True),     # two sources, dilation 2, residual
    ((16,), 24, 2, 2, 1, (120, 160), 2, False),    # k2 / s2 downsampling, Cout not a multiple of 16
    ((64, 64), 48, 3, 1, 1, (15, 20), 1, False),   # K = 1152 -> 18 steps: rejected (whole K > 8 steps)
])
def test_conv2d_whole_k_tile(srcs, cout, k, stride, dil, hw, n, res):
    """Tactic 39: the 64x64 register-staged tile with every k-step's loads issued up front (K <= 512) == F.conv2d
    (bias, relu, optional residual); a K beyond 8 steps is rejected (-5), not run."""
    O = ops()
    torch.manual_seed(39)
    xs = [torch.randn(n, c, *hw, device=DEV) for c in srcs]
    cin = sum(srcs)
    w = torch.randn(cout, cin, k, k, device=DEV) / math.sqrt(cin * k * k)
    b = torch.randn(cout, device=DEV) * 0.1
    pad = (k // 2) * dil if k % 2 else 0
    xcat = torch.cat(xs, 1).half().float()
    ref = F.relu(F.conv2d(xcat, w.half().float(), b, stride=stride, padding=pad, dilation=dil))
    r = torch.randn_like(ref) if res else None
    if res:
        ref = ref + r.half().float()
    wp, kpad, _ = O.pack_conv_weight(w)
    args = dict(bias=b.contiguous(), stride=stride, pad=pad, dil=dil, act="relu",
                res=nhwc(r).half() if res else None, tile_cfg=39)
    if kpad > 512:
        with pytest.raises(RuntimeError):
            O.conv2d([nhwc(t).half() for t in xs], wp, kpad, cout, k, k, **args)
        return
    out = O.conv2d([nhwc(t).half() for t in xs], wp, kpad, cout, k, k, **args)
    torch.cuda.synchronize()
    assert rel_err(nchw(out), ref) < 3e-3


@pytest.mark.parametrize("cfg", [37, 38])
@pytest.mark.parametrize("srcs,cout,hw,n,res", [
    ((128, 128), 256, (30, 40), 1, False),  # coarse GRU level shape, two sources
    ((64,), 96, (15, 20), 2, True),        # Cout not a multiple of 64 (workspace rows padded to 128), residual
    ((128, 64, 64), 384, (13, 21), 1, False),  # three sources, rows not a multiple of any tile
])
def test_conv2d_workgroup_splitk(srcs, cout, hw, n, res, cfg):
    """Workgroup split-K (tactics 37 / 38): S workgroups store fp32 partial tiles of one output tile's K slices, a
    second launch sums them in fixed order and runs the epilogue (bias, activation, residual) == F.conv2d; two runs
    give identical bits."""
    O = ops()
    torch.manual_seed(37)
    xs = [torch.randn(n, c, *hw, device=DEV) for c in srcs]
    cin = sum(srcs)
    w = torch.randn(cout, cin, 3, 3, device=DEV) / math.sqrt(cin * 9)
    b = torch.randn(cout, device=DEV) * 0.1
    r = torch.randn(n, cout, *hw, device=DEV) if res else None
    xcat = torch.cat(xs, 1).half().float()
    ref = F.relu(F.conv2d(xcat, w.half().float(), b, padding=1))
    if res:
        ref = ref + r.half().float()
    wp, kpad, _ = O.pack_conv_weight(w)
    ws = O.splitk_workspace(1 << 22, 16)
    outs = []
    for _ in range(2):
        out = O.conv2d([nhwc(t).half() for t in xs], wp, kpad, cout, 3, 3, bias=b.contiguous(), act="relu",
                       res=nhwc(r).half() if res else None, tile_cfg=cfg, workspace=ws)
        torch.cuda.synchronize()
        outs.append(out.clone())
    assert rel_err(nchw(outs[0]), ref) < 3e-3
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("n,h,w,xs,grid", [(1, 30, 40, (256,), 128), (2, 60, 80, (128, 128), 64),
                                           (1, 13, 21, (128,), 7)])
def test_gru_level_one_launch(n, h, w, xs, grid):
    """sa_gru_level: the ZRQ conv, a grid-wide barrier and the q conv in ONE launch on `grid`
    workgroups (split-K slices dealt round-robin) == the fp32 ConvGRU; replays reuse the barrier words (generation
    counter) and give identical bits; the timeout flag stays clear."""
    O = ops()
    torch.manual_seed(6)
    hd = 128
    net = torch.randn(n, hd, h, w, device=DEV).tanh()
    x = torch.randn(n, sum(xs), h, w, device=DEV)
    cz, cr, cq = (torch.randn(n, hd, h, w, device=DEV) * 0.5 for _ in range(3))
    cin = hd + sum(xs)
    wz, wr, wq = (torch.randn(hd, cin, 3, 3, device=DEV) / math.sqrt(cin * 9) for _ in range(3))
    bz, br, bq = (torch.randn(hd, device=DEV) * 0.1 for _ in range(3))
    hx = torch.cat([net, x], 1).half().float()
    z = torch.sigmoid(F.conv2d(hx, wz.half().float(), bz, padding=1) + cz.half().float())
    r = torch.sigmoid(F.conv2d(hx, wr.half().float(), br, padding=1) + cr.half().float())
    rh = (r * net.half().float()).half().float()
    q = torch.tanh(F.conv2d(torch.cat([rh, x.half().float()], 1), wq.half().float(), bq, padding=1) + cq.half().float())
    ref = (1 - z) * net.half().float() + z * q
    ctx = nhwc(torch.cat([cz, cr, cq], 1)).half()
    xh = [nhwc(t).half() for t in torch.split(x, list(xs), 1)]
    wqx = wq.clone()
    wqx[:, :hd] = 0
    wzrq, kpad, _ = O.pack_conv_weight(torch.cat([wz, wr, wqx], 0))
    wqh, kph, _ = O.pack_conv_weight(wq[:, :hd].contiguous())
    bar = torch.zeros(4, dtype=torch.int32, device=DEV)
    ws = O.splitk_workspace(1 << 22, 4096)
    outs = []
    for _ in range(3):
        net_h = nhwc(net).half()
        zb = torch.empty(n, h, w, hd, device=DEV, dtype=torch.float16)
        rhb, qx = torch.empty_like(zb), torch.empty_like(zb)
        za = O.conv2d([net_h, *xh], wzrq, kpad, 3 * hd, 3, 3, bias=torch.cat([bz, br, bq]).contiguous(), out=qx,
                      epi="gru_zrq", ctx=ctx, aux=zb, hbuf=net_h, rh=rhb, splitk=0, workspace=ws, launch=False)
        qa = O.conv2d([rhb], wqh, kph, hd, 3, 3, out=net_h, epi="gru_q", res=qx, aux=zb, hbuf=net_h, splitk=0,
                      workspace=ws, launch=False)
        O.gru_level(za, qa, bar, grid)
        torch.cuda.synchronize()
        outs.append(net_h.clone())
    assert rel_err(nchw(outs[0]), ref) < 4e-3
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    assert bar[0].item() == 0 and bar[1].item() == 3 and bar[2].item() == 0


@pytest.mark.parametrize("cfg", [26, 27, 28, 29, 30, 31, 32, 33])
@pytest.mark.parametrize("srcs,cout,hw,n", [
    ((128, 256), 256, (120, 160), 1),   # RAFT 1/4 z/r (two sources, 2 n-tiles), patches tile the image exactly
    ((128,), 128, (60, 80), 2),          # 1/8 level: 8x32 patches overhang the right edge
    ((64, 64, 128), 384, (30, 40), 1),   # three sources, 3 n-tiles, patches overhang both edges
    ((64,), 128, (13, 21), 2),           # tiny image: one partial patch per image
])
def test_conv2d_halo_vs_torch(srcs, cout, hw, n, cfg):
    """Halo-reuse 3x3 tiles (cfg 26: 8 x 32 output patches, 27: 16 x 16; 28 / 29 planar; 30 / 31: 16 x 32 / 12 x 32
    patches over 32-channel chunks, 128 x 64 / 96 x 64 wave tiles): the input patch of each channel chunk is loaded
    once and read by all 9 taps; must equal F.conv2d (zero padding at every image border, multi-source concatenation,
    bias + activation epilogue, run twice)."""
    O = ops()
    torch.manual_seed(21)
    xs = [torch.randn(n, c, *hw, device=DEV) for c in srcs]
    cin = sum(srcs)
    w = torch.randn(cout, cin, 3, 3, device=DEV) / math.sqrt(cin * 9)
    b = torch.randn(cout, device=DEV) * 0.1
    ref = F.leaky_relu(F.conv2d(torch.cat([x.half().float() for x in xs], 1), w.half().float(), b, padding=1), 0.1)
    wp, kpad, _ = O.pack_conv_weight(w)
    for _ in range(2):
        out = O.conv2d([nhwc(x).half() for x in xs], wp, kpad, cout, 3, 3, bias=b.contiguous(), act="leaky",
                       alpha=0.1, tile_cfg=cfg)
        torch.cuda.synchronize()
        assert rel_err(nchw(out), ref) < 2e-3


@pytest.mark.parametrize("cfg,n", [(26, 4), (28, 4), (30, 8), (31, 6), (32, 8), (33, 6)])
def test_conv2d_halo_tail_split(cfg, n):
    """splitk 0 on the halo tiles: 300 (cfg 26 / 28 / 31) or 320 (cfg 30) tiles on 256 CUs, so the last 44 / 64 are
    cut into K-ranges of whole channel chunks (uneven: 6 chunks of 64 over 4 ranges; 12 chunks of 32 for 30 / 31)
    reduced by the last arriver.  Must equal F.conv2d and the unsplit launch to fp32-summation-order noise, for the
    store epilogue and the GRU q epilogue (in-place hidden-state update)."""
    O = ops()
    torch.manual_seed(23)
    h, w = 120, 160
    xs = [torch.randn(n, 128, h, w, device=DEV) for _ in range(3)]
    wt = torch.randn(128, 384, 3, 3, device=DEV) / math.sqrt(384 * 9)
    b = torch.randn(128, device=DEV) * 0.1
    ref = F.leaky_relu(F.conv2d(torch.cat([x.half().float() for x in xs], 1), wt.half().float(), b, padding=1), 0.1)
    wp, kpad, _ = O.pack_conv_weight(wt)
    ws = O.splitk_workspace(1 << 24, 4096)
    xh = [nhwc(x).half() for x in xs]
    whole = O.conv2d(xh, wp, kpad, 128, 3, 3, bias=b.contiguous(), act="leaky", alpha=0.1, tile_cfg=cfg, splitk=1)
    for _ in range(2):
        out = O.conv2d(xh, wp, kpad, 128, 3, 3, bias=b.contiguous(), act="leaky", alpha=0.1, tile_cfg=cfg, splitk=0,
                       workspace=ws)
        torch.cuda.synchronize()
        assert rel_err(nchw(out), ref) < 2e-3
        assert (out.float() - whole.float()).abs().max().item() < 2e-2
    # GRU q epilogue (net <- (1 - z) net + z tanh(conv(r*h) + qx)) over a 2-chunk input: split in two
    hd = 128
    net = torch.randn(n, hd, h, w, device=DEV).tanh()
    rh = torch.randn(n, hd, h, w, device=DEV) * 0.5
    qx = torch.randn(n, hd, h, w, device=DEV) * 0.5
    z = torch.rand(n, hd, h, w, device=DEV)
    wq = torch.randn(hd, hd, 3, 3, device=DEV) / math.sqrt(hd * 9)
    q = torch.tanh(F.conv2d(rh.half().float(), wq.half().float(), padding=1) + qx.half().float())
    refn = (1 - z.half().float()) * net.half().float() + z.half().float() * q
    wqp, kq, _ = O.pack_conv_weight(wq)
    net_h = nhwc(net).half()
    O.conv2d([nhwc(rh).half()], wqp, kq, hd, 3, 3, out=net_h, epi="gru_q", res=nhwc(qx).half(), aux=nhwc(z).half(),
             hbuf=net_h, tile_cfg=cfg, splitk=0, workspace=ws)
    torch.cuda.synchronize()
    assert rel_err(nchw(net_h), refn) < 4e-3


@pytest.mark.parametrize("cfg", [26, 27, 28, 29, 30, 31, 32, 33])
def test_conv2d_halo_gru_and_stats(cfg):
    """Halo tiles with the fused epilogues: the ZRQ / Q GRU pair and per-(image, channel) instance-norm statistics
    (patch rows map to image pixels, so the statistics must still be exact)."""
    O = ops()
    torch.manual_seed(22)
    n, hd, h, w = 2, 128, 24, 40
    net = torch.randn(n, hd, h, w, device=DEV).tanh()
    x = torch.randn(n, 256, h, w, device=DEV)
    cz, cr, cq = (torch.randn(n, hd, h, w, device=DEV) * 0.5 for _ in range(3))
    wz, wr, wq = (torch.randn(hd, hd + 256, 3, 3, device=DEV) / math.sqrt((hd + 256) * 9) for _ in range(3))
    bz, br, bq = (torch.randn(hd, device=DEV) * 0.1 for _ in range(3))
    hx = torch.cat([net, x], 1).half().float()
    z = torch.sigmoid(F.conv2d(hx, wz.half().float(), bz, padding=1) + cz.half().float())
    r = torch.sigmoid(F.conv2d(hx, wr.half().float(), br, padding=1) + cr.half().float())
    rh = (r * net.half().float()).half().float()
    q = torch.tanh(F.conv2d(torch.cat([rh, x.half().float()], 1), wq.half().float(), bq, padding=1) + cq.half().float())
    ref = (1 - z) * net.half().float() + z * q
    net_h = nhwc(net).half()
    ctx = nhwc(torch.cat([cz, cr, cq], 1)).half()
    xh = nhwc(x).half()
    wqx = wq.clone()
    wqx[:, :hd] = 0
    wzrq, kpad, _ = O.pack_conv_weight(torch.cat([wz, wr, wqx], 0))
    wqh, kph, _ = O.pack_conv_weight(wq[:, :hd].contiguous())
    zb = torch.empty(n, h, w, hd, device=DEV, dtype=torch.float16)
    rhb, qx = torch.empty_like(zb), torch.empty_like(zb)
    O.conv2d([net_h, xh], wzrq, kpad, 3 * hd, 3, 3, bias=torch.cat([bz, br, bq]).contiguous(), out=qx,
             epi="gru_zrq", ctx=ctx, aux=zb, hbuf=net_h, rh=rhb, tile_cfg=cfg)
    O.conv2d([rhb], wqh, kph, hd, 3, 3, out=net_h, epi="gru_q", res=qx, aux=zb, hbuf=net_h, tile_cfg=cfg)
    torch.cuda.synchronize()
    assert rel_err(nchw(zb), z) < 3e-3
    assert rel_err(nchw(net_h), ref) < 4e-3
    # statistics: sum / sum of squares per (image, channel) of the stored output
    xin = torch.randn(n, 128, h, w, device=DEV)
    ws = torch.randn(128, 128, 3, 3, device=DEV) / math.sqrt(128 * 9)
    wsp, kps, _ = O.pack_conv_weight(ws)
    st = torch.zeros(16, n, 128, 2, dtype=torch.int64, device=DEV)
    if cfg in (30, 31, 32, 33):  # kHaloW's epilogue is compiled without statistics: the launcher refuses the shape
        with pytest.raises(RuntimeError):
            O.conv2d(nhwc(xin).half(), wsp, kps, 128, 3, 3, stats=st, stats_slots=16, tile_cfg=cfg)
        return
    O.conv2d(nhwc(xin).half(), wsp, kps, 128, 3, 3, stats=st, stats_slots=16, tile_cfg=cfg)
    torch.cuda.synchronize()
    # the epilogue accumulates the fp32 values before their fp16 store
    o = F.conv2d(xin.half().float(), ws.half().float(), padding=1).double()
    tot = st.sum(0).double() / 16777216.0
    assert torch.allclose(tot[..., 0], o.sum((2, 3)), rtol=1e-4, atol=2e-3)
    assert torch.allclose(tot[..., 1], (o * o).sum((2, 3)), rtol=1e-4, atol=2e-3)


@pytest.mark.parametrize("cfg", [-1, 4, 7, 11, 19, 26, 28, 30, 31, 32, 33])
@pytest.mark.parametrize("oc", [1, 2])
def test_flow_head_tap_projection(cfg, oc):
    """Flow head with conv2's tap projections fused into conv1's epilogue (SA_EPI_TAPPROJ: conv1's 256 channels are
    never stored) + the 3x3 stencil, against F.conv2d(relu(conv1)) -> conv2 in fp32 on the fp16-rounded hidden
    features; BN = 64 tile configs are refused."""
    O = ops()
    torch.manual_seed(31)
    n, h, w = 2, 30, 44
    x = torch.randn(n, 128, h, w, device=DEV)
    w1 = torch.randn(256, 128, 3, 3, device=DEV) / math.sqrt(128 * 9)
    b1 = torch.randn(256, device=DEV) * 0.1
    w2 = torch.randn(oc, 256, 3, 3, device=DEV) / math.sqrt(256 * 9)
    b2 = torch.randn(oc, device=DEV) * 0.1
    hid = F.relu(F.conv2d(x.half().float(), w1.half().float(), b1, padding=1)).half().float()
    flow0 = torch.randn(n, h, w, oc, device=DEV)
    ref = flow0 + F.conv2d(hid, w2.half().float(), b2, padding=1).permute(0, 2, 3, 1)
    wp, kpad, _ = O.pack_conv_weight(w1)
    taps = 9 * oc
    tapw = torch.zeros(taps, 256, device=DEV, dtype=torch.float16)
    for t in range(9):
        for o in range(oc):
            tapw[t * oc + o] = w2[o, :, t // 3, t % 3].half()
    P = torch.full((n, h, w, 2 * taps), float("nan"), device=DEV)
    O.conv2d(nhwc(x).half(), wp, kpad, 256, 3, 3, bias=b1.contiguous(), act="relu", out=P, epi="tapproj",
             tapw=tapw, taps=taps, tile_cfg=cfg)
    flow = flow0.clone()
    O.tapproj_stencil(P, taps, oc, b2.contiguous(), flow)
    torch.cuda.synchronize()
    assert rel_err(flow - flow0, ref - flow0) < 3e-3
    with pytest.raises(RuntimeError):
        O.conv2d(nhwc(x).half(), wp, kpad, 256, 3, 3, bias=b1.contiguous(), act="relu", out=P, epi="tapproj",
                 tapw=tapw, taps=taps, tile_cfg=5)


def test_conv2d_flow_acc_and_stats():
    O = ops()
    torch.manual_seed(4)
    n, h, w = 2, 10, 14
    x = torch.randn(n, 256, h, w, device=DEV)
    wt = torch.randn(1, 256, 3, 3, device=DEV) / 48
    b = torch.tensor([0.3], device=DEV)
    flow = torch.randn(n, h, w, device=DEV)
    ref = flow + F.conv2d(x.half().float(), wt.half().float(), b, padding=1)[:, 0]
    wp, kpad, _ = O.pack_conv_weight(wt)
    O.conv2d(nhwc(x).half(), wp, kpad, 1, 3, 3, bias=b, out=flow.view(n, h, w, 1), epi="flow_acc")
    torch.cuda.synchronize()
    assert rel_err(flow, ref) < 2e-3
    # instance-norm statistics fused in the epilogue + apply kernel
    w2 = torch.randn(64, 256, 3, 3, device=DEV) / 48
    wp2, kp2, _ = O.pack_conv_weight(w2)
    stats = torch.zeros(n, 64, 2, dtype=torch.int64, device=DEV)
    y = O.conv2d(nhwc(x).half(), wp2, kp2, 64, 3, 3, stats=stats)
    out = O.instnorm_apply(y, stats, act="relu")
    torch.cuda.synchronize()
    yr = F.conv2d(x.half().float(), w2.half().float(), padding=1)
    assert rel_err(stats[..., 0].double() / 2 ** 24, yr.sum((2, 3))) < 1e-2
    ref2 = F.relu(F.instance_norm(yr))
    assert rel_err(nchw(out), ref2) < 5e-3
    # slotted statistics (the engine's contention-spreading layout) fold to the same sums
    st16 = torch.zeros(16, n, 64, 2, dtype=torch.int64, device=DEV)
    for cfg in (1, 3, 5):
        st1 = torch.zeros(n, 64, 2, dtype=torch.int64, device=DEV)
        O.conv2d(nhwc(x).half(), wp2, kp2, 64, 3, 3, stats=st1, tile_cfg=cfg)
        st16.zero_()
        y16 = O.conv2d(nhwc(x).half(), wp2, kp2, 64, 3, 3, stats=st16, stats_slots=16, tile_cfg=cfg)
        # the apply kernel folds the 16 copies itself (the engine's path): bitwise the apply of the reduced sums,
        # with and without a normalised residual
        r16 = st16.clone()
        a_slots = O.instnorm_apply(y16, st16, act="relu", slots=16)
        ar_slots = O.instnorm_apply(y16, st16, act="relu", res=y16, res_stats=r16, act2="relu", slots=16)
        O.stats_reduce(st16, 16)
        O.stats_reduce(st16, 16)  # idempotent
        torch.cuda.synchronize()
        assert torch.equal(st16[0], st1) and st16[1:].abs().sum().item() == 0
        assert torch.equal(a_slots, O.instnorm_apply(y16, st16[0], act="relu"))
        assert torch.equal(ar_slots, O.instnorm_apply(y16, st16[0], act="relu", res=y16, res_stats=st16[0],
                                                      act2="relu"))


def test_pool_interp():
    O = ops()
    torch.manual_seed(5)
    x = torch.randn(2, 64, 15, 21, device=DEV)
    xh = nhwc(x).half()
    p = O.avgpool3s2(xh)
    assert rel_err(nchw(p), F.avg_pool2d(x.half().float(), 3, 2, 1)) < 2e-3
    for ac in (True, False):
        it = O.interp_bilinear(xh, (31, 40), align_corners=ac)
        ref = F.interpolate(x.half().float(), (31, 40), mode="bilinear", align_corners=ac)
        assert rel_err(nchw(it), ref) < 2e-3
    pk = O.avgpool_k(xh, 2)
    assert rel_err(nchw(pk), F.avg_pool2d(x.half().float(), 2)) < 2e-3


def test_corr_pyramid_and_lookup_vs_oracle():
    from stereoalgorithms_amd.models.raft_stereo import CorrBlock1D, coords_grid
    O = ops()
    torch.manual_seed(6)
    b, c, h, w = 2, 256, 6, 40
    f1 = torch.randn(b, c, h, w, device=DEV)
    f2 = torch.randn(b, c, h, w, device=DEV)
    f1h, f2h = nhwc(f1).half(), nhwc(f2).half()
    buf, levels = O.corr1d_pyramid(f1h, f2h, levels=4)
    cb = CorrBlock1D(f1.half().float(), f2.half().float(), 4, 4)
    for l in range(4):
        ref = cb.pyramid[l].view(b, h, w, -1)
        assert rel_err(levels[l], ref) < 1e-4
    flow = torch.randn(b, h, w, device=DEV) * 6 - 3
    feat = O.corr1d_lookup(buf, flow, b, h, w, w)
    coords = coords_grid(b, h, w, DEV)
    coords[:, 0] += flow
    ref = cb(coords)  # [b,36,h,w]
    torch.cuda.synchronize()
    assert feat.shape[-1] == 40
    assert rel_err(nchw(feat[..., :36]), ref) < 2e-3
    assert feat[..., 36:].abs().max().item() == 0


def test_raft_motion_head_vs_torch():
    """Fused correlation lookup + relu(convc1) + relu(convf1) == the unfused PyTorch composition."""
    from stereoalgorithms_amd.models.raft_stereo import CorrBlock1D, coords_grid
    O = ops()
    torch.manual_seed(9)
    b, c, h, w = 2, 256, 7, 44
    f1 = torch.randn(b, c, h, w, device=DEV)
    f2 = torch.randn(b, c, h, w, device=DEV)
    buf, _ = O.corr1d_pyramid(nhwc(f1).half(), nhwc(f2).half(), levels=4)
    flow = torch.randn(b, h, w, device=DEV) * 5 - 2
    wc = torch.randn(64, 36, 1, 1, device=DEV) / 6
    bc = torch.randn(64, device=DEV) * 0.1
    wf = torch.randn(64, 2, 7, 7, device=DEV) / 10
    bf = torch.randn(64, device=DEV) * 0.1
    cor, flo, fc = O.raft_motion_head(buf, flow, b, h, w, w, wc, bc, wf, bf)
    cb = CorrBlock1D(f1.half().float(), f2.half().float(), 4, 4)
    coords = coords_grid(b, h, w, DEV)
    coords[:, 0] += flow
    corr = cb(coords)
    ref_c = F.relu(F.conv2d(corr, wc, bc))
    fl2 = torch.stack([flow, torch.zeros_like(flow)], 1)
    ref_f = F.relu(F.conv2d(fl2, wf, bf, padding=3))
    torch.cuda.synchronize()
    assert rel_err(nchw(cor), ref_c) < 3e-3
    assert rel_err(nchw(flo), ref_f) < 3e-3
    assert torch.allclose(fc[..., 0].float(), flow, atol=1e-2) and fc[..., 1].abs().max().item() == 0


@pytest.mark.parametrize("variant", [1, 2, 3])
@pytest.mark.parametrize("b,h,w", [(2, 7, 44), (1, 24, 32), (1, 13, 37), (2, 20, 64)])
def test_raft_motion_encoder_vs_torch(b, h, w, variant):
    """The whole motion encoder in one kernel == lookup -> convc1/convf1 -> convc2/convf2 -> conv (fp32 torch on
    the same fp16-rounded operands), including tiles that overhang the image (zero padding of every conv)."""
    from stereoalgorithms_amd.models.raft_stereo import CorrBlock1D, coords_grid
    O = ops()
    torch.manual_seed(10)
    c = 256
    f1 = torch.randn(b, c, h, w, device=DEV)
    f2 = torch.randn(b, c, h, w, device=DEV)
    buf, _ = O.corr1d_pyramid(nhwc(f1).half(), nhwc(f2).half(), levels=4)
    flow = torch.randn(b, h, w, device=DEV) * 5 - 2
    wc = torch.randn(64, 36, 1, 1, device=DEV) / 6
    bc = torch.randn(64, device=DEV) * 0.1
    wf = torch.randn(64, 2, 7, 7, device=DEV) / 10
    bf = torch.randn(64, device=DEV) * 0.1
    w2c = torch.randn(64, 64, 3, 3, device=DEV) / 24
    b2c = torch.randn(64, device=DEV) * 0.1
    w2f = torch.randn(64, 64, 3, 3, device=DEV) / 24
    b2f = torch.randn(64, device=DEV) * 0.1
    w3 = torch.randn(126, 128, 3, 3, device=DEV) / 34
    b3 = torch.randn(126, device=DEV) * 0.1
    out = O.raft_motion_encoder(buf, flow, b, h, w, w, wc, bc, wf, bf, w2c, b2c, w2f, b2f, w3, b3, variant=variant)
    cb = CorrBlock1D(f1.half().float(), f2.half().float(), 4, 4)
    coords = coords_grid(b, h, w, DEV)
    coords[:, 0] += flow
    corr = cb(coords).half().float()
    fl2 = torch.stack([flow, torch.zeros_like(flow)], 1)
    hf = lambda t: t.half().float()
    cor1 = hf(F.relu(F.conv2d(corr, hf(wc), bc)))
    flo1 = hf(F.relu(F.conv2d(hf(fl2), hf(wf), bf, padding=3)))
    cor2 = hf(F.relu(F.conv2d(cor1, hf(w2c), b2c, padding=1)))
    flo2 = hf(F.relu(F.conv2d(flo1, hf(w2f), b2f, padding=1)))
    ref = F.relu(F.conv2d(torch.cat([cor2, flo2], 1), hf(w3), b3, padding=1))
    torch.cuda.synchronize()
    assert rel_err(nchw(out[..., :126]), ref) < 5e-3
    assert torch.allclose(out[..., 126].float(), flow, atol=1e-2) and out[..., 127].abs().max().item() == 0


def test_convex_upsample_vs_oracle():
    from stereoalgorithms_amd.models.raft_stereo import RAFTStereo
    O = ops()
    torch.manual_seed(7)
    m = RAFTStereo("raftstereo-realtime")
    b, h, w, f = 2, 6, 9, 8
    mask = torch.randn(b, 9 * f * f, h, w, device=DEV)
    flow = torch.randn(b, 2, h, w, device=DEV)
    ref = m.upsample_flow(flow, mask.half().float())[:, 0]
    out = O.convex_upsample(nhwc(mask).half(), flow[:, 0].contiguous(), f, sign=-1.0)
    torch.cuda.synchronize()
    assert rel_err(out, -ref) < 1e-4


def test_preprocess_modes():
    O = ops()
    torch.manual_seed(8)
    img = torch.randint(0, 256, (2, 17, 23, 3), dtype=torch.uint8, device=DEV)
    rgb = img.flip(-1).float()
    for mode, fn in [("raw", lambda v: v), ("unit", lambda v: v / 255), ("signed", lambda v: 2 * v / 255 - 1),
                     ("imagenet", lambda v: (v / 255 - torch.tensor([0.485, 0.456, 0.406], device=DEV))
                      / torch.tensor([0.229, 0.224, 0.225], device=DEV))]:
        out = O.preprocess(img, mode)
        torch.cuda.synchronize()
        assert rel_err(out[..., :3], fn(rgb)) < 1e-3
        assert out[..., 3:].abs().max().item() == 0


def test_remap_matches_numpy_reference():
    from stereoalgorithms_amd.utils.geometry import remap_bilinear_u8
    O = ops()
    rng = np.random.default_rng(0)
    src = rng.integers(0, 256, (1, 20, 30, 3), dtype=np.uint8)
    ys, xs = np.mgrid[0:18, 0:25].astype(np.float32)
    maps = np.stack([xs * 1.1 + 0.37 * np.sin(ys) - 1.3, ys * 0.97 + 0.21 * np.cos(xs) + 0.6], -1)[None]
    out = O.remap_bgr(torch.from_numpy(src).to(DEV), torch.from_numpy(maps).to(DEV)).cpu().numpy()
    ref = remap_bilinear_u8(src[0], maps[0])
    assert np.abs(out[0].astype(int) - ref.astype(int)).max() <= 1


def test_reproject_matches_Q():
    O = ops()
    torch.manual_seed(9)
    b, h, w = 1, 8, 12
    d = torch.rand(b, h, w, device=DEV) * 40 + 1
    img = torch.randint(0, 256, (b, h, w, 3), dtype=torch.uint8, device=DEV)
    Q = np.array([[1, 0, 0, -320.5], [0, 1, 0, -240.2], [0, 0, 0, 500.0], [0, 0, 1 / 60.0, 0]], np.float64)
    dout, cloud = O.reproject(-d, img, Q, sign=-1.0)
    torch.cuda.synchronize()
    ys, xs = torch.meshgrid(torch.arange(h, device=DEV).float(), torch.arange(w, device=DEV).float(), indexing="ij")
    Wh = d[0] / 60.0
    X = (xs - 320.5) / Wh
    Z = 500.0 / Wh
    assert torch.allclose(dout, d)
    assert torch.allclose(cloud[0, ..., 0], X, rtol=1e-4, atol=1e-3)
    assert torch.allclose(cloud[0, ..., 2], Z.expand_as(X), rtol=1e-4)
    assert torch.equal(cloud[0, ..., 3:].round().to(torch.uint8), img[0].flip(-1))


@pytest.mark.parametrize("srcs,cout,k,stride,dil,splitk", [
    ((64, 128), 128, 3, 1, 1, 1),
    ((128, 64, 64), 256, 3, 2, 1, 1),
    ((64,), 64, 3, 1, 2, 1),
    ((128,), 96, 5, 1, 1, 1),
    ((128, 128), 128, 3, 1, 1, 3),
])
def test_conv2d_uniform_k_fast_path(srcs, cout, k, stride, dil, splitk):
    """Every source a multiple of 64 channels: the wave-uniform im2col gather (per-row tap masks,
    multi-source channel walk, dilation, stride, split-K) equals torch."""
    O = ops()
    torch.manual_seed(11)
    n, h, w = 2, 19, 27
    xs = [torch.randn(n, c, h, w, device=DEV) for c in srcs]
    cin = sum(srcs)
    wt = torch.randn(cout, cin, k, k, device=DEV) / math.sqrt(cin * k * k)
    pad = dil * (k // 2)
    ref = F.conv2d(torch.cat(xs, 1).half().float(), wt.half().float(), stride=stride, padding=pad, dilation=dil)
    wp, kpad, _ = O.pack_conv_weight(wt, [(c, c) for c in srcs])
    ws = O.splitk_workspace() if splitk != 1 else None
    out = O.conv2d([nhwc(x).half() for x in xs], wp, kpad, cout, k, k, stride=stride, pad=pad, dil=dil,
                   splitk=splitk, workspace=ws)
    torch.cuda.synchronize()
    assert rel_err(nchw(out), ref) < 2e-3


def test_conv3d_uniform_k_fast_path():
    O = ops()
    torch.manual_seed(12)
    x = torch.randn(2, 64, 6, 9, 11, device=DEV).half().float()
    wt = torch.randn(64, 64, 3, 3, 3, device=DEV) / math.sqrt(64 * 27)
    for stride in (1, 2):
        ref = F.conv3d(x, wt, stride=stride, padding=1)
        wp, kpad, _ = O.pack_conv3d_weight(wt)
        out = O.conv3d(x.permute(0, 2, 3, 4, 1).contiguous().half(), wp, kpad, 64, 3, stride)
        torch.cuda.synchronize()
        assert rel_err(out.permute(0, 4, 1, 2, 3), ref) < 2e-3
