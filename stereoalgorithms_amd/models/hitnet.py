"""HITNet PyTorch oracle (fp32, NCHW), presets ``hitnet-d400`` and ``hitnet-xl``.

Reference pins: HitNet/src/HitNet.cpp:13-17,69-78 — one 6-channel input ``input`` [1,6,480,640] =
[left RGB; right RGB] / 255 (HitNet_preprocess.cu:19-51), output ``reference_output_disparity`` H*W
positive disparity; the benchmarked export is ``middlebury_d400`` (HitNet/test/main.cpp:9,
README_en.md:171,192, max disparity 400 px at full resolution); README_en.md:171 also lists
``flyingthings_finalpass_xl`` (no latency published, README_en.md:192-194).  The reference ships only that
I/O contract (the networks are PINTO TF->ONNX exports of the authors' saved models, not in the repo and
not downloadable here), so this is a re-implementation of the published architecture (Tankovich et al.,
"HITNet: Hierarchical Iterative Tile Refinement Network for Real-time Stereo Matching", CVPR 2021, §3)
with our own parameter names.  Parity with the upstream weights is therefore unpinned.

Architecture (paper section in brackets):

  * Feature extractor [§3.1]: U-Net, 5 levels e_0 .. e_4 at 1 .. 1/16, LeakyReLU(0.2); strided 2x2 convs
    down, 2x2 transposed convs up, skip concatenation + 1x1 merge + 3x3 conv.  Channels (16,16,24,24,32)
    for d400, (32,32,48,48,64) for XL.
  * Initialisation [§3.2] on levels 0..3 (4x4 tiles, so the tile grids are 1/4 .. 1/32 of the input; a
    480x640 input has no integral 1/64 grid, which pins the coarsest hypothesis level to 3): a 4x4 /
    stride-4 tile embedding of the left features and the same conv at stride (4,1) on the right; L1 cost of
    the 16-channel tile features over every integer disparity of the level (maxdisp >> l), argmin -> d_init;
    descriptor p = MLP(cost, tile feature) (13 channels).  A hypothesis is h = [d, dx, dy, p] (16 channels),
    d in level-l pixels, slanted plane d + dx * u + dy * v over the tile.
  * Propagation [§3.3], coarse -> fine: level 3 refines its own init; levels 2..0 refine TWO candidates
    jointly, the slanted-plane 2x upsampling of the coarser level's winner and the level's own init.  Each
    candidate gets a local cost from warping: the 16 tile pixels of the left features against the right
    features sampled (linear interpolation along x, zeros outside) at the candidate's plane disparity and
    at +-1, L1 over channels -> 48 costs.  The update network sees all candidates at once
    ([cost_k, h_k] for every k concatenated), 1x1 conv -> residual blocks with a dilation schedule ->
    3x3 conv -> per candidate (delta h_k, confidence w_k); the refined candidate with the highest confidence
    wins (inference-mode HITNet: argmax of the confidences).
  * Final refinement [§3.3, the propagation steps below the tile resolution]: the level-0 winner is split
    into 2x2 tiles (plane evaluated at each sub-tile centre) and refined once more with the same warping
    cost (4 pixels x 3 shifts) and a residual update network (one hypothesis, no init), then split into
    1x1 tiles (per pixel, full resolution) and refined again (1 pixel x 3 shifts).  Output = max(d, 0).

Choices not fixed by the published description (documented deviations, all shared by the native engine):
update-network width 32 (XL 64); residual dilations (1, 2, 4) per level (XL (1, 2, 4, 8, 1)); refinement
widths 32 / 16 (XL 48 / 24) with dilations (1, 2) / (1, 1); XL max disparity 320; the local cost uses the
level's full feature vector (paper: learned tile features of the same width).

This module is the numerics oracle for csrc/models/hitnet.cpp and the source of seeded random weights.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

PRESETS = {
    "hitnet-d400": dict(maxdisp=400, ch=(16, 16, 24, 24, 32), width=32, dils=(1, 2, 4),
                        refine=((32, (1, 2)), (16, (1, 1)))),
    "hitnet-xl": dict(maxdisp=320, ch=(32, 32, 48, 48, 64), width=64, dils=(1, 2, 4, 8, 1),
                      refine=((48, (1, 2)), (24, (1, 1)))),
}
HYP_LEVELS = 4  # tile hypotheses on feature levels 0..3
SLOPE = 0.2


def lrelu(x):
    return F.leaky_relu(x, SLOPE)


class UpBlock(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.deconv = nn.ConvTranspose2d(cin, cout, 2, 2)
        self.merge = nn.Conv2d(2 * cout, cout, 1)
        self.conv = nn.Conv2d(cout, cout, 3, 1, 1)

    def forward(self, x, skip):
        x = lrelu(self.deconv(x))
        x = lrelu(self.merge(torch.cat((x, skip), 1)))
        return lrelu(self.conv(x))


class FeatureUNet(nn.Module):
    def __init__(self, ch):
        super().__init__()
        down = [nn.ModuleList([nn.Conv2d(3, ch[0], 3, 1, 1), nn.Conv2d(ch[0], ch[0], 3, 1, 1)])]
        for l in range(1, 5):
            down.append(nn.ModuleList([nn.Conv2d(ch[l - 1], ch[l], 2, 2), nn.Conv2d(ch[l], ch[l], 3, 1, 1),
                                       nn.Conv2d(ch[l], ch[l], 3, 1, 1)]))
        self.down = nn.ModuleList(down)
        self.up = nn.ModuleList([UpBlock(ch[l + 1], ch[l]) for l in range(4)])

    def forward(self, x):
        d = []
        for blk in self.down:
            for conv in blk:
                x = lrelu(conv(x))
            d.append(x)
        e = [None] * 5
        e[4] = d[4]
        for l in range(3, -1, -1):
            e[l] = self.up[l](e[l + 1], d[l])
        return e


class TileInit(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.tile = nn.Conv2d(c, 16, 4, 4)
        self.desc = nn.Conv2d(17, 13, 1)

    def tiles(self, el, er):
        """4x4 tile embeddings: left at stride 4 [B,16,h,w], right at stride (4,1) [B,16,h,W-3]."""
        return self.tile(el), F.conv2d(er, self.tile.weight, self.tile.bias, stride=(4, 1))

    def forward(self, el, er, ndisp):
        return self.hypothesis(*self.tiles(el, er), ndisp)

    def hypothesis(self, tl, tr, ndisp):
        b, c, h, w = tl.shape
        wr = tr.shape[-1]
        big = torch.finfo(tl.dtype).max
        costs = []
        xs = torch.arange(w, device=tl.device) * 4
        for d in range(ndisp):
            j = xs - d
            valid = (j >= 0) & (j < wr)
            g = tr[..., j.clamp(0, wr - 1)]
            cst = (tl - g).abs().sum(1)
            costs.append(torch.where(valid.view(1, 1, w), cst, torch.full_like(cst, big)))
        cv = torch.stack(costs, 1)  # [B,D,h,w]
        cmin, dinit = cv.min(1)  # first index on ties
        p = lrelu(self.desc(torch.cat((cmin.unsqueeze(1), tl), 1)))
        z = torch.zeros_like(cmin).unsqueeze(1)
        return torch.cat((dinit.float().unsqueeze(1), z, z, p), 1)


class ResBlock(nn.Module):
    def __init__(self, c, dil):
        super().__init__()
        self.conv1 = nn.Conv2d(c, c, 3, 1, dil, dilation=dil)
        self.conv2 = nn.Conv2d(c, c, 3, 1, dil, dilation=dil)

    def forward(self, x):
        return lrelu(x + self.conv2(lrelu(self.conv1(x))))


def cost_channels(t: int) -> int:
    return 3 * t * t


class UpdateNet(nn.Module):
    """Joint update of ``ncand`` hypotheses of tile size ``t``: input [cost_k (3 t^2), h_k (16)] for every
    candidate k, output per candidate 16 deltas (+ a confidence when ncand > 1, or always for levels)."""

    def __init__(self, t: int, ncand: int, width: int, dils, conf: bool = True):
        super().__init__()
        self.t, self.ncand, self.conf = t, ncand, conf
        self.cin = cost_channels(t) + 16
        self.nout = 17 if conf else 16
        self.inp = nn.Conv2d(ncand * self.cin, width, 1)
        self.res = nn.ModuleList([ResBlock(width, d) for d in dils])
        self.out = nn.Conv2d(width, ncand * self.nout, 3, 1, 1)

    def forward(self, costs, hyps):
        """costs/hyps: lists over candidates of [B,3t^2,h,w] / [B,16,h,w] -> (refined list, confidences)."""
        x = torch.cat([torch.cat((c, h), 1) for c, h in zip(costs, hyps)], 1)
        x = lrelu(self.inp(x))
        for r in self.res:
            x = r(x)
        y = self.out(x)
        outs, confs = [], []
        for k, h in enumerate(hyps):
            yk = y[:, k * self.nout:(k + 1) * self.nout]
            hn = h + yk[:, :16]
            outs.append(torch.cat((hn[:, :1].clamp_min(0), hn[:, 1:]), 1))
            confs.append(yk[:, 16:17] if self.conf else None)
        return outs, confs


def tile_offsets(t: int, device):
    """(u, v) pixel offsets of the t*t tile pixels relative to the tile centre, channel k = v*t + u."""
    r = torch.arange(t, device=device, dtype=torch.float32) - (t - 1) / 2.0
    v, u = torch.meshgrid(r, r, indexing="ij")
    return u.reshape(t * t), v.reshape(t * t)


def plane_pixels(h, t: int):
    """Per-pixel plane disparity of t x t tiles: [B,1,t*th,t*tw]."""
    u, v = tile_offsets(t, h.device)
    d = h[:, 0:1] + h[:, 1:2] * u.view(1, -1, 1, 1) + h[:, 2:3] * v.view(1, -1, 1, 1)  # [B,t*t,th,tw]
    return F.pixel_shuffle(d, t) if t > 1 else d


def warp_cost(el, er, h, t: int = 4):
    """Local L1 cost of each tile's t*t pixels at the plane disparity (+-1): [B,3t^2,th,tw],
    channel s*t^2 + v*t + u."""
    b, c, H, W = el.shape
    dpix = plane_pixels(h, t)  # [B,1,H,W]
    xs = torch.arange(W, device=el.device, dtype=torch.float32).view(1, 1, 1, W)
    out = []
    for s in (-1.0, 0.0, 1.0):
        xr = xs - (dpix + s)  # right x (level pixels), linear interpolation, zero outside
        x0 = torch.floor(xr)
        a = xr - x0
        acc = torch.zeros(b, c, H, W, device=el.device)
        for k, wt in ((0, 1 - a), (1, a)):
            xi = x0 + k
            ok = (xi >= 0) & (xi <= W - 1)
            g = torch.gather(er, 3, xi.clamp(0, W - 1).long().expand(b, c, H, W))
            acc = acc + g * (wt * ok)
        cost = (el - acc).abs().sum(1, keepdim=True)  # [B,1,H,W]
        out.append(F.pixel_unshuffle(cost, t) if t > 1 else cost)  # [B,t*t,th,tw]
    return torch.cat(out, 1)


def upsample_hyp(h):
    """Slanted-plane 2x upsampling of tile hypotheses to the next finer feature level (d doubles)."""
    b, c, th, tw = h.shape
    up = F.interpolate(h, scale_factor=2, mode="nearest")
    oy = (torch.arange(2 * th, device=h.device) % 2 * 2 - 1).float().view(1, 1, 2 * th, 1)
    ox = (torch.arange(2 * tw, device=h.device) % 2 * 2 - 1).float().view(1, 1, 1, 2 * tw)
    d = 2 * (up[:, 0:1] + up[:, 1:2] * ox + up[:, 2:3] * oy)
    return torch.cat((d, up[:, 1:]), 1)


def split_hyp(h, t: int):
    """Split t x t tiles into (t/2) x (t/2) tiles of the same level: the plane is evaluated at each sub-tile
    centre (offsets +-t/4 pixels), slopes and descriptor copied."""
    b, c, th, tw = h.shape
    up = F.interpolate(h, scale_factor=2, mode="nearest")
    q = t / 4.0
    oy = ((torch.arange(2 * th, device=h.device) % 2) * 2 - 1).float().view(1, 1, 2 * th, 1) * q
    ox = ((torch.arange(2 * tw, device=h.device) % 2) * 2 - 1).float().view(1, 1, 1, 2 * tw) * q
    d = up[:, 0:1] + up[:, 1:2] * ox + up[:, 2:3] * oy
    return torch.cat((d, up[:, 1:]), 1)


def expand_final(h, t: int = 1):
    """Disparity map from tile hypotheses of size t (plane evaluated per pixel), clamped at 0."""
    return plane_pixels(h, t)[:, 0].clamp_min(0)


class HITNet(nn.Module):
    def __init__(self, maxdisp=400, ch=(16, 16, 24, 24, 32), width=32, dils=(1, 2, 4),
                 refine=((32, (1, 2)), (16, (1, 1)))):
        super().__init__()
        self.maxdisp, self.ch = maxdisp, ch
        self.feature = FeatureUNet(ch)
        self.init = nn.ModuleList([TileInit(ch[l]) for l in range(HYP_LEVELS)])
        self.prop = nn.ModuleList([UpdateNet(4, 1 if l == HYP_LEVELS - 1 else 2, width, dils)
                                   for l in range(HYP_LEVELS)])
        self.refine = nn.ModuleList([UpdateNet(t, 1, w, d, conf=False) for t, (w, d) in zip((2, 1), refine)])

    def levels(self, el, er):
        """Tile hypotheses coarse -> fine; returns the per-level winners (index = level)."""
        hyps = [None] * HYP_LEVELS
        h = None
        for l in range(HYP_LEVELS - 1, -1, -1):
            hi = self.init[l](el[l], er[l], self.maxdisp >> l)
            cands = [hi] if h is None else [upsample_hyp(h), hi]
            outs, confs = self.prop[l]([warp_cost(el[l], er[l], c) for c in cands], cands)
            best, conf = outs[0], confs[0]
            for o, cf in zip(outs[1:], confs[1:]):  # strictly greater wins: ties keep the upsampled candidate
                take = cf > conf
                best = torch.where(take, o, best)
                conf = torch.where(take, cf, conf)
            hyps[l] = h = best
        return hyps

    def forward(self, x6):
        """x6: [B,6,H,W] = [left RGB; right RGB] / 255 -> disparity [B,H,W]."""
        b = x6.shape[0]
        e = self.feature(torch.cat((x6[:, :3], x6[:, 3:]), 0))
        el = [t[:b] for t in e]
        er = [t[b:] for t in e]
        h = self.levels(el, er)[0]
        for t, net in zip((2, 1), self.refine):
            h = split_hyp(h, 2 * t)
            (h,), _ = net([warp_cost(el[0], er[0], h, t)], [h])
        return expand_final(h, 1)


def scale_init(m: HITNet, gain: float = (6.0 / (1 + SLOPE ** 2)) ** 0.5, update_gain: float = 0.25) -> HITNet:
    """Variance-preserving init for the full-configuration tests: PyTorch's default conv init (uniform with
    var 1 / (3 fan_in)) shrinks a leaky-ReLU signal ~2.4x per layer, so after the 14-layer feature U-Net the
    coarse features of a random network are ~1e-7 -- below fp16's normal range -- and every tile-init argmin
    compares noise.  Multiplying the feature and tile-embedding weights by sqrt(6 / (1 + slope^2)) (He init for
    leaky ReLU) keeps the features O(1), so the fp16 engine and the fp32 oracle see the same matching problem.

    The update networks' output convs (the deltas on the hypotheses) are scaled by ``update_gain``: at the default
    init the XL networks (width 64, five dilated blocks per level) turn fp16 rounding of the hypotheses into > 1 px
    disparity changes on ~6 % of the pixels away from any near-tie decision (an fp16-rounded copy of the oracle
    itself, while 1e-5 input noise in fp32 changes nothing), i.e. the random network is ill-conditioned in fp16;
    with deltas 4x smaller it is not (>= 0.99 within 1 px), and the disparity stays ~24 px on average."""
    with torch.no_grad():
        for mod in list(m.feature.modules()) + [t.tile for t in m.init]:
            if isinstance(mod, (nn.Conv2d, nn.ConvTranspose2d)):
                mod.weight.mul_(gain)
        for net in list(m.prop) + list(m.refine):
            net.out.weight.mul_(update_gain)
            net.out.bias.mul_(update_gain)
    return m


def near_tie_mask(m: HITNet, x6, rel: float = 1e-2, eps: float = 0.0):
    """Full-resolution mask of the pixels whose result hangs on a near-tie decision of the network: the tile-init
    argmin of any ancestor tile whose best two costs are within ``rel * cost + eps``, or the confidence argmax
    of any ancestor tile whose two candidates' confidences are within ``rel * |conf| + eps``.  An implementation
    that rounds differently (fp16 operands, another summation order) may legitimately decide those the other
    way; everywhere else its disparity must track the oracle's.  Returns (disparity [B,H,W], mask [B,H,W])."""
    b, _, H, W = x6.shape
    e = m.feature(torch.cat((x6[:, :3], x6[:, 3:]), 0))
    el = [t[:b] for t in e]
    er = [t[b:] for t in e]
    tie = torch.zeros(b, H, W, dtype=torch.bool, device=x6.device)

    def mark(mask_tiles, l):  # level-l 4x4 tiles cover (4 << l)^2 input pixels
        f = 4 << l
        up = mask_tiles.repeat_interleave(f, 1).repeat_interleave(f, 2)[:, :H, :W]
        tie[:, :up.shape[1], :up.shape[2]] |= up

    h = None
    for l in range(HYP_LEVELS - 1, -1, -1):
        tl, tr = m.init[l].tiles(el[l], er[l])
        nd = m.maxdisp >> l
        wr = tr.shape[-1]
        xs = torch.arange(tl.shape[-1], device=tl.device) * 4
        costs = []
        for d in range(nd):
            j = xs - d
            valid = (j >= 0) & (j < wr)
            cst = (tl - tr[..., j.clamp(0, wr - 1)]).abs().sum(1)
            costs.append(torch.where(valid.view(1, 1, -1), cst, torch.full_like(cst, float("inf"))))
        two = torch.stack(costs, 1).topk(2, dim=1, largest=False).values
        mark((two[:, 1] - two[:, 0]) <= rel * two[:, 0].abs() + eps, l)
        hi = m.init[l](el[l], er[l], nd)
        cands = [hi] if h is None else [upsample_hyp(h), hi]
        outs, confs = m.prop[l]([warp_cost(el[l], er[l], c) for c in cands], cands)
        best, conf = outs[0], confs[0]
        for o, cf in zip(outs[1:], confs[1:]):
            mark(((cf - conf).abs() <= rel * conf.abs() + eps)[:, 0], l)
            take = cf > conf
            best = torch.where(take, o, best)
            conf = torch.where(take, cf, conf)
        h = best
    for t, net in zip((2, 1), m.refine):
        h = split_hyp(h, 2 * t)
        (h,), _ = net([warp_cost(el[0], er[0], h, t)], [h])
    return expand_final(h, 1), tie


def build(preset: str = "hitnet-d400", seed: int = 0) -> HITNet:
    torch.manual_seed(seed)
    return HITNet(**PRESETS[preset]).eval()
