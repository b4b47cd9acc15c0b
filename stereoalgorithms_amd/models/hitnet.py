"""HITNet PyTorch oracle (fp32, NCHW), preset ``hitnet-d400``.

Reference pin: HitNet/src/HitNet.cpp:13-17,69-78 — one 6-channel input ``input`` [1,6,480,640] =
[left RGB; right RGB] / 255 (HitNet_preprocess.cu:19-51), output ``reference_output_disparity`` H*W
positive disparity; the benchmarked export is ``middlebury_d400`` (HitNet/test/main.cpp:9,
README_en.md:171,192), i.e. a maximum disparity of 400 px at full resolution.  The reference only ships
that I/O contract (the network is a PINTO TF->ONNX export), so this is a re-implementation of the
published architecture (Tankovich et al., "HITNet: Hierarchical Iterative Tile Refinement Network for
Real-time Stereo Matching", CVPR 2021) with our own parameter names:

  * U-Net feature extractor, 5 levels (1 .. 1/16), channels 16,16,24,24,32, LeakyReLU(0.2); strided
    2x2 convs down, 2x2 transposed convs up, skip concatenation + 1x1 merge + 3x3 conv.
  * Tile hypotheses on levels 0..3: a 4x4/stride-4 tile embedding of the left features and the same
    conv at stride (4,1) on the right; L1 matching cost over every integer disparity of the level
    (400 >> l), argmin -> d_init; descriptor p = MLP(cost, tile feature) (13 channels).
    A hypothesis is h = [d, dx, dy, p] (16 channels), d in level-l pixels.
  * Propagation coarse -> fine: level 3 refines its own init; levels 2..0 refine two candidates
    (the slanted-plane upsampled hypothesis of the coarser level and the level's own init).  Each
    candidate gets a local cost: the 4x4 tile pixels warped into the right features along x at
    d + dx*u + dy*v (+-1 shifts), L1 over channels -> 48 features; [cost, h] -> 1x1 conv + two
    dilated residual blocks + 3x3 conv -> (delta h, confidence).  The refined candidate with the highest
    confidence wins (hard selection, inference-mode HITNet).
  * Final slanted-plane expansion of the level-0 tiles to full resolution.

This module is the numerics oracle for csrc/models/hitnet.cpp and the source of seeded random weights.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

PRESETS = {"hitnet-d400": dict(maxdisp=400)}
CH = [16, 16, 24, 24, 32]
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
    def __init__(self):
        super().__init__()
        down = [nn.ModuleList([nn.Conv2d(3, CH[0], 3, 1, 1), nn.Conv2d(CH[0], CH[0], 3, 1, 1)])]
        for l in range(1, 5):
            down.append(nn.ModuleList([nn.Conv2d(CH[l - 1], CH[l], 2, 2), nn.Conv2d(CH[l], CH[l], 3, 1, 1),
                                       nn.Conv2d(CH[l], CH[l], 3, 1, 1)]))
        self.down = nn.ModuleList(down)
        self.up = nn.ModuleList([UpBlock(CH[l + 1], CH[l]) for l in range(4)])

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


class Propagation(nn.Module):
    def __init__(self, dils=(1, 2)):
        super().__init__()
        self.inp = nn.Conv2d(64, 32, 1)
        self.res = nn.ModuleList([ResBlock(32, d) for d in dils])
        self.out = nn.Conv2d(32, 17, 3, 1, 1)

    def forward(self, cost, h):
        x = lrelu(self.inp(torch.cat((cost, h), 1)))
        for r in self.res:
            x = r(x)
        y = self.out(x)
        hn = h + y[:, :16]
        hn = torch.cat((hn[:, :1].clamp_min(0), hn[:, 1:]), 1)
        return hn, y[:, 16:17]


def tile_offsets(device):
    """(u, v) pixel offsets of the 16 tile pixels relative to the tile centre, channel k = v*4 + u."""
    r = torch.arange(4, device=device, dtype=torch.float32) - 1.5
    v, u = torch.meshgrid(r, r, indexing="ij")
    return u.reshape(16), v.reshape(16)


def warp_cost(el, er, h):
    """Local L1 cost of each tile's 16 pixels at the plane disparity (+-1): [B,48,h,w], channel s*16 + v*4 + u."""
    b, c, H, W = el.shape
    th, tw = h.shape[-2:]
    u, v = tile_offsets(el.device)
    # per-pixel plane disparity at full level resolution
    d = h[:, 0:1] + h[:, 1:2] * u.view(1, 16, 1, 1) + h[:, 2:3] * v.view(1, 16, 1, 1)  # [B,16,th,tw]
    dpix = F.pixel_shuffle(d, 4)  # [B,1,H,W]: channel v*4+u -> pixel (4y+v, 4x+u)
    xs = torch.arange(W, device=el.device, dtype=torch.float32).view(1, 1, 1, W)
    out = []
    for s in (-1.0, 0.0, 1.0):
        xr = xs - (dpix + s)  # right x (level pixels), linear interpolation, zero outside
        x0 = torch.floor(xr)
        a = xr - x0
        acc = torch.zeros(b, c, H, W, device=el.device)
        for t, wt in ((0, 1 - a), (1, a)):
            xi = x0 + t
            ok = (xi >= 0) & (xi <= W - 1)
            g = torch.gather(er, 3, xi.clamp(0, W - 1).long().expand(b, c, H, W))
            acc = acc + g * (wt * ok)
        cost = (el - acc).abs().sum(1, keepdim=True)  # [B,1,H,W]
        out.append(F.pixel_unshuffle(cost, 4))  # [B,16,th,tw]
    return torch.cat(out, 1)


def upsample_hyp(h):
    """Slanted-plane 2x upsampling of tile hypotheses to the next finer level."""
    b, c, th, tw = h.shape
    up = F.interpolate(h, scale_factor=2, mode="nearest")
    oy = (torch.arange(2 * th, device=h.device) % 2 * 2 - 1).float().view(1, 1, 2 * th, 1)
    ox = (torch.arange(2 * tw, device=h.device) % 2 * 2 - 1).float().view(1, 1, 1, 2 * tw)
    d = 2 * (up[:, 0:1] + up[:, 1:2] * ox + up[:, 2:3] * oy)
    return torch.cat((d, up[:, 1:]), 1)


def expand_final(h):
    u, v = tile_offsets(h.device)
    d = h[:, 0:1] + h[:, 1:2] * u.view(1, 16, 1, 1) + h[:, 2:3] * v.view(1, 16, 1, 1)
    return F.pixel_shuffle(d, 4)[:, 0].clamp_min(0)


class HITNet(nn.Module):
    def __init__(self, maxdisp=400):
        super().__init__()
        self.maxdisp = maxdisp
        self.feature = FeatureUNet()
        self.init = nn.ModuleList([TileInit(CH[l]) for l in range(HYP_LEVELS)])
        self.prop = nn.ModuleList([Propagation() for _ in range(HYP_LEVELS)])

    def forward(self, x6):
        """x6: [B,6,H,W] = [left RGB; right RGB] / 255 -> disparity [B,H,W]."""
        b = x6.shape[0]
        e = self.feature(torch.cat((x6[:, :3], x6[:, 3:]), 0))
        el = [t[:b] for t in e]
        er = [t[b:] for t in e]
        h = None
        for l in range(HYP_LEVELS - 1, -1, -1):
            hi = self.init[l](el[l], er[l], self.maxdisp >> l)
            cands = [hi] if h is None else [upsample_hyp(h), hi]
            best, conf = None, None
            for c in cands:
                hn, cf = self.prop[l](warp_cost(el[l], er[l], c), c)
                if best is None:
                    best, conf = hn, cf
                else:  # strictly greater wins: ties keep the earlier (upsampled) candidate
                    take = cf > conf
                    best = torch.where(take, hn, best)
                    conf = torch.where(take, cf, conf)
            h = best
        return expand_final(h)


def build(preset: str = "hitnet-d400", seed: int = 0) -> HITNet:
    torch.manual_seed(seed)
    return HITNet(**PRESETS[preset]).eval()
