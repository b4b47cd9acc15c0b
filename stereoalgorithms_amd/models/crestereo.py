"""CREStereo PyTorch oracle (fp32, NCHW) + presets ``crestereo-iter{2,5,10}``.

The reference pins the I/O contract of its CREStereo engines (inputs ``left``/``right`` [1,3,480,640]
RGB 0..255; output ``output`` [1,2,480,640] whose channel 0 is the positive disparity:
CREStereo/src/TRTCREStereo.cpp:15-18,130-137) and the three exported variants
``crestereo_init_iter{2,5,10}_480x640`` (README_en.md:222,244-246; "init" = no flow_init input).  The
network is upstream CREStereo (megvii-research, CVPR 2022) re-implemented here with its parameter
names: BasicEncoder (instance norm) -> 256-ch 1/4 features split into GRU hidden/context; 1/8 and
1/16 avg-pooled pyramids; LoFTR linear-attention self + cross layers at 1/16 with (bug-compatible)
sine position encoding; Adaptive Group Correlation (4 groups, alternating 1x9 / 3x3 windows, learned
offsets at 1/16 and 1/8); SepConvGRU update block; cascaded 1/16 -> 1/8 -> 1/4 refinement and convex
upsampling.  This module is the numerics oracle for csrc/models/crestereo.cpp and the source of
seeded random-init weights.
"""
from __future__ import annotations

import copy
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from .raft_stereo import ResidualBlock, randomize_norm_stats

PRESETS = {"crestereo-iter2": 2, "crestereo-iter5": 5, "crestereo-iter10": 10}


class BasicEncoder(nn.Module):
    """CREStereo feature extractor: conv1 7x7/2 -> layer1 (64) -> layer2 (96, /2) -> layer3 (128) -> 1x1."""

    def __init__(self, output_dim=256, norm_fn="instance"):
        super().__init__()
        self.norm_fn = norm_fn
        self.norm1 = nn.InstanceNorm2d(64)
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3)
        self.relu1 = nn.ReLU(inplace=True)
        self.in_planes = 64
        self.layer1 = self._make_layer(64, 1)
        self.layer2 = self._make_layer(96, 2)
        self.layer3 = self._make_layer(128, 1)
        self.conv2 = nn.Conv2d(128, output_dim, kernel_size=1)

    def _make_layer(self, dim, stride):
        layers = (ResidualBlock(self.in_planes, dim, self.norm_fn, stride),
                  ResidualBlock(dim, dim, self.norm_fn, 1))
        self.in_planes = dim
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.relu1(self.norm1(self.conv1(x)))
        return self.conv2(self.layer3(self.layer2(self.layer1(x))))


class BasicMotionEncoder(nn.Module):
    def __init__(self, cor_planes=36):
        super().__init__()
        self.convc1 = nn.Conv2d(cor_planes, 256, 1, padding=0)
        self.convc2 = nn.Conv2d(256, 192, 3, padding=1)
        self.convf1 = nn.Conv2d(2, 128, 7, padding=3)
        self.convf2 = nn.Conv2d(128, 64, 3, padding=1)
        self.conv = nn.Conv2d(64 + 192, 128 - 2, 3, padding=1)

    def forward(self, flow, corr):
        cor = F.relu(self.convc2(F.relu(self.convc1(corr))))
        flo = F.relu(self.convf2(F.relu(self.convf1(flow))))
        out = F.relu(self.conv(torch.cat([cor, flo], dim=1)))
        return torch.cat([out, flow], dim=1)


class SepConvGRU(nn.Module):
    def __init__(self, hidden_dim=128, input_dim=256):
        super().__init__()
        c = hidden_dim + input_dim
        self.convz1 = nn.Conv2d(c, hidden_dim, (1, 5), padding=(0, 2))
        self.convr1 = nn.Conv2d(c, hidden_dim, (1, 5), padding=(0, 2))
        self.convq1 = nn.Conv2d(c, hidden_dim, (1, 5), padding=(0, 2))
        self.convz2 = nn.Conv2d(c, hidden_dim, (5, 1), padding=(2, 0))
        self.convr2 = nn.Conv2d(c, hidden_dim, (5, 1), padding=(2, 0))
        self.convq2 = nn.Conv2d(c, hidden_dim, (5, 1), padding=(2, 0))

    def forward(self, h, x):
        for cz, cr, cq in ((self.convz1, self.convr1, self.convq1), (self.convz2, self.convr2, self.convq2)):
            hx = torch.cat([h, x], dim=1)
            z = torch.sigmoid(cz(hx))
            r = torch.sigmoid(cr(hx))
            q = torch.tanh(cq(torch.cat([r * h, x], dim=1)))
            h = (1 - z) * h + z * q
        return h


class FlowHead(nn.Module):
    def __init__(self, input_dim=128, hidden_dim=256):
        super().__init__()
        self.conv1 = nn.Conv2d(input_dim, hidden_dim, 3, padding=1)
        self.conv2 = nn.Conv2d(hidden_dim, 2, 3, padding=1)

    def forward(self, x):
        return self.conv2(F.relu(self.conv1(x)))


class BasicUpdateBlock(nn.Module):
    def __init__(self, hidden_dim=128, cor_planes=36, mask_size=4):
        super().__init__()
        self.encoder = BasicMotionEncoder(cor_planes)
        self.gru = SepConvGRU(hidden_dim=hidden_dim, input_dim=128 + hidden_dim)
        self.flow_head = FlowHead(hidden_dim, hidden_dim=256)
        self.mask = nn.Sequential(nn.Conv2d(128, 256, 3, padding=1), nn.ReLU(inplace=True),
                                  nn.Conv2d(256, mask_size ** 2 * 9, 1, padding=0))

    def forward(self, net, inp, corr, flow):
        motion = self.encoder(flow, corr)
        net = self.gru(net, torch.cat([inp, motion], dim=1))
        return net, 0.25 * self.mask(net), self.flow_head(net)


# ------------------------------------------------------------------------------ LoFTR attention
def elu_feature_map(x):
    return F.elu(x) + 1


class LinearAttention(nn.Module):
    def __init__(self, eps=1e-6):
        super().__init__()
        self.eps = eps

    def forward(self, q, k, v):
        Q, K = elu_feature_map(q), elu_feature_map(k)
        s = v.size(1)
        v = v / s
        KV = torch.einsum("nshd,nshv->nhdv", K, v)
        Z = 1 / (torch.einsum("nlhd,nhd->nlh", Q, K.sum(dim=1)) + self.eps)
        return torch.einsum("nlhd,nhdv,nlh->nlhv", Q, KV, Z) * s


class LoFTREncoderLayer(nn.Module):
    def __init__(self, d_model=256, nhead=8):
        super().__init__()
        self.dim, self.nhead = d_model // nhead, nhead
        self.q_proj = nn.Linear(d_model, d_model, bias=False)
        self.k_proj = nn.Linear(d_model, d_model, bias=False)
        self.v_proj = nn.Linear(d_model, d_model, bias=False)
        self.attention = LinearAttention()
        self.merge = nn.Linear(d_model, d_model, bias=False)
        self.mlp = nn.Sequential(nn.Linear(d_model * 2, d_model * 2, bias=False), nn.ReLU(True),
                                 nn.Linear(d_model * 2, d_model, bias=False))
        self.norm1 = nn.LayerNorm(d_model)
        self.norm2 = nn.LayerNorm(d_model)

    def forward(self, x, source):
        bs = x.size(0)
        q = self.q_proj(x).view(bs, -1, self.nhead, self.dim)
        k = self.k_proj(source).view(bs, -1, self.nhead, self.dim)
        v = self.v_proj(source).view(bs, -1, self.nhead, self.dim)
        msg = self.merge(self.attention(q, k, v).reshape(bs, -1, self.nhead * self.dim))
        msg = self.norm1(msg)
        msg = self.norm2(self.mlp(torch.cat([x, msg], dim=2)))
        return x + msg


class LocalFeatureTransformer(nn.Module):
    def __init__(self, d_model=256, nhead=8, layer_names=("self",)):
        super().__init__()
        self.layer_names = list(layer_names)
        layer = LoFTREncoderLayer(d_model, nhead)
        self.layers = nn.ModuleList(copy.deepcopy(layer) for _ in self.layer_names)
        for p in self.parameters():
            if p.dim() > 1:
                nn.init.xavier_uniform_(p)

    def forward(self, f0, f1):
        for layer, name in zip(self.layers, self.layer_names):
            if name == "self":
                f0, f1 = layer(f0, f0), layer(f1, f1)
            else:
                f0 = layer(f0, f1)
                f1 = layer(f1, f0)
        return f0, f1


def position_encoding_sine(d_model: int, h: int, w: int, device=None):
    """LoFTR sine encoding with CREStereo's operator-precedence quirk in the frequency term:
    ``-math.log(10000.0) / d_model // 2`` evaluates to -1.0, so div_term = exp(-[0, 2, 4, ...])."""
    y = torch.ones(h, w).cumsum(0).float()[None]
    x = torch.ones(h, w).cumsum(1).float()[None]
    div = torch.exp(torch.arange(0, d_model // 2, 2).float() * (-math.log(10000.0) / d_model // 2))[:, None, None]
    pe = torch.zeros(d_model, h, w)
    pe[0::4] = torch.sin(x * div)
    pe[1::4] = torch.cos(x * div)
    pe[2::4] = torch.sin(y * div)
    pe[3::4] = torch.cos(y * div)
    return pe[None].to(device)


# ------------------------------------------------------------------------------ AGCL
def bilinear_sampler(img, coords):
    H, W = img.shape[-2:]
    xg, yg = coords.split([1, 1], dim=-1)
    grid = torch.cat([2 * xg / (W - 1) - 1, 2 * yg / (H - 1) - 1], dim=-1)
    return F.grid_sample(img, grid, align_corners=True)


def coords_grid(b, h, w, device):
    ys, xs = torch.meshgrid(torch.arange(h, device=device), torch.arange(w, device=device), indexing="ij")
    return torch.stack([xs, ys], 0).float()[None].repeat(b, 1, 1, 1)


def window(small_patch):
    return (3, 3) if small_patch else (1, 9)


class AGCL:
    """Adaptive Group Correlation Layer: 4 channel groups, local 1x9 or 3x3 windows."""

    def __init__(self, fmap1, fmap2, att=None):
        self.fmap1, self.fmap2 = fmap1, fmap2
        if att is not None:  # cross attention on the (static) 1/16 features, computed once
            n, c, h, w = fmap1.shape
            l, r = att(fmap1.permute(0, 2, 3, 1).reshape(n, h * w, c), fmap2.permute(0, 2, 3, 1).reshape(n, h * w, c))
            self.fmap1, self.fmap2 = [x.reshape(n, h, w, c).permute(0, 3, 1, 2) for x in (l, r)]
        n, _, h, w = fmap1.shape
        self.coords = coords_grid(n, h, w, fmap1.device)

    @staticmethod
    def local_corr(left, right, psize):
        n, c, h, w = left.shape
        py, px = psize[0] // 2, psize[1] // 2
        rp = F.pad(right, (px, px, py, py), mode="replicate")
        out = [torch.mean(left * rp[:, :, dy:dy + h, dx:dx + w], dim=1, keepdim=True)
               for dy in range(2 * py + 1) for dx in range(2 * px + 1)]
        return torch.cat(out, dim=1)

    def corr_iter(self, flow, small_patch):
        coords = (self.coords + flow).permute(0, 2, 3, 1)
        right = bilinear_sampler(self.fmap2, coords)
        lefts, rights = self.fmap1.chunk(4, dim=1), right.chunk(4, dim=1)
        return torch.cat([self.local_corr(l, r, window(small_patch)) for l, r in zip(lefts, rights)], dim=1)

    def corr_offset(self, flow, extra_offset, small_patch):
        n, c, h, w = self.fmap1.shape
        psize = window(small_patch)
        ry, rx = psize[0] // 2, psize[1] // 2
        xg, yg = torch.meshgrid(torch.arange(-rx, rx + 1, device=flow.device),
                                torch.arange(-ry, ry + 1, device=flow.device), indexing="xy")
        offs = torch.stack((xg, yg)).reshape(2, -1).permute(1, 0).float()  # [9, 2] (x, y), row-major window
        extra = extra_offset.reshape(n, 9, 2, h, w).permute(0, 1, 3, 4, 2)  # [n, 9, h, w, 2]
        coords = (self.coords + flow).permute(0, 2, 3, 1)[:, None] + offs[None, :, None, None, :] + extra
        coords = coords.reshape(n, -1, w, 2)
        out = []
        for l, r in zip(self.fmap1.chunk(4, dim=1), self.fmap2.chunk(4, dim=1)):
            rs = bilinear_sampler(r, coords).reshape(n, c // 4, 9, h, w)
            out.append(torch.mean(l[:, :, None] * rs, dim=1))
        return torch.cat(out, dim=1)


class CREStereo(nn.Module):
    def __init__(self, iters: int = 5, hidden_dim: int = 128):
        super().__init__()
        self.iters = iters
        self.hidden_dim = hidden_dim
        self.fnet = BasicEncoder(output_dim=256, norm_fn="instance")
        self.update_block = BasicUpdateBlock(hidden_dim=hidden_dim, cor_planes=4 * 9, mask_size=4)
        self.self_att_fn = LocalFeatureTransformer(256, 8, ["self"])
        self.cross_att_fn = LocalFeatureTransformer(256, 8, ["cross"])
        self.conv_offset_16 = nn.Conv2d(256, 18, 3, padding=1)
        self.conv_offset_8 = nn.Conv2d(256, 18, 3, padding=1)
        self.range_16 = 1
        self.range_8 = 1

    @staticmethod
    def convex_upsample(flow, mask, rate=4):
        n, _, h, w = flow.shape
        mask = torch.softmax(mask.view(n, 1, 9, rate, rate, h, w), dim=2)
        up = F.unfold(rate * flow, [3, 3], padding=1).view(n, 2, 9, 1, 1, h, w)
        up = torch.sum(mask * up, dim=2).permute(0, 1, 4, 2, 5, 3)
        return up.reshape(n, 2, rate * h, rate * w)

    def forward(self, image1, image2, iters=None):
        """image1/2: [B,3,H,W] RGB 0..255 -> [B,2,H,W] (channel 0 = disparity)."""
        iters = iters or self.iters
        image1 = 2 * (image1 / 255.0) - 1.0
        image2 = 2 * (image2 / 255.0) - 1.0
        b = image1.shape[0]
        fm = self.fnet(torch.cat([image1, image2], 0))
        fmap1, fmap2 = fm[:b], fm[b:]
        hd = self.hidden_dim
        fmap1_dw8, fmap2_dw8 = F.avg_pool2d(fmap1, 2, stride=2), F.avg_pool2d(fmap2, 2, stride=2)
        offset_dw8 = self.range_8 * (torch.sigmoid(self.conv_offset_8(fmap1_dw8)) - 0.5) * 2.0
        net, inp = torch.split(fmap1, [hd, hd], dim=1)
        net, inp = torch.tanh(net), F.relu(inp)
        net_dw8, inp_dw8 = F.avg_pool2d(net, 2, stride=2), F.avg_pool2d(inp, 2, stride=2)
        fmap1_dw16, fmap2_dw16 = F.avg_pool2d(fmap1, 4, stride=4), F.avg_pool2d(fmap2, 4, stride=4)
        offset_dw16 = self.range_16 * (torch.sigmoid(self.conv_offset_16(fmap1_dw16)) - 0.5) * 2.0
        net_dw16, inp_dw16 = F.avg_pool2d(net, 4, stride=4), F.avg_pool2d(inp, 4, stride=4)
        h16, w16 = fmap1_dw16.shape[2:]
        pe = position_encoding_sine(256, h16, w16, fmap1.device)
        f1 = (fmap1_dw16 + pe).permute(0, 2, 3, 1).reshape(b, h16 * w16, 256)
        f2 = (fmap2_dw16 + pe).permute(0, 2, 3, 1).reshape(b, h16 * w16, 256)
        f1, f2 = self.self_att_fn(f1, f2)
        fmap1_dw16, fmap2_dw16 = [x.reshape(b, h16, w16, 256).permute(0, 3, 1, 2) for x in (f1, f2)]

        corr_fn = AGCL(fmap1, fmap2)
        corr_fn_dw8 = AGCL(fmap1_dw8, fmap2_dw8)
        corr_fn_att_dw16 = AGCL(fmap1_dw16, fmap2_dw16, att=self.cross_att_fn)

        flow_dw16 = torch.zeros(b, 2, h16, w16, device=fmap1.device)
        flow = None
        for itr in range(iters // 2):
            corrs = corr_fn_att_dw16.corr_offset(flow_dw16, offset_dw16, small_patch=itr % 2 == 1)
            net_dw16, up_mask, delta = self.update_block(net_dw16, inp_dw16, corrs, flow_dw16)
            flow_dw16 = flow_dw16 + delta
            flow = self.convex_upsample(flow_dw16, up_mask, rate=4)
        if flow is None:  # iters < 2: start the 1/8 stage from zero flow at 1/4
            flow = torch.zeros(b, 2, 4 * h16, 4 * w16, device=fmap1.device)
        scale = fmap1_dw8.shape[2] / flow.shape[2]
        flow_dw8 = -scale * F.interpolate(flow, size=fmap1_dw8.shape[2:], mode="bilinear", align_corners=True)
        for itr in range(iters // 2):
            corrs = corr_fn_dw8.corr_offset(flow_dw8, offset_dw8, small_patch=itr % 2 == 1)
            net_dw8, up_mask, delta = self.update_block(net_dw8, inp_dw8, corrs, flow_dw8)
            flow_dw8 = flow_dw8 + delta
            flow = self.convex_upsample(flow_dw8, up_mask, rate=4)
        scale = fmap1.shape[2] / flow.shape[2]
        flow = -scale * F.interpolate(flow, size=fmap1.shape[2:], mode="bilinear", align_corners=True)
        flow_up = None
        for itr in range(iters):
            corrs = corr_fn.corr_iter(flow, small_patch=itr % 2 == 1)
            net, up_mask, delta = self.update_block(net, inp, corrs, flow)
            flow = flow + delta
            flow_up = -self.convex_upsample(flow, up_mask, rate=4)
        return flow_up


def build(preset: str = "crestereo-iter5", seed: int = 0) -> CREStereo:
    torch.manual_seed(seed)
    m = CREStereo(iters=PRESETS[preset]).eval()
    randomize_norm_stats(m, seed)
    return m


def scale_heads(m: CREStereo, flow_gain: float = 4.0, flow_bias: float = -0.3, mask_gain: float = 6.0,
                seed: int = 0) -> CREStereo:
    """Well-scaled flow / mask heads for full-configuration numerics tests (see raft_stereo.scale_heads):
    the cascade then produces disparities of several pixels with spatial structure, so the AGCL windows,
    the deformable offsets and the convex upsampling are exercised away from zero flow."""
    g = torch.Generator().manual_seed(seed + 11)
    ub = m.update_block
    with torch.no_grad():
        c2 = ub.flow_head.conv2
        c2.weight.mul_(flow_gain)
        c2.bias.zero_()
        c2.bias[0] = flow_bias
        mk = ub.mask[2]
        mk.weight.mul_(mask_gain)
        mk.bias.copy_(0.5 * torch.randn(mk.bias.shape, generator=g))
    return m
