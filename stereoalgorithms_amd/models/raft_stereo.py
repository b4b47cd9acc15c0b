"""RAFT-Stereo PyTorch oracle (fp32, NCHW) + presets.

The reference repo only ships the I/O contract of RAFT-Stereo (inputs ``left``/``right``
[1,3,480,640] RGB 0..255, output ``flow_up`` = negative disparity; RAFTStereo/src/TRTRAFTStereo.cpp:13-20)
and the export recipes for the two variants it benchmarks (README_en.md:88-101).  The network is
upstream RAFT-Stereo; this module re-implements it with the upstream parameter names so that its
``state_dict`` (saved as safetensors) is exactly what the native engine (csrc/models/raft_stereo.cpp)
loads.  It is the numerics oracle for the engine and the source of seeded random-init weights.
"""
from __future__ import annotations

from dataclasses import dataclass, field, asdict

import torch
import torch.nn as nn
import torch.nn.functional as F


@dataclass
class RaftStereoConfig:
    n_downsample: int = 2
    n_gru_layers: int = 3
    slow_fast_gru: bool = False
    shared_backbone: bool = False
    valid_iters: int = 32
    hidden_dims: list = field(default_factory=lambda: [128, 128, 128])
    corr_levels: int = 4
    corr_radius: int = 4
    context_norm: str = "batch"
    mixed_precision: bool = False


PRESETS = {
    # upstream defaults: sceneflow checkpoint, 32 iterations at inference
    "raftstereo-sceneflow": RaftStereoConfig(),
    # README_en.md:95-101 realtime export flags
    "raftstereo-realtime": RaftStereoConfig(n_downsample=3, n_gru_layers=2, slow_fast_gru=True,
                                            shared_backbone=True, valid_iters=7, mixed_precision=True),
}


class ResidualBlock(nn.Module):
    def __init__(self, in_planes, planes, norm_fn="group", stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(in_planes, planes, kernel_size=3, padding=1, stride=stride)
        self.conv2 = nn.Conv2d(planes, planes, kernel_size=3, padding=1)
        self.relu = nn.ReLU(inplace=True)
        down = not (stride == 1 and in_planes == planes)
        if norm_fn == "batch":
            self.norm1, self.norm2 = nn.BatchNorm2d(planes), nn.BatchNorm2d(planes)
            if down:
                self.norm3 = nn.BatchNorm2d(planes)
        elif norm_fn == "instance":
            self.norm1, self.norm2 = nn.InstanceNorm2d(planes), nn.InstanceNorm2d(planes)
            if down:
                self.norm3 = nn.InstanceNorm2d(planes)
        elif norm_fn == "none":
            self.norm1, self.norm2 = nn.Sequential(), nn.Sequential()
            if down:
                self.norm3 = nn.Sequential()
        else:
            raise ValueError(norm_fn)
        self.downsample = None
        if down:
            self.downsample = nn.Sequential(nn.Conv2d(in_planes, planes, kernel_size=1, stride=stride), self.norm3)

    def forward(self, x):
        y = self.relu(self.norm1(self.conv1(x)))
        y = self.relu(self.norm2(self.conv2(y)))
        if self.downsample is not None:
            x = self.downsample(x)
        return self.relu(x + y)


def _norm(norm_fn, c):
    return {"batch": lambda: nn.BatchNorm2d(c), "instance": lambda: nn.InstanceNorm2d(c),
            "none": lambda: nn.Sequential()}[norm_fn]()


class BasicEncoder(nn.Module):
    def __init__(self, output_dim=128, norm_fn="batch", downsample=3):
        super().__init__()
        self.norm_fn = norm_fn
        self.norm1 = _norm(norm_fn, 64)
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=1 + (downsample > 2), padding=3)
        self.relu1 = nn.ReLU(inplace=True)
        self.in_planes = 64
        self.layer1 = self._make_layer(64, 1)
        self.layer2 = self._make_layer(96, 1 + (downsample > 1))
        self.layer3 = self._make_layer(128, 1 + (downsample > 0))
        self.conv2 = nn.Conv2d(128, output_dim, kernel_size=1)

    def _make_layer(self, dim, stride):
        layers = (ResidualBlock(self.in_planes, dim, self.norm_fn, stride),
                  ResidualBlock(dim, dim, self.norm_fn, 1))
        self.in_planes = dim
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.relu1(self.norm1(self.conv1(x)))
        return self.conv2(self.layer3(self.layer2(self.layer1(x))))


class MultiBasicEncoder(nn.Module):
    def __init__(self, output_dim, norm_fn="batch", downsample=3):
        super().__init__()
        self.norm_fn = norm_fn
        self.norm1 = _norm(norm_fn, 64)
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=1 + (downsample > 2), padding=3)
        self.relu1 = nn.ReLU(inplace=True)
        self.in_planes = 64
        self.layer1 = self._make_layer(64, 1)
        self.layer2 = self._make_layer(96, 1 + (downsample > 1))
        self.layer3 = self._make_layer(128, 1 + (downsample > 0))
        self.layer4 = self._make_layer(128, 2)
        self.layer5 = self._make_layer(128, 2)
        self.outputs08 = nn.ModuleList(
            nn.Sequential(ResidualBlock(128, 128, norm_fn, 1), nn.Conv2d(128, d[2], 3, padding=1)) for d in output_dim)
        self.outputs16 = nn.ModuleList(
            nn.Sequential(ResidualBlock(128, 128, norm_fn, 1), nn.Conv2d(128, d[1], 3, padding=1)) for d in output_dim)
        self.outputs32 = nn.ModuleList(nn.Conv2d(128, d[0], 3, padding=1) for d in output_dim)

    _make_layer = BasicEncoder._make_layer

    def forward(self, x, dual_inp=False, num_layers=3):
        x = self.relu1(self.norm1(self.conv1(x)))
        x = self.layer3(self.layer2(self.layer1(x)))
        v = None
        if dual_inp:
            v = x
            x = x[: x.shape[0] // 2]
        outs = [[f(x) for f in self.outputs08]]
        if num_layers >= 2:
            y = self.layer4(x)
            outs.append([f(y) for f in self.outputs16])
        if num_layers >= 3:
            z = self.layer5(y)
            outs.append([f(z) for f in self.outputs32])
        return (outs, v) if dual_inp else (outs, None)


class BasicMotionEncoder(nn.Module):
    def __init__(self, cfg: RaftStereoConfig):
        super().__init__()
        cor_planes = cfg.corr_levels * (2 * cfg.corr_radius + 1)
        self.convc1 = nn.Conv2d(cor_planes, 64, 1, padding=0)
        self.convc2 = nn.Conv2d(64, 64, 3, padding=1)
        self.convf1 = nn.Conv2d(2, 64, 7, padding=3)
        self.convf2 = nn.Conv2d(64, 64, 3, padding=1)
        self.conv = nn.Conv2d(64 + 64, 128 - 2, 3, padding=1)

    def forward(self, flow, corr):
        cor = F.relu(self.convc2(F.relu(self.convc1(corr))))
        flo = F.relu(self.convf2(F.relu(self.convf1(flow))))
        out = F.relu(self.conv(torch.cat([cor, flo], dim=1)))
        return torch.cat([out, flow], dim=1)


class ConvGRU(nn.Module):
    def __init__(self, hidden_dim, input_dim, kernel_size=3):
        super().__init__()
        p = kernel_size // 2
        self.convz = nn.Conv2d(hidden_dim + input_dim, hidden_dim, kernel_size, padding=p)
        self.convr = nn.Conv2d(hidden_dim + input_dim, hidden_dim, kernel_size, padding=p)
        self.convq = nn.Conv2d(hidden_dim + input_dim, hidden_dim, kernel_size, padding=p)

    def forward(self, h, cz, cr, cq, *x_list):
        x = torch.cat(x_list, dim=1)
        hx = torch.cat([h, x], dim=1)
        z = torch.sigmoid(self.convz(hx) + cz)
        r = torch.sigmoid(self.convr(hx) + cr)
        q = torch.tanh(self.convq(torch.cat([r * h, x], dim=1)) + cq)
        return (1 - z) * h + z * q


class FlowHead(nn.Module):
    def __init__(self, input_dim=128, hidden_dim=256, output_dim=2):
        super().__init__()
        self.conv1 = nn.Conv2d(input_dim, hidden_dim, 3, padding=1)
        self.conv2 = nn.Conv2d(hidden_dim, output_dim, 3, padding=1)
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        return self.conv2(self.relu(self.conv1(x)))


def pool2x(x):
    return F.avg_pool2d(x, 3, stride=2, padding=1)


def interp(x, dest):
    return F.interpolate(x, dest.shape[2:], mode="bilinear", align_corners=True)


class BasicMultiUpdateBlock(nn.Module):
    def __init__(self, cfg: RaftStereoConfig):
        super().__init__()
        hd = cfg.hidden_dims
        self.cfg = cfg
        self.encoder = BasicMotionEncoder(cfg)
        self.gru08 = ConvGRU(hd[2], 128 + hd[1] * (cfg.n_gru_layers > 1))
        self.gru16 = ConvGRU(hd[1], hd[0] * (cfg.n_gru_layers == 3) + hd[2])
        self.gru32 = ConvGRU(hd[0], hd[1])
        self.flow_head = FlowHead(hd[2], hidden_dim=256, output_dim=2)
        factor = 2 ** cfg.n_downsample
        self.mask = nn.Sequential(nn.Conv2d(hd[2], 256, 3, padding=1), nn.ReLU(inplace=True),
                                  nn.Conv2d(256, factor ** 2 * 9, 1, padding=0))

    def forward(self, net, inp, corr=None, flow=None, iter08=True, iter16=True, iter32=True, update=True):
        n = self.cfg.n_gru_layers
        if iter32:
            net[2] = self.gru32(net[2], *inp[2], pool2x(net[1]))
        if iter16:
            if n > 2:
                net[1] = self.gru16(net[1], *inp[1], pool2x(net[0]), interp(net[2], net[1]))
            else:
                net[1] = self.gru16(net[1], *inp[1], pool2x(net[0]))
        if iter08:
            mf = self.encoder(flow, corr)
            if n > 1:
                net[0] = self.gru08(net[0], *inp[0], mf, interp(net[1], net[0]))
            else:
                net[0] = self.gru08(net[0], *inp[0], mf)
        if not update:
            return net
        delta_flow = self.flow_head(net[0])
        mask = 0.25 * self.mask(net[0])
        return net, mask, delta_flow


class CorrBlock1D:
    """All-pairs 1-D correlation + avg-pooled pyramid; lookup = 1-D bilinear with zero padding."""

    def __init__(self, fmap1, fmap2, num_levels=4, radius=4):
        self.num_levels, self.radius = num_levels, radius
        b, d, h, w1 = fmap1.shape
        w2 = fmap2.shape[3]
        corr = torch.einsum("aijk,aijh->ajkh", fmap1, fmap2) / torch.sqrt(torch.tensor(d).float())
        corr = corr.reshape(b * h * w1, 1, 1, w2)
        self.pyramid = [corr]
        for _ in range(num_levels):
            corr = F.avg_pool2d(corr, [1, 2], stride=[1, 2])
            self.pyramid.append(corr)
        self.shape = (b, h, w1)

    def __call__(self, coords):
        r = self.radius
        b, h, w1 = self.shape
        x = coords[:, :1].permute(0, 2, 3, 1).reshape(b * h * w1, 1, 1, 1)
        out = []
        dx = torch.linspace(-r, r, 2 * r + 1, device=coords.device).view(1, 1, 2 * r + 1, 1)
        for i in range(self.num_levels):
            corr = self.pyramid[i]
            wl = corr.shape[-1]
            x0 = dx + x / 2 ** i
            grid = torch.cat([2 * x0 / (wl - 1) - 1, torch.zeros_like(x0)], dim=-1)
            s = F.grid_sample(corr, grid, align_corners=True)
            out.append(s.view(b, h, w1, -1))
        return torch.cat(out, dim=-1).permute(0, 3, 1, 2).contiguous().float()


def coords_grid(b, h, w, device):
    ys, xs = torch.meshgrid(torch.arange(h, device=device), torch.arange(w, device=device), indexing="ij")
    return torch.stack([xs, ys], 0).float()[None].repeat(b, 1, 1, 1)


class RAFTStereo(nn.Module):
    def __init__(self, cfg: RaftStereoConfig | str = "raftstereo-sceneflow"):
        super().__init__()
        if isinstance(cfg, str):
            self.preset = cfg
            cfg = PRESETS[cfg]
        else:
            self.preset = "custom"
        self.cfg = cfg
        hd = cfg.hidden_dims
        self.cnet = MultiBasicEncoder(output_dim=[hd, hd], norm_fn=cfg.context_norm, downsample=cfg.n_downsample)
        self.update_block = BasicMultiUpdateBlock(cfg)
        self.context_zqr_convs = nn.ModuleList(
            nn.Conv2d(hd[i], hd[i] * 3, 3, padding=1) for i in range(cfg.n_gru_layers))
        if cfg.shared_backbone:
            self.conv2 = nn.Sequential(ResidualBlock(128, 128, "instance", stride=1), nn.Conv2d(128, 256, 3, padding=1))
        else:
            self.fnet = BasicEncoder(output_dim=256, norm_fn="instance", downsample=cfg.n_downsample)

    def upsample_flow(self, flow, mask):
        n, d, h, w = flow.shape
        f = 2 ** self.cfg.n_downsample
        mask = torch.softmax(mask.view(n, 1, 9, f, f, h, w), dim=2)
        up = F.unfold(f * flow, [3, 3], padding=1).view(n, d, 9, 1, 1, h, w)
        up = torch.sum(mask * up, dim=2).permute(0, 1, 4, 2, 5, 3)
        return up.reshape(n, d, f * h, f * w)

    def forward(self, image1, image2, iters=None, test_mode=True):
        """image1/2: [B,3,H,W] RGB 0..255.  Returns (low-res flow, flow_up [B,1,H,W])."""
        cfg = self.cfg
        iters = iters or cfg.valid_iters
        image1 = (2 * (image1 / 255.0) - 1.0).contiguous()
        image2 = (2 * (image2 / 255.0) - 1.0).contiguous()
        if cfg.shared_backbone:
            cnet_list, x = self.cnet(torch.cat((image1, image2), 0), dual_inp=True, num_layers=cfg.n_gru_layers)
            fmap1, fmap2 = self.conv2(x).split(x.shape[0] // 2, dim=0)
        else:
            cnet_list, _ = self.cnet(image1, num_layers=cfg.n_gru_layers)
            fmaps = self.fnet(torch.cat([image1, image2], 0))
            fmap1, fmap2 = fmaps.split(image1.shape[0], dim=0)
        net_list = [torch.tanh(x[0]) for x in cnet_list]
        inp_list = [torch.relu(x[1]) for x in cnet_list]
        inp_list = [list(conv(i).split(conv.out_channels // 3, dim=1))
                    for i, conv in zip(inp_list, self.context_zqr_convs)]
        corr_fn = CorrBlock1D(fmap1.float(), fmap2.float(), num_levels=cfg.corr_levels, radius=cfg.corr_radius)
        b, _, h, w = net_list[0].shape
        coords0 = coords_grid(b, h, w, image1.device)
        coords1 = coords0.clone()
        n = cfg.n_gru_layers
        flow_up = None
        for itr in range(iters):
            corr = corr_fn(coords1)
            flow = coords1 - coords0
            if n == 3 and cfg.slow_fast_gru:
                net_list = self.update_block(net_list, inp_list, iter32=True, iter16=False, iter08=False, update=False)
            if n >= 2 and cfg.slow_fast_gru:
                net_list = self.update_block(net_list, inp_list, iter32=n == 3, iter16=True, iter08=False, update=False)
            net_list, up_mask, delta_flow = self.update_block(net_list, inp_list, corr, flow, iter32=n == 3,
                                                              iter16=n >= 2)
            delta_flow[:, 1] = 0.0
            coords1 = coords1 + delta_flow
            if test_mode and itr < iters - 1:
                continue
            flow_up = self.upsample_flow(coords1 - coords0, up_mask)[:, :1]
        return coords1 - coords0, flow_up


def build(preset: str, seed: int = 0) -> RAFTStereo:
    """Seeded random-init RAFT-Stereo of a named preset (eval mode)."""
    torch.manual_seed(seed)
    m = RAFTStereo(preset).eval()
    randomize_norm_stats(m, seed)
    return m


def randomize_norm_stats(m: nn.Module, seed: int = 0):
    """Non-trivial BatchNorm affine/running statistics so that BN folding is actually exercised
    (PyTorch's default init is the identity transform)."""
    g = torch.Generator().manual_seed(seed + 7)
    for mod in m.modules():
        if isinstance(mod, nn.BatchNorm2d):
            c = mod.num_features
            with torch.no_grad():
                mod.weight.copy_(0.75 + 0.5 * torch.rand(c, generator=g))
                mod.bias.copy_(0.1 * torch.randn(c, generator=g))
                mod.running_mean.copy_(0.1 * torch.randn(c, generator=g))
                mod.running_var.copy_(0.75 + 0.5 * torch.rand(c, generator=g))


def config_dict(preset: str) -> dict:
    return asdict(PRESETS[preset])


def scale_heads(m: RAFTStereo, flow_gain: float = 6.0, flow_bias: float = -0.35, mask_gain: float = 6.0,
                seed: int = 0) -> RAFTStereo:
    """Well-scaled heads for full-configuration numerics tests.

    Random-init RAFT-Stereo predicts near-zero updates (mean disparity ~0.04 px after 32 iterations), so
    the correlation lookup only ever samples around zero offset and convex upsampling sees a near-uniform
    mask.  This scales the flow head's last conv (and biases its x channel towards negative flow =
    positive disparity) and the mask head's last conv, so that disparity grows to several pixels over the
    iterations with spatial structure, the lookup walks across pyramid taps / levels and the upsampling
    softmax is peaked.  Everything stays a plain RAFT-Stereo state_dict."""
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
