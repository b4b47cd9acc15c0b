"""Fast-ACVNet+ PyTorch oracle (fp32, NCHW), preset ``fastacvnet-plus``.

Reference pin: FastACVNet_plus/src/TRTFastACVNet_plus.cpp:15-18 (inputs ``left_image``/``right_image``
[1,3,480,640] ImageNet-normalised RGB, FastACVNet_plus_preprocess.cu:21-29; output ``output`` H*W positive
disparity) for the ``fast_acvnet_plus_generalization_opset16_480x640`` export (README_en.md:272,293-295).
The network is upstream Fast-ACVNet+ (Xu et al., "Accurate and Efficient Stereo Matching via Attention
Concatenation Volume"), re-implemented with its parameter names:

  MobileNetV2 (timm mobilenetv2_100 layout) features at 1/4..1/32 -> FPN-style transposed-conv
  up-fusion to 1/4 (+ shallow stems at 1/2 and 1/4) -> normalised (cosine) correlation volume over
  maxdisp/4 = 48 planes -> 3-D conv hourglass with image-guided channel attention -> softmax ->
  top-24 "fine-to-important" disparity sampling -> attention-weighted concatenation volume at the
  sampled disparities (right features warped by integer shifts) -> 3-D hourglass -> top-2 softmax
  regression -> learned 3x3 superpixel (spx) upsampling to full resolution, x4.

This module is the numerics oracle for csrc/models/fast_acvnet.cpp and the source of seeded
random-init weights.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .raft_stereo import randomize_norm_stats

PRESETS = {"fastacvnet-plus": dict(maxdisp=192, topk=24)}


class BasicConv(nn.Module):
    def __init__(self, cin, cout, deconv=False, is_3d=False, bn=True, relu=True, **kw):
        super().__init__()
        self.relu, self.use_bn = relu, bn
        if is_3d:
            self.conv = (nn.ConvTranspose3d if deconv else nn.Conv3d)(cin, cout, bias=False, **kw)
            self.bn = nn.BatchNorm3d(cout)
        else:
            self.conv = (nn.ConvTranspose2d if deconv else nn.Conv2d)(cin, cout, bias=False, **kw)
            self.bn = nn.BatchNorm2d(cout)

    def forward(self, x):
        x = self.conv(x)
        if self.use_bn:
            x = self.bn(x)
        if self.relu:
            x = F.leaky_relu(x, 0.01)
        return x


class Conv2x(nn.Module):
    def __init__(self, cin, cout, deconv=False, is_3d=False, concat=True, keep_concat=True, bn=True, relu=True):
        super().__init__()
        self.concat = concat
        kernel = (4, 4, 4) if (deconv and is_3d) else (4 if deconv else 3)
        self.conv1 = BasicConv(cin, cout, deconv, is_3d, bn=True, relu=True, kernel_size=kernel, stride=2, padding=1)
        if concat:
            mul = 2 if keep_concat else 1
            self.conv2 = BasicConv(cout * 2, cout * mul, False, is_3d, bn, relu, kernel_size=3, stride=1, padding=1)
        else:
            self.conv2 = BasicConv(cout, cout, False, is_3d, bn, relu, kernel_size=3, stride=1, padding=1)

    def forward(self, x, rem):
        x = self.conv1(x)
        if x.shape[-2:] != rem.shape[-2:]:
            x = F.interpolate(x, size=rem.shape[-2:], mode="nearest")
        x = torch.cat((x, rem), 1) if self.concat else x + rem
        return self.conv2(x)


# ------------------------------------------------------------------------ MobileNetV2 (timm layout)
class DepthwiseSeparable(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.conv_dw = nn.Conv2d(cin, cin, 3, 1, 1, groups=cin, bias=False)
        self.bn1 = nn.BatchNorm2d(cin)
        self.conv_pw = nn.Conv2d(cin, cout, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)

    def forward(self, x):
        return self.bn2(self.conv_pw(F.relu6(self.bn1(self.conv_dw(x)))))


class InvertedResidual(nn.Module):
    def __init__(self, cin, cout, stride, exp=6):
        super().__init__()
        mid = cin * exp
        self.has_skip = stride == 1 and cin == cout
        self.conv_pw = nn.Conv2d(cin, mid, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(mid)
        self.conv_dw = nn.Conv2d(mid, mid, 3, stride, 1, groups=mid, bias=False)
        self.bn2 = nn.BatchNorm2d(mid)
        self.conv_pwl = nn.Conv2d(mid, cout, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(cout)

    def forward(self, x):
        y = F.relu6(self.bn1(self.conv_pw(x)))
        y = F.relu6(self.bn2(self.conv_dw(y)))
        y = self.bn3(self.conv_pwl(y))
        return x + y if self.has_skip else y


def _stage(cin, cout, n, stride):
    return nn.Sequential(*[InvertedResidual(cin if i == 0 else cout, cout, stride if i == 0 else 1) for i in range(n)])


# stage specs of mobilenetv2_100: (cout, repeats, stride); stage 0 is the depthwise-separable block
MBV2 = [(16, 1, 1), (24, 2, 2), (32, 3, 2), (64, 4, 2), (96, 3, 1), (160, 3, 2)]


class Feature(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv_stem = nn.Conv2d(3, 32, 3, 2, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(32)
        blocks = [nn.Sequential(DepthwiseSeparable(32, 16))]
        cin = 16
        for cout, n, s in MBV2[1:]:
            blocks.append(_stage(cin, cout, n, s))
            cin = cout
        # timm Feature split: layers = [1, 2, 3, 5, 6]
        self.block0 = nn.Sequential(blocks[0])
        self.block1 = nn.Sequential(blocks[1])
        self.block2 = nn.Sequential(blocks[2])
        self.block3 = nn.Sequential(blocks[3], blocks[4])
        self.block4 = nn.Sequential(blocks[5])

    def forward(self, x):
        x = F.relu6(self.bn1(self.conv_stem(x)))
        x2 = self.block0(x)
        x4 = self.block1(x2)
        x8 = self.block2(x4)
        x16 = self.block3(x8)
        x32 = self.block4(x16)
        return [x4, x8, x16, x32]


class FeatUp(nn.Module):
    def __init__(self):
        super().__init__()
        chans = [16, 24, 32, 96, 160]
        self.deconv32_16 = Conv2x(chans[4], chans[3], deconv=True, concat=True)
        self.deconv16_8 = Conv2x(chans[3] * 2, chans[2], deconv=True, concat=True)
        self.deconv8_4 = Conv2x(chans[2] * 2, chans[1], deconv=True, concat=True)
        self.conv4 = BasicConv(chans[1] * 2, chans[1] * 2, kernel_size=3, stride=1, padding=1)

    def forward(self, fl, fr):
        x4, x8, x16, x32 = fl
        y4, y8, y16, y32 = fr
        x16, y16 = self.deconv32_16(x32, x16), self.deconv32_16(y32, y16)
        x8, y8 = self.deconv16_8(x16, x8), self.deconv16_8(y16, y8)
        x4, y4 = self.deconv8_4(x8, x4), self.deconv8_4(y8, y4)
        return [self.conv4(x4), x8, x16, x32], [self.conv4(y4), y8, y16, y32]


class ChannelAtt(nn.Module):
    def __init__(self, cv_chan, im_chan):
        super().__init__()
        self.im_att = nn.Sequential(BasicConv(im_chan, im_chan // 2, kernel_size=1, stride=1, padding=0),
                                    nn.Conv2d(im_chan // 2, cv_chan, 1))

    def forward(self, cv, im):
        return torch.sigmoid(self.im_att(im)).unsqueeze(2) * cv


class Hourglass(nn.Module):
    """3-D hourglass with image-guided channel attention (hourglass / hourglass_att upstream)."""

    def __init__(self, c):
        super().__init__()
        k3 = dict(is_3d=True, bn=True, relu=True, kernel_size=3, padding=1)
        self.conv1 = nn.Sequential(BasicConv(c, 2 * c, stride=2, **k3), BasicConv(2 * c, 2 * c, stride=1, **k3))
        self.conv2 = nn.Sequential(BasicConv(2 * c, 4 * c, stride=2, **k3), BasicConv(4 * c, 4 * c, stride=1, **k3))
        self.conv2_up = BasicConv(4 * c, 2 * c, deconv=True, is_3d=True, bn=True, relu=True, kernel_size=(4, 4, 4),
                                  padding=(1, 1, 1), stride=(2, 2, 2))
        self.conv1_up = BasicConv(2 * c, 1, deconv=True, is_3d=True, bn=False, relu=False, kernel_size=(4, 4, 4),
                                  padding=(1, 1, 1), stride=(2, 2, 2))
        self.agg_0 = nn.Sequential(BasicConv(4 * c, 2 * c, is_3d=True, kernel_size=1, padding=0, stride=1),
                                   BasicConv(2 * c, 2 * c, is_3d=True, kernel_size=3, padding=1, stride=1))
        self.feature_att_8 = ChannelAtt(2 * c, 64)
        self.feature_att_16 = ChannelAtt(4 * c, 192)
        self.feature_att_up_8 = ChannelAtt(2 * c, 64)

    def forward(self, x, imgs):
        conv1 = self.feature_att_8(self.conv1(x), imgs[1])
        conv2 = self.feature_att_16(self.conv2(conv1), imgs[2])
        conv1 = torch.cat((self.conv2_up(conv2), conv1), dim=1)
        conv1 = self.feature_att_up_8(self.agg_0(conv1), imgs[1])
        return self.conv1_up(conv1)


def norm_correlation_volume(l, r, maxdisp):
    b, c, h, w = l.shape
    ln = l / (torch.norm(l, 2, 1, True) + 1e-5)
    rn = r / (torch.norm(r, 2, 1, True) + 1e-5)
    vol = l.new_zeros(b, 1, maxdisp, h, w)
    for i in range(maxdisp):
        if i > 0:
            vol[:, :, i, :, i:] = (ln[:, :, :, i:] * rn[:, :, :, :-i]).mean(1, keepdim=True)
        else:
            vol[:, :, i] = (ln * rn).mean(1, keepdim=True)
    return vol


def warp_right(right, disp_samples):
    """right [B,C,H,W] sampled at x - d (zeros outside) for integer-valued d [B,D,H,W] -> [B,C,D,H,W]."""
    b, c, h, w = right.shape
    d = disp_samples.shape[1]
    xs = torch.arange(w, device=right.device, dtype=right.dtype).view(1, 1, 1, w)
    ys = torch.arange(h, device=right.device, dtype=right.dtype).view(1, 1, h, 1).expand(b, d, h, w)
    gx = (xs - disp_samples) / ((w - 1.0) / 2.0) - 1.0
    gy = ys / ((h - 1.0) / 2.0) - 1.0
    grid = torch.stack([gx, gy], dim=4).view(b, d * h, w, 2)
    return F.grid_sample(right, grid, mode="bilinear", padding_mode="zeros", align_corners=True).view(b, c, d, h, w)


def context_upsample(depth_low, up_weights):
    b, c, h, w = depth_low.shape
    unf = F.unfold(depth_low, 3, 1, 1).reshape(b, -1, h, w)
    unf = F.interpolate(unf, (h * 4, w * 4), mode="nearest").reshape(b, 9, h * 4, w * 4)
    return (unf * up_weights).sum(1)


class FastACVNetPlus(nn.Module):
    def __init__(self, maxdisp=192, topk=24):
        super().__init__()
        self.maxdisp, self.topk = maxdisp, topk
        self.feature = Feature()
        self.feature_up = FeatUp()
        self.stem_2 = nn.Sequential(BasicConv(3, 32, kernel_size=3, stride=2, padding=1),
                                    nn.Conv2d(32, 32, 3, 1, 1, bias=False), nn.BatchNorm2d(32), nn.ReLU())
        self.stem_4 = nn.Sequential(BasicConv(32, 48, kernel_size=3, stride=2, padding=1),
                                    nn.Conv2d(48, 48, 3, 1, 1, bias=False), nn.BatchNorm2d(48), nn.ReLU())
        self.spx = nn.Sequential(nn.ConvTranspose2d(2 * 32, 9, kernel_size=4, stride=2, padding=1))
        self.spx_2 = Conv2x(32, 32, True)
        self.spx_4 = nn.Sequential(BasicConv(96, 32, kernel_size=3, stride=1, padding=1),
                                   nn.Conv2d(32, 32, 3, 1, 1, bias=False), nn.BatchNorm2d(32), nn.ReLU())
        self.conv = BasicConv(96, 48, kernel_size=3, padding=1, stride=1)
        self.desc = nn.Conv2d(48, 48, kernel_size=1, padding=0, stride=1)
        self.corr_stem = BasicConv(1, 8, is_3d=True, kernel_size=3, stride=1, padding=1)
        self.corr_feature_att_4 = ChannelAtt(8, 96)
        self.hourglass_att = Hourglass(8)
        self.concat_feature = nn.Sequential(BasicConv(96, 32, kernel_size=3, stride=1, padding=1),
                                            nn.Conv2d(32, 16, 3, 1, 1, bias=False))
        self.concat_stem = BasicConv(32, 16, is_3d=True, kernel_size=3, stride=1, padding=1)
        self.concat_feature_att_4 = ChannelAtt(16, 96)
        self.hourglass = Hourglass(16)

    def forward(self, left, right):
        """left/right: [B,3,H,W] ImageNet-normalised RGB -> disparity [B,H,W]."""
        fl, fr = self.feature_up(self.feature(left), self.feature(right))
        stem_2x, stem_2y = self.stem_2(left), self.stem_2(right)
        stem_4x, stem_4y = self.stem_4(stem_2x), self.stem_4(stem_2y)
        fl[0] = torch.cat((fl[0], stem_4x), 1)
        fr[0] = torch.cat((fr[0], stem_4y), 1)
        match_l, match_r = self.desc(self.conv(fl[0])), self.desc(self.conv(fr[0]))
        corr = self.corr_stem(norm_correlation_volume(match_l, match_r, self.maxdisp // 4))
        att_weights = self.hourglass_att(self.corr_feature_att_4(corr, fl[0]), fl)  # [B,1,48,h,w]
        prob = F.softmax(att_weights, dim=2)
        # ONNX TopK semantics (equal values: lower index first) == stable descending sort
        _, ind = prob.sort(dim=2, descending=True, stable=True)
        ind_k = ind[:, :, :self.topk].sort(2, False)[0]
        att_topk = torch.gather(prob, 2, ind_k)
        samples = ind_k.squeeze(1).float()  # [B,24,h,w]
        cl, cr = self.concat_feature(fl[0]), self.concat_feature(fr[0])
        vol = torch.cat((cl.unsqueeze(2).expand(-1, -1, samples.shape[1], -1, -1), warp_right(cr, samples)), 1)
        vol = self.concat_feature_att_4(self.concat_stem(att_topk * vol), fl[0])
        cost = self.hourglass(vol, fl).squeeze(1)  # [B,24,h,w]
        _, ci = cost.sort(dim=1, descending=True, stable=True)
        pi = ci[:, :2]
        p2 = F.softmax(torch.gather(cost, 1, pi), 1)
        pred = (torch.gather(samples, 1, pi) * p2).sum(1, keepdim=True)
        xspx = self.spx_2(self.spx_4(fl[0]), stem_2x)
        spx_pred = F.softmax(self.spx(xspx), 1)
        return context_upsample(pred, spx_pred) * 4


def near_tie_mask(m: FastACVNetPlus, left, right, rel: float = 2e-2):
    """Forward pass plus a full-resolution mask of the pixels whose result hangs on a near-tie selection:
    the attention top-k cut (the k-th and (k+1)-th probabilities within ``rel``) or the final top-2 cut (the
    2nd and 3rd cost logits within ``rel`` of the logit spread) of any 1/4-resolution pixel in the 3x3
    neighbourhood the superpixel upsampling reads.  An implementation with other rounding may pick the other
    candidate there; elsewhere it must track the oracle.  Returns (disparity [B,H,W], mask [B,H,W])."""
    fl, fr = m.feature_up(m.feature(left), m.feature(right))
    stem_2x, stem_2y = m.stem_2(left), m.stem_2(right)
    stem_4x, stem_4y = m.stem_4(stem_2x), m.stem_4(stem_2y)
    fl[0] = torch.cat((fl[0], stem_4x), 1)
    fr[0] = torch.cat((fr[0], stem_4y), 1)
    match_l, match_r = m.desc(m.conv(fl[0])), m.desc(m.conv(fr[0]))
    corr = m.corr_stem(norm_correlation_volume(match_l, match_r, m.maxdisp // 4))
    att_weights = m.hourglass_att(m.corr_feature_att_4(corr, fl[0]), fl)
    prob = F.softmax(att_weights, dim=2)
    sp, ind = prob.sort(dim=2, descending=True, stable=True)
    k = m.topk
    tie = (sp[:, 0, k - 1] - sp[:, 0, k]) <= rel * sp[:, 0, k - 1]
    ind_k = ind[:, :, :k].sort(2, False)[0]
    att_topk = torch.gather(prob, 2, ind_k)
    samples = ind_k.squeeze(1).float()
    cl, cr = m.concat_feature(fl[0]), m.concat_feature(fr[0])
    vol = torch.cat((cl.unsqueeze(2).expand(-1, -1, samples.shape[1], -1, -1), warp_right(cr, samples)), 1)
    vol = m.concat_feature_att_4(m.concat_stem(att_topk * vol), fl[0])
    cost = m.hourglass(vol, fl).squeeze(1)
    sc, ci = cost.sort(dim=1, descending=True, stable=True)
    spread = (sc[:, 0] - sc[:, -1]).clamp_min(1e-12)
    tie = tie | ((sc[:, 1] - sc[:, 2]) <= rel * spread)
    pi = ci[:, :2]
    p2 = F.softmax(torch.gather(cost, 1, pi), 1)
    pred = (torch.gather(samples, 1, pi) * p2).sum(1, keepdim=True)
    xspx = m.spx_2(m.spx_4(fl[0]), stem_2x)
    spx_pred = F.softmax(m.spx(xspx), 1)
    disp = context_upsample(pred, spx_pred) * 4
    tie = F.max_pool2d(tie.float().unsqueeze(1), 3, 1, 1)  # the upsampling reads each 1/4 pixel's 3x3 neighbours
    tie = F.interpolate(tie, scale_factor=4, mode="nearest")[:, 0] > 0
    return disp, tie


def forward_forced(m: FastACVNetPlus, left, right, samples, top2=None):
    """Teacher-forced forward pass: every continuous stage is computed here in fp32 from the images, the two
    discrete selections are taken from the caller -- ``samples`` [B,k,h,w] (the top-k disparity indices,
    ascending) and optionally ``top2`` [B,2,h,w] (the candidate slots of the final regression; default: this
    pass's own top-2).  Returns (disparity [B,H,W], attention logits [B,D,h,w], cost logits [B,k,h,w]) so a test
    can check that the forced selections are legitimate top-k / top-2 choices of the oracle's own logits (up to
    a near-tie tolerance) and that everything else tracks the oracle end to end."""
    fl, fr = m.feature_up(m.feature(left), m.feature(right))
    stem_2x, stem_2y = m.stem_2(left), m.stem_2(right)
    stem_4x, stem_4y = m.stem_4(stem_2x), m.stem_4(stem_2y)
    fl[0] = torch.cat((fl[0], stem_4x), 1)
    fr[0] = torch.cat((fr[0], stem_4y), 1)
    match_l, match_r = m.desc(m.conv(fl[0])), m.desc(m.conv(fr[0]))
    corr = m.corr_stem(norm_correlation_volume(match_l, match_r, m.maxdisp // 4))
    att_weights = m.hourglass_att(m.corr_feature_att_4(corr, fl[0]), fl)
    prob = F.softmax(att_weights, dim=2)
    ind_k = samples.long().unsqueeze(1)
    att_topk = torch.gather(prob, 2, ind_k)
    samples = samples.float()
    cl, cr = m.concat_feature(fl[0]), m.concat_feature(fr[0])
    vol = torch.cat((cl.unsqueeze(2).expand(-1, -1, samples.shape[1], -1, -1), warp_right(cr, samples)), 1)
    vol = m.concat_feature_att_4(m.concat_stem(att_topk * vol), fl[0])
    cost = m.hourglass(vol, fl).squeeze(1)
    pi = top2.long() if top2 is not None else cost.sort(dim=1, descending=True, stable=True)[1][:, :2]
    p2 = F.softmax(torch.gather(cost, 1, pi), 1)
    pred = (torch.gather(samples, 1, pi) * p2).sum(1, keepdim=True)
    xspx = m.spx_2(m.spx_4(fl[0]), stem_2x)
    spx_pred = F.softmax(m.spx(xspx), 1)
    return context_upsample(pred, spx_pred) * 4, att_weights[:, 0], cost


def build(preset: str = "fastacvnet-plus", seed: int = 0) -> FastACVNetPlus:
    torch.manual_seed(seed)
    m = FastACVNetPlus(**PRESETS[preset]).eval()
    randomize_norm_stats(m, seed)
    for mod in m.modules():  # 3-D batch norms too
        if isinstance(mod, nn.BatchNorm3d):
            g = torch.Generator().manual_seed(seed + mod.num_features)
            with torch.no_grad():
                mod.weight.copy_(0.75 + 0.5 * torch.rand(mod.num_features, generator=g))
                mod.bias.copy_(0.1 * torch.randn(mod.num_features, generator=g))
                mod.running_mean.copy_(0.1 * torch.randn(mod.num_features, generator=g))
                mod.running_var.copy_(0.75 + 0.5 * torch.rand(mod.num_features, generator=g))
    return m


def sharpen(m: FastACVNetPlus, factor: float = 100.0) -> FastACVNetPlus:
    """Scale the two cost heads (hourglass ``conv1_up``) so a random-init network has peaked softmaxes.
    With random weights the attention / cost logits are ~1e-2 and nearly flat, so the top-24 and top-2
    selections flip on fp16 rounding; trained networks are peaked.  Used by the numerics tests so the
    engine-vs-oracle comparison measures arithmetic error, not tie-breaking."""
    with torch.no_grad():
        m.hourglass_att.conv1_up.conv.weight.mul_(factor)
        m.hourglass.conv1_up.conv.weight.mul_(factor)
    return m
