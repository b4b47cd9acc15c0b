"""Torch-facing wrappers over the hand-written HIP kernels (NHWC fp16 on the GPU).

These are thin: they validate shapes, pack weights, fill the C launch structs and launch on the
current torch stream.  Used by the numerics tests (each op vs. a PyTorch fp32 reference) and by
Python-level tooling; the production path is the native engine (``models.engine``).
"""
from __future__ import annotations

import ctypes as C
import math
from typing import Sequence

import torch

from .. import _native as N

__all__ = [
    "splitk_workspace", "pack_conv_weight", "conv2d", "flow_head_tail", "flow_head_tail2", "stats_reduce", "instnorm_apply", "avgpool3s2", "avgpool_k", "interp_bilinear",
    "corr1d_pyramid", "corr1d_lookup", "raft_motion_head", "convex_upsample", "preprocess", "remap_bgr", "reproject",
    "agcl_corr", "linear_attention", "layernorm", "ew", "interp_flow", "convex_upsample_c",
    "pack_conv3d_weight", "deconv_as_conv_weight", "conv3d", "dwconv3x3", "norm_corr_volume", "topk_disparity",
    "concat_volume", "topk_regress", "spx_upsample",
]


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ptr(t: torch.Tensor | None):
    return C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)


def _pix_stride(t: torch.Tensor) -> int:
    """NHWC tensor (possibly a channel slice): elements between consecutive pixels."""
    assert t.dim() == 4 and t.stride(3) == 1, "expect NHWC with unit channel stride"
    n, h, w, c = t.shape
    s = t.stride(2)
    assert t.stride(1) == w * s and (n == 1 or t.stride(0) == h * w * s), "pixels must be uniformly strided"
    return s


def stats_reduce(stats, slots):
    """Fold ``slots`` copies of instance-norm statistics into copy 0 (copies 1.. are cleared)."""
    N.check(N.dev().sa_stats_reduce(stats.data_ptr(), slots, stats.numel() // slots, _stream()), "sa_stats_reduce")
    return stats


def flow_head_tail(y, w, bias, flow):
    """Fused tap projection + 3x3 stencil of a C -> 1 conv: fp16 NHWC ``y`` [n,h,w,C] (pixel stride may exceed C),
    ``w`` [9, C] (tap ky*3+kx), fp32 ``flow`` [n,h,w] += bias + conv(y) in place."""
    n, h, wd, c = y.shape
    w16 = torch.zeros(16, c, dtype=torch.float16, device=y.device)
    w16[:9] = w.to(torch.float16)
    assert flow.dtype == torch.float32 and flow.is_contiguous() and flow.shape == (n, h, wd)
    N.check(N.dev().sa_flow_head_tail(y.data_ptr(), _pix_stride(y), c, w16.data_ptr(), bias.data_ptr(),
                                      flow.data_ptr(), n, h, wd, _stream()), "sa_flow_head_tail")
    return flow


def flow_head_tail2(y, w, bias, flow):
    """Two-channel variant (CREStereo's flow head conv2 256 -> 2): ``w`` [2, C, 3, 3], fp32 ``flow`` [n,h,w,2]
    += bias + conv(y) in place."""
    n, h, wd, c = y.shape
    w16 = torch.zeros(32, c, dtype=torch.float16, device=y.device)
    w16[:18] = w.permute(2, 3, 0, 1).reshape(18, c).to(torch.float16)  # row (ky*3+kx)*2 + o
    assert flow.dtype == torch.float32 and flow.is_contiguous() and flow.shape == (n, h, wd, 2)
    N.check(N.dev().sa_flow_head_tail_oc(y.data_ptr(), _pix_stride(y), c, w16.data_ptr(), 2, bias.data_ptr(),
                                         flow.data_ptr(), n, h, wd, _stream()), "sa_flow_head_tail_oc")
    return flow


def raft_motion_head(pyr_buf, flow, b, h, w1, w2, convc1_w, convc1_b, convf1_w, convf1_b, levels=4, radius=4):
    """Fused lookup + relu(convc1) + relu(convf1 on [flow_x, 0]): returns (cor1, flo1, flowcopy) fp16
    NHWC.  ``convc1_w`` [64, L*(2r+1), 1, 1], ``convf1_w`` [64, 2, 7, 7] (torch layouts)."""
    nc = levels * (2 * radius + 1)
    wc = convc1_w.reshape(64, nc).t().contiguous().float()
    wf = convf1_w[:, 0].reshape(64, 49).t().contiguous().float()
    dev = flow.device
    cor = torch.empty(b, h, w1, 64, dtype=torch.float16, device=dev)
    flo = torch.empty(b, h, w1, 64, dtype=torch.float16, device=dev)
    fc = torch.empty(b, h, w1, 8, dtype=torch.float16, device=dev)
    N.check(N.dev().sa_raft_motion_head(pyr_buf.data_ptr(), flow.contiguous().data_ptr(), b, h, w1, w2, levels, radius,
                                        wc.data_ptr(), convc1_b.float().contiguous().data_ptr(), wf.data_ptr(),
                                        convf1_b.float().contiguous().data_ptr(), cor.data_ptr(), 64, flo.data_ptr(),
                                        64, fc.data_ptr(), 8, _stream()), "sa_raft_motion_head")
    return cor, flo, fc[..., :2]


def raft_motion_encoder(pyr_buf, flow, b, h, w1, w2, convc1_w, convc1_b, convf1_w, convf1_b, convc2_w, convc2_b,
                        convf2_w, convf2_b, conv_w, conv_b, levels=4, radius=4, variant=-1):
    """The fused RAFT motion encoder (sa_raft_motion_encoder): fp16 NHWC [b, h, w1, 128] =
    [relu(conv([relu(convc2(cor1)), relu(convf2(flo1))])) (126) | flow_x | 0].  Torch-layout weights."""
    nc = levels * (2 * radius + 1)
    dev = flow.device
    wb = torch.zeros(128, 96, dtype=torch.float32, device=dev)  # block-diagonal stage-1 B
    wb[:64, :nc] = convc1_w.reshape(64, nc).float()
    wb[64:, nc:nc + 49] = convf1_w[:, 0].reshape(64, 49).float()
    wb = wb.half().contiguous()
    b1 = torch.cat([convc1_b.float(), convf1_b.float()]).contiguous()
    w2c, kc, _ = pack_conv_weight(convc2_w)
    w2f, kf, _ = pack_conv_weight(convf2_w)
    w3, k3, _ = pack_conv_weight(conv_w)
    assert kc == 576 and kf == 576 and k3 == 1152
    out = torch.empty(b, h, w1, 128, dtype=torch.float16, device=dev)
    f = lambda t: t.float().contiguous()
    bias = [f(convc2_b), f(convf2_b), f(conv_b)]
    N.dev().sa_raft_motion_encoder_variant(variant)
    N.check(N.dev().sa_raft_motion_encoder(pyr_buf.data_ptr(), flow.contiguous().data_ptr(), b, h, w1, w2, levels,
                                           radius, wb.data_ptr(), b1.data_ptr(), w2c.data_ptr(), bias[0].data_ptr(),
                                           w2f.data_ptr(), bias[1].data_ptr(), w3.data_ptr(), bias[2].data_ptr(),
                                           out.data_ptr(), 128, _stream()), "sa_raft_motion_encoder")
    N.dev().sa_raft_motion_encoder_variant(-1)
    return out


def splitk_workspace(floats: int = 1 << 22, counters: int = 4096, device="cuda"):
    return (torch.empty(floats, dtype=torch.float32, device=device),
            torch.zeros(counters, dtype=torch.int32, device=device))


def pack_conv_weight(w: torch.Tensor, segs: Sequence[tuple[int, int]] | None = None):
    """[Cout, Cin, KH, KW] -> fp16 [round_up(Cout,128), Kpad], K ordered (kh, kw, ci_padded)."""
    cout, cin, kh, kw = w.shape
    segs = list(segs) if segs else [(cin, (cin + 7) // 8 * 8)]
    assert sum(r for r, _ in segs) == cin
    cin_pad = sum(p for _, p in segs)
    wp = torch.zeros(cout, kh, kw, cin_pad, dtype=torch.float32, device=w.device)
    rc = pc = 0
    wt = w.permute(0, 2, 3, 1).float()
    for r, p in segs:
        wp[..., pc:pc + r] = wt[..., rc:rc + r]
        rc += r
        pc += p
    k = kh * kw * cin_pad
    kpad = (k + 63) // 64 * 64  # 64-aligned K -> DMA-staged BK=64 kernel path
    cpad = (cout + 127) // 128 * 128
    out = torch.zeros(cpad, kpad, dtype=torch.float16, device=w.device)
    out[:cout, :k] = wp.reshape(cout, k).half()
    return out.contiguous(), kpad, cin_pad


def conv2d(xs, wpacked, kpad, cout, kh, kw, bias=None, stride=1, pad=None, dil=1, act="none",
           act2="none", res=None, out=None, epi="store", scale=1.0, alpha=0.01, stats=None,
           ctx=None, aux=None, hbuf=None, rh=None, tile_cfg=-1, splitk=1, workspace=None, up=0, cout_real=0,
           gate=None, stats_slots=1, cin_real=0, tapw=None, taps=0, launch=True, in_stats=None, in_slots=1,
           in_eps=1e-5):
    """NHWC fp16 implicit-GEMM conv.  ``splitk``: 1 = off, 0 = auto, >1 = forced; needs
    ``workspace`` = (fp32 slab tensor, int32 counter tensor zero-initialised).  ``up`` = 2: transposed
    conv, the 4 parity classes (cout = 4 * cout_real) are scattered to a 2x output.  ``gate``: fp16
    NHWC multiplier applied after the activation.  ``in_stats`` (int64 [in_slots][N][Cin][2], the direct
    64-channel kernel only): ``xs`` is a conv's raw output and the conv reads relu(IN(xs)) instead."""
    if isinstance(xs, torch.Tensor):
        xs = [xs]
    n, h, w, _ = xs[0].shape
    sh = sw = stride if isinstance(stride, int) else None
    if sh is None:
        sh, sw = stride
    if pad is None:
        ph, pw = (kh // 2) * dil, (kw // 2) * dil
    elif isinstance(pad, int):
        ph = pw = pad
    else:
        ph, pw = pad
    ho = (h + 2 * ph - dil * (kh - 1) - 1) // sh + 1
    wo = (w + 2 * pw - dil * (kw - 1) - 1) // sw + 1
    a = N.SaConvArgs()
    cin = 0
    for i, x in enumerate(xs):
        assert x.dtype == torch.float16 and x.is_cuda
        a.src[i].ptr = x.data_ptr()
        a.src[i].channels = x.shape[3]
        a.src[i].stride = _pix_stride(x)
        cin += x.shape[3]
    a.nsrc = len(xs)
    a.cin_real = cin_real  # single zero-padded source: real channels (the 7x7 stem kernel stages only those)
    a.N, a.H, a.W, a.Cin = n, h, w, cin
    a.KH, a.KW, a.sh, a.sw, a.ph, a.pw, a.dh, a.dw = kh, kw, sh, sw, ph, pw, dil, dil
    a.Ho, a.Wo = ho, wo
    if out is None:
        dt = torch.float32 if epi == "store_f32" else torch.float16
        if up:
            out = torch.empty(n, 2 * ho, 2 * wo, cout_real, dtype=dt, device=xs[0].device)
        else:
            out = torch.empty(n, ho, wo, cout, dtype=dt, device=xs[0].device)
    a.up, a.cout_real = up, cout_real
    if gate is not None:
        a.gate, a.gate_stride = gate.data_ptr(), _pix_stride(gate)
    a.weight = wpacked.data_ptr()
    a.bias = bias.data_ptr() if bias is not None else None
    a.Cout, a.Kpad = cout, kpad
    a.out = out.data_ptr() if out is not None else None
    a.out_stride = (out.stride(2) if out.dim() == 4 else 1) if out is not None else 0
    a.epi, a.act, a.act2 = N.EPI[epi], N.ACT[act], N.ACT[act2]
    a.alpha, a.scale = alpha, scale
    if res is not None:
        a.res, a.res_stride = res.data_ptr(), _pix_stride(res)
    if ctx is not None:
        a.ctx, a.ctx_stride = ctx.data_ptr(), _pix_stride(ctx)
    if aux is not None:
        a.aux, a.aux_stride = aux.data_ptr(), _pix_stride(aux)
    if hbuf is not None:
        a.hbuf, a.h_stride = hbuf.data_ptr(), _pix_stride(hbuf)
    if rh is not None:
        a.rh, a.rh_stride = rh.data_ptr(), _pix_stride(rh)
    if stats is not None:
        assert stats.dtype == torch.int64  # fixed point, value * 2^24
        a.stats = stats.data_ptr()
        a.stats_slots = stats_slots
    if tapw is not None:  # epi "tapproj": fp16 [taps][cout] projection weights; out fp32 [n,h,w,(cout//128)*taps]
        a.tapw, a.taps = tapw.data_ptr(), taps
    if in_stats is not None:
        assert in_stats.dtype == torch.int64
        a.in_stats, a.in_slots, a.in_eps = in_stats.data_ptr(), in_slots, in_eps
    a.tile_cfg = tile_cfg
    a.splitk = splitk
    if workspace is not None:
        ws, cnt = workspace
        assert ws.dtype == torch.float32 and cnt.dtype == torch.int32
        a.ws, a.counters, a.ws_floats, a.n_counters = ws.data_ptr(), cnt.data_ptr(), ws.numel(), cnt.numel()
    if not launch:  # the filled SaConvArgs (e.g. for gru_level), nothing enqueued
        return a
    N.check(N.dev().sa_conv2d(C.byref(a), _stream()), "sa_conv2d")
    return out


def gru_level(za, qa, bar, grid=128):
    """One ConvGRU level in one launch (sa_gru_level): ``za`` / ``qa`` are conv2d(..., launch=False) args of the
    z/r(/q-x) conv (epi gru_zr / gru_zrq) and the q conv (epi gru_q), both with a split-K workspace; ``bar`` an int32
    tensor of 4 zeros owned by this level (grid barrier words, [2] = timeout flag)."""
    assert bar.dtype == torch.int32 and bar.numel() >= 4 and bar.is_cuda
    N.check(N.dev().sa_gru_level(C.byref(za), C.byref(qa), bar.data_ptr(), int(grid), _stream()), "sa_gru_level")


def tapproj_stencil(P, taps, oc, bias, flow):
    """flow [n,h,w,oc] fp32 += bias + 3x3 neighbourhood sums of the two n-tile partials in P [n,h,w,2*taps]."""
    n, h, w, _ = flow.shape
    N.check(N.dev().sa_tapproj_stencil(P.data_ptr(), taps, oc, bias.data_ptr() if bias is not None else None,
                                       flow.data_ptr(), n, h, w, _stream()), "sa_tapproj_stencil")
    return flow


def instnorm_apply(x, stats, act="none", res=None, res_stats=None, act2="none", eps=1e-5, out=None, slots=1,
                   res_act="none"):
    """slots > 1: stats (and res_stats) hold that many [N][C][2] copies, summed by the kernel.  ``res_act``: the
    activation of the normalised residual (with ``res_stats``)."""
    n, h, w, c = x.shape
    out = torch.empty_like(x) if out is None else out
    a = N.SaNormArgs()
    a.x, a.x_stride = x.data_ptr(), _pix_stride(x)
    a.stats = stats.data_ptr()
    if res is not None:
        a.res, a.res_stride = res.data_ptr(), _pix_stride(res)
    if res_stats is not None:
        a.res_stats = res_stats.data_ptr()
    a.out, a.out_stride = out.data_ptr(), _pix_stride(out)
    a.N, a.HW, a.C = n, h * w, c
    a.act, a.act2 = N.ACT[act], N.ACT[act2]
    a.eps, a.alpha = eps, 0.01
    a.stat_slots = slots
    a.res_act = N.ACT[res_act]
    N.check(N.dev().sa_instnorm_apply(C.byref(a), _stream()), "sa_instnorm_apply")
    return out


def avgpool3s2(x, out=None):
    n, h, w, c = x.shape
    ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    out = torch.empty(n, ho, wo, c, dtype=x.dtype, device=x.device) if out is None else out
    N.check(N.dev().sa_avgpool3s2(_ptr(x), _pix_stride(x), _ptr(out), _pix_stride(out), n, h, w, c,
                                  _stream()), "avgpool3s2")
    return out


def avgpool_k(x, k, out=None):
    n, h, w, c = x.shape
    out = torch.empty(n, h // k, w // k, c, dtype=x.dtype, device=x.device) if out is None else out
    N.check(N.dev().sa_avgpool_k(_ptr(x), _pix_stride(x), _ptr(out), _pix_stride(out), n, h, w, c, k,
                                 _stream()), "avgpool_k")
    return out


def interp_bilinear(x, size, align_corners=True, mul=1.0, out=None):
    n, h, w, c = x.shape
    ho, wo = size
    out = torch.empty(n, ho, wo, c, dtype=x.dtype, device=x.device) if out is None else out
    N.check(N.dev().sa_interp_bilinear(_ptr(x), _pix_stride(x), _ptr(out), _pix_stride(out), n, h, w, c,
                                       ho, wo, int(align_corners), float(mul), _stream()), "interp")
    return out


def corr1d_pyramid(f1, f2, levels=4):
    """f1, f2: [B,H,W,C] fp16 -> list of fp32 levels [B,H,W1,W2>>l] (views of one buffer)."""
    b, h, w1, c = f1.shape
    w2 = f2.shape[2]
    sizes = []
    wl = w2
    for _ in range(levels):
        sizes.append(wl)
        wl >>= 1
    buf = torch.empty(sum(b * h * w1 * s for s in sizes), dtype=torch.float32, device=f1.device)
    assert f1.is_contiguous() and f2.is_contiguous()
    N.check(N.dev().sa_corr1d_pyramid(_ptr(f1), _ptr(f2), c, b, h, w1, w2, c, levels, _ptr(buf), _stream()),
            "corr1d_pyramid")
    out, off = [], 0
    for s in sizes:
        out.append(buf[off:off + b * h * w1 * s].view(b, h, w1, s))
        off += b * h * w1 * s
    return buf, out


def corr1d_lookup(pyr_buf, flow, b, h, w1, w2, levels=4, radius=4, out_channels=None,
                  flow_out=None, flow_out2=None):
    nfeat = levels * (2 * radius + 1)
    oc = out_channels or (nfeat + 7) // 8 * 8
    out = torch.empty(b, h, w1, oc, dtype=torch.float16, device=flow.device)
    fo_ptr, fo_s, fo_c = (0, 0, 0) if flow_out is None else (flow_out.data_ptr(), _pix_stride(flow_out), flow_out.shape[3])
    fo2_ptr, fo2_s = (0, 0) if flow_out2 is None else (flow_out2.data_ptr(), _pix_stride(flow_out2))
    N.check(N.dev().sa_corr1d_lookup(_ptr(pyr_buf), _ptr(flow), b, h, w1, w2, levels, radius, _ptr(out), oc, oc,
                                     C.c_void_p(fo_ptr), fo_s, fo_c, C.c_void_p(fo2_ptr), fo2_s, _stream()),
            "corr1d_lookup")
    return out


def convex_upsample(mask, flow, factor, sign=1.0):
    b, h, w, _ = mask.shape
    out = torch.empty(b, h * factor, w * factor, dtype=torch.float32, device=mask.device)
    N.check(N.dev().sa_convex_upsample(_ptr(mask), _pix_stride(mask), _ptr(flow), b, h, w, factor, float(sign),
                                       _ptr(out), _stream()), "convex_upsample")
    return out


def preprocess(bgr, mode="signed", out=None, c_off=0, zero_to=8, out_channels=8):
    b, h, w, _ = bgr.shape
    assert bgr.dtype == torch.uint8 and bgr.is_contiguous()
    out = torch.zeros(b, h, w, out_channels, dtype=torch.float16, device=bgr.device) if out is None else out
    N.check(N.dev().sa_preprocess(_ptr(bgr), b, h, w, N.PRE[mode], _ptr(out), _pix_stride(out), c_off, zero_to,
                                  _stream()), "preprocess")
    return out


def remap_bgr(src, maps):
    """src u8 [B,Hs,Ws,3]; maps fp32 [nmaps,H,W,2] (x, y) -> [B,H,W,3]"""
    b, hs, ws, _ = src.shape
    nm, h, w, _ = maps.shape
    out = torch.empty(b, h, w, 3, dtype=torch.uint8, device=src.device)
    N.check(N.dev().sa_remap_bgr(_ptr(src), b, hs, ws, _ptr(maps.contiguous()), nm, h, w, _ptr(out), _stream()),
            "remap")
    return out


def reproject(disp, left_bgr, Q, sign=1.0):
    """disp fp32 [B,H,W]; Q 4x4 (host array-like) -> (signed disparity, cloud [B,H,W,6])"""
    b, h, w = disp.shape
    q = (C.c_float * 16)(*[float(v) for v in torch.as_tensor(Q, dtype=torch.float64).flatten().tolist()])
    dout = torch.empty_like(disp)
    cloud = torch.empty(b, h, w, 6, dtype=torch.float32, device=disp.device)
    N.check(N.dev().sa_reproject(_ptr(disp.contiguous()), 1, float(sign), _ptr(left_bgr.contiguous()), b, h, w,
                                 C.cast(q, C.c_void_p), _ptr(dout), _ptr(cloud), _stream()), "reproject")
    return dout, cloud


# ------------------------------------------------------------------------------ CREStereo ops
def agcl_corr(f1, f2, flow, offset=None, small_patch=False, iter_mode=False, out_channels=40):
    """f1/f2: fp16 NHWC [N,H,W,C]; flow fp32 [N,H,W,2]; offset fp16 [N,H,W,>=18] -> fp16 [N,H,W,oc]."""
    n, h, w, c = f1.shape
    out = torch.empty(n, h, w, out_channels, dtype=torch.float16, device=f1.device)
    a = N.SaAgclArgs()
    a.f1, a.f1_stride = f1.data_ptr(), _pix_stride(f1)
    a.f2, a.f2_stride = f2.data_ptr(), _pix_stride(f2)
    assert flow.dtype == torch.float32 and flow.is_contiguous() and flow.shape == (n, h, w, 2)
    a.flow = flow.data_ptr()
    if offset is not None:
        a.offset, a.offset_stride = offset.data_ptr(), _pix_stride(offset)
    a.N, a.H, a.W, a.C = n, h, w, c
    a.small_patch, a.iter_mode = int(small_patch), int(iter_mode)
    a.out, a.out_stride, a.out_channels = out.data_ptr(), out_channels, out_channels
    N.check(N.dev().sa_agcl_corr(C.byref(a), _stream()), "sa_agcl_corr")
    return out


def agcl_conv1x1(f1, f2, flow, weight, bias, small_patch=False):
    """Iter-mode AGCL fused with a 1x1 conv 36 -> 256 + bias + relu (CREStereo's convc1): f1/f2 fp16 NHWC
    [N,H,W,256], flow fp32 [N,H,W,2], weight [256,36(,1,1)], bias [256] -> fp16 [N,H,W,256]."""
    n, h, w, c = f1.shape
    w2 = weight.reshape(weight.shape[0], -1)
    assert w2.shape == (256, 36) and bias.shape == (256,)
    w16 = torch.zeros(256, 64, dtype=torch.float16, device=f1.device)
    w16[:, :36] = w2.to(torch.float16)
    b32 = bias.float().contiguous()
    out = torch.empty(n, h, w, 256, dtype=torch.float16, device=f1.device)
    a = N.SaAgclArgs()
    a.f1, a.f1_stride = f1.data_ptr(), _pix_stride(f1)
    a.f2, a.f2_stride = f2.data_ptr(), _pix_stride(f2)
    assert flow.dtype == torch.float32 and flow.is_contiguous() and flow.shape == (n, h, w, 2)
    a.flow = flow.data_ptr()
    a.N, a.H, a.W, a.C = n, h, w, c
    a.small_patch, a.iter_mode = int(small_patch), 1
    N.check(N.dev().sa_agcl_conv1x1(C.byref(a), w16.data_ptr(), b32.data_ptr(), 256, out.data_ptr(), 256, _stream()),
            "sa_agcl_conv1x1")
    return out


def cre_motion_head_pre(corr, flow, wc, bc, wf, bf):
    """cre_motion_head from a correlation already computed (offset mode: agcl_corr first): corr fp16 [N,H,W,>=36]
    (pixel stride = its last dim), flow fp32 [N,H,W,2] -> (cor [N,H,W,256], flo [N,H,W,128], fcopy [N,H,W,2])."""
    n, h, w, cc = corr.shape
    dev = corr.device
    wc16 = torch.zeros(256, 64, dtype=torch.float16, device=dev)
    wc16[:, :36] = wc.reshape(256, 36).to(torch.float16)
    wf16 = torch.zeros(128, 128, dtype=torch.float16, device=dev)
    wf16[:, :98] = wf.reshape(128, 98).to(torch.float16)
    bc32, bf32 = bc.float().contiguous(), bf.float().contiguous()
    cor = torch.empty(n, h, w, 256, dtype=torch.float16, device=dev)
    flo = torch.empty(n, h, w, 128, dtype=torch.float16, device=dev)
    fcopy = torch.empty(n, h, w, 2, dtype=torch.float16, device=dev)
    assert corr.dtype == torch.float16 and corr.is_contiguous() and cc >= 36
    assert flow.dtype == torch.float32 and flow.is_contiguous() and flow.shape == (n, h, w, 2)
    a = N.SaAgclArgs()
    a.flow = flow.data_ptr()
    a.N, a.H, a.W, a.C = n, h, w, 256
    a.out, a.out_stride, a.out_channels = corr.data_ptr(), cc, 36
    hd = N.SaCreHeadArgs()
    hd.w16, hd.bias, hd.cor, hd.cor_stride = wc16.data_ptr(), bc32.data_ptr(), cor.data_ptr(), 256
    hd.wf16, hd.fbias, hd.flo, hd.flo_stride = wf16.data_ptr(), bf32.data_ptr(), flo.data_ptr(), 128
    hd.fcopy, hd.fcopy_stride = fcopy.data_ptr(), 2
    N.check(N.dev().sa_cre_motion_head_pre(C.byref(a), C.byref(hd), _stream()), "sa_cre_motion_head_pre")
    return cor, flo, fcopy


def cre_motion_head(f1, f2, flow, wc, bc, wf, bf, small_patch=False):
    """CREStereo motion-encoder head in one launch (iter mode): relu(convc1(AGCL)) -> [N,H,W,256], relu(convf1(flow))
    -> [N,H,W,128] (7x7, pad 3) and the fp16 flow copy -> [N,H,W,2].  wc [256,36(,1,1)], wf [128,2,7,7]."""
    n, h, w, c = f1.shape
    dev = f1.device
    wc16 = torch.zeros(256, 64, dtype=torch.float16, device=dev)
    wc16[:, :36] = wc.reshape(256, 36).to(torch.float16)
    wf16 = torch.zeros(128, 128, dtype=torch.float16, device=dev)
    wf16[:, :98] = wf.reshape(128, 98).to(torch.float16)  # k = c * 49 + ky * 7 + kx
    bc32, bf32 = bc.float().contiguous(), bf.float().contiguous()
    cor = torch.empty(n, h, w, 256, dtype=torch.float16, device=dev)
    flo = torch.empty(n, h, w, 128, dtype=torch.float16, device=dev)
    fcopy = torch.empty(n, h, w, 2, dtype=torch.float16, device=dev)
    a = N.SaAgclArgs()
    a.f1, a.f1_stride = f1.data_ptr(), _pix_stride(f1)
    a.f2, a.f2_stride = f2.data_ptr(), _pix_stride(f2)
    assert flow.dtype == torch.float32 and flow.is_contiguous() and flow.shape == (n, h, w, 2)
    a.flow = flow.data_ptr()
    a.N, a.H, a.W, a.C = n, h, w, c
    a.small_patch, a.iter_mode = int(small_patch), 1
    hd = N.SaCreHeadArgs()
    hd.w16, hd.bias, hd.cor, hd.cor_stride = wc16.data_ptr(), bc32.data_ptr(), cor.data_ptr(), 256
    hd.wf16, hd.fbias, hd.flo, hd.flo_stride = wf16.data_ptr(), bf32.data_ptr(), flo.data_ptr(), 128
    hd.fcopy, hd.fcopy_stride = fcopy.data_ptr(), 2
    N.check(N.dev().sa_cre_motion_head(C.byref(a), C.byref(hd), _stream()), "sa_cre_motion_head")
    return cor, flo, fcopy


def linear_attention(q, k, v, heads=8, eps=1e-6):
    """q: fp16 [N, L, heads*dim], k/v: [N, S, heads*dim] (last dim may be a slice) -> fp16 [N, L, heads*dim]."""
    n, l, d = q.shape
    s = k.shape[1]
    out = torch.empty(n, l, d, dtype=torch.float16, device=q.device)
    ws = torch.empty(N.dev().sa_linear_attention_ws_floats(n, s, heads, d // heads), dtype=torch.float32,
                     device=q.device)
    N.check(N.dev().sa_linear_attention(_ptr(q), q.stride(1), _ptr(k), k.stride(1), _ptr(v), v.stride(1), _ptr(out),
                                        out.stride(1), n, l, s, heads, d // heads, eps, _ptr(ws), _stream()),
            "sa_linear_attention")
    return out


def layernorm(x, gamma, beta, res=None, eps=1e-5):
    rows, c = x.shape[0] * x.shape[1], x.shape[-1]
    out = torch.empty_like(x)
    N.check(N.dev().sa_layernorm(_ptr(x), x.stride(1), _ptr(gamma), _ptr(beta), _ptr(res),
                                 res.stride(1) if res is not None else 0, _ptr(out), out.stride(1), rows, c, eps,
                                 _stream()), "sa_layernorm")
    return out


def ew(x, act="none", scale=1.0, add=None, bcast=None, period=1):
    """x: fp16 NHWC (channel slices allowed) -> fp16 contiguous act(x*scale + add + bcast)."""
    n, h, w, c = x.shape
    out = torch.empty(n, h, w, c, dtype=torch.float16, device=x.device)
    a = N.SaEwArgs()
    a.x, a.x_stride = x.data_ptr(), _pix_stride(x)
    if add is not None:
        a.add, a.add_stride = add.data_ptr(), _pix_stride(add)
    if bcast is not None:
        a.bcast, a.bcast_period = bcast.data_ptr(), period
    a.out, a.out_stride = out.data_ptr(), c
    a.P, a.C, a.act, a.scale = n * h * w, c, N.ACT[act], scale
    N.check(N.dev().sa_ew(C.byref(a), _stream()), "sa_ew")
    return out


def interp_flow(x, ho, wo, mul=1.0):
    n, h, w, c = x.shape
    out = torch.empty(n, ho, wo, c, dtype=torch.float32, device=x.device)
    N.check(N.dev().sa_interp_flow(_ptr(x), _ptr(out), n, h, w, c, ho, wo, mul, _stream()), "sa_interp_flow")
    return out


def convex_upsample_c(mask, flow, factor, sign=1.0, oc=2):
    n, h, w, fc = flow.shape
    out = torch.empty(n, h * factor, w * factor, oc, dtype=torch.float32, device=flow.device)
    N.check(N.dev().sa_convex_upsample_c(_ptr(mask), _pix_stride(mask), _ptr(flow), fc, n, h, w, factor, sign,
                                         _ptr(out), oc, _stream()), "sa_convex_upsample_c")
    return out


# ------------------------------------------------------------------------------ Fast-ACVNet+ ops
def pack_conv3d_weight(w: torch.Tensor, cin_pad: int | None = None):
    """[Cout, Cin, KD, KH, KW] -> fp16 [round_up(Cout,128), Kpad], K ordered (kd, kh, kw, ci_padded)."""
    cout, cin, kd, kh, kw = w.shape
    cin_pad = cin_pad or (cin + 7) // 8 * 8
    wp = torch.zeros(cout, kd, kh, kw, cin_pad, dtype=torch.float32, device=w.device)
    wp[..., :cin] = w.permute(0, 2, 3, 4, 1).float()
    k = kd * kh * kw * cin_pad
    kpad = (k + 63) // 64 * 64
    out = torch.zeros((cout + 127) // 128 * 128, kpad, dtype=torch.float16, device=w.device)
    out[:cout, :k] = wp.reshape(cout, k).half()
    return out.contiguous(), kpad, cin_pad


def deconv_as_conv_weight(wt: torch.Tensor) -> torch.Tensor:
    """ConvTranspose{2,3}d(k=4, s=2, p=1) weight [Cin, Cout, 4, 4(, 4)] -> equivalent 3x3(x3) stride-1 conv
    weight [P*Cout, Cin, (3,) 3, 3] whose output channel p*Cout + o is parity class p (bit0 = x, bit1 = y,
    bit2 = z) of output channel o:  out[2i + a] = sum_d in[i + d] * Wt[a + 1 - 2d], d in {-1, 0, 1}."""
    is3d = wt.dim() == 5
    ci, co = wt.shape[:2]
    npar = 8 if is3d else 4
    w = torch.zeros(npar * co, ci, *([3] * (3 if is3d else 2)), dtype=wt.dtype, device=wt.device)
    for p in range(npar):
        pb, pa, pc = p & 1, (p >> 1) & 1, p >> 2
        for dy in range(3):
            ky = pa + 1 - 2 * (dy - 1)
            for dx in range(3):
                kx = pb + 1 - 2 * (dx - 1)
                if not (0 <= ky < 4 and 0 <= kx < 4):
                    continue
                if not is3d:
                    w[p * co:(p + 1) * co, :, dy, dx] = wt[:, :, ky, kx].t()
                    continue
                for dz in range(3):
                    kz = pc + 1 - 2 * (dz - 1)
                    if 0 <= kz < 4:
                        w[p * co:(p + 1) * co, :, dz, dy, dx] = wt[:, :, kz, ky, kx].t()
    return w


def conv3d(x, wpacked, kpad, cout, k=3, stride=1, pad=None, bias=None, act="none", alpha=0.01, gate=None,
           up=0, cout_real=0, out=None, tile_cfg=-1, epi="store"):
    """NDHWC fp16 volume [N, D, H, W, C] conv (implicit GEMM over (kd, kh, kw, ci)).  ``gate``: fp16
    [N, H, W, >=cout] multiplied after the activation (broadcast over depth).  ``up`` = 3 scatters the
    8 parity classes of a transposed conv (cout = 8 * cout_real)."""
    n, d, h, w, c = x.shape
    assert x.dtype == torch.float16 and x.is_contiguous()
    pad = k // 2 if pad is None else pad
    a = N.SaConvArgs()
    a.src[0].ptr, a.src[0].channels, a.src[0].stride = x.data_ptr(), c, c
    a.nsrc = 1
    a.N, a.H, a.W, a.Cin = n, h, w, c
    a.KH = a.KW = a.KD = k
    a.sh = a.sw = a.sd = stride
    a.ph = a.pw = a.pd = pad
    a.dh = a.dw = 1
    a.Ho, a.Wo = (h + 2 * pad - k) // stride + 1, (w + 2 * pad - k) // stride + 1
    a.Di, a.Do = d, (d + 2 * pad - k) // stride + 1
    oc = cout_real if up else cout
    if out is None:
        shape = (n, 2 * a.Do, 2 * a.Ho, 2 * a.Wo, oc) if up else (n, a.Do, a.Ho, a.Wo, oc)
        out = torch.zeros(shape, dtype=torch.float32 if epi == "store_f32" else torch.float16, device=x.device)
    a.weight = wpacked.data_ptr()
    a.bias = bias.data_ptr() if bias is not None else None
    a.Cout, a.Kpad = cout, kpad
    a.out, a.out_stride = out.data_ptr(), out.shape[-1]
    a.epi, a.act, a.alpha, a.scale = N.EPI[epi], N.ACT[act], alpha, 1.0
    a.tile_cfg, a.splitk = tile_cfg, 1
    a.up, a.cout_real = up, cout_real
    if gate is not None:
        a.gate, a.gate_stride = gate.data_ptr(), _pix_stride(gate)
    N.check(N.dev().sa_conv2d(C.byref(a), _stream()), "sa_conv2d(3d)")
    return out


def dwconv3x3(x, w, b, stride=1, act="none"):
    """Depthwise 3x3 (pad 1) on fp16 NHWC; w fp32 [C, 9], b fp32 [C]."""
    n, h, wd, c = x.shape
    ho, wo = (h - 1) // stride + 1, (wd - 1) // stride + 1
    out = torch.empty(n, ho, wo, c, dtype=torch.float16, device=x.device)
    N.check(N.dev().sa_dwconv3x3(_ptr(x), _pix_stride(x), _ptr(w.float().contiguous()), _ptr(b.float().contiguous()),
                                 _ptr(out), c, n, h, wd, c, stride, N.ACT[act], _stream()), "sa_dwconv3x3")
    return out


def norm_corr_volume(l, r, D, out_channels=8):
    n, h, w, c = l.shape
    out = torch.empty(n, D, h, w, out_channels, dtype=torch.float16, device=l.device)
    N.check(N.dev().sa_norm_corr_volume(_ptr(l), _pix_stride(l), _ptr(r), _pix_stride(r), n, h, w, c, D, _ptr(out),
                                        out_channels, _stream()), "sa_norm_corr_volume")
    return out


def topk_disparity(att, K):
    """att: fp16 or fp32 volume [N, D, H, W, s] (channel 0) -> (prob, disp) fp32 [N, H, W, K]."""
    n, d, h, w, s = att.shape
    prob = torch.empty(n, h, w, K, dtype=torch.float32, device=att.device)
    disp = torch.empty_like(prob)
    f32 = int(att.dtype == torch.float32)
    N.check(N.dev().sa_topk_disparity(_ptr(att), s, f32, n, d, h, w, K, _ptr(prob), _ptr(disp), _stream()),
            "sa_topk_disparity")
    return prob, disp


def concat_volume(l, r, prob, disp, out_channels=None):
    n, h, w, c = l.shape
    K = prob.shape[-1]
    oc = out_channels or 2 * c
    out = torch.empty(n, K, h, w, oc, dtype=torch.float16, device=l.device)
    N.check(N.dev().sa_concat_volume(_ptr(l), _pix_stride(l), _ptr(r), _pix_stride(r), _ptr(prob), _ptr(disp), n, h, w,
                                     c, K, _ptr(out), oc, _stream()), "sa_concat_volume")
    return out


def topk_regress(cost, disp, top=2):
    """cost: fp16 or fp32 volume [N, K, H, W, s] (channel 0), disp fp32 [N, H, W, K] -> fp32 [N, H, W]."""
    n, k, h, w, s = cost.shape
    out = torch.empty(n, h, w, dtype=torch.float32, device=cost.device)
    f32 = int(cost.dtype == torch.float32)
    N.check(N.dev().sa_topk_regress(_ptr(cost), s, f32, _ptr(disp), n, k, h, w, top, _ptr(out), _stream()),
            "sa_topk_regress")
    return out


def spx_upsample(spx, pred, f=4, scale=4.0):
    """spx: fp16 NHWC [N, f*h, f*w, >=9] logits, pred fp32 [N, h, w] -> fp32 [N, f*h, f*w]."""
    n, h, w = pred.shape
    out = torch.empty(n, h * f, w * f, dtype=torch.float32, device=pred.device)
    N.check(N.dev().sa_spx_upsample(_ptr(spx), _pix_stride(spx), _ptr(pred.contiguous()), n, h, w, f, scale,
                                    _ptr(out), _stream()), "sa_spx_upsample")
    return out
